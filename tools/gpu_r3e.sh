#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/attn_debug.py 2>&1 | grep -v amdgpu.ids | grep -v "err by d" || exit 1
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/r3e_attn.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3e_attn.log | tail -1; grep FAILED gpurun_out/r3e_attn.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  echo "new"; timeout -k 10 60 python tools/attn_bench.py --what fwd,bwd 2>&1 | grep kernel || exit 1

done
