#!/bin/bash
# new d-256 attention forward: kernel tests, then timing against the old kernel, then the step tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/r3c_attn.log 2>&1 || { echo "attn tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r3c_attn.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r3c_attn.log | tail -1
for i in 1 2; do
  echo "new"; timeout -k 10 60 python tools/attn_bench.py --what fwd 2>&1 | grep kernel || exit 1
  echo "old"; PTK_ATTN_FWD_OLD=1 timeout -k 10 60 python tools/attn_bench.py --what fwd 2>&1 | grep kernel || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_stage1_gpu.py tests/test_graph_gpu.py > gpurun_out/r3c_s1.log 2>&1; rc=$?
echo "stage1 rc=$rc"; grep -E "passed|failed" gpurun_out/r3c_s1.log | tail -1; grep FAILED gpurun_out/r3c_s1.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r3c_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3c_bench.log; exit 1; }
tail -1 gpurun_out/r3c_bench.log
