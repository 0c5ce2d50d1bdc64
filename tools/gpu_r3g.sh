#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ce_stats_gpu.py tests/test_kernels_gpu.py tests/test_stage1_gpu.py -k "ce_ or cross or golden or arch" > gpurun_out/r3g.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r3g.log | tail -1; grep -E "FAILED|Error" gpurun_out/r3g.log | head
[ $rc -eq 0 ] || exit $rc
for i in $(seq ${AB_REPS:-2}); do
  for e in PTK_CE_TWO_PASS=1 PTK_CE_TWO_PASS=0; do
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$e', d['value'], d['ms_per_step'], d['loss'])"
  done
done
