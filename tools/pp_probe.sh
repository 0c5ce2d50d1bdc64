#!/bin/bash
# Ping-pong 8-wave GEMM (mode 32) vs the persistent 4-wave GEMM (mode 8): bit-identity tests, then the
# step's w4 shapes timed on both paths (tools/gemm_probe.py).  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "pingpong" > gpurun_out/ppt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ppt.log; exit 1; }
tail -2 gpurun_out/ppt.log
for i in 1 2; do
  for shape in "22528 13824 1152 3" "22528 6912 1152 5" "22528 1152 1024 0" "22528 1536 1152 0" "18432 3072 1024 0"; do
    for mode in 8 32; do
      set -- $shape
      timeout -k 10 120 python tools/gemm_probe.py $1 $2 $3 $4 $mode 20 2>/dev/null || exit 1
    done
  done
done
