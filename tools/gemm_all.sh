#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "big_tile or all_epilogues or geglu or epilogues" > gpurun_out/w4t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w4t.log; exit 1; }
tail -1 gpurun_out/w4t.log
timeout -k 10 600 python tools/gemm_bench.py --all > gpurun_out/gall3.log 2>&1
