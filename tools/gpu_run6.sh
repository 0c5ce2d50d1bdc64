#!/bin/bash
# split-tail kernel: correctness tests, then the shape probe
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "split_tail or p8_matches" > gpurun_out/r6_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6_tests.log; exit 1; }
tail -3 gpurun_out/r6_tests.log
timeout -k 10 400 python -u tools/p8_probe.py > gpurun_out/r6_probe.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/r6_probe.log; exit 1; }
cat gpurun_out/r6_probe.log
