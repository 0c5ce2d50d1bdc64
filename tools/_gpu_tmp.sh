set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "weight_grad" > gpurun_out/r5w_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
