set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5y_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5y_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r5y_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5y_smoke.log 2>&1 || { echo smoke failed; tail -10 gpurun_out/r5y_smoke.log; exit 1; }
tail -2 gpurun_out/r5y_smoke.log
