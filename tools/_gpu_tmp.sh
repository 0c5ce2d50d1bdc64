set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5wg_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r5wg_tests.log; exit 1; }
tail -1 gpurun_out/r5wg_tests.log
