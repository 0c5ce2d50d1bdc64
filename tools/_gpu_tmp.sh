set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r5z_tests.log; exit 1; }
tail -1 gpurun_out/r5z_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r5z_smoke.log; exit 1; }
grep smoke: gpurun_out/r5z_smoke.log
timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5z_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5z_cfg4.log; exit 1; }
tail -1 gpurun_out/r5z_cfg4.log | cut -c1-200
