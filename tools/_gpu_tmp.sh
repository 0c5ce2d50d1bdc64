set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5m_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5m_cfg4.log; exit 1; }
tail -1 gpurun_out/r5m_cfg4.log | cut -c1-300
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" gpurun_out/r5m_tests.log | head -20; exit 1; }
tail -3 gpurun_out/r5m_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5m_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5m_bench.log; exit 1; }
tail -1 gpurun_out/r5m_bench.log | cut -c1-250
