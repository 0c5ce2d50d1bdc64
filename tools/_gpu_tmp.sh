set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_stage1_gpu.py -x -v --timeout 400 --timeout-method thread -k "cfg2w or cfg2-2-128" > gpurun_out/r5e_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5e_tests.log | tail -3; grep -E "FAILED|Error|assert" gpurun_out/r5e_tests.log | head -10
grep -E "cfg2w|arch\[cfg2-bs2" gpurun_out/parity_metrics.jsonl | grep -E "d_proj\"|grad.model|loss" | head -30
exit $rc
