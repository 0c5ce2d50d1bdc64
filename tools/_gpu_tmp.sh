set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5m_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5m_cfg4.log; exit 1; }
tail -1 gpurun_out/r5m_cfg4.log | cut -c1-300
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" gpurun_out/r5m_tests.log | head -20; exit 1; }
tail -3 gpurun_out/r5m_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5m_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5m_bench.log; exit 1; }
tail -1 gpurun_out/r5m_bench.log | cut -c1-250
SH="g_qkv g_o g_dgu_dx g_down sig_qkv_b sig_fc1_b proj_fc1 proj_dA sq8192"
for r in 1 2; do
MODES=32 timeout -k 10 200 python -u tools/p8_probe.py $SH > gpurun_out/r5m_p8_base$r.log 2>&1 || { echo probe failed; tail -3 gpurun_out/r5m_p8_base$r.log; exit 1; }
PTK_LIB=ablibs/libptk_p8cread.so MODES=32 timeout -k 10 200 python -u tools/p8_probe.py $SH > gpurun_out/r5m_p8_cread$r.log 2>&1 || { echo probe failed; tail -3 gpurun_out/r5m_p8_cread$r.log; exit 1; }
done
paste -d' ' <(grep -o '"name": "[a-z0-9_]*\|"p8_us": [0-9.]*' gpurun_out/r5m_p8_base1.log | paste - -) <(grep -o '"p8_us": [0-9.]*' gpurun_out/r5m_p8_cread1.log) <(grep -o '"p8_us": [0-9.]*' gpurun_out/r5m_p8_base2.log) <(grep -o '"p8_us": [0-9.]*' gpurun_out/r5m_p8_cread2.log)
