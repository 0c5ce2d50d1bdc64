set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "p8_matches" > gpurun_out/r5g_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5g_tests.log | tail -3; grep -E "FAILED|Error|assert" gpurun_out/r5g_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
MODES=32,128,0 timeout -k 10 400 python -u tools/p8_probe.py g_gu_geglu g_dh_geglu_bwd g_down g_dgu_dx g_qkv g_o g_dO g_dqkv sig_qkv_b sig_o_br sig_fc1_b sig_fc2_br > gpurun_out/r5g_probe.log 2>&1 || { echo probe failed; tail -5 gpurun_out/r5g_probe.log; exit 1; }
grep -v amdgpu gpurun_out/r5g_probe.log
