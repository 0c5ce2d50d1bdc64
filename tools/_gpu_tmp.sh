set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1


SH="g_qkv g_o g_dgu_dx g_down sig_qkv_b sig_fc1_b sig_fc2 proj_fc1 proj_dA g_gu_geglu g_dh_geglu_bwd sq8192"
MODES=32,256 timeout -k 10 400 python -u tools/p8_probe.py $SH > gpurun_out/r5p_probe.log 2>&1 || { echo probe failed; tail -3 gpurun_out/r5p_probe.log; exit 1; }
cat gpurun_out/r5p_probe.log | grep name
