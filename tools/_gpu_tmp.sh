set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CHECK=1 MODES=8,2048,32 timeout -k 10 400 python -u tools/p8_probe.py g_qkv g_down g_gu_geglu g_dh_geglu_bwd sq8192 sig_fc1_b proj_fc2 > gpurun_out/r5r_probe.log 2>&1 || { echo probe failed; tail -5 gpurun_out/r5r_probe.log; exit 1; }
grep name gpurun_out/r5r_probe.log | cut -c1-300
