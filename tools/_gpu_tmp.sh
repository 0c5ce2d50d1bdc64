set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH="g_qkv g_o g_dO g_dqkv g_down g_dgu_dx sig_qkv_b sig_o_br sig_fc1_b"
MODES=32,0 timeout -k 10 400 python -u tools/p8_probe.py $SH > gpurun_out/r5x_probe.log 2>&1 || { echo probe failed; tail -3 gpurun_out/r5x_probe.log; exit 1; }
grep name gpurun_out/r5x_probe.log | cut -c1-200
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5x_b1_$r.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5x_b1_$r.log; exit 1; }
tail -1 gpurun_out/r5x_b1_$r.log | cut -c1-160
PTK_TM224=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5x_b0_$r.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5x_b0_$r.log; exit 1; }
tail -1 gpurun_out/r5x_b0_$r.log | cut -c1-160
done
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5x_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5x_cfg4.log; exit 1; }
tail -1 gpurun_out/r5x_cfg4.log | cut -c1-200
