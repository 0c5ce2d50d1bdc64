set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5s_flash.log 2>&1 || { echo flash tests failed; grep -E "FAIL|Error|assert" gpurun_out/r5s_flash.log | head -20; exit 1; }
tail -2 gpurun_out/r5s_flash.log
for r in 1 2; do
PTK_ATTN_PERSIST=1 timeout -k 10 120 python -u tools/attn_bench.py --what bwd > gpurun_out/r5s_attn_p1_$r.log 2>&1 || { echo attn failed; tail -3 gpurun_out/r5s_attn_p1_$r.log; exit 1; }
PTK_ATTN_PERSIST=0 timeout -k 10 120 python -u tools/attn_bench.py --what bwd > gpurun_out/r5s_attn_p0_$r.log 2>&1 || { echo attn failed; tail -3 gpurun_out/r5s_attn_p0_$r.log; exit 1; }
done
grep -h "{" gpurun_out/r5s_attn_p1_1.log gpurun_out/r5s_attn_p0_1.log gpurun_out/r5s_attn_p1_2.log gpurun_out/r5s_attn_p0_2.log | cut -c1-250
timeout -k 10 300 python -u tools/census_probe2.py stage2 16 15 8 > gpurun_out/r5r_census_s2.log 2>&1 || { echo census failed; tail -5 gpurun_out/r5r_census_s2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5r_census_s2.log
timeout -k 10 300 python -u tools/census_probe2.py cfg5 16 8 15 14 > gpurun_out/r5r_census_c5.log 2>&1 || { echo census failed; tail -5 gpurun_out/r5r_census_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5r_census_c5.log
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5r_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5r_cfg4.log; exit 1; }
tail -1 gpurun_out/r5r_cfg4.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5r_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5r_bench.log; exit 1; }
tail -1 gpurun_out/r5r_bench.log | cut -c1-200
PTK_STREAMK=0 PTK_ATTN_PERSIST=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5r_bench_off.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5r_bench_off.log; exit 1; }
tail -1 gpurun_out/r5r_bench_off.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5r_bench2.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5r_bench2.log; exit 1; }
tail -1 gpurun_out/r5r_bench2.log | cut -c1-200
