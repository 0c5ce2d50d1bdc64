set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "projector" > gpurun_out/r5p_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r5p_tests.log; exit 1; }
tail -2 gpurun_out/r5p_tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5p_b1_$r.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5p_b1_$r.log; exit 1; }
tail -1 gpurun_out/r5p_b1_$r.log | cut -c1-150
PTK_WGRAD_TN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5p_b0_$r.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5p_b0_$r.log; exit 1; }
tail -1 gpurun_out/r5p_b0_$r.log | cut -c1-150
done
