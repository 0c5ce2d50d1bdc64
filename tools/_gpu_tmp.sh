set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "flash" > gpurun_out/r5i_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5i_tests.log | tail -3; grep -E "FAILED|Error|assert" gpurun_out/r5i_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for p in 0 1; do
  PTK_ATTN_PERSIST=$p timeout -k 10 120 python -u tools/attn_bench.py --what fwd > gpurun_out/r5i_ab.log 2>&1 || { echo attn bench failed; tail -5 gpurun_out/r5i_ab.log; exit 1; }
  echo "persist=$p $(grep -v amdgpu gpurun_out/r5i_ab.log | tr '\n' ' ' | cut -c1-400)"
done; done
for r in 1 2; do for p in 0 1; do
  PTK_ATTN_PERSIST=$p timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5i_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5i_bench.log; exit 1; }
  echo "persist=$p $(tail -1 gpurun_out/r5i_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')"
done; done
