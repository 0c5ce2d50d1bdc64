set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "p8_matches or geglu or epilogues" > gpurun_out/r5f_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r5f_tests.log | tail -3; grep -E "FAILED|Error|assert" gpurun_out/r5f_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
for lean in 1 0; do
  echo "lean=$lean"
  MODES=8,32 PTK_LEAN_EPI=$lean timeout -k 10 300 python -u tools/p8_probe.py g_gu_geglu g_dh_geglu_bwd > gpurun_out/r5f_probe.log 2>&1 || { echo probe failed; tail -5 gpurun_out/r5f_probe.log; exit 1; }
  grep -v amdgpu gpurun_out/r5f_probe.log
done
for r in 1 2; do for lean in 0 1; do
  PTK_LEAN_EPI=$lean timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5f_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5f_bench.log; exit 1; }
  echo "lean=$lean $(tail -1 gpurun_out/r5f_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_mfma_frac"], d["roofline"]["achieved"])')"
done; done
