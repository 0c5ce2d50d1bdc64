set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for lib in "" ablibs/libptk_duearly.so; do
  echo "lib=${lib:-new}"
  MODES=32,64 PTK_LIB=$lib timeout -k 10 200 python -u tools/p8_probe.py g_down g_o g_gu_geglu g_dh_geglu_bwd > gpurun_out/r5b_probe.log 2>&1 || { echo probe failed; tail -5 gpurun_out/r5b_probe.log; exit 1; }
  grep -v amdgpu gpurun_out/r5b_probe.log
done
