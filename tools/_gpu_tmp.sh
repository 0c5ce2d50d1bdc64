set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CONFIG=cfg4 ROUNDS=2 STEPS=2 timeout -k 10 1100 bash tools/ab.sh new ablibs/libptk_f32.so ablibs/libptk_f128.so > gpurun_out/r5f_ab.log 2>&1 || { echo ab failed; tail -5 gpurun_out/r5f_ab.log; exit 1; }
cat gpurun_out/r5f_ab.log
