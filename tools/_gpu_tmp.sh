set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PTK_LIB=ablibs/libptk_g4r32.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stage2_vs_reference or stage2_architecture" > gpurun_out/r5g4_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r5g4_tests.log; exit 1; }
tail -1 gpurun_out/r5g4_tests.log
CONFIG=cfg4 ROUNDS=2 STEPS=2 timeout -k 10 1100 bash tools/ab.sh new ablibs/libptk_g4r32.so ablibs/libptk_g2r16.so > gpurun_out/r5g4_ab.log 2>&1 || { echo ab failed; tail -5 gpurun_out/r5g4_ab.log; exit 1; }
cat gpurun_out/r5g4_ab.log
