set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stage2_vs_reference or norm_wgrad or rms" > gpurun_out/r5n_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r5n_tests.log; exit 1; }
tail -1 gpurun_out/r5n_tests.log
CONFIG=cfg4 ROUNDS=2 STEPS=2 timeout -k 10 1000 bash tools/ab.sh new ablibs/libptk_wg1.so > gpurun_out/r5n_ab.log 2>&1 || { echo ab failed; tail -5 gpurun_out/r5n_ab.log; exit 1; }
cat gpurun_out/r5n_ab.log
