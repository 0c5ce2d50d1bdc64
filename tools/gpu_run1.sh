set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t1.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/b1.log 2>&1
echo "bench rc=$?"; tail -2 gpurun_out/b1.log
