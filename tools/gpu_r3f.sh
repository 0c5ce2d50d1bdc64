#!/bin/bash
# full GPU suite, default bench, rocprofv3 kernel stats of a short bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3f_tests.log | tail -1; grep FAILED gpurun_out/r3f_tests.log | head
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3f_bench.log; exit 1; }
tail -1 gpurun_out/r3f_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3f_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/r3f_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r3f_prof.log; exit 1; }
tail -1 $R/gpurun_out/r3f_prof.log
ls -R $R/gpurun_out/r3f_prof | head -20
