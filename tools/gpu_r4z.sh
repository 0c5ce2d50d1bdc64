#!/bin/bash
# round-4 final check on this tree: full GPU suite, smoke, default bench (with the CPU baseline), bench with the
# stage timers, rocprofv3 kernel statistics of the default bench, cfg4 / cfg5 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > gpurun_out/r4z_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4z_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4z_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4z_smoke.log; exit 1; }
grep smoke gpurun_out/r4z_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4z_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4z_bench.log; exit 1; }
tail -1 gpurun_out/r4z_bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --stage-timers > gpurun_out/r4z_bench_stages.log 2>&1 || { echo "stage bench failed"; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4z_bench_cfg4.log 2>&1 || { echo "cfg4 failed"; tail -3 gpurun_out/r4z_bench_cfg4.log; exit 1; }
tail -1 gpurun_out/r4z_bench_cfg4.log | cut -c1-200
timeout -k 10 400 python -u bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4z_bench_cfg5.log 2>&1 || { echo "cfg5 failed"; tail -3 gpurun_out/r4z_bench_cfg5.log; exit 1; }
tail -1 gpurun_out/r4z_bench_cfg5.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4z_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/r4z_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r4z_prof.log; exit 1; }
db=$(find $R/gpurun_out/r4z_prof -name "*.db" | head -1); python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r4z_stats.csv
head -12 $R/gpurun_out/r4z_stats.csv | cut -c1-150
