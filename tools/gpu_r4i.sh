#!/bin/bash
# round-4: norm kernels with every row input loaded up front + p8 priority split on by default:
# model-level oracle tests (the residual norms have no standalone entry point), bench, per-kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_stage1_gpu.py tests/test_stage2_gpu.py tests/test_kernels_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4i_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4i_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4i_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4i_bench.log; exit 1; }
tail -1 gpurun_out/r4i_bench.log | cut -c1-300
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4i_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r4i_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r4i_prof.log; exit 1; }
db=$(find $R/gpurun_out/r4i_prof -name "*.db" | head -1); python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r4i_stats.csv
grep -E "norm|qknorm" $R/gpurun_out/r4i_stats.csv | cut -c1-160
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stage_timers_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/r4i_timers.log 2>&1; rc=$?; echo "timers rc=$rc"; grep -E "passed|failed" gpurun_out/r4i_timers.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stage-timers > gpurun_out/r4i_bench_stages.log 2>&1 || { echo "stage bench failed"; tail -5 gpurun_out/r4i_bench_stages.log; exit 1; }
tail -1 gpurun_out/r4i_bench_stages.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d.get('stages_ms_per_step')))"
timeout -k 10 200 python -u tools/fa_stamps.py 0 fwd64 > gpurun_out/r4i_fa64_stamps.log 2>&1; echo "fa64 stamps rc=$?"; tail -3 gpurun_out/r4i_fa64_stamps.log
