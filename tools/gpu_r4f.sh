#!/bin/bash
# round-4: full GPU suite (new census-asserted cfg5 / Stage-2 oracle tests), bench, cfg4 stream-K A/B, lm_head
# stats-only kernel time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4f_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4f_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log | cut -c1-400
for v in 0 1; do PTK_NO_STREAMK=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4f_cfg4_nosk$v.log 2>&1 || { echo "cfg4 failed"; tail -3 gpurun_out/r4f_cfg4_nosk$v.log; exit 1; }; echo "cfg4 PTK_NO_STREAMK=$v: $(tail -1 gpurun_out/r4f_cfg4_nosk$v.log | cut -c1-200)"; done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1; do PTK_LM_STATS_ONLY=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4f_lm$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r4f_lm$v.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r4f_lm$v.log; exit 1; }; db=$(find $R/gpurun_out/r4f_lm$v -name "*.db" | head -1); python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r4f_lm${v}_stats.csv; grep -E "gemm_big_kernel<0, 0>|ce_stats" $R/gpurun_out/r4f_lm${v}_stats.csv | cut -c1-160; done
