#!/bin/bash
# round-4 check: full GPU suite, graph-destroy probe, default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4a_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4a_tests.log | head
[ $rc -eq 0 ] || exit $rc
DESTROY=1 timeout -k 10 300 python -u tools/graph_debug.py > gpurun_out/r4a_graph_destroy.log 2>&1; echo "graph_debug rc=$?"; cat gpurun_out/r4a_graph_destroy.log | grep -v Warn | tail -8
timeout -k 10 300 python -u tools/census_probe2.py stage2 16 2 4 6 8 10 12 14 > gpurun_out/r4a_census_s2.log 2>&1; echo "census s2 rc=$?"; grep -v Warn gpurun_out/r4a_census_s2.log | tail -9
timeout -k 10 300 python -u tools/census_probe2.py cfg5 16 1 2 4 6 8 10 12 14 > gpurun_out/r4a_census_c5.log 2>&1; echo "census cfg5 rc=$?"; grep -v Warn gpurun_out/r4a_census_c5.log | tail -10
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4a_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4a_bench.log; exit 1; }
tail -1 gpurun_out/r4a_bench.log
