#!/bin/bash
# round-4: stream-K kernel tests, bench, then the full GPU suite and the census probes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -v -x --timeout 120 --timeout-method thread -k "stream_k or persistent or p8 or w4" > gpurun_out/r4b_sk.log 2>&1
rc=$?; echo "sk tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4b_sk.log | tail -1; grep -E "FAILED|Error|assert" gpurun_out/r4b_sk.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4b_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4b_bench.log; exit 1; }
tail -1 gpurun_out/r4b_bench.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4b_tests.log | tail -1; grep -E "FAILED" gpurun_out/r4b_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/census_probe2.py stage2 16 2 4 6 8 10 12 14 > gpurun_out/r4b_census_s2.log 2>&1; echo "census s2 rc=$?"; grep -v Warn gpurun_out/r4b_census_s2.log | tail -9
timeout -k 10 300 python -u tools/census_probe2.py cfg5 16 1 2 4 6 8 10 12 14 > gpurun_out/r4b_census_c5.log 2>&1; echo "census cfg5 rc=$?"; grep -v Warn gpurun_out/r4b_census_c5.log | tail -10
DESTROY=1 timeout -k 10 300 python -u tools/graph_debug.py > gpurun_out/r4b_graph_destroy.log 2>&1; echo "graph_debug rc=$?"; grep -v Warn gpurun_out/r4b_graph_destroy.log | tail -8
