#!/bin/bash
# round-4: census probes of the final dispatch (stream-K off by default), census-asserted tests, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/census_probe2.py stage2 16 2 4 6 8 10 12 14 > gpurun_out/r4g_census_s2.log 2>&1; echo "census s2 rc=$?"; grep -v Warn gpurun_out/r4g_census_s2.log | tail -9
timeout -k 10 300 python -u tools/census_probe2.py cfg5 16 1 2 4 6 8 10 12 14 > gpurun_out/r4g_census_c5.log 2>&1; echo "census cfg5 rc=$?"; grep -v Warn gpurun_out/r4g_census_c5.log | tail -10
timeout -k 10 300 python -u tools/census_probe.py 32 30 > gpurun_out/r4g_census_c2.log 2>&1; echo "census cfg2 rc=$?"; grep -v Warn gpurun_out/r4g_census_c2.log | tail -3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4g_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4g_bench.log; exit 1; }
tail -1 gpurun_out/r4g_bench.log | cut -c1-300
