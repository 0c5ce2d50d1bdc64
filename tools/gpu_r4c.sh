#!/bin/bash
# round-4: persistent-GEMM tests, stream-K A/B per shape, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "stream_k or persistent or p8 or w4" > gpurun_out/r4c_sk.log 2>&1
rc=$?; echo "sk tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4c_sk.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4c_sk.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sk_ab.py > gpurun_out/r4c_sk_ab.log 2>&1; echo "sk_ab rc=$?"; grep -v Warn gpurun_out/r4c_sk_ab.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4c_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4c_bench.log; exit 1; }
tail -1 gpurun_out/r4c_bench.log
