#!/bin/bash
# after reverting the split tail: GEMM correctness first, then the whole suite, bench, rocprof
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp32_accumulate_gpu.py tests/test_kernels_gpu.py -k "fp32_accumulate or p8 or persistent" > gpurun_out/r3b_gemm.log 2>&1 || { echo "gemm tests failed"; grep -E "FAILED|Error" gpurun_out/r3b_gemm.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/r3b_gemm.log | tail -1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3b_tests.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r3b_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3b_bench.log; exit 1; }
tail -1 gpurun_out/r3b_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3b_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/r3b_prof.log 2>&1 || { echo "prof failed"; exit 1; }
tail -1 $R/gpurun_out/r3b_prof.log
cd $R
timeout -k 10 300 bash tools/fa_abl.sh > gpurun_out/r3b_faabl.log 2>&1; echo "faabl rc=$?"
