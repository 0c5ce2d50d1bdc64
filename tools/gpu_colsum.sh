#!/bin/bash
# projector / Stage-1 GPU tests, then the colsum kernels' times in a short profiled bench
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_stage1_gpu.py -k "projector or proj or stage1 or census or golden or bias" > gpurun_out/colsum_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/colsum_tests.log | tail -1; grep FAILED gpurun_out/colsum_tests.log | head
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/colsum_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/colsum_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/colsum_prof.log; exit 1; }
tail -1 $R/gpurun_out/colsum_prof.log | cut -c1-160
db=$(find $R/gpurun_out/colsum_prof -name "*.db" | head -1)
python3 - $db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for n, gx, gy, k, t in c.execute("select name, grid_x, grid_y, count(*), avg(end-start) from kernels where name like '%colsum%' or name like '%transpose_kernel%' group by name, grid_x, grid_y"):
    print(n.split('(')[0][-26:], gx, gy, k, round(t / 1e3, 1), "us")
PY
rm -rf $R/gpurun_out/colsum_prof
