#!/bin/bash
# dK/dV read-ahead depth: flash tests on the in-tree library (DKV_PD 2), then rocprofv3 kernel times of a short
# bench under DKV_PD 0 / 2 / 3 builds (PTK_LIB), same box
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attn" > gpurun_out/dkvpd_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/dkvpd_tests.log | tail -1; grep FAILED gpurun_out/dkvpd_tests.log | head
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for lib in ${DKV_LIBS:-new}; do
  tag=$(basename $lib .so)
  l=$lib; [ "$l" = new ] && l=""
  PTK_LIB=$l timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/dkvpd_$tag -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/dkvpd_$tag.log 2>&1 || { echo "prof failed $tag"; tail -3 $R/gpurun_out/dkvpd_$tag.log; exit 1; }
  db=$(find $R/gpurun_out/dkvpd_$tag -name "*.db" | head -1)
  python3 - $db $tag <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for n, k, t in c.execute("select name, count(*), avg(end-start) from kernels where name like '%attn_bwd%' group by name"):
    print(sys.argv[2], n.split('(')[0][-28:], k, round(t / 1e3, 1), "us")
PY
  rm -rf $R/gpurun_out/dkvpd_$tag
done
done
