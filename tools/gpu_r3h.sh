#!/bin/bash
# rocprofv3 kernel traces of a short bench with the lm_head-statistics CE (0) and the two-pass CE (1)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  PTK_CE_TWO_PASS=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r3h_prof$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 2 > $R/gpurun_out/r3h_prof$v.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r3h_prof$v.log; exit 1; }
  db=$(find $R/gpurun_out/r3h_prof$v -name "*.db" | head -1)
  python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r3h_stats$v.csv
  python3 - $db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
n = "name" if "name" in cols else "kernel_name"
rows = c.execute(f"select {n}, end - start from kernels order by end - start desc limit 12").fetchall()
for name, d in rows: print(d / 1e3, "us", name[:110])
for name, tot, k in c.execute(f"select {n}, sum(end-start), count(*) from kernels where {n} like '%ce%' group by {n}"):
    print("CE-like", name[:90], k, tot / k / 1e3, "us avg")
PY
done
