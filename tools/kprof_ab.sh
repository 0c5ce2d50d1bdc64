#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel stats of bench.py (2 steps) for build/libptk_prev.so and the in-tree
# libptk.so; prints the kernels whose name matches $1 (regex) with their average duration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && cd gpurun_out && export TMPDIR=/tmp
for lib in build/libptk_prev.so ""; do
  rm -rf kab
  PTK_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d kab -o run -- python3 ../bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> kab.err || { tail -3 kab.err; exit 1; }
  python3 - "$1" "${lib:-new}" <<'PY'
import csv, re, sys
pat, tag = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open("kab/run_kernel_stats.csv")):
    if re.search(pat, r["Name"]):
        print(f"{tag:22s} {float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5s}  {r['Name'][:90]}")
PY
done
