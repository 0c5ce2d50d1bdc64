#!/bin/bash
# rocprofv3 kernel stats of the cfg4 (Stage 2) bench: 2 optimizer steps at gas 8 after 1 warm-up
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/cfg4_prof -o run -- python3 $R/bench.py --config cfg4 --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/cfg4_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/cfg4_prof.log; exit 1; }
tail -1 $R/gpurun_out/cfg4_prof.log | cut -c1-200
db=$(find $R/gpurun_out/cfg4_prof -name "*.db" | head -1)
python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r3_cfg4_kernel_stats.csv
