#!/bin/bash
# default bench (with the CPU baseline), rocprofv3 kernel stats of a short bench, SQ MFMA-busy counters
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/r3_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3_bench.log; exit 1; }
tail -1 gpurun_out/r3_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/r3_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r3_prof.log; exit 1; }
tail -1 $R/gpurun_out/r3_prof.log
db=$(find $R/gpurun_out/r3_prof -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r3_kernel_stats.csv
timeout -k 10 300 python3 -u $R/bench.py --config cfg4 --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r3_bench_cfg4.log 2>&1 || { echo "cfg4 bench failed"; tail -5 $R/gpurun_out/r3_bench_cfg4.log; exit 1; }
tail -1 $R/gpurun_out/r3_bench_cfg4.log
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/r3_sqpmc -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/r3_sqpmc.log 2>&1 || { echo "pmc failed"; tail -3 $R/gpurun_out/r3_sqpmc.log; exit 1; }
f=$(find $R/gpurun_out/r3_sqpmc -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_summary.py $f --top 30 > $R/gpurun_out/r3_sq_mfma.md && head -40 $R/gpurun_out/r3_sq_mfma.md
