set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r05_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline) > gpurun_out/r05_sq.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/r05_sq.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r05_sq/run_counter_collection.csv --top 16 > gpurun_out/r05_sq_summary.md 2>&1 || { echo summary failed; tail -5 gpurun_out/r05_sq_summary.md; exit 1; }
cat gpurun_out/r05_sq_summary.md
