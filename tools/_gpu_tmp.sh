set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05_final_cfg5.log 2>&1 || { echo cfg5 failed; tail -5 gpurun_out/r05_final_cfg5.log; exit 1; }
tail -1 gpurun_out/r05_final_cfg5.log | cut -c1-200
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_rep_$r.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r05_rep_$r.log; exit 1; }
tail -1 gpurun_out/r05_rep_$r.log | cut -c1-120
done
