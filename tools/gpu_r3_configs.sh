#!/bin/bash
# the other Stage-1 configs on one GPU: cfg1 (bs 2), cfg5 (Gemma3-4B), cfg2 at T = 512
set -o pipefail
mkdir -p gpurun_out
for args in "--config cfg1" "--config cfg5" "--text-len 512"; do
  timeout -k 10 300 python -u bench.py $args --no-cpu-baseline > gpurun_out/r3_cfg.log 2>&1 || { echo "bench $args failed"; tail -5 gpurun_out/r3_cfg.log; exit 1; }
  tail -1 gpurun_out/r3_cfg.log
done
