#!/bin/bash
# Same-box A/B of the vision prefetch: bench.py with and without --no-prefetch, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for flag in "" --prefetch; do
    timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline $flag > gpurun_out/abp.json 2> gpurun_out/abp.err || { tail -5 gpurun_out/abp.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abp.json')); print('${flag:-inline}', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
