#!/bin/bash
# Same-box A/B of the bench over an environment switch: tools/ab_env.sh VAR=value  (alternated with VAR unset)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-2}); do
  for e in "$1" ""; do
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('${e:-default}', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
