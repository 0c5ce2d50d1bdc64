#!/bin/bash
# Same-box A/B of the bench: build/libptk_prev.so (tools/build_prev.sh) vs the in-tree libptk.so,
# alternated, each run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for lib in build/libptk_prev.so ""; do
    PTK_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { cat gpurun_out/ab.err | tail -5; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('${lib:-new}', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
