#!/bin/bash
# Same-box A/B of the bench over library builds, alternated, each run under its own time limit.
#   tools/ab.sh [lib ...]   (default: build/libptk_prev.so from tools/build_prev.sh vs the in-tree libptk.so;
#                            "new" = the in-tree library)
# env: STEPS (default 5), ROUNDS (default 2), CONFIG (default cfg2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=("$@")
[ ${#LIBS[@]} -eq 0 ] && LIBS=(build/libptk_prev.so new)
for i in $(seq ${ROUNDS:-2}); do
  for lib in "${LIBS[@]}"; do
    l=$lib; [ "$l" = new ] && l=""
    PTK_LIB=$l timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --config ${CONFIG:-cfg2} --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  done
done
