#!/bin/bash
# time the attention forward for the default build and each ablation build (tools: make faabl)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "base"; timeout -k 10 60 python tools/attn_bench.py --what fwd || exit $?
for n in 1 2 3 4 5 6 7; do
  echo "abl$n"; PTK_LIB=build/libptk_faabl$n.so timeout -k 10 60 python tools/attn_bench.py --what fwd || exit $?
done
