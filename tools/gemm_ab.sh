#!/bin/bash
# Same-box A/B of GEMM library builds on step shapes: tools/gemm_ab.sh lib...  ("new" = in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for lib in "$@"; do
    l=$lib; [ "$l" = new ] && l=""
    PTK_LIB=$l timeout -k 10 180 python tools/gemm_ab.py $GEMM_SHAPES 2>/dev/null || exit 1
  done
done
