#!/bin/bash
# Same-box timing of persistent 4-wave GEMM builds (schedule variants / ablations) on step shapes.
#   tools/w4_var.sh lib...   ("new" = the in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    l=$lib; [ "$l" = new ] && l=""
    for shape in "22528 6912 1152 0" "8192 8192 8192 0" "18432 3072 1024 0"; do
      set -- $shape
      PTK_LIB=$l timeout -k 10 120 python tools/gemm_probe.py $1 $2 $3 $4 8 10 2>/dev/null | sed "s|^|$lib |" || exit 1
    done
  done
done
