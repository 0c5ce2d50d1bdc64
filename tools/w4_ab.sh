#!/bin/bash
# Same-box check + A/B of the persistent 4-wave GEMM: kernel tests (mode 8 and the auto-selected
# shapes), then tools/gemm_probe.py on the step's w4 shapes for build/libptk_prev.so vs the in-tree
# library, then the bench A/B (tools/ab.sh).  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "big_tile or all_epilogues or geglu or epilogues" > gpurun_out/w4t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w4t.log; exit 1; }
tail -2 gpurun_out/w4t.log
for i in 1 2; do
  for lib in build/libptk_prev.so ""; do
    for shape in "22528 13824 1152 3" "22528 6912 1152 0" "18432 3072 1024 0" "22528 1152 6912 0" "8192 8192 8192 0"; do
      set -- $shape
      PTK_LIB=$lib timeout -k 10 120 python tools/gemm_probe.py $1 $2 $3 $4 8 10 2>/dev/null | sed "s|^|${lib:-new} |" || exit 1
    done
  done
done
bash tools/ab.sh
