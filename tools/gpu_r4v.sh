#!/bin/bash
# round-4: the dQ kernel's Q, dO and O rows by LDS-DMA as whole rows (two phases) instead of per-lane fragment
# loads: attention + golden tests, dQ stamps new / previous, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py tests/test_dkv_fused_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flash or attn or golden or dkv" > gpurun_out/r4v_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4v_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4v_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in fastamps fastamps_old; do
  for w in "512 bwd" "0 bwd"; do
    FA_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/fa_stamps.py $w > gpurun_out/r4v_fa.log 2>&1 || { echo "fa stamps failed: $lib $w"; tail -3 gpurun_out/r4v_fa.log; exit 1; }
    echo "$lib $w: $(grep -v amdgpu.ids gpurun_out/r4v_fa.log | tr '\n' ' ' | cut -c1-420)"
  done
done
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_oldflash.so 2>&1 | grep -v amdgpu.ids
