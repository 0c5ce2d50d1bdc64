#!/bin/bash
# round-4: attention forwards (Gemma d 256) load the Q rows by LDS-DMA as whole rows instead of per-lane fragments:
# attention + golden tests, stamps of both forwards under the new / previous flash.hip, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flash or attn or golden" > gpurun_out/r4r_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4r_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4r_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in fastamps fastamps_old; do
  for w in "512 fwd" "0 fwd"; do
    FA_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/fa_stamps.py $w > gpurun_out/r4r_fa.log 2>&1 || { echo "fa stamps failed: $lib $w"; tail -3 gpurun_out/r4r_fa.log; exit 1; }
    echo "$lib $w: $(grep -v amdgpu.ids gpurun_out/r4r_fa.log | tr '\n' ' ' | cut -c1-400)"
  done
done
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_oldflash.so 2>&1 | grep -v amdgpu.ids
