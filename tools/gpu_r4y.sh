#!/bin/bash
# round-4: GEGLU-backward epilogue's first g / u row block loaded before the tile's last K-tile pair (new) vs at
# the epilogue's start (ablibs/libptk_gpre0.so): GEMM + golden tests, dh GEMM timing, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or golden or census or architecture" > gpurun_out/r4y_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4y_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4y_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
GEMM_SHAPES="g_dh_geglu_bwd g_gu g_down" bash tools/gemm_ab.sh new ablibs/libptk_gpre0.so 2>&1 | grep -v amdgpu.ids || exit 1
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_gpre0.so 2>&1 | grep -v amdgpu.ids
