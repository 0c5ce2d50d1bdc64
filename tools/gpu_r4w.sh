#!/bin/bash
# round-4: the 128x128 GEMM with the MFMA operands swapped (transposed accumulator layout) so the epilogue stages its
# accumulators by 16-B LDS stores instead of 4-B ones: GEMM + golden tests, step-shape GEMM timings new / previous, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or golden or census or architecture" > gpurun_out/r4w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4w_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4w_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
GEMM_SHAPES="g_qkv g_dO sig_o sig_fc2" bash tools/gemm_ab.sh new ablibs/libptk_ntold.so 2>&1 | grep -v amdgpu.ids || exit 1
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_ntold.so 2>&1 | grep -v amdgpu.ids
