#!/bin/bash
# round-4: persistent epilogues without the alpha scale (alpha != 1 dispatched to the 128^2 / 256^2 kernels):
# GEMM + golden tests, step A/B against the previous build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or golden" > gpurun_out/r4u_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4u_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4u_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_prev.so 2>&1 | grep -v amdgpu.ids
