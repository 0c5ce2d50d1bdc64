#!/bin/bash
# round-4: persistent GEMM epilogue diagnostics (stamps build): is the ~11k-cycle epilogue the chip-wide write
# burst?  Same shapes on half the CUs (PTK_GEMM_GRID=128), and the w4 kernels (gate|up GEGLU, dh GEGLU-bwd, down)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { timeout -k 10 120 python -u tools/p8_stamps.py "$@" >> gpurun_out/r4k_stamps.log 2>&1 || { echo "stamps failed: $*"; tail -3 gpurun_out/r4k_stamps.log; exit 1; }; }
run 22528 1152 1024 0 g_o p8
PTK_GEMM_GRID=128 run 22528 1152 1024 0 g_o_grid128 p8
PTK_GEMM_GRID=64 run 22528 1152 1024 0 g_o_grid64 p8
run 22528 13824 1152 0 gate_up_plain p8
PTK_GEMM_GRID=128 run 22528 13824 1152 0 gate_up_plain_grid128 p8
run 22528 13824 1152 0 gate_up_geglu w4 3
run 22528 13824 1152 1 gate_up_geglu w4 3
run 22528 6912 1152 0 dh_geglu_bwd w4 5
run 22528 6912 1152 1 dh_geglu_bwd w4 5
PTK_GEMM_GRID=128 run 22528 6912 1152 0 dh_geglu_bwd_grid128 w4 5
run 22528 1152 6912 0 down w4 0
grep -v -e Warn -e amdgpu.ids gpurun_out/r4k_stamps.log | cut -c1-900
