#!/bin/bash
# round-4: the line-pair exchange by bank-masked DPP moves instead of DPP + selects: GEMM + golden tests, stamps
# (new vs previous build), step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or golden" > gpurun_out/r4t_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4t_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4t_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in w4stamps w4stamps_prev; do
  for sh in "22528 6912 1152 0 dh_gbwd_$lib w4 5" "22528 1152 1024 0 g_o_$lib p8" "18432 3072 1024 0 sig_qkv_$lib p8"; do
    PTK_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/p8_stamps.py $sh >> gpurun_out/r4t_stamps.log 2>&1 || { echo "stamps failed: $sh"; tail -3 gpurun_out/r4t_stamps.log; exit 1; }
  done
done
grep -v -e Warn -e amdgpu.ids gpurun_out/r4t_stamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['seg0']
    print(d['shape'], 'us', d['us'], 'epi', s['epilogue_issue_cyc'], 'ktile', s['rest_loop_cyc_per_ktile'])
"
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_prevlines.so 2>&1 | grep -v amdgpu.ids
