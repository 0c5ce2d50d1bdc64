#!/bin/bash
# round-4: GEGLU-backward g, u loaded as whole lines (PTK_W4_LINES bit 2) on top of the whole-line stores:
# kernel + golden tests, dh stamps under lines 3 / 1 / 0, whole-step A/B against lines 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage1_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or golden" > gpurun_out/r4p_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4p_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4p_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in w4stamps w4stamps_lines1 w4stamps_lines0; do
  PTK_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/p8_stamps.py 22528 6912 1152 0 dh_gbwd_$lib w4 5 >> gpurun_out/r4p_stamps.log 2>&1 || { echo "stamps failed"; tail -3 gpurun_out/r4p_stamps.log; exit 1; }
done
grep -v -e Warn -e amdgpu.ids gpurun_out/r4p_stamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['seg1']
    print(d['shape'], 'us', d['us'], 'epi', s['epilogue_issue_cyc'], 'ktile', s['rest_loop_cyc_per_ktile'], 'first', s['first_ktile_cyc'])
"
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_lines1.so 2>&1 | grep -v amdgpu.ids
