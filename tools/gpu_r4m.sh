#!/bin/bash
# round-4: GEGLU-backward epilogue with three row blocks of g, u in flight (PTK_GBWD_SETS=3) vs two: kernel tests,
# stamps of the dh shape under both, whole-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage_timers_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4m_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4m_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in w4stamps w4stamps2; do
  PTK_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/p8_stamps.py 22528 6912 1152 0 dh_geglu_bwd_$lib w4 5 >> gpurun_out/r4m_stamps.log 2>&1 || { echo "stamps failed"; tail -3 gpurun_out/r4m_stamps.log; exit 1; }
done
grep -v -e Warn -e amdgpu.ids gpurun_out/r4m_stamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['seg1']
    print(d['shape'], 'us', d['us'], 'epi', s['epilogue_issue_cyc'], 'ktile', s['rest_loop_cyc_per_ktile'], 'first', s['first_ktile_cyc'])
"
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_gbwd2.so 2>&1 | grep -v amdgpu.ids
