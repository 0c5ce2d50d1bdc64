#!/bin/bash
# round-4: epilogue store-pattern diagnostics (stamps build): normal 16 rows x 64 B per store instruction vs
# 8 rows x 128 B (mode 2) vs the normal pattern onto 16 L2-resident rows (mode 3); also at grid 64
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { timeout -k 10 120 python -u tools/p8_stamps.py "$@" >> gpurun_out/r4l_stamps.log 2>&1 || { echo "stamps failed: $*"; tail -3 gpurun_out/r4l_stamps.log; exit 1; }; }
for m in 0 2 3; do run 22528 1152 1024 $m g_o p8; done
for m in 0 2 3; do PTK_GEMM_GRID=64 run 22528 1152 1024 $m g_o_grid64 p8; done
for m in 0 2 3; do run 18432 3072 1024 $m sig_qkv p8; done
for m in 0 2 3; do run 22528 1152 6912 $m down w4; done
grep -v -e Warn -e amdgpu.ids gpurun_out/r4l_stamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s0=d['seg0']
    print(d['shape'], d['kernel'], 'mode', d['epi_mode'], 'us', d['us'], 'epi', s0['epilogue_issue_cyc'], 'ktile', s0['rest_loop_cyc_per_ktile'], 'seg1 first', d.get('seg1',{}).get('first_ktile_cyc'))
"
