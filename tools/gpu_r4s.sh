#!/bin/bash
# round-4: the GEGLU and GEGLU-backward projections on the 8-wave persistent kernel (PTK_P8=1: now with the
# younger-half priority and the whole-line stores) vs the 4-wave one: stamps of both shapes on both kernels, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for k in p8 w4; do
  for sh in "22528 13824 1152 0 gate_up_$k $k 3" "22528 6912 1152 0 dh_gbwd_$k $k 5"; do
    timeout -k 10 120 python -u tools/p8_stamps.py $sh >> gpurun_out/r4s_stamps.log 2>&1 || { echo "stamps failed: $sh"; tail -3 gpurun_out/r4s_stamps.log; exit 1; }
  done
done
grep -v -e Warn -e amdgpu.ids gpurun_out/r4s_stamps.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['seg1']
    print(d['shape'], 'us', d['us'], 'epi', s['epilogue_issue_cyc'], 'ktile', s['rest_loop_cyc_per_ktile'], 'first', s['first_ktile_cyc'])
"
ROUNDS=3 STEPS=10 bash tools/ab_env.sh PTK_P8=1 2>&1 | grep -v amdgpu.ids
