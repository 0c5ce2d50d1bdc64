#!/bin/bash
# round-4 diagnostic: dh + GEGLU-backward epilogue cycles per tile on the full grid, half and a quarter of the CUs
# (stamps build, PTK_GEMM_GRID): an epilogue bound by chip-wide HBM bandwidth shortens on fewer CUs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
for grid in 256 128 64; do
  for act in 5 0; do
    PTK_GEMM_GRID=$grid PTK_STAMPS_LIB=ablibs/libptk_w4stamps.so timeout -k 10 120 python -u tools/p8_stamps.py 22528 6912 1152 0 "dh_act${act}_grid${grid}" w4 $act 2>&1 | grep -v amdgpu.ids | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
s=[d[k] for k in d if k.startswith('seg')]
print(d['shape'], 'us', d['us'], 'epi', sorted(x['epilogue_issue_cyc'] for x in s)[len(s)//2], 'ktile', sorted(x['rest_loop_cyc_per_ktile'] for x in s)[len(s)//2], 'first', sorted(x['first_ktile_cyc'] for x in s)[len(s)//2])" || exit 1
  done
done
