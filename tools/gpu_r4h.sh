#!/bin/bash
# round-4: same-box A/B of p8 issue-priority variants (tools/ab.sh alternation)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=3 STEPS=10 bash tools/ab.sh new ablibs/libptk_p8prio.so ablibs/libptk_p8mprio.so 2>&1 | tee gpurun_out/r4h_ab.txt
