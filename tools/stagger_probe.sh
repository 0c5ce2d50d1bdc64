#!/bin/bash
# Persistent 4-wave GEMM: time the GEGLU (gate|up) and GEGLU-backward (dh) shapes with half of each
# XCD's workgroups started late by PTK_W4_STAGGER units (~1k cycles), so that half the CUs store
# their epilogue while the other half runs MFMAs.  Same results; timing only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in 0 ${STAGGERS:-12 25 50 0}; do
  for shape in "22528 13824 1152 3" "22528 6912 1152 5"; do
    set -- $shape
    PTK_W4_STAGGER=$s timeout -k 10 120 python tools/gemm_probe.py $1 $2 $3 $4 8 20 | sed "s|^|stagger=$s |" || exit 1
  done
done
