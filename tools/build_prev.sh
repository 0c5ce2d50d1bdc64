#!/bin/bash
# Build libptk.so of a git revision (default HEAD) into build/libptk_prev.so for same-box A/B timing:
#   PTK_LIB=build/libptk_prev.so python bench.py ...
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" projectiontrainer_amd/csrc include | tar -x -C "$TMP"
make -C "$TMP/projectiontrainer_amd/csrc" -j8 > /dev/null
cp "$TMP/projectiontrainer_amd/libptk.so" "$ROOT/build/libptk_prev.so"
rm -rf "$TMP"
echo "built $REV -> build/libptk_prev.so"
