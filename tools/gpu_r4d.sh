#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/sk_probe.py 22528 1536 1152 > gpurun_out/r4d_probe1.log 2>&1; echo "probe rc=$?"; grep -v Warn gpurun_out/r4d_probe1.log
timeout -k 10 200 python -u tools/sk_probe.py 22528 1152 4608 > gpurun_out/r4d_probe2.log 2>&1; echo "probe rc=$?"; grep -v Warn gpurun_out/r4d_probe2.log
