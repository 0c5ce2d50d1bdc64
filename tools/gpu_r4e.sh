#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/sk_probe.py 22528 1536 1152 > gpurun_out/r4e_probe1.log 2>&1; echo "probe rc=$?"; grep -v Warn gpurun_out/r4e_probe1.log | cut -c1-200
timeout -k 10 200 python -u tools/sk_probe.py 22528 1152 4608 > gpurun_out/r4e_probe2.log 2>&1; echo "probe rc=$?"; grep -v Warn gpurun_out/r4e_probe2.log | cut -c1-200
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "stream_k or persistent or p8 or w4" > gpurun_out/r4e_sk.log 2>&1
rc=$?; echo "sk tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4e_sk.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4e_sk.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sk_ab.py > gpurun_out/r4e_sk_ab.log 2>&1; echo "sk_ab rc=$?"; grep -v Warn gpurun_out/r4e_sk_ab.log
PTK_HIP_MEMSET=1 DESTROY=1 timeout -k 10 300 python -u tools/graph_debug.py > gpurun_out/r4e_graph_memset.log 2>&1; echo "graph_debug memset rc=$?"; grep -v Warn gpurun_out/r4e_graph_memset.log | tail -8
