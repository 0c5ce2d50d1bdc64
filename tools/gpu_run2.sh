set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "p8_matches_w4 or persistent_vs_fp32 or projector_module" -v --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "p8 tests rc=$rc"; tail -12 gpurun_out/t2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/graph_debug.py > gpurun_out/graph_debug.log 2>&1; echo "graph rc=$?"; cat gpurun_out/graph_debug.log | grep -v amdgpu.ids
timeout -k 10 400 python -u tools/p8_probe.py > gpurun_out/p8_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/p8_probe.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_dist.py tests/test_graph_gpu.py tests/test_stage2_gpu.py -m gpu -v --timeout 250 --timeout-method thread > gpurun_out/t2b.log 2>&1
echo "dist/graph/stage2 rc=$?"; tail -15 gpurun_out/t2b.log
