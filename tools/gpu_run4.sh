set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/p8_probe.py proj_dW2 proj_dW1 proj_dA g_dgu_dx proj_fc1 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b4.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/b4.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1; echo "prof rc=$?"
