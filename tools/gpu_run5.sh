set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/graph_debug.py 2>&1 | grep -v amdgpu.ids
