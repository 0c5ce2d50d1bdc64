set -o pipefail
timeout -k 10 200 python -u tools/p8_debug.py 2>&1 | grep -v amdgpu.ids
