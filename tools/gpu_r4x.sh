#!/bin/bash
# round-4: Stage-2 weight-grad operand transpose with 16-B accesses, 128x64 tiles (new) vs the 64x64 8-B kernel
# (ablibs/libptk_tr8.so): transpose + Stage-2 tests, kernel timings on the cfg4 shapes, cfg4 bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage2_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread -k "transpose or stage2 or s2" > gpurun_out/r4x_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4x_tests.log | tail -1; grep -E "^E  |FAILED" gpurun_out/r4x_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in new ablibs/libptk_tr8.so; do
  l=$lib; [ "$l" = new ] && l=""
  PTK_LIB=$l timeout -k 10 120 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids || exit 1
import os, torch
from projectiontrainer_amd import kernels as Kn
dev = torch.device("cuda:0")
out = []
for cols in (1152, 1536, 6912, 13824):
    x = torch.randn(14336, cols, device=dev).to(torch.bfloat16)
    for _ in range(3): Kn.transpose_rows(x, 14336, 14336)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): Kn.transpose_rows(x, 14336, 14336)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    out.append(f"cols {cols}: {us:.1f} us ({2 * x.numel() * 2 / us / 1e6:.2f} TB/s)")
print(os.environ.get("PTK_LIB") or "new", "; ".join(out))
PY
done
for i in 1 2; do
  for lib in new ablibs/libptk_tr8.so; do
    l=$lib; [ "$l" = new ] && l=""
    PTK_LIB=$l timeout -k 10 400 python bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4x_cfg4.json 2> gpurun_out/r4x_cfg4.err || { tail -5 gpurun_out/r4x_cfg4.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4x_cfg4.json')); print('$lib', d['value'], d['ms_per_step'])"
  done
done
