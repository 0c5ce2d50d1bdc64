#!/bin/bash
# hipBLASLt-for-plain-GEMMs A/B: per-shape probe (MFMA kernels vs hipBLASLt) and whole-step benches of
# cfg2 / cfg4 with PTK_BLASLT=0 (MFMA only) vs the default shape rule.  Each step time-limited; stops at
# the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
PTK_BLASLT=0 timeout -k 10 200 python -u tools/blaslt_probe.py > gpurun_out/r02_blaslt_probe2.txt 2>&1 || exit $?
PTK_BLASLT=1 timeout -k 10 200 python -u tools/blaslt_probe.py >> gpurun_out/r02_blaslt_probe2.txt 2>&1 || exit $?
for v in 0 2; do
  PTK_BLASLT=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02_ab2_cfg2_$v.json 2> gpurun_out/r02_ab2_cfg2_$v.err || exit $?
  PTK_BLASLT=$v timeout -k 10 200 python -u bench.py --config cfg4 --steps 5 --warmup 2 > gpurun_out/r02_ab2_cfg4_$v.json 2> gpurun_out/r02_ab2_cfg4_$v.err || exit $?
done
echo ab_done
