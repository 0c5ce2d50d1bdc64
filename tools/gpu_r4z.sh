#!/bin/bash
# round-4 final check on this tree: full GPU suite, smoke, (with ablibs/ present: an attention A/B, stamps + step
# A/B against ablibs/libptk_oldflash.so), default bench (with the CPU baseline), stage timers, cfg5 line, rocprofv3 stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > gpurun_out/r4z_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4z_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4z_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4z_smoke.log; exit 1; }
grep smoke gpurun_out/r4z_smoke.log
[ -f ablibs/libptk_fastamps_old.so ] && for lib in fastamps fastamps_old; do
  for w in "512 fwd" "0 fwd" "512 bwd"; do
    FA_STAMPS_LIB=ablibs/libptk_$lib.so timeout -k 10 120 python -u tools/fa_stamps.py $w > gpurun_out/r4z_fa.log 2>&1 || { echo "fa stamps failed: $lib $w"; tail -3 gpurun_out/r4z_fa.log; exit 1; }
    echo "$lib $w: $(grep -v amdgpu.ids gpurun_out/r4z_fa.log | tr '\n' ' ' | cut -c1-600)" >> gpurun_out/r4z_fa_all.log
  done
done
if [ -f ablibs/libptk_oldflash.so ]; then
  cut -c1-300 gpurun_out/r4z_fa_all.log
  ROUNDS=2 STEPS=10 bash tools/ab.sh new ablibs/libptk_oldflash.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4z_ab.txt
fi
timeout -k 10 500 python -u bench.py > gpurun_out/r4z_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4z_bench.log; exit 1; }
tail -1 gpurun_out/r4z_bench.log | cut -c1-300
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --stage-timers > gpurun_out/r4z_bench_stages.log 2>&1 || { echo "stage bench failed"; exit 1; }
timeout -k 10 200 python -u bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4z_bench_cfg5.log 2>&1 || { echo "cfg5 failed"; tail -3 gpurun_out/r4z_bench_cfg5.log; exit 1; }
tail -1 gpurun_out/r4z_bench_cfg5.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4z_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/r4z_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r4z_prof.log; exit 1; }
db=$(find $R/gpurun_out/r4z_prof -name "*.db" | head -1); python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r4z_stats.csv
head -12 $R/gpurun_out/r4z_stats.csv | cut -c1-150
