#!/bin/bash
# Parametrised GPU-box checks of this tree (replaces the per-round one-off scripts).
#   ROUND=r05 tools/gpu_round.sh [part ...]
# parts (default: tests smoke bench prof): tests | smoke | bench | stages | cfg5 | cfg4 | prof | pmc
#   tests   full `pytest -m gpu` (TESTS=<pytest args> / KEXPR=<-k expression> select a subset)
#   smoke   __graft_entry__.smoke()
#   bench   default bench.py line (with the CPU baseline)
#   stages  bench.py --stage-timers (per-stage breakdown)
#   cfg5 / cfg4   the Gemma3-4B Stage-1 and the Stage-2 bench lines
#   prof    rocprofv3 --kernel-trace --stats of bench.py (kernel statistics CSV)
#   pmc     the two FETCH / WRITE counter passes of the dominant kernel (tools/pmc_traffic.py)
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
T=${ROUND:-rXX}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PARTS=("$@")
[ ${#PARTS[@]} -eq 0 ] && PARTS=(tests smoke bench prof)
fail() { echo "$1 failed (rc $2)"; tail -5 "$3"; exit 1; }
for part in "${PARTS[@]}"; do
  log=gpurun_out/${T}_$part.log
  case $part in
    tests)
      KARGS=()
      [ -n "${KEXPR:-}" ] && KARGS=(-k "$KEXPR")
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread ${TESTS:-} "${KARGS[@]}" > $log 2>&1
      rc=$?; grep -E "passed|failed" $log | tail -1; grep -E "FAILED|Error" $log | head -5
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail smoke $? $log
      grep smoke: $log ;;
    bench)
      timeout -k 10 600 python -u bench.py > $log 2>&1 || fail bench $? $log
      tail -1 $log | cut -c1-400 ;;
    stages)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --stage-timers > $log 2>&1 || fail stages $? $log
      tail -1 $log | cut -c1-300 ;;
    cfg5)
      timeout -k 10 300 python -u bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $log 2>&1 || fail cfg5 $? $log
      tail -1 $log | cut -c1-300 ;;
    cfg4)
      timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline > $log 2>&1 || fail cfg4 $? $log
      tail -1 $log | cut -c1-300 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps ${PROF_STEPS:-5} --warmup 2) > $log 2>&1 \
        || fail prof $? $log
      tail -1 $log | cut -c1-300 ;;
    pmc)
      K=${PMC_KERNEL:-gemm_w4_kernel<3}
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "$K" \
          --output-format csv -d $R/gpurun_out/${T}_pmc_$c -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline) \
          > gpurun_out/${T}_pmc_$c.log 2>&1 || fail "pmc $c" $? gpurun_out/${T}_pmc_$c.log
      done
      python3 tools/pmc_traffic.py gpurun_out/${T}_pmc_FETCH_SIZE/run_counter_collection.csv \
        gpurun_out/${T}_pmc_WRITE_SIZE/run_counter_collection.csv "$K" gpurun_out/${T}_pmc_traffic.json > $log 2>&1 \
        || fail pmc $? $log
      tail -1 $log | cut -c1-300 ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
