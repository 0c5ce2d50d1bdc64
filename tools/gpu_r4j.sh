#!/bin/bash
# round-4: stage timers test + per-stage step breakdown, SigLIP forward stamps, q/k-norm backward piece loads (stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_stage_timers_gpu.py tests/test_dkv_fused_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r4j_tests.log | tail -1; grep -E "^E  " gpurun_out/r4j_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --stage-timers > gpurun_out/r4j_bench_stages.log 2>&1 || { echo "stage bench failed"; tail -5 gpurun_out/r4j_bench_stages.log; exit 1; }
tail -1 gpurun_out/r4j_bench_stages.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']); [print(k, v) for k, v in d.get('stages_ms_per_step', {}).items()]"
timeout -k 10 200 python -u tools/fa_stamps.py 0 fwd64 > gpurun_out/r4j_fa64_stamps.log 2>&1; echo "fa64 stamps rc=$?"; tail -3 gpurun_out/r4j_fa64_stamps.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4j_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r4j_prof.log 2>&1 || { echo "prof failed"; tail -3 $R/gpurun_out/r4j_prof.log; exit 1; }
db=$(find $R/gpurun_out/r4j_prof -name "*.db" | head -1); python3 $R/tools/rocpd_stats.py $db $R/gpurun_out/r4j_stats.csv
grep -E "qknorm|residual_norm" $R/gpurun_out/r4j_stats.csv | cut -c1-60,200-260
cd $R
for sh in "22528 1152 1024 0 g_o" "22528 1152 1024 1 g_o" "18432 3072 1024 0 sig_qkv" "18432 3072 1024 1 sig_qkv" "22528 1536 1152 0 g_qkv" "22528 13824 1152 0 gate_up_plain" "22528 13824 1152 1 gate_up_plain" "22528 1152 13824 0 dgu_dX"; do
  timeout -k 10 120 python -u tools/p8_stamps.py $sh >> gpurun_out/r4j_p8_stamps.log 2>&1 || { echo "p8 stamps failed: $sh"; tail -3 gpurun_out/r4j_p8_stamps.log; exit 1; }
done
grep -v Warn gpurun_out/r4j_p8_stamps.log | cut -c1-600
