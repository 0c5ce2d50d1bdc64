set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_stage1_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5u_s1.log 2>&1 || { echo s1 tests failed; grep -E "FAIL|Error|assert" gpurun_out/r5u_s1.log | head -30; exit 1; }
tail -2 gpurun_out/r5u_s1.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5u_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r5u_bench.log; exit 1; }
tail -1 gpurun_out/r5u_bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5u_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r5u_prof.log 2>&1 || { echo prof failed; tail -3 $GRAFT_REPO_ROOT/gpurun_out/r5u_prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r5u_prof.log | cut -c1-200
