set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "weight_grad" -x -v --timeout 200 --timeout-method thread > gpurun_out/r5n_wg.log 2>&1 || { echo wg tests failed; grep -E "FAIL|Error|assert" gpurun_out/r5n_wg.log | head -20; exit 1; }
tail -2 gpurun_out/r5n_wg.log
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5n_cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/r5n_cfg4.log; exit 1; }
tail -1 gpurun_out/r5n_cfg4.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5n_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r5n_prof.log 2>&1 || { echo prof failed; tail -3 $GRAFT_REPO_ROOT/gpurun_out/r5n_prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r5n_prof.log | cut -c1-200
