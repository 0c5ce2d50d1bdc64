#!/bin/bash
# GPU-box check runner: each step has its own time limit; stops at the first
# step that ends in anything but success (0) or a plain test failure (1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {
  local name=$1 to=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    kernels) run kernels 400 python -m pytest tests/test_kernels_gpu.py -q -x -rs ;;
    stage1)  run stage1 600 python -m pytest tests/test_stage1_gpu.py -q -x -rs ;;
    gputests) run gputests 900 python -m pytest tests -m gpu -q -x -rs ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benchfull) run benchfull 900 python bench.py ;;
    gemmbench) run gemmbench 300 python tools/gemm_bench.py ;;
    prof)    run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    pmcfetch) run pmcfetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "gemm_(big|w4)_kernel<3" --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcwrite) run pmcwrite 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "gemm_(big|w4)_kernel<3" --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmcdkv) run pmcdkv 600 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex "dkv256" --output-format csv -d gpurun_out/pmc_dkv -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    stage2)  run stage2 600 python -m pytest tests/test_stage2_gpu.py -q -x -rs ;;
    prof2)   run prof2 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --config cfg4 --steps 3 --warmup 1 ;;
    bench4)  run bench4 600 python bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu-baseline ;;
    sqpmc4)  run sqpmc4 600 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqpmc4 -o run -- python3 bench.py --config cfg4 --gas 1 --steps 2 --warmup 1 --no-cpu-baseline ;;
    sqpmc)   run sqpmc 600 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqpmc -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcattn1) run pmcattn1 600 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "attn_" --output-format csv -d gpurun_out/pmc_attn1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcattn2) run pmcattn2 600 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "attn_" --output-format csv -d gpurun_out/pmc_attn2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step" ;;
  esac
done
