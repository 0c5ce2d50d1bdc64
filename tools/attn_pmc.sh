#!/bin/bash
# Two SQ counter passes over the attention microbenchmark, for the default kernels and an env-selected variant.
# usage: bash tools/attn_pmc.sh TAG [ENV=VAL ...]   (writes gpurun_out/pmc_TAG_{1,2}/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
for kv in "$@"; do export "$kv"; done
what=${ATTN_WHAT:-fwd}
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "attn_" --output-format csv -d gpurun_out/pmc_${tag}_1 -o run -- python3 tools/attn_bench.py --what $what --reps 3 > gpurun_out/pmc_${tag}_1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-include-regex "attn_" --output-format csv -d gpurun_out/pmc_${tag}_2 -o run -- python3 tools/attn_bench.py --what $what --reps 3 > gpurun_out/pmc_${tag}_2.log 2>&1 || exit $?
python3 tools/pmc_dump.py gpurun_out/pmc_${tag}_1/run_counter_collection.csv gpurun_out/pmc_${tag}_2/run_counter_collection.csv > gpurun_out/pmc_${tag}.txt
