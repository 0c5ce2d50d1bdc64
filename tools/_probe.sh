cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd gpurun_out && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "attn_" --output-format csv -d pmc -o run -- python3 ../bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
  for k in attn_bwd_dkv256 attn_bwd_dq_kernel attn_fwd_kernel\<256 attn_fwd_kernel\<64; do python3 ../tools/pmc_sum.py pmc/run_counter_collection.csv "$k" "$k"; done
  rm -rf pmc
done
