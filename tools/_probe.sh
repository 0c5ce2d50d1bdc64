cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for s in "8192 8192 8192"; do
  for lib in "" build/libptk_abl1.so build/libptk_abl3.so build/libptk_abl4.so build/libptk_abl5.so build/libptk_abl2.so; do
    echo "$lib"; PTK_LIB=$lib timeout -k 10 60 python tools/gemm_probe.py $s 0 8 30 || exit 1
  done
done
