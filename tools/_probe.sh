cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for s in "8192 8192 8192" "22528 13824 1152"; do
  for lib in "" build/libptk_aux1.so build/libptk_aux2.so build/libptk_aux16.so ""; do
    echo "$lib"; PTK_LIB=$lib timeout -k 10 60 python tools/gemm_probe.py $s 0 2 30 || exit 1
  done
done
