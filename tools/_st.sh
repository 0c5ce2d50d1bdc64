cd $GRAFT_REPO_ROOT
for args in "22528 13824 1152 3 0" "22528 13824 1152 3 1" "22528 13824 1152 3 2" "22528 13824 1152 0 0" "22528 13824 1152 0 1" "22528 13824 1152 0 2" "8192 8192 8192 0 0"; do
  timeout -k 10 120 python tools/gemm_stamps.py $args || exit 1
done
