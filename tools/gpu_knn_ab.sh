# distCUDA2 A/B of knn builds (variants/libhidegs_TAG.so) against the product: bash tools/gpu_knn_ab.sh TAG ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/knn_ab.log; : > $L
for v in "" "$@"; do
  echo "== ${v:-product}" >> $L
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/knn_time.py >> $L 2>&1 || exit 1
done
