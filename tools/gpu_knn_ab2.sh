# distCUDA2 variants: bit-exactness (the knn GPU tests against each variant) then timing, twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in "$@"; do
  HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/knnab_test_$v.log 2>&1 || exit 1
done
bash tools/knn_variants.sh "$@" > gpurun_out/knnab_time.log 2>&1 && bash tools/knn_variants.sh "$@" >> gpurun_out/knnab_time.log 2>&1
echo rc=$?
