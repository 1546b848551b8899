# distCUDA2 neighbour-seed filter variant: bit-exactness (the knn GPU tests against the variant) and timing.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
HIDEGS_LIB=variants/libhidegs_seedf.so timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/seedf_test.log 2>&1 && \
bash tools/knn_variants.sh seedf > gpurun_out/seedf_time.log 2>&1 && \
bash tools/knn_variants.sh seedf >> gpurun_out/seedf_time.log 2>&1
echo rc=$?
