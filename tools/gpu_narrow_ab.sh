# Narrow-digit scatter instances: the binning GPU tests on the product, then the unskewed bench view and
# the 4K frame, product vs the variants named (tools/gpu_common_ab.sh, tools/sort_ab.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/narrow_test.log 2>&1 && \
bash tools/gpu_common_ab.sh "$@" && \
for r in 1 2; do for v in "" "$@"; do HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/sort_ab.py >> gpurun_out/narrow_sortab.log 2>&1 || exit 1; done; done
echo rc=$?
