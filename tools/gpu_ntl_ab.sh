# Scatter non-temporal input loads: sort tests against the variant, then the D2 view and sort_ab, product vs variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
HIDEGS_LIB=variants/libhidegs_ntl.so timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q -k "raster_keys or tile_pairs" --timeout 120 --timeout-method thread > gpurun_out/narrow_test.log 2>&1 || exit 1
bash tools/gpu_common_ab.sh ntl || exit 1
for r in 1 2; do for v in "" ntl; do HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/sort_ab.py >> gpurun_out/narrow_sortab.log 2>&1 || exit 1; done; done
echo rc=$?
