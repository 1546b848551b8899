# 128-digit scatter instances at every size (n4k) vs the product's 12M-pair limit, with non-temporal loads.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
HIDEGS_LIB=variants/libhidegs_n4k.so timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q -k "raster_keys or tile_pairs or config5" --timeout 120 --timeout-method thread > gpurun_out/n4k_test.log 2>&1 || exit 1
for r in 1 2 3; do for v in "" n4k; do HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/sort_ab.py >> gpurun_out/n4k_sortab.log 2>&1 || exit 1; done; done
echo rc=$?
