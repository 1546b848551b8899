# Small views (config 2 scale): the binning step, product vs the tile-path segmented thresholds named
# (variants/libhidegs_TAG.so), at several view sizes; binning tests against the most aggressive variant first.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/small_ab.log; : > $L
HIDEGS_LIB=variants/libhidegs_tsa1.so timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not variant and not overflow and not maximum" > gpurun_out/small_ab_test.log 2>&1 || exit 1
for r in 1 2; do for n in 20000 50000 100000 200000; do for v in "" "$@"; do
  echo "== ${v:-product} $n" >> $L
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 100 python -u tools/small_view_time.py $n >> $L 2>&1 || exit 1
done; done; done
echo rc=$?
