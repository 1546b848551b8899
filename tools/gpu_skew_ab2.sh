# Binning GPU tests on the product, then skewed D2 views (tools/skew_time.py) product vs the variants, twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/skab_test.log 2>&1 || exit 1
for r in 1 2; do for v in "" "$@"; do
  echo "== ${v:-product}" >> gpurun_out/skab.log
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/skew_time.py none 0.15:0.1 0.5:0.02 >> gpurun_out/skab.log 2>&1 || exit 1
done; done
echo rc=$?
