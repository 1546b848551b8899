# Hot-tile scouts A/B: binning parity tests on the default build, then tools/skew_time.py per variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/binning_tests.log 2>&1 && \
echo "== default" > gpurun_out/skew_ab.log && timeout -k 10 200 python -u tools/skew_time.py >> gpurun_out/skew_ab.log 2>&1 && \
for v in "$@"; do echo "== $v" >> gpurun_out/skew_ab.log && HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 200 python -u tools/skew_time.py >> gpurun_out/skew_ab.log 2>&1 || exit 1; done
