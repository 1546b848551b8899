cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/giant.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_binning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread >> $L 2>&1 &&
timeout -k 10 200 python -u tools/extreme_time.py >> $L 2>&1 &&
timeout -k 10 200 python -u tools/skew_time.py >> $L 2>&1 &&
HIDEGS_LIB=variants/libhidegs_qtrace.so timeout -k 10 200 python -u tools/queue_trace.py 1000000 8500000 >> $L 2>&1
