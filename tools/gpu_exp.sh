cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
HIDEGS_LIB=variants/libhidegs_qtrace.so timeout -k 10 300 python -u tools/queue_trace.py skew:0.05:0.1 > gpurun_out/qtrace.log 2>&1
