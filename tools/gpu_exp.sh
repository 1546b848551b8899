cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_skew_ab.sh "$@" && timeout -k 10 300 python -u tools/extreme_time.py > gpurun_out/ext.log 2>&1 && \
for v in "$@"; do echo "== $v" >> gpurun_out/ext.log; HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 300 python -u tools/extreme_time.py >> gpurun_out/ext.log 2>&1 || exit 1; done
