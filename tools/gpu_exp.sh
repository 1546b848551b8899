cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
: > gpurun_out/exp.log
for v in "" "$@"; do echo "== ${v:-default}" >> gpurun_out/exp.log; HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/skew_time.py none 0.15:0.1 >> gpurun_out/exp.log 2>&1 || exit 1; done
for v in "$@"; do echo "== tests $v" >> gpurun_out/exp.log; HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "not variant and not overflow" >> gpurun_out/exp.log 2>&1 || exit 1; done
