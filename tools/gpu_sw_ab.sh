cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/sw.log; : > $L
for v in "" sw16 "" sw16; do echo "== ${v:-product}" >> $L; HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/skew_time.py none >> $L 2>&1 || exit 1; done
