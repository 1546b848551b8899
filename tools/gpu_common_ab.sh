# The unskewed bench view only, product vs variants alternating (noise of a few us between runs):
# bash tools/gpu_common_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/common_ab.log; : > $L
for r in 1 2 3; do for v in "" "$@"; do
  echo "== ${v:-product}" >> $L
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/skew_time.py none >> $L 2>&1 || exit 1
done; done
