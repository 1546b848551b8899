# A/B of partition-queue builds (variants/libhidegs_TAG.so) on the skewed and one-tile views:
# bash tools/gpu_queue_ab.sh TAG ...   (the product build first)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/queue_ab.log; : > $L
for v in "" "$@"; do
  echo "== ${v:-product}" >> $L
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/extreme_time.py >> $L 2>&1 || exit 1
  HIDEGS_LIB=${v:+variants/libhidegs_$v.so} timeout -k 10 200 python -u tools/skew_time.py >> $L 2>&1 || exit 1
done
