# Per-pass cost of segment_sort: run tools/seg_time.py against variant libraries (tools/build_variant.py).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/seg_time.py || exit 1
for v in "$@"; do HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 120 python tools/seg_time.py || exit 1; done
