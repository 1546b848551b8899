# distCUDA2 kernel timing against variant libraries (tools/build_variant.py).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/knn_time.py || exit 1
for v in "$@"; do echo "== $v"; HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 120 python tools/knn_time.py || exit 1; done
