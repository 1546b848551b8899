# Masked Adam timing against variant libraries (tools/build_variant.py).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/adam_time.py || exit 1
for v in "$@"; do HIDEGS_LIB=variants/libhidegs_$v.so timeout -k 10 120 python tools/adam_time.py || exit 1; done
