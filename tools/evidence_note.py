"""Write profiles/<NAME>.md: the evidence that the driver's round-end GPU tiers will find a suite that
runs start to finish on this tree, from a tools/gpu_round6.sh run in gpurun_out/:
the commit, the kernel sources' hash, the `pytest -m gpu` pass line and wall time, the smoke's wall time,
the in-tree .so files the test process mapped, the command that builds every one of them, and the lines
the tests printed about when asynchronous errors surfaced.

usage: python tools/evidence_note.py NAME [COMMIT]   (COMMIT: the commit the gpurun snapshot was taken at;
       default HEAD -- give it when tools/ or profiles/ commits landed after the run)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")


def read(name):
    with open(os.path.join(G, name)) as f:
        return f.read().strip()


def main():
    name = sys.argv[1]
    need = ["gputest.log", "smoke.log", "t_gputest0", "t_gputest1", "t_smoke1", "maps_gputest.txt", "sources.sha256"]
    missing = [n for n in need if not os.path.exists(os.path.join(G, n))]
    if missing:  # a failed or partial session: write nothing
        sys.exit(f"evidence_note: missing {missing}")
    rev = sys.argv[2] if len(sys.argv) > 2 else "HEAD"
    head = subprocess.run(["git", "rev-parse", rev], cwd=ROOT, capture_output=True, text=True).stdout.strip()
    dirty = "" if rev != "HEAD" else subprocess.run(
        ["git", "status", "--porcelain", "--", ".", ":!profiles", ":!gpurun_out"], cwd=ROOT, capture_output=True,
        text=True).stdout.strip()
    t0, t1, t2 = (float(read(n)) for n in ("t_gputest0", "t_gputest1", "t_smoke1"))
    log = read("gputest.log").splitlines()
    summary = log[-1]
    # pytest -q -s prints its progress dots on the same line as the test's own output
    printed = [m.group(0) for ln in log for m in [re.search(r"(HIDEGS_E_ASYNC|stall_|crash_).*", ln)] if m]
    slow = []
    in_dur = False
    for ln in log:
        if "slowest" in ln and "durations" in ln:
            in_dur = True
            continue
        if in_dur:
            if not ln.strip() or ln.startswith("="):
                break
            slow.append(ln)
    maps = read("maps_gputest.txt").splitlines()
    sys.path.insert(0, ROOT)
    from hidegs_amd import build
    lib_cmd = " ".join(["hipcc", *build.FLAGS]).replace(build.INCLUDE, "include")
    with open(os.path.join(ROOT, "profiles", f"{name}.md"), "w") as f:
        f.write(f"# {name}: the GPU suite and smoke on the round's tree\n\n")
        f.write(f"* Commit: `{head}`{' (with uncommitted changes: ' + dirty.replace(chr(10), '; ') + ')' if dirty else ''}.\n")
        f.write(f"* Kernel sources hash (`bench.sources_sha256`, taken on the box): `{read('sources.sha256')}`.\n")
        f.write("* Command: `tools/gpu_round6.sh` (one gpurun call): `pytest tests -m gpu -x -q --timeout 120 "
                "--timeout-method thread`, then `python -c 'import __graft_entry__ as g; g.smoke()'`.\n")
        f.write(f"* `pytest -m gpu`: **{summary}**; wall time {t1 - t0:.1f} s (including the first `import torch`).\n")
        f.write(f"* `smoke()`: wall time {t2 - t1:.1f} s. Its output:\n\n```\n{read('smoke.log')}\n```\n\n")
        f.write("* In-tree shared objects the test process mapped (`tests/conftest.py`, `HIDEGS_MAPS_OUT`):\n")
        for m in maps:
            f.write(f"  * `{m}`\n")
        f.write("* Every one of them is produced by `__graft_entry__.build()`, which the driver runs on the CPU:\n")
        f.write(f"  * `hidegs_amd/libhidegs.so`: `hidegs_amd.build.build()`: each of {', '.join(build.SOURCES)} "
                f"compiled by `{lib_cmd} -c`, linked by `hipcc --offload-arch=gfx950 -shared -fPIC`;\n")
        for tag, (defs, changed) in build.VARIANTS.items():
            f.write(f"  * `hidegs_amd/variants/libhidegs_{tag}.so`: the same, with {' '.join(defs)} on "
                    f"{', '.join(changed)} (test-only builds that drive error paths);\n")
        f.write("  * `oracle/_build/liboracle.so`: `oracle.build()` (gcc, `oracle/Makefile`): the CPU oracle, test "
                "infrastructure only;\n")
        f.write("  * `tests/c_abi/abi_client` (a program, run as a child): `hidegs_amd.build.build_abi_client()`.\n")
        if printed:
            f.write("\nWhat the tests printed (asynchronous error timing, fail-fast):\n\n```\n" + "\n".join(printed) + "\n```\n")
        if slow:
            f.write("\nSlowest tests:\n\n```\n" + "\n".join(slow) + "\n```\n")


if __name__ == "__main__":
    main()
