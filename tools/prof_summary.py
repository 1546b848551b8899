"""Summarise rocprofv3 CSV output per (kernel, grid size): kernel-trace durations and
PMC FETCH_SIZE / WRITE_SIZE per launch.

usage: python tools/prof_summary.py KT_DIR [FETCH_DIR WRITE_DIR] > profiles/<name>.md
FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads half the bytes of a
wide coalesced streaming read (MI355X_MICROARCH.md, HBM), so the table gives the raw value
and hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 as the corrected estimate.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(d, suffix):
    f = glob.glob(os.path.join(d, "*" + suffix))
    if not f:
        return []
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    kt = rows(sys.argv[1], "kernel_trace.csv")
    agg = defaultdict(list)
    for r in kt:
        agg[(r["Kernel_Name"], int(r.get("Grid_Size") or r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[2:]:
        for r in rows(d, "counter_collection.csv"):
            pmc[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | grid (threads) | launches | avg us | min us | max us | FETCH_SIZE KiB | WRITE_SIZE KiB | corrected HBM MB/launch |")
    print("|---|---|---|---|---|---|---|---|---|")
    out = {}
    for (name, grid), ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        c = pmc.get((name, grid), {})
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) if c.get("FETCH_SIZE") else None
        w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) if c.get("WRITE_SIZE") else None
        hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
        print(f"| {name} | {grid} | {len(ds)} | {sum(ds)/len(ds)/1e3:.2f} | {min(ds)/1e3:.2f} | {max(ds)/1e3:.2f} | "
              f"{'' if f is None else f'{f:.0f}'} | {'' if w is None else f'{w:.0f}'} | "
              f"{'' if hbm is None else f'{hbm/1e6:.1f}'} |")
        out[f"{name}@{grid}"] = {"avg_us": sum(ds) / len(ds) / 1e3, "launches": len(ds), "fetch_kib": f,
                                 "write_kib": w, "hbm_bytes_per_launch": hbm}
    if os.environ.get("PROF_JSON"):
        with open(os.environ["PROF_JSON"], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
