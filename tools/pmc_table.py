"""Average PMC counter values per kernel from rocprofv3 CSV dirs (tools/pmc_sort.sh output).

usage: python tools/pmc_table.py gpurun_out/pmc1 gpurun_out/pmc2 ...
"""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("void hidegs::(anonymous namespace)::", "")
                key = (name, r.get("Grid_Size", ""), r.get("Dispatch_Id", r.get("Correlation_Id", "")))
                vals[(name, r.get("Grid_Size", ""))][r["Counter_Name"]].append((key[2], float(r["Counter_Value"])))
for (name, grid), cs in sorted(vals.items()):
    print(f"{name} grid={grid}")
    for c, lst in sorted(cs.items()):
        per = defaultdict(float)
        for disp, v in lst:
            per[disp] += v
        avg = sum(per.values()) / max(len(per), 1)
        print(f"   {c:24s} {avg:16.1f}  (launches {len(per)})")
