"""Average rocprofv3 PMC counters per kernel name (all launches) into a JSON file.

usage: python tools/pmc_json.py PMC_DIR OUT.json [KERNEL_SUBSTRING ...]
Keys are kernel names with template/argument decoration cut at the first '(' or '<'; values map
counter name -> average value per launch, plus "launches".
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    want = sys.argv[3:]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for fn in files:
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
                if want and not any(w in name for w in want):
                    continue
                acc[name][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    res = {}
    for name, per in acc.items():
        by_counter = defaultdict(list)
        for (disp, cn), vals in per.items():
            by_counter[cn].append(sum(vals))  # one value per dispatch (summed over dimensions)
        res[name] = {cn: sum(v) / len(v) for cn, v in by_counter.items()}
        res[name]["launches"] = max(len(v) for v in by_counter.values())
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
