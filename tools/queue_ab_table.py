"""Table of whole-sort times per build from gpurun_out/queue_ab.log (tools/gpu_queue_ab.sh output)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/queue_ab.log"
tag, rows = None, {}
for ln in open(path):
    if ln.startswith("=="):
        tag = ln[3:].strip()
        continue
    m = re.match(r"(.{14,30}?)\s+n=\d+: sort\s+([\d.]+) us", ln)
    if m:
        rows.setdefault(m.group(1).strip(), {})[tag] = m.group(2)
        continue
    m = re.match(r"\s*([\d.:a-z]+): K .*?  sort\s+([\d.]+) us", ln)
    if m:
        rows.setdefault("D2 " + m.group(1), {})[tag] = m.group(2)
for k, v in rows.items():
    print(f"{k:28s}", "  ".join(f"{t} {x}" for t, x in v.items()))
