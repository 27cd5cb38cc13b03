#!/usr/bin/env python3
"""Per-round timeline from a rocprofv3 kernel_trace.csv: each kernel's start
offset, duration and the idle gap before it on its queue (last N kernels)."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
last_end = {}
for r in rows:
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
    gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
    last_end[q] = e
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("sdagpu::(anonymous namespace)::", "")
                  .replace("void ", ""))[:44]
    print(f"q{q:>2} {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:8.1f}  {name}")
