#!/usr/bin/env python3
"""One complete round from a rocprofv3 kernel_trace.csv (between the last two
k_gate_wait dispatches, i.e. round starts): per kernel start offset, duration
and idle gap on its queue; kernels shorter than --min-us are folded away."""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--min-us", type=float, default=20.0)
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if "k_gate_wait" in r["Kernel_Name"]]
a, b = starts[-2], starts[-1]
print(f"round span {(b - a) / 1e6:.3f} ms")
last = {}
for r in rows:
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
    if not a <= s < b:
        continue
    gap = (s - last[q]) / 1e3 if q in last else 0.0
    last[q] = e
    if (e - s) / 1e3 < args.min_us:
        continue
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("sdagpu::(anonymous namespace)::", "")
                  .replace("void ", ""))[:44]
    print(f"q{q:>2} {(s - a) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:8.1f}  {name}")
