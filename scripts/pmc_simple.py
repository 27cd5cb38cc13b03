#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter_collection.csv files (one per PMC pass).

usage: pmc_simple.py pass1.csv [pass2.csv ...]
Prints, per kernel, the mean of every counter per dispatch and a few ratios:
  valu_ms   SQ_INSTS_VALU x 64 / (256 CUs x 64 lanes x 2.4 GHz): the time the VALU
            instructions alone need at the integer issue peak
  lds%conf  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  ms        mean dispatch duration in that (instrumented, serialised) run
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("sdagpu::", ""))
    return n.replace("void ", "")[-40:]


per = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for path in sys.argv[1:]:
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (path, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
rows = []
for k, cs in per.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    ms = sum(dur[k]) / len(dur[k])
    rows.append((ms * len(dur[k]), k, ms, len(dur[k]), m))
for _, k, ms, n, m in sorted(rows, reverse=True)[:14]:
    valu_ms = m.get("SQ_INSTS_VALU", 0) * 64 / (256 * 64 * 2.4e9) * 1e3
    conf = m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, m.get("SQ_ACTIVE_INST_LDS", 0))
    print(f"{k:40s} n={n:3d} ms={ms:8.3f} valu_ms={valu_ms:7.3f} lds_conf={conf:5.2f}")
    print("    " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
