"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel.

Columns: dispatches, total kernel ms, VALU instructions per wave, and the split
of wave time into issuing (ACTIVE_INST_ANY), issue-stalled (WAIT_INST_ANY) and
parked on waitcnt/barrier (WAIT_ANY) -- disjoint, ~sum to WAVE_CYCLES on gfx950.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    n = n.replace("void ", "")
    return n[-60:]


def main(path):
    rows = defaultdict(lambda: defaultdict(float))
    durs = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
        durs[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{'kernel':60s} {'disp':>4s} {'ms':>8s} {'valu/wave':>10s} {'issue%':>7s} "
          f"{'stall%':>7s} {'wait%':>7s} {'valu/act%':>9s}")
    for k, c in sorted(rows.items(), key=lambda kv: -sum(durs[kv[0]].values())):
        ms = sum(durs[k].values())
        if ms < 0.05:
            continue
        waves = max(c["SQ_WAVES"], 1)
        wc = max(c["SQ_WAVE_CYCLES"], 1)
        print(f"{k:60s} {len(durs[k]):4d} {ms:8.3f} {c['SQ_INSTS_VALU'] / waves:10.0f} "
              f"{100 * c['SQ_ACTIVE_INST_ANY'] / wc:7.1f} {100 * c['SQ_WAIT_INST_ANY'] / wc:7.1f} "
              f"{100 * c['SQ_WAIT_ANY'] / wc:7.1f} "
              f"{100 * c['SQ_ACTIVE_INST_VALU'] / max(c['SQ_ACTIVE_INST_ANY'], 1):9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
