#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total/avg per round."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rounds = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"{'kernel':64s} {'calls':>5s} {'ms/round':>9s} {'avg ms':>8s} {'%':>5s}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:18]:
    name = r['Name'].replace('sdagpu::(anonymous namespace)::', '').replace('void ', '')[:64]
    print(f"{name:64s} {r['Calls']:>5s} {float(r['TotalDurationNs'])/1e6/rounds:9.3f} {float(r['AverageNs'])/1e6:8.3f} {float(r['Percentage']):5.1f}")
print(f"total kernel time per round: {tot/1e6/rounds:.2f} ms")
