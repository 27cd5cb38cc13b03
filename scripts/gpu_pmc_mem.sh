#!/bin/bash
# Memory-path counters per kernel of the headline round (vector L1 accesses and stalls, L1->L2 requests, TA busy).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_FLAT_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmcm -o p -- python $R/bench.py --steps 2 --warmup 1 > $O/pmc_mem.log 2>&1 || { tail -20 $O/pmc_mem.log; exit 1; }
python - $(find $O/pmcm -name "*counter_collection.csv" | head -1) <<'PY' | tee $O/pmc_mem_table.txt
import csv, sys, re, collections
d = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("sdagpu::(anonymous namespace)::", "").replace("void ", ""))[:34]
    d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE": n[k] += 1
print(f"{'kernel':34s} {'disp':>4s} {'L1 acc M':>9s} {'L1->L2 rd M':>11s} {'L1->L2 wr M':>11s} {'TA wave M':>9s} {'TA busy%':>8s} {'TD busy%':>8s} {'L1 pend stall%':>14s}")
for k, c in sorted(d.items(), key=lambda kv: -kv[1]["TCP_TOTAL_CACHE_ACCESSES_sum"])[:8]:
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0  # summed over 8 XCDs
    cu_cyc = cyc * 256
    print(f"{k:34s} {n[k]:4d} {c['TCP_TOTAL_CACHE_ACCESSES_sum']/1e6:9.1f} {c['TCP_TCC_READ_REQ_sum']/1e6:11.1f} {c['TCP_TCC_WRITE_REQ_sum']/1e6:11.1f} {c['TA_FLAT_WAVEFRONTS_sum']/1e6:9.2f} {100*c['TA_TA_BUSY_sum']/cu_cyc:8.1f} {100*c['TD_TD_BUSY_sum']/cu_cyc:8.1f} {100*c['TCP_PENDING_STALL_CYCLES_sum']/cu_cyc:14.1f}")
PY
rm -rf $O/pmcm
