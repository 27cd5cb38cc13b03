#!/bin/bash
# One PMC pass (issue mix) over the headline bench; prints the per-kernel table with the columns that pass feeds.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/pmc1 -o p -- python $R/bench.py --steps 2 --warmup 1 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
python - $(find $O/pmc1 -name "*counter_collection.csv" | head -1) <<'PY'
import csv, sys, re, collections
d = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("sdagpu::(anonymous namespace)::", "").replace("void ", ""))[:36]
    d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
print(f"{'kernel':36s} {'disp':>4s} {'VALU Ginstr':>11s} {'lane-ops/B':>10s} {'LDS Minstr':>10s} {'LDS act Mcyc':>12s} {'conflict Mcyc':>13s} {'wait_lds':>10s}")
for k, c in sorted(d.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"])[:8]:
    per = 3.0  # rounds in the run (1 warm-up + 2 timed) -- plus the check round
    print(f"{k:36s} {n[k]:4d} {c['SQ_INSTS_VALU']/1e9:11.3f} {c['SQ_INSTS_VALU']*64/5.56e9/per:10.2f} {c['SQ_INSTS_LDS']/1e6:10.1f} {c['SQ_ACTIVE_INST_LDS']/1e6:12.1f} {c['SQ_LDS_BANK_CONFLICT']/1e6:13.1f} {c['SQ_WAIT_INST_LDS']/1e6:10.1f}")
PY
rm -rf $O/pmc1
