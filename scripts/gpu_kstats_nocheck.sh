#!/bin/bash
# Per-kernel MINIMUM and median times over 8 unchecked rounds (scripts/exp_round.py): for timing
# kernel variants whose output may be wrong.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rt -o rt -- python $R/scripts/exp_round.py 8 > $O/kstats.log 2>&1 || { tail -20 $O/kstats.log; exit 1; }
python - $(find $O/rt -name "*kernel_trace.csv" | head -1) <<'PY'
import csv, sys, re, statistics, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("sdagpu::(anonymous namespace)::", "").replace("void ", ""))[:40]
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in sorted(d.items(), key=lambda kv: -max(kv[1])):
    big = [x for x in v if x > 0.3 * max(v)]
    if max(v) < 0.3: continue
    print(f"{n:40s} n={len(big):3d} min {min(big):7.3f} median {statistics.median(big):7.3f} ms")
PY
rm -rf $O/rt
