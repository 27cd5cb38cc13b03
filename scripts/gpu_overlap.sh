#!/bin/bash
# A/B of the seal-side tag pass schedules: default, per-clerk overlap, fused; timeline of the overlap run.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for v in "base:SDA_MAC_OVERLAP=0" "overlap:SDA_MAC_OVERLAP=1" "fused:SDA_FUSED_SEAL_MAC=1"; do
  name=${v%%:*}; kv=${v#*:}
  export $kv
  timeout -k 10 120 python $R/bench.py --steps 10 --warmup 3 > $O/ab_$name.log 2>&1 || { tail -20 $O/ab_$name.log; exit 1; }
  unset ${kv%%=*}
  echo "$name $(tail -1 $O/ab_$name.log | grep -o '"ms_per_step": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
export SDA_MAC_OVERLAP=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rt -o rt -- python $R/bench.py --steps 3 --warmup 2 > $O/ab_trace.log 2>&1 || { tail -20 $O/ab_trace.log; exit 1; }
python $R/scripts/round_timeline.py $(find $O/rt -name "*kernel_trace.csv" | head -1) --min-us 15 > $O/ab_overlap_timeline.txt
rm -rf $O/rt
cat $O/ab_overlap_timeline.txt
