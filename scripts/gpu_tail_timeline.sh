#!/bin/bash
# Kernel timeline of headline rounds (every kernel of 2 us and more, with its queue) from
# several processes: shows where a round's result path runs against the next round's kernels.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tt$i -o tt -- python $R/bench.py --steps 8 --warmup 3 > $O/tail_trace$i.log 2>&1 || { tail -20 $O/tail_trace$i.log; exit 1; }
  python - <<PY
import json
l=[x for x in open("$O/tail_trace$i.log") if x.startswith("{")][-1]
print("run $i ms_per_step", json.loads(l)["ms_per_step"])
PY
  python $R/scripts/round_timeline.py $(find $O/tt$i -name "*kernel_trace.csv" | head -1) --min-us 2 > $O/tail_timeline$i.txt
  head -1 $O/tail_timeline$i.txt
  rm -rf $O/tt$i
done
