#!/bin/bash
# Per-kernel times with nothing overlapping: usage gpu_kstats_serial.sh CONFIG [CONFIG...]
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for c in "$@"; do
  echo "== config $c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rts -o rt -- python $R/scripts/serial_kstats.py $c 3 > $O/kstats_serial$c.log 2>&1 || { tail -20 $O/kstats_serial$c.log; exit 1; }
  python $R/scripts/kstats.py $(find $O/rts -name "*kernel_stats.csv" | head -1) 4 > $O/kstats_serial$c.txt
  rm -rf $O/rts
  head -22 $O/kstats_serial$c.txt
done
