#!/bin/bash
# One-GPU headline round under rocprofv3: kernel trace + stats, then one PMC pass per counter set
# (issue mix, wave-time split, HBM reads, HBM writes). Summaries land in gpurun_out/round_*.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rt -o rt -- python $R/bench.py --steps 5 --warmup 2 > $O/round_trace.log 2>&1 || { tail -20 $O/round_trace.log; exit 1; }
cp $(find $O/rt -name "*kernel_stats.csv" | head -1) $O/round_kernel_stats.csv
python $R/scripts/kstats.py $O/round_kernel_stats.csv 7 > $O/round_kernel_stats.txt
python $R/scripts/round_timeline.py $(find $O/rt -name "*kernel_trace.csv" | head -1) --min-us 15 > $O/round_timeline.txt
rm -rf $O/rt
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pmc pass $i: $set"
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc$i -o p -- python $R/bench.py --steps 2 --warmup 1 > $O/round_pmc$i.log 2>&1 || { tail -20 $O/round_pmc$i.log; exit 1; }
  cp $(find $O/pmc$i -name "*counter_collection.csv" | head -1) $O/round_pmc$i.csv
  rm -rf $O/pmc$i
done
python $R/scripts/round_pmc_table.py $O/round_pmc1.csv $O/round_pmc2.csv $O/round_pmc3.csv $O/round_pmc4.csv $O/round_pmc5.csv $O/round_kernel_stats.csv 7 > $O/round_pmc_table.txt
cat $O/round_pmc_table.txt
