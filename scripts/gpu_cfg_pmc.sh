#!/bin/bash
# Issue-mix and wave-time counters of a benchmark configuration, kernels serialised
# (scripts/serial_kstats.py): usage gpu_cfg_pmc.sh CONFIG
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
c=$1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM"; do
  i=$((i+1))
  echo "pmc pass $i: $set"
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/cpmc$i -o p -- python $R/scripts/serial_kstats.py $c 1 > $O/cfg${c}_pmc$i.log 2>&1 || { tail -20 $O/cfg${c}_pmc$i.log; exit 1; }
  cp $(find $O/cpmc$i -name "*counter_collection.csv" | head -1) $O/cfg${c}_pmc$i.csv
  rm -rf $O/cpmc$i
done
python $R/scripts/pmc_simple.py $O/cfg${c}_pmc1.csv $O/cfg${c}_pmc2.csv > $O/cfg${c}_pmc.txt
cat $O/cfg${c}_pmc.txt
