#!/bin/bash
# Issue-mix counters of the encode + encrypt kernel alone (scripts/exp_encode_alone.py):
# usage gpu_encode_pmc.sh [MODULUS [BOXES [VALUES]]]
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM"; do
  i=$((i+1))
  echo "pmc pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/epmc$i -o p -- python $R/scripts/exp_encode_alone.py "$@" > $O/enc_pmc$i.log 2>&1 || { tail -20 $O/enc_pmc$i.log; exit 1; }
  cp $(find $O/epmc$i -name "*counter_collection.csv" | head -1) $O/enc_pmc$i.csv
  rm -rf $O/epmc$i
done
python $R/scripts/pmc_simple.py $O/enc_pmc1.csv $O/enc_pmc2.csv > $O/enc_pmc.txt
grep -A1 "k_encode_encrypt" $O/enc_pmc.txt
