#!/bin/bash
# Counters of the panel-resident share GEMM alone (configs 6 and 8): issue mix and waits
# in the first pass, the memory path's queues and MFMA / VALU co-execution in the second.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MODE=${1:-1:2}
P1="SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_WAIT_INST_LDS"
for c in 6 8; do
  n=0
  for pmc in "$P1" "$P2"; do
    n=$((n + 1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $R/gpurun_out/pmc_panel${c}_$n -o g -- python $R/scripts/exp_gemm_fold.py $c --only $MODE > $R/gpurun_out/pmc_panel${c}_$n.log 2>&1 || { tail -20 $R/gpurun_out/pmc_panel${c}_$n.log; exit 1; }
  done
  python $R/scripts/pmc_simple.py $(find $R/gpurun_out/pmc_panel${c}_1 $R/gpurun_out/pmc_panel${c}_2 -name "*counter_collection.csv") > $R/gpurun_out/pmc_panel$c.txt
  head -2 $R/gpurun_out/pmc_panel$c.txt
done
