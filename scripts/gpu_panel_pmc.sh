#!/bin/bash
# Issue counters of the panel-resident share GEMM alone (configs 6 and 8), one rocprofv3 pass.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in 6 8; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/pmc_panel$c -o g -- python $R/scripts/exp_gemm_fold.py $c --only 1:2 > $R/gpurun_out/pmc_panel$c.log 2>&1 || { tail -20 $R/gpurun_out/pmc_panel$c.log; exit 1; }
  f=$(find $R/gpurun_out/pmc_panel$c -name "*counter_collection.csv" | head -1)
  python $R/scripts/pmc_simple.py "$f" > $R/gpurun_out/pmc_panel$c.txt
  head -4 $R/gpurun_out/pmc_panel$c.txt
done
