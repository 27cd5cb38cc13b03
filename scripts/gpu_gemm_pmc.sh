#!/bin/bash
# PMC counters of the modular GEMM (one rocprofv3 pass per counter set; kernel-trace only).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 -L > $R/gpurun_out/counters_avail.txt 2>&1 || true
grep -c . $R/gpurun_out/counters_avail.txt
timeout -k 10 120 python $R/scripts/bench_modgemm.py
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $R/gpurun_out/pmc_gemm -o g -- python $R/scripts/bench_modgemm.py > $R/gpurun_out/pmc_gemm.log 2>&1 || { tail -20 $R/gpurun_out/pmc_gemm.log; exit 1; }
f=$(find $R/gpurun_out/pmc_gemm -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "modgemm" not in k:
        continue
    agg["modgemm"][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[r["Counter_Name"]] += 1
for name, v in sorted(agg["modgemm"].items()):
    print(f"{name:32s} {v / max(1, cnt[name]):16.0f} per dispatch ({cnt[name]} dispatches)")
PY
