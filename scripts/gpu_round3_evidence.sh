#!/bin/bash
# The measurements behind the round's README / BASELINE / DESIGN numbers, in one go:
# every configuration checked (+ kernel tables of 6 and 8), config 11's kernel table, the
# share GEMM alone (general against panel-resident kernel, counters of the latter), the
# MFMA / VALU co-issue micro-benchmark, and the headline bench as the driver runs it.
set -e
mkdir -p gpurun_out
O=gpurun_out
bash scripts/gpu_final_configs.sh 2 3 5 6 7 8 9 10 11
bash scripts/gpu_kstats_cfg.sh 11 > /dev/null && echo "kernel stats of config 11 done"
timeout -k 10 300 python -u scripts/exp_gemm_fold.py > $O/gemm_panel_vs_general.txt 2>&1 || { tail -20 $O/gemm_panel_vs_general.txt; exit 1; }
grep "^config" $O/gemm_panel_vs_general.txt
bash scripts/gpu_panel_pmc.sh 1:2 > $O/panel_pmc_run.log 2>&1 || { tail -20 $O/panel_pmc_run.log; exit 1; }
cat $O/pmc_panel6.txt $O/pmc_panel8.txt | grep -A1 "_panel<" > $O/modgemm_panel_pmc.txt
cat $O/modgemm_panel_pmc.txt | cut -c1-200
hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops scripts/ubench_mfma_valu.hip -o /tmp/ubench_mv 2>/dev/null
timeout -k 10 60 /tmp/ubench_mv > $O/ubench_mfma_valu.txt
cat $O/ubench_mfma_valu.txt
timeout -k 10 300 python bench_configs.py --config 4 --check > $O/final_config4.json 2> $O/final_config4.err || { tail -20 $O/final_config4.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/final_config4.json").read().strip().splitlines()[-1])
print("config 4", d["name"], "s/round", round(d["ms_per_round"] / 1e3, 2), "correct", d["correct"], "HBM high water GB",
      round(d["hbm_high_water_bytes"] / 1e9, 1), flush=True)
PY
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_headline.json 2> $O/bench_headline.err || { tail -20 $O/bench_headline.err; exit 1; }
tail -1 $O/bench_headline.json | cut -c1-300
