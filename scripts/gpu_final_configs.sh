#!/bin/bash
# Every benchmark configuration of bench_configs.py with its output checked (one JSON
# line each into gpurun_out/final_configN.json), then per-kernel times of the two
# many-clerk configurations. usage: gpu_final_configs.sh [CONFIG ...] (default: all but 4)
set -e
mkdir -p gpurun_out
O=gpurun_out
cfgs=${@:-2 3 5 6 7 8 9 10 11}
for c in $cfgs; do
  extra="--steps 5 --warmup 2"
  [ "$c" = 4 ] && extra=""
  timeout -k 10 600 python bench_configs.py --config $c $extra --check > $O/final_config$c.json 2> $O/final_config$c.err || { tail -20 $O/final_config$c.err; exit 1; }
  python - "$O/final_config$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("config", d["config"], d["name"], "ms/round", round(d["ms_per_round"], 2), "elements/s %.3g" % d["value"],
      "correct", d["correct"], "HBM high water GB", round(d["hbm_high_water_bytes"] / 1e9, 1), flush=True)
PY
done
for c in 6 8; do
  case " $cfgs " in *" $c "*) bash scripts/gpu_kstats_cfg.sh $c > /dev/null && cp $O/kstats_cfg$c.txt $O/final_config${c}_kernel_stats.txt && bash scripts/gpu_kstats_serial.sh $c > /dev/null && cp $O/kstats_serial$c.txt $O/final_config${c}_kernel_stats_serial.txt && echo "kernel stats of config $c done";; esac
done
