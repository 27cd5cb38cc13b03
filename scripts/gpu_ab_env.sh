#!/bin/bash
# A/B of environment switches on the headline bench: usage gpu_ab_env.sh VAR=VAL [VAR=VAL ...]
# Each setting: kernel tests, then 10 timed rounds; then per-kernel times of the last setting.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for kv in base "$@"; do
  if [ "$kv" != base ]; then export $kv; fi
  timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/ab_tests_$kv.log 2>&1 || { tail -30 $O/ab_tests_$kv.log; exit 1; }
  timeout -k 10 120 python $R/bench.py --steps 10 --warmup 3 > $O/ab_$kv.log 2>&1 || { tail -20 $O/ab_$kv.log; exit 1; }
  echo "$kv: $(tail -1 $O/ab_tests_$kv.log) $(tail -1 $O/ab_$kv.log | grep -o '"ms_per_step": [0-9.]*')"
  last=$kv
  if [ "$kv" != base ]; then unset ${kv%%=*}; fi
done
if [ "$last" != base ]; then export $last; fi
bash $R/scripts/gpu_kstats.sh
