#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u bench_configs.py --config 8 --check --steps 2 --warmup 1 > gpurun_out/config8.json 2> gpurun_out/config8.err || { tail -20 gpurun_out/config8.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/config8.json').read().strip().splitlines()[-1]);print('config8',d['ms_per_round'],d['correct'])"
timeout -k 10 600 python bench_configs.py --config 6 --check --steps 2 --warmup 1 > gpurun_out/pss155_1kx1m.json 2> gpurun_out/config6.err || { tail -20 gpurun_out/config6.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/pss155_1kx1m.json').read().strip().splitlines()[-1]);print('config6',d['ms_per_round'],d['correct'])"
