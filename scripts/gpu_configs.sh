# GPU tests, headline bench, and the BASELINE configs on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --stages > gpurun_out/bench_full.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 3 --check > gpurun_out/config3.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 5 --check > gpurun_out/config5.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 4 --participants 256 --check > gpurun_out/config4_small.log 2>&1 && \
timeout -k 10 400 python bench_configs.py --config 4 > gpurun_out/config4.log 2>&1
