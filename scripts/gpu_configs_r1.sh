# BASELINE configs 3, 4 (one full 10k x 125M round), 5 on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python bench_configs.py --config 3 --check > gpurun_out/config3.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 5 --check > gpurun_out/config5.log 2>&1 && \
timeout -k 10 400 python -u bench_configs.py --config 4 --steps 1 --warmup 0 > gpurun_out/config4.log 2>&1
