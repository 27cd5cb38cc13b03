# Share kernels: numerics (16-bit halves and three draws per word), A/B timing, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_share16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t48.log 2>&1 && \
timeout -k 10 200 python -u scripts/debug/share_bench.py > gpurun_out/share_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stages > gpurun_out/bench48.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stages >> gpurun_out/bench48.log 2>&1
