# Full GPU test suite, smoke(), headline bench and a kernel-trace profile (round timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_full.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- \
    python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof3.log 2>&1
