# Kernel tests, two headline benches and a kernel-trace profile (round timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -f gpurun_out/bench2.log
mkdir -p gpurun_out/prof2
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stages >> gpurun_out/bench2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stages >> gpurun_out/bench2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- \
    python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1
