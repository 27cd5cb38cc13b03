set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_modgemm.py tests/test_gpu_streaming.py -x -q > gpurun_out/gpu_mfma.log 2>&1 && \
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --stages > gpurun_out/bench_full.log 2>&1
