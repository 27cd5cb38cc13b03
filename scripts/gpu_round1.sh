set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/info.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --participants 100 --steps 3 --warmup 1 --stages > gpurun_out/bench_small.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --stages > gpurun_out/bench_full.log 2>&1
