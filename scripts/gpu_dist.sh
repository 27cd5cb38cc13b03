# GPU tests + 1-GPU bench + 2-rank rehearsal of the distributed bench on one GPU (gloo)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --stages > gpurun_out/bench_full.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --participants 100 --dist-backend gloo > gpurun_out/bench_dist2.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 2 --warmup 1 --participants 40 --dim 200000 --dist-backend gloo > gpurun_out/bench_dist4.log 2>&1
