# Full GPU suite, smoke, 1-GPU bench, distributed path (RCCL, world 1) in both layouts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/f_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --stages > gpurun_out/f_bench.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --force-dist --steps 10 --warmup 3 > gpurun_out/f_bench_dist_owner.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --force-dist --layout committee --steps 10 --warmup 3 > gpurun_out/f_bench_dist_comm.log 2>&1
