# Owner layout at world 2 (two ranks sharing the one GPU, gloo staging) + kernel stats of the headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof12
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --dist-backend gloo --participants 200 --steps 3 --warmup 1 > gpurun_out/o2_bench.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof12 -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof12_bench.log 2>&1
