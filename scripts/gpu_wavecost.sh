set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29562 bench.py --force-dist --waves 4 --steps 5 --warmup 2 --stages > gpurun_out/wave4.log 2>&1 && \
timeout -k 10 300 $R --master-port 29563 bench.py --force-dist --waves 2 --steps 5 --warmup 2 --stages > gpurun_out/wave2.log 2>&1 && \
timeout -k 10 300 $R --master-port 29564 bench.py --force-dist --layout owner --steps 5 --warmup 2 --stages > gpurun_out/owner1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --stages > gpurun_out/single.log 2>&1
