# clerk-stage micro-benchmark + PMC breakdown of its kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
timeout -k 10 300 python scripts/bench_clerk.py > gpurun_out/bench_clerk.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcc -o run -- python3 scripts/bench_clerk.py --reps 1 --modes 0,1 > gpurun_out/pmcc.log 2>&1
