set -e
mkdir -p gpurun_out
echo "== tests" 
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "unchecked or round" 2>&1 | tail -5
echo "== bench"
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_d_single.log 2>&1
cut -c1-260 gpurun_out/r3_d_single.log | tail -1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_d_single2.log 2>&1
cut -c1-260 gpurun_out/r3_d_single2.log | tail -1
