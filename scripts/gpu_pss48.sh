# Packed-Shamir small-field share kernel: round numerics (PSS_4_8_3, dropout, streaming) + configs 3 and 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tpss.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 3 --check > gpurun_out/config3.log 2>&1 && \
timeout -k 10 300 python bench_configs.py --config 5 --check > gpurun_out/config5.log 2>&1
