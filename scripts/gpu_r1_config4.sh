# BASELINE config 4 (10k x 125M, PSS_4_8_3, streamed) on the current kernels, checked against the plain sum.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench_configs.py --config 4 --check > gpurun_out/c4_w32.log 2>&1 && \
timeout -k 10 400 python -u bench_configs.py --config 4 --wave 64 > gpurun_out/c4_w64.log 2>&1
