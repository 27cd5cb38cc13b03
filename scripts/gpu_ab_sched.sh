# A/B of side-stream key-agreement scheduling on the headline round:
# SDA_OPEN_AFTER_SHARE (clerk keys queued behind the share kernel) and
# SDA_KEY_PRIO="open,powers" (wave priority of the open setup / Poly1305 tables).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {
  SDA_OPEN_AFTER_SHARE=$1 SDA_KEY_PRIO=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stages \
      > gpurun_out/ab_run.log 2>&1 || exit 1
  echo "after_share=$1 prio=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_run.log) $(grep stage_ms gpurun_out/ab_run.log)" >> gpurun_out/ab.log
}
for rep in 1 2; do
  run 1 1,1
  run 1 0,1
  run 1 0,0
  run 1 1,0
done
