set -e
mkdir -p gpurun_out
timeout -k 10 120 bash docs/cli-walkthrough.sh --device gpu 2>&1 | tail -1
timeout -k 10 120 bash docs/cli-walkthrough.sh --device gpu --mask chacha --sharing shamir --clerks 8 2>&1 | tail -1
for w in 1 2 4; do
  timeout -k 10 200 python bench.py --force-dist --waves $w > gpurun_out/r3_e_committee_w1_waves$w.log 2>&1 || { tail -20 gpurun_out/r3_e_committee_w1_waves$w.log; exit 1; }
  echo "committee world 1 waves $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_e_committee_w1_waves$w.log)"
done
timeout -k 10 200 python bench.py --force-dist --loopback --waves 4 > gpurun_out/r3_e_loopback_waves4.log 2>&1 || { tail -20 gpurun_out/r3_e_loopback_waves4.log; exit 1; }
echo "loopback waves 4: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_e_loopback_waves4.log) $(grep -o '"compute_stream_vs_rccl": "[^"]*"' gpurun_out/r3_e_loopback_waves4.log)"
timeout -k 10 200 python bench.py --force-dist --layout owner > gpurun_out/r3_e_owner_w1.log 2>&1 || { tail -20 gpurun_out/r3_e_owner_w1.log; exit 1; }
echo "owner world 1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_e_owner_w1.log)"
