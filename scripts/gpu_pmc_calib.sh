#!/bin/bash
# What FETCH_SIZE / WRITE_SIZE and the raw L2 -> fabric request counters report for
# kernels of known traffic (scripts/pmc_calib.py).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/calib$i -o p -- python $R/scripts/pmc_calib.py > $O/calib$i.log 2>&1 || { tail -20 $O/calib$i.log; exit 1; }
  cp $(find $O/calib$i -name "*counter_collection.csv" | head -1) $O/calib$i.csv
  rm -rf $O/calib$i
done
python - $O/calib1.csv $O/calib2.csv $O/calib3.csv $O/calib4.csv $O/calib5.csv <<'PY' | tee $O/pmc_calibration.txt
import csv, sys, re, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sys.argv[1:]:
    for r in csv.DictReader(open(p)):
        k = re.sub(r"<.*", "", r["Kernel_Name"].replace("void ", "").replace("at::native::", ""))[:40]
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("1 GiB = 1.0737 GB moved per direction by the copy; read only by the sum; written only by the fill")
for k, c in d.items():
    m = {n: sorted(v)[len(v) // 2] for n, v in c.items()}  # median over the dispatches
    if m.get("TCC_EA0_RDREQ_sum", 0) + m.get("TCC_EA0_WRREQ_sum", 0) < 1e5:
        continue
    print(k)
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(m.items())))
    rd64 = m.get("TCC_EA0_RDREQ_sum", 0) - m.get("TCC_BUBBLE_sum", 0) - m.get("TCC_EA0_RDREQ_32B_sum", 0)
    print(f"   FETCH_SIZE {m.get('FETCH_SIZE', 0) * 1024 / 1e9:.3f} GB   WRITE_SIZE {m.get('WRITE_SIZE', 0) * 1024 / 1e9:.3f} GB   "
          f"read requests x 128 B {m.get('TCC_EA0_RDREQ_sum', 0) * 128 / 1e9:.3f} GB   x 64 B {m.get('TCC_EA0_RDREQ_sum', 0) * 64 / 1e9:.3f} GB   "
          f"write requests x 64 B {m.get('TCC_EA0_WRREQ_sum', 0) * 64 / 1e9:.3f} GB")
PY
