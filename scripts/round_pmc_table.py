#!/usr/bin/env python3
"""Per-kernel resource table of the headline round from rocprofv3 PMC passes.

usage: round_pmc_table.py pmc1.csv pmc2.csv fetch.csv write.csv grbm.csv kernel_stats.csv ROUNDS_IN_STATS

Counters are averaged per dispatch and multiplied by the dispatches per round
taken from the un-instrumented kernel_stats (PMC runs serialise kernels and
inflate their durations, so times come from the plain trace).

  lane-ops/B   SQ_INSTS_VALU x 64 lanes / ciphertext bytes of the round
  valu%        time the kernel would need at the measured integer issue peak
               (one wave64 VALU instruction per cycle per CU, 2.4 GHz, 256 CUs
               = 3.9e13 lane-ops/s) over its measured time
  GHz          GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / kernel time of the
               instrumented run: the clock the kernel really ran at (the chip
               drops below 2.4 GHz under sustained integer load)
  valu@clk%    valu% recomputed at that clock
  lds%         SQ_ACTIVE_INST_LDS x 4 / (1024 SIMDs x cycles)
  conf%        SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (share of LDS-busy
               cycles lost to bank conflicts)
  rd GB        FETCH_SIZE as rocprofv3 derives it. On this chip it counts every L2 ->
               fabric read request as 64 bytes: TCC_BUBBLE (the 128-byte requests) reads
               zero, and kernels that load 16 bytes per lane issue 128-byte requests
               (scripts/gpu_pmc_calib.sh: a 1 GiB buffer copy reports 0.537 GB read, a
               1 GiB sum with narrower loads 1.074 GB). So a kernel's true read volume
               lies between `rd GB` and twice that ...
  rd x2        ... the upper end (every request 128 bytes)
  model        what the kernel must read + write by its shapes (headline round: 1000 x
               1M values of 4 bytes in, 3e9 shares of 2 bytes, 5.56e9 ciphertext bytes)
  wr GB        WRITE_SIZE (64-byte write requests: matches the model)
  TB/s         (model if known, else rd + wr) / kernel time
"""
import csv
import re
import sys
from collections import defaultdict

CLK = 2.4e9
CUS = 256
XCDS = 8
PEAK = CUS * 64 * CLK
CIPHERTEXT_BYTES = 5.56e9  # 3000 boxes x 1M values x ~1.85 varint bytes
# (read GB, written GB) a launch of the headline round moves by its shapes, per round
MODEL_GB = {
    "k_share_additive48<0, 6>": (4.0, 6.0),       # int32 secrets in, 3 x 1e9 u16 shares out
    "k_share_additive48<0>": (4.0, 6.0),
    "k_encode_encrypt<unsigned short, false>": (6.0 + 0.03, CIPHERTEXT_BYTES / 1e9),
    "k_mac_chunks<0, false>": (CIPHERTEXT_BYTES / 1e9 + 0.08, 0.0),   # + 26 KB of tables per box
    "k_mac_chunks<1, false>": (CIPHERTEXT_BYTES / 1e9 + 0.08, CIPHERTEXT_BYTES / 1e9),
    "k_decode_sum_z<2, false>": (CIPHERTEXT_BYTES / 1e9, 0.25),
    "k_decode_sum_z<2>": (CIPHERTEXT_BYTES / 1e9, 0.25),
}


def short(name):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("sdagpu::", ""))
    return n.replace("void ", "")[-44:]


def load(path):
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def clocks(path):
    """GHz per kernel: GRBM_GUI_ACTIVE cycles over the dispatch's own duration."""
    cyc, ns = defaultdict(float), defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        k = short(r["Kernel_Name"])
        cyc[k] += float(r["Counter_Value"])
        ns[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: cyc[k] / ns[k] / XCDS for k in cyc if ns[k] > 0}


def main(argv):
    pm = [load(p) for p in argv[1:5]]
    gr = clocks(argv[5])
    argv = argv[:5] + argv[6:]
    rounds = float(argv[6])
    stats = {}
    for r in csv.DictReader(open(argv[5])):
        stats[short(r["Name"])] = (float(r["Calls"]) / rounds, float(r["TotalDurationNs"]) / 1e6 / rounds)
    print(f"{'kernel':44s} {'n/rnd':>6s} {'ms/rnd':>7s} {'lane-ops/B':>10s} {'valu%':>6s} {'GHz':>5s} {'v@clk%':>6s} {'lds%':>6s} "
          f"{'conf%':>6s} {'mfma%':>6s} {'issue%':>6s} {'stall%':>6s} {'wait%':>6s} {'rd GB':>6s} {'rd x2':>6s} {'wr GB':>6s} "
          f"{'model r+w':>11s} {'TB/s':>5s}")
    tot = defaultdict(float)
    for k, (calls, ms) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        if ms < 0.03:
            continue
        a, b, f, w = (p.get(k, {}) for p in pm)
        valu = a.get("SQ_INSTS_VALU", 0) * calls
        cyc = ms * 1e-3 * CLK
        lds = a.get("SQ_ACTIVE_INST_LDS", 0) * calls * 4 / (4 * CUS * cyc)
        ghz = gr.get(k, 0.0)
        vclk = valu * 64 / (CUS * 64 * ghz * 1e9) / (ms * 1e-3) if ghz else 0.0
        conf = a.get("SQ_LDS_BANK_CONFLICT", 0) / max(a.get("SQ_ACTIVE_INST_LDS", 0), 1)
        mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * calls / (4 * CUS * cyc)
        wc = max(b.get("SQ_WAVE_CYCLES", 0), 1)
        rd = f.get("FETCH_SIZE", 0) * calls * 1024 / 1e9
        wr = w.get("WRITE_SIZE", 0) * calls * 1024 / 1e9
        model = MODEL_GB.get(k)
        if model is None:  # template arguments added since (e.g. the tile's code length)
            model = next((v for name, v in MODEL_GB.items()
                          if k.startswith(name.rstrip(">") + ",")), None)
        mtxt = f"{model[0]:5.2f}+{model[1]:4.2f}" if model else ""
        moved = sum(model) if model else rd + wr
        print(f"{k:44s} {calls:6.1f} {ms:7.3f} {valu * 64 / CIPHERTEXT_BYTES:10.1f} "
              f"{100 * valu * 64 / PEAK / (ms * 1e-3):6.1f} {ghz:5.2f} {100 * vclk:6.1f} {100 * lds:6.1f} {100 * conf:6.1f} {100 * mfma:6.1f} "
              f"{100 * b.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {100 * b.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * b.get('SQ_WAIT_ANY', 0) / wc:6.1f} {rd:6.2f} {2 * rd:6.2f} {wr:6.2f} {mtxt:>11s} {moved / ms:5.2f}")
        tot["ms"] += ms
        tot["vclk_ms"] += vclk * ms
        tot["valu"] += valu
        tot["rd"] += rd
        tot["wr"] += wr
    print(f"{'sum':44s} {'':6s} {tot['ms']:7.3f} {tot['valu'] * 64 / CIPHERTEXT_BYTES:10.1f} "
          f"{100 * tot['valu'] * 64 / PEAK / (tot['ms'] * 1e-3):6.1f} {'':54s} {tot['rd']:6.2f} {tot['wr']:6.2f}")
    print(f"VALU time of the whole round at the issue peak (2.4 GHz): {tot['valu'] * 64 / PEAK * 1e3:.2f} ms; "
          f"at the clocks the kernels ran at: {tot['vclk_ms']:.2f} ms")


if __name__ == "__main__":
    main(sys.argv)
