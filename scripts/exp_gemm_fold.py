#!/usr/bin/env python3
"""Experiment: share GEMM of configs 6 / 8 alone, per kernel (general / panel-resident) and epilogue fold
(0 integer, 2 double-precision)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd._native import gpu  # noqa: E402
from sda_amd.models.configs import bench_config  # noqa: E402
from sda_amd.ops import gpu as G  # noqa: E402

# usage: exp_gemm_fold.py [config ...] [--only PANEL:FOLD]
args = sys.argv[1:]
only = None
if "--only" in args:
    i = args.index("--only")
    only = tuple(int(v) for v in args[i + 1].split(":"))
    del args[i:i + 2]
for c in [int(a) for a in args] or (6, 8):
    cfg = bench_config(c)
    ps = cfg.sharing()
    p, n, K = ps.field_modulus, ps.share_count, ps.secret_count + ps.privacy_threshold_
    P, B = cfg.participants, cfg.dimension // ps.secret_count
    Kp = G.padded_k(K)
    L = G.limb_count(p, Kp)
    A = torch.randint(0, 127, (L, n, Kp), dtype=torch.int8, device="cuda")  # any digits time alike
    X = torch.randint(0, 127, (L, P, B, Kp), dtype=torch.int8, device="cuda")
    out = torch.empty(n, P, B, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(n * P * G.tiles(B), dtype=torch.int32, device="cuda")
    # the write roofline: the GEMM's output buffer filled by a plain store kernel
    out.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        out.zero_()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"config {c}: filling the {out.numel() * 4 / 1e9:.1f} GB output alone takes {ms:.2f} ms "
          f"({out.numel() * 4 / ms / 1e9:.2f} TB/s)", flush=True)
    ref = None
    for panel, mode in ((only,) if only else ((0, 0), (0, 2), (1, 0), (1, 2))):
        gpu().set_gemm_fold_f64(mode)
        gpu().set_gemm_panel(panel)
        for _ in range(2):
            cnt.zero_()
            G.modgemm_i8(A, X, p, out, ldc_z=B, ldc_m=P * B, ldc_n=1, limit=n * P * B, cnt=cnt)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            G.modgemm_i8(A, X, p, out, ldc_z=B, ldc_m=P * B, ldc_n=1, limit=n * P * B, cnt=cnt)
        e1.record()
        torch.cuda.synchronize()
        chk = int(out[::97, ::13, ::101].to(torch.int64).sum().item())
        ref = chk if ref is None else ref
        print(f"config {c} panel {panel} fold mode {mode}: {e0.elapsed_time(e1) / 3:.2f} ms  checksum {'same' if chk == ref else 'DIFFERENT'}", flush=True)
    gpu().set_gemm_fold_f64(2)  # the defaults
    gpu().set_gemm_panel(-1)
    del A, X, out, cnt
    torch.cuda.empty_cache()
