#!/usr/bin/env python3
"""Times the int8-limb MFMA modular GEMM at the packed-Shamir share shape
(S = M . X per participant: n x (t + k) times (t + k) x batches) and reports the
matrix-core rate: int8 MACs counted over all 9 limb products."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd.models.schemes import PSS_155_728_100  # noqa: E402
from sda_amd.ops import gpu as G  # noqa: E402


def main():
    ps = PSS_155_728_100
    p, n, K = ps.prime_modulus, ps.share_count, ps.secret_count + ps.privacy_threshold_
    P, B = 64, 10000  # participants x batches (1M dims / 100 secrets per batch)
    Kp = G.padded_k(K)
    L = G.limb_count(p, Kp)
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.randint(0, p, (n, K), dtype=torch.int32, device=dev, generator=g)
    Al = G.limbs_of(A, Kp, p)
    X = torch.randint(0, 128, (L, P, B, Kp), dtype=torch.int8, device=dev, generator=g)
    out = torch.empty(n, P, B, dtype=torch.int32, device=dev)

    def run():
        G.modgemm_i8(Al, X, p, out, ldc_z=B, ldc_m=P * B, ldc_n=1, limit=n * P * B)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    macs = n * Kp * B * P * L * L
    print(f"modgemm_i8 {n}x{Kp} . {Kp}x{B} x {P} participants, {L} limbs: {ms:.3f} ms, "
          f"{2 * macs / ms / 1e9:.1f} TOPS int8 ({macs / 1e9:.1f} GMAC), "
          f"{n * P * B / ms / 1e6:.2f} G outputs/s, C write {n * P * B * 4 / ms / 1e6:.0f} GB/s")
    # spot check against int64 matmul
    z = 5
    Xz = sum(X[l, z].cpu().to(torch.int64) << (7 * l) for l in range(L))  # [B][Kp]
    ref = ((A.cpu().to(torch.int64) @ Xz[:2000, :K].T) % p).to(dev)
    out = out[:, :, :2000]
    assert torch.equal(out[:, z, :].to(torch.int64), ref), "modgemm mismatch"
    print("spot check ok")


if __name__ == "__main__":
    main()
