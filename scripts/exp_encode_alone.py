#!/usr/bin/env python3
"""Experiment: the encode + encrypt kernel alone on boxes shaped like a many-clerk round's
(usage: exp_encode_alone.py [MODULUS [BOXES [VALUES]]]): ms per launch and bytes per second."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd.ops import gpu as G  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 746497
M = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
L = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
dev = torch.device("cuda")
vals = torch.randint(0, m, (M, L), dtype=torch.int32, device=dev)
T = G.tiles(L)
cnt = torch.empty(M, T, dtype=torch.int32, device=dev)
G.count(vals, cnt)
pt_len = torch.zeros(M, dtype=torch.int32, device=dev)
G.segscan(cnt, pt_len)
stride = (G.SEAL_OVERHEAD + L * G.varint_max_len(m) + 63) // 64 * 64
ct = torch.empty(M * stride, dtype=torch.uint8, device=dev)
keys = torch.randint(0, 256, (M * G.MSGKEY_BYTES,), dtype=torch.uint8, device=dev)
mb = G.varint_max_len(m)
for _ in range(2):
    G.encode_encrypt(vals, cnt, keys, ct, stride, max_code_bytes=mb)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    G.encode_encrypt(vals, cnt, keys, ct, stride, max_code_bytes=mb)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
nbytes = int(pt_len.to(torch.int64).sum().item())
print(f"encode m={m} {M} boxes x {L} values: {ms:.2f} ms, {nbytes / 1e9:.2f} GB of ciphertext, "
      f"{nbytes / ms / 1e6:.0f} GB/s", flush=True)
