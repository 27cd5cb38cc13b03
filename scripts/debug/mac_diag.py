"""Locate Poly1305 chunk partials that differ between the matrix-core and the
Horner paths (seal side and open side) on a few large boxes."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from sda_amd._native import gpu
from sda_amd.engine import KeyTable
from sda_amd.ops import gpu as G
from sda_amd.ops.sealed import Arena, open_setup, seal_data, seal_setup

M, L, m = int(os.environ.get("MAC_M", 64)), 1_000_000, 433
P130 = (1 << 130) - 5
dev = torch.device("cuda")
vals = torch.randint(0, m, (M, L), dtype=torch.int16, device=dev)
keys = KeyTable.generate(1, dev)
kidx = torch.zeros(M, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
arena = Arena.empty(M, L, m, dev)
gpu().set_mac_mfma(0)
ks = seal_setup(arena, kidx, keys.pks, os.urandom(32), 0, err).with_powers()
seal_data(arena, ks, vals, err)
ko = open_setup(arena, kidx, keys.sks, keys.pks, err)
torch.cuda.synchronize()
print("seal (horner) err", int(err.item()))
saved = arena.ct.clone()
K = arena.K
pre = torch.empty(M, K * G.SUB_PER_CHUNK, dtype=torch.int32, device=dev)


def parts(mode, decrypt, kset):
    gpu().set_mac_mfma(mode)
    arena.ct.copy_(saved)
    p = torch.zeros(M * K * 8, dtype=torch.int32, device=dev)
    ok = torch.zeros(M, dtype=torch.int32, device=dev)
    e = torch.zeros(1, dtype=torch.int32, device=dev)
    if decrypt:
        G.mac_chunks(M, K, kset.keys, kset.pows, arena.ct, arena.stride, arena.pt_len, p, decrypt=True,
                     sub_cnt=pre)
    else:
        G.mac_chunks(M, K, kset.keys, kset.pows, arena.ct, arena.stride, arena.pt_len, p, decrypt=False)
    G.mac_final(M, K, kset.keys, arena.ct, arena.stride, arena.pt_len, p, verify=True, ok=ok, err=e)
    torch.cuda.synchronize()
    v = p.view(M, K, 8)[:, :, :5].to(torch.int64).cpu().tolist()
    vals_ = [[sum((x & 0xFFFFFFFF) << (26 * u) for u, x in enumerate(c)) % P130 for c in row] for row in v]
    return vals_, ok.cpu().tolist(), int(e.item())


lens = arena.pt_len.cpu().tolist()
for decrypt, kset in ((False, ks), (True, ko)):
    a, oka, ea = parts(0, decrypt, kset)
    b, okb, eb = parts(1, decrypt, kset)
    print(f"decrypt={decrypt}: horner err={ea} bad={oka.count(0)}; mfma err={eb} bad={okb.count(0)}")
    shown = 0
    for j in range(M):
        diff = [k for k in range(K) if a[j][k] != b[j][k]]
        if diff and shown < 6:
            shown += 1
            N = lens[j]
            print(f"  msg {j}: N={N} N%16={N % 16} chunks={-(-(N + 32) // 16384)} differing chunks={diff[:10]}"
                  f" (last chunk index {(N + 32 - 1) // 16384})")
