"""A/B timing of the Poly1305 chunk kernel: matrix-core segments (mode 1) vs
per-lane Horner everywhere (mode 0), seal side (MAC only) and open side (MAC +
in-place decrypt + terminator counts), on the headline round's 3000 boxes of
1M values (m = 433). Every timed pass is verified by k_mac_final."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from sda_amd._native import gpu
from sda_amd.engine import KeyTable
from sda_amd.ops import gpu as G
from sda_amd.ops.sealed import Arena, open_setup, seal_data, seal_setup

M, L, m = int(os.environ.get("MAC_M", 3000)), 1_000_000, 433
dev = torch.device("cuda")
vals = torch.randint(0, m, (M, L), dtype=torch.int16, device=dev)
keys = KeyTable.generate(1, dev)
kidx = torch.zeros(M, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
arena = Arena.empty(M, L, m, dev)
ks = seal_setup(arena, kidx, keys.pks, os.urandom(32), 0, err).with_powers()
seal_data(arena, ks, vals, err)
ko = open_setup(arena, kidx, keys.sks, keys.pks, err)
torch.cuda.synchronize()
assert int(err.item()) == 0
saved = arena.ct.clone()
K = arena.K
partials = torch.empty(M * K * 8, dtype=torch.int32, device=dev)
pre = torch.empty(M, K * G.SUB_PER_CHUNK, dtype=torch.int32, device=dev)
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

for mode in (0, 1, 0, 1):
    gpu().set_mac_mfma(mode)
    arena.ct.copy_(saved)  # the previous open pass decrypted in place
    a, b = ev(), ev()
    G.mac_chunks(M, K, ks.keys, ks.pows, arena.ct, arena.stride, arena.pt_len, partials, decrypt=False)
    a.record()
    for _ in range(5):
        G.mac_chunks(M, K, ks.keys, ks.pows, arena.ct, arena.stride, arena.pt_len, partials,
                     decrypt=False)
    b.record()
    ok = torch.zeros(M, dtype=torch.int32, device=dev)
    G.mac_final(M, K, ks.keys, arena.ct, arena.stride, arena.pt_len, partials, verify=True, ok=ok,
                err=err)
    torch.cuda.synchronize()
    seal_ms = a.elapsed_time(b) / 5
    bad_seal = (ok == 0).nonzero().flatten().tolist()
    open_ms = []
    for _ in range(3):
        arena.ct.copy_(saved)
        a, b = ev(), ev()
        a.record()
        G.mac_chunks(M, K, ko.keys, ko.pows, arena.ct, arena.stride, arena.pt_len, partials,
                     decrypt=True, sub_cnt=pre)
        b.record()
        G.mac_final(M, K, ko.keys, arena.ct, arena.stride, arena.pt_len, partials, verify=True,
                    ok=ok, err=err)
        torch.cuda.synchronize()
        open_ms.append(a.elapsed_time(b))
        bad_open = (ok == 0).nonzero().flatten().tolist()
        if bad_seal or bad_open:
            lens = arena.pt_len.cpu().tolist()
            print("  bad seal", bad_seal[:8], "bad open", bad_open[:8],
                  "lens", [lens[i] for i in (bad_seal + bad_open)[:8]], flush=True)
    e = int(err.item())
    print(f"mode={mode} ({'mfma' if mode else 'horner'}): seal MAC {seal_ms:.3f} ms, "
          f"open MAC+decrypt {min(open_ms):.3f} ms, err={e}", flush=True)
    assert e == 0
