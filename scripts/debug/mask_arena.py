import sys, os; sys.path.insert(0, os.getcwd())
import torch
from sda_amd.engine import DeviceAggregator
from sda_amd.models import PSS_155_728_100, AggregationSpec, FullMask
from sda_amd.ops import gpu as G
from sda_amd.ops.sealed import Arena, seal, open_
from sda_amd._native import native
p = PSS_155_728_100.prime_modulus
spec = AggregationSpec(777, p, PSS_155_728_100, FullMask(p))
agg = DeviceAggregator(spec)
P, D = 2, 777
x = torch.randint(0, p, (P, D), dtype=torch.int32, device="cuda")
err = torch.zeros(1, dtype=torch.int32, device="cuda")
key = native().crypto.random_bytes(32)
shares, cnt, mvals, mcnt = agg._share(x, key, 0, err)
torch.cuda.synchronize()
print("after share err", int(err.item()), "mask max", int(mvals.max()), "shares max", int(shares.max()), "min", int(shares.min()))
mcnt_ref = torch.empty_like(mcnt); G.count(mvals, mcnt_ref)
print("mask cnt kernel vs count:", mcnt.tolist(), mcnt_ref.tolist())
n = agg.n
kidx = torch.full((P,), n, dtype=torch.int32, device="cuda")
e2 = torch.zeros(1, dtype=torch.int32, device="cuda")
ar = seal(mvals, kidx, agg.keys.pks, key, 5000, e2, p, cnt=mcnt.clone())
out = open_(ar, kidx, agg.keys.sks, agg.keys.pks, e2, out_dtype=torch.int32)
print("mask arena err", int(e2.item()), "roundtrip", bool(torch.equal(out, mvals)))
e3 = torch.zeros(1, dtype=torch.int32, device="cuda")
ar = seal(mvals, kidx, agg.keys.pks, key, 6000, e3, p)
out = open_(ar, kidx, agg.keys.sks, agg.keys.pks, e3, out_dtype=torch.int32)
print("mask arena recount err", int(e3.item()), "roundtrip", bool(torch.equal(out, mvals)))
sh = shares.view(n * P, -1)
kc = torch.arange(n, dtype=torch.int32, device="cuda").repeat_interleave(P)
e4 = torch.zeros(1, dtype=torch.int32, device="cuda")
ar = seal(sh, kc, agg.keys.pks, key, 7000, e4, p)
out = open_(ar, kc, agg.keys.sks, agg.keys.pks, e4, out_dtype=torch.int32)
print("clerk arena err", int(e4.item()), "roundtrip", bool(torch.equal(out, sh)))
