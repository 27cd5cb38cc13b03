import sys, os; sys.path.insert(0, os.getcwd())
import torch
from sda_amd.engine import DeviceAggregator, reference_sum, AggregationError
from sda_amd.models import PSS_155_728_100, AggregationSpec, FullMask, Additive
p = PSS_155_728_100.prime_modulus
cases = {
    "add3_fullmask_bigmod": (AggregationSpec(777, p, Additive(3, p), FullMask(p)), None, {}),
    "add3_fullmask_bigmod_4096": (AggregationSpec(5000, p, Additive(3, p), FullMask(p)), None, {}),
    "pss155_fullmask": (AggregationSpec(777, p, PSS_155_728_100, FullMask(p)), None, {}),
    "pss155_dropout": (AggregationSpec(777, p, PSS_155_728_100), [c for c in range(728) if c % 3 != 1], {}),
}
for name, (spec, live, kw) in cases.items():
    agg = DeviceAggregator(spec, **kw)
    x = torch.randint(0, p, (2, spec.dimension), dtype=torch.int32, device="cuda")
    try:
        res = agg.run_round(x, clerks=live)
        print(name, "ok" if torch.equal(res.output, reference_sum(x, p)) else "MISMATCH", flush=True)
    except AggregationError as e:
        print(name, "ERROR", e, flush=True)
