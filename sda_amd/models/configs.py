"""The five BASELINE.json configurations as named presets."""
from __future__ import annotations

from .schemes import Additive, AggregationSpec, NoMask, PSS_4_8_3, pss_5_of_8

BENCH_CONFIGS = {
    # 1: README CLI example (plumbing)
    "cli_3x10": dict(participants=3, spec=lambda: AggregationSpec(10, 433, Additive(3, 433))),
    # 2: headline -- 1k participants x 1M dims, 3-way additive, one MI355X
    "add3_1kx1m": dict(participants=1000,
                       spec=lambda: AggregationSpec(1_000_000, 433, Additive(3, 433), NoMask(),
                                                    title="1k x 1M additive-3")),
    # 3: packed Shamir k=3 n=8 (PSS_4_8_3)
    "pss483_1kx1m": dict(participants=1000,
                         spec=lambda: AggregationSpec(1_000_000, 433, PSS_4_8_3, NoMask(),
                                                      title="1k x 1M PSS_4_8_3")),
    # 4: 10k x 125M (GPT-2-small gradient), 8 clerks -- streamed in waves
    "add8_10kx125m": dict(participants=10_000,
                          spec=lambda: AggregationSpec(125_000_000, 433, Additive(8, 433),
                                                       NoMask(), title="10k x 125M additive-8")),
    # 5: packed Shamir 5-of-8 with clerk dropout
    "pss5of8_1kx1m": dict(participants=1000,
                          spec=lambda: AggregationSpec(1_000_000, 433, pss_5_of_8(), NoMask(),
                                                       title="1k x 1M PSS 5-of-8")),
}


def bench_config(name: str):
    cfg = BENCH_CONFIGS[name]
    return cfg["participants"], cfg["spec"]()
