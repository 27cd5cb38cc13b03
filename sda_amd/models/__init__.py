"""Aggregation job presets: schemes and the benchmark configurations."""
from .schemes import (  # noqa: F401
    AggregationSpec, Additive, PackedShamir, NoMask, FullMask, ChaChaMask,
    PSS_4_8_3, PSS_4_26_3, PSS_155_728_100, PSS_155_19682_100, pss_5_of_8,
)
from .configs import BENCH_CONFIGS, bench_config  # noqa: F401
