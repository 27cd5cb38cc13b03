"""The benchmark configurations as named presets (the single table
`bench_configs.py` runs; numbers 1-5 are BASELINE.json's `configs` list in order).

Each preset: participants per rank, vector dimension, the aggregation spec, the
clerks that deliver results (None = all; config 5 drops three of eight), whether
the round is streamed in participant waves, and the packed-Shamir backend.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Sequence

from .schemes import (PSS_4_8_3, PSS_155_728_100, PSS_155_19682_100, Additive, AggregationSpec,
                      ChaChaMask, FullMask, NoMask, PackedShamir, pss_5_of_8)


@dataclass(frozen=True)
class BenchConfig:
    number: int
    name: str
    participants: int              # per rank (config 4: in total, split over the ranks)
    dimension: int
    sharing: Callable[[], object]  # () -> sharing scheme (some need the native field helpers)
    clerks: Optional[Sequence[int]] = None
    streamed: bool = False
    wave: int = 32
    pss_backend: str = "auto"
    what: str = ""
    masking: str = "none"          # none | full | chacha (client/src/crypto/masking/*.rs)

    def spec(self, dimension: Optional[int] = None) -> AggregationSpec:
        s = self.sharing()
        D = dimension or self.dimension
        mask = {"none": lambda: NoMask(), "full": lambda: FullMask(s.field_modulus),
                "chacha": lambda: ChaChaMask(s.field_modulus, D)}[self.masking]()
        return AggregationSpec(D, s.field_modulus, s, mask, title=self.name)


def small_prime_5_of_8(prime: int = 241) -> PackedShamir:
    """t = 2, k = 3, n = 8 over a prime < 256. The matrix formulation only needs
    t + k + 1 = 6 distinct secret-side points and n = 8 share points disjoint
    from them: p = 241 has p - 1 = 240 = 16 * 15, so omega_secrets of order 16
    and omega_shares of order 15 (coprime orders: the two point sets only share
    1, which neither uses beyond the fixed zero at 1)."""
    from .._native import native

    f = native().field
    g = next(w for w in range(2, prime) if f.mult_order(w, prime) == prime - 1)
    ws = f.mod_pow(g, (prime - 1) // 16, prime)
    wn = f.mod_pow(g, (prime - 1) // 15, prime)
    return PackedShamir(3, 8, 2, prime, ws, wn)


BENCH_CONFIGS = {
    c.number: c for c in [
        BenchConfig(1, "cli_3x10", 3, 10, lambda: Additive(3, 433),
                    what="README walkthrough through sdad + sda (CPU plumbing)"),
        BenchConfig(2, "add3_1kx1m", 1000, 1_000_000, lambda: Additive(3, 433),
                    what="headline: 1k x 1M, additive-3, one MI355X (= bench.py)"),
        BenchConfig(3, "pss483_1kx1m", 1000, 1_000_000, lambda: PSS_4_8_3,
                    what="1k x 1M per GPU, packed Shamir k=3 n=8, committee layout over xGMI"),
        BenchConfig(4, "pss483_10kx125m", 10_000, 125_000_000, lambda: PSS_4_8_3, streamed=True,
                    what="10k x 125M (GPT-2-small gradient), 8 clerks, streamed in participant "
                         "waves with accumulator checkpoints"),
        BenchConfig(5, "pss5of8_dropout", 1000, 1_000_000, pss_5_of_8, clerks=(0, 2, 3, 5, 7),
                    what="packed Shamir 5-of-8 (t=2, k=3) with clerks 1, 4, 6 dropped"),
        BenchConfig(6, "pss155_728_1kx1m", 1000, 1_000_000, lambda: PSS_155_728_100,
                    pss_backend="mfma",
                    what="the reference's large parameter set: 728 clerks, k=100, t=155, shares "
                         "and reconstruction on the int8-limb MFMA GEMM"),
        BenchConfig(7, "pss5of8_u8_dropout", 1000, 1_000_000, small_prime_5_of_8,
                    clerks=(0, 2, 3, 5, 7),
                    what="config 5 over a prime below 256: field elements stored as int8-sized "
                         "values (u8 shares)"),
        BenchConfig(8, "pss155_19682_16x1m", 16, 1_000_000, lambda: PSS_155_19682_100,
                    pss_backend="mfma",
                    what="the reference's largest parameter set: 19,682 clerks, k=100, t=155 "
                         "(315k sealed boxes of 10,000 shares for 16 participants per GPU)"),
        BenchConfig(9, "add3_fullmask_1kx1m", 1000, 1_000_000, lambda: Additive(3, 433),
                    masking="full",
                    what="headline shape with a full mask: every participant also seals its "
                         "1M-value mask for the recipient, who opens and sums them"),
        BenchConfig(10, "add3_chachamask_1kx1m", 1000, 1_000_000, lambda: Additive(3, 433),
                    masking="chacha",
                    what="headline shape with a ChaCha mask: participants expand a rand-0.3 "
                         "ChaChaRng seed over the vector, the recipient re-expands all 1000 seeds"),
        BenchConfig(11, "add3_chachamask_m31_1kx1m", 1000, 1_000_000,
                    lambda: Additive(3, 2 ** 31 - 1), masking="chacha",
                    what="ChaCha mask over the largest supported modulus (2^31 - 1): 32-bit "
                         "shares, five-byte varints, a rejected draw every ~1e10"),
    ]
}


def bench_config(number: int) -> BenchConfig:
    return BENCH_CONFIGS[number]
