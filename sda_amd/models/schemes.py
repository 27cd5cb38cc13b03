"""Aggregation job specifications (the reference's "job format" as data).

Mirrors the scheme enums of the reference protocol crate
(protocol/src/crypto.rs:43-188) and the Aggregation resource
(protocol/src/resources.rs:43-67). Derived properties follow the reference:
``input_size`` / ``output_size`` / ``privacy_threshold`` /
``reconstruction_threshold`` (crypto.rs:101-155).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Union


@dataclass(frozen=True)
class NoMask:
    kind: str = "none"

    def has_mask(self) -> bool:
        return False

    def to_wire(self):
        return "None"


@dataclass(frozen=True)
class FullMask:
    modulus: int
    kind: str = "full"

    def has_mask(self) -> bool:
        return True

    def to_wire(self):
        return {"Full": {"modulus": self.modulus}}


@dataclass(frozen=True)
class ChaChaMask:
    modulus: int
    dimension: int
    seed_bitsize: int = 128
    kind: str = "chacha"

    def has_mask(self) -> bool:
        return True

    @property
    def seed_words(self) -> int:
        return (self.seed_bitsize + 31) // 32

    def to_wire(self):
        return {"ChaCha": {"modulus": self.modulus, "dimension": self.dimension,
                           "seed_bitsize": self.seed_bitsize}}


MaskingScheme = Union[NoMask, FullMask, ChaChaMask]


@dataclass(frozen=True)
class Additive:
    share_count: int
    modulus: int
    kind: str = "additive"

    def input_size(self) -> int:
        return 1

    def output_size(self) -> int:
        return self.share_count

    def privacy_threshold(self) -> int:
        return self.share_count - 1

    def reconstruction_threshold(self) -> int:
        return self.share_count

    @property
    def field_modulus(self) -> int:
        return self.modulus

    def to_wire(self):
        return {"Additive": {"share_count": self.share_count, "modulus": self.modulus}}


@dataclass(frozen=True)
class PackedShamir:
    secret_count: int
    share_count: int
    privacy_threshold_: int
    prime_modulus: int
    omega_secrets: int
    omega_shares: int
    kind: str = "packed_shamir"

    def input_size(self) -> int:
        return self.secret_count

    def output_size(self) -> int:
        return self.share_count

    def privacy_threshold(self) -> int:
        return self.privacy_threshold_

    def reconstruction_threshold(self) -> int:
        return self.privacy_threshold_ + self.secret_count

    @property
    def field_modulus(self) -> int:
        return self.prime_modulus

    def to_wire(self):
        return {"PackedShamir": {"secret_count": self.secret_count,
                                 "share_count": self.share_count,
                                 "privacy_threshold": self.privacy_threshold_,
                                 "prime_modulus": self.prime_modulus,
                                 "omega_secrets": self.omega_secrets,
                                 "omega_shares": self.omega_shares}}

    def native(self):
        from .._native import native

        return native().field.PackedShamirParams(
            self.secret_count, self.share_count, self.privacy_threshold_,
            self.prime_modulus, self.omega_secrets, self.omega_shares)


SharingScheme = Union[Additive, PackedShamir]

# threshold-secret-sharing 0.2 parameter sets (protocol/src/crypto.rs PackedShamir fields)
PSS_4_8_3 = PackedShamir(3, 8, 4, 433, 354, 150)
PSS_4_26_3 = PackedShamir(3, 26, 4, 433, 354, 17)
PSS_155_728_100 = PackedShamir(100, 728, 155, 746497, 95660, 610121)
PSS_155_19682_100 = PackedShamir(100, 19682, 155, 5038849, 4318906, 1814687)


def pss_5_of_8(prime: int = 433) -> PackedShamir:
    """Packed Shamir with reconstruction threshold 5 out of 8 clerks (t=2, k=3).

    t+k+1 = 6 evaluation points is not an FFT size, so the tss crate cannot
    express it; the matrix formulation only needs distinct points. Requires
    16 * 9 | p - 1 (true for p = 433).
    """
    from .._native import native

    f = native().field
    g = next(w for w in range(2, prime) if f.mult_order(w, prime) == prime - 1)
    # order 16 (>= 6 secret-side points) and order 9 (= n + 1 share points):
    # coprime orders, so no share point can coincide with any secret-side point
    ws = f.mod_pow(g, (prime - 1) // 16, prime)
    wn = f.mod_pow(g, (prime - 1) // 9, prime)
    return PackedShamir(3, 8, 2, prime, ws, wn)


@dataclass
class AggregationSpec:
    """What a device round needs: dimension, modulus and the schemes."""

    dimension: int
    modulus: int
    sharing: SharingScheme
    masking: MaskingScheme = field(default_factory=NoMask)
    title: str = "aggregation"

    def __post_init__(self):
        if self.dimension <= 0:
            raise ValueError("dimension must be positive")
        fm = self.sharing.field_modulus
        if not (2 <= fm < 2 ** 31):
            raise ValueError("field modulus must be in [2, 2^31) for the GPU engine")
        if isinstance(self.masking, ChaChaMask) and self.masking.dimension != self.dimension:
            raise ValueError("ChaCha mask dimension must equal the vector dimension")
        if self.masking.has_mask() and self.masking.modulus != fm:
            raise ValueError("mask modulus must equal the sharing modulus")

    @property
    def field_modulus(self) -> int:
        return self.sharing.field_modulus

    @property
    def n_clerks(self) -> int:
        return self.sharing.output_size()

    @property
    def batches(self) -> int:
        k = self.sharing.input_size()
        return (self.dimension + k - 1) // k
