"""Packed-Shamir parity with the threshold-secret-sharing 0.2 construction.

The reference delegates sharing and reconstruction to the tss crate
(client/src/crypto/sharing/packed_shamir.rs:40-43,73-77): share = values
[0, secrets, randomness] at the powers of omega_secrets -> inverse radix-2 FFT
-> zero-pad -> radix-3 FFT at the powers of omega_shares -> drop point 0;
reconstruct = interpolate through {1} u {omega_shares^(i+1)} and evaluate at
omega_secrets^(1..k). The crate itself is not available here (no Rust
toolchain, no crate cache), so the oracle is an independent Python model of
that FFT construction (tests/helpers.py: tss_share) plus big-integer Lagrange
interpolation; equality is modulo p (the crate's `%` may return negative
representatives, the engines keep canonical ones). Parity with crate *binaries*
stays unpinned.

Checked here (CPU): our matrix formulation (csrc/src/pss.cc) produces exactly
the FFT construction's shares for identical randomness, for every reference
parameter set; FFT-model shares reconstruct through our Lagrange matrices from
all clerks and from dropout subsets; the integration-test vector of the
reference (integration-tests/tests/full_loop.rs:57-64,148) comes out.
"""
import random

import pytest

from helpers import tss_share
from sda_amd.models.schemes import (PSS_4_8_3, PSS_4_26_3, PSS_155_728_100, PSS_155_19682_100)

SETS = {"PSS_4_8_3": PSS_4_8_3, "PSS_4_26_3": PSS_4_26_3, "PSS_155_728_100": PSS_155_728_100}


def _model_share(ps, secrets, rnd):
    return tss_share(secrets, rnd, ps.privacy_threshold_, ps.share_count, ps.secret_count,
                     ps.prime_modulus, ps.omega_secrets, ps.omega_shares)


def _interp_eval(points, values, xs, p):
    """Lagrange interpolation through (points, values), evaluated at xs (big ints)."""
    out = []
    for x in xs:
        acc = 0
        for i, (xi, yi) in enumerate(zip(points, values)):
            num, den = 1, 1
            for j, xj in enumerate(points):
                if j != i:
                    num = num * (x - xj) % p
                    den = den * (xi - xj) % p
            acc = (acc + yi * num * pow(den, p - 2, p)) % p
        out.append(acc)
    return out


def _model_reconstruct(ps, indices, shares):
    p = ps.prime_modulus
    pts = [1] + [pow(ps.omega_shares, i + 1, p) for i in indices]
    vals = [0] + list(shares)
    xs = [pow(ps.omega_secrets, e, p) for e in range(1, ps.secret_count + 1)]
    return _interp_eval(pts, vals, xs, p)


@pytest.mark.parametrize("name", list(SETS))
def test_share_equals_fft_construction(native, name):
    ps = SETS[name]
    nat, p = ps.native(), ps.prime_modulus
    nat.validate()
    rng = random.Random(hash(name) & 0xFFFF)
    for _ in range(6 if ps.share_count < 100 else 2):
        s = [rng.randrange(p) for _ in range(ps.secret_count)]
        r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
        ours = [v % p for v in nat.share(s, r)]
        assert ours == _model_share(ps, s, r)


def test_share_equals_fft_construction_19682(native):
    """The largest reference set: one batch (the model's size-19683 DFT is O(n^2))."""
    ps = PSS_155_19682_100
    nat, p = ps.native(), ps.prime_modulus
    rng = random.Random(19682)
    s = [rng.randrange(p) for _ in range(ps.secret_count)]
    r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
    ours = [v % p for v in nat.share(s, r)]
    # spot-check 40 shares against direct polynomial evaluation of the FFT model
    from helpers import fft2_inverse

    coeffs = fft2_inverse([0] + s + r, ps.omega_secrets, p)
    for i in rng.sample(range(ps.share_count), 40):
        x = pow(ps.omega_shares, i + 1, p)
        assert ours[i] == sum(c * pow(x, e, p) for e, c in enumerate(coeffs)) % p


@pytest.mark.parametrize("name", ["PSS_4_8_3", "PSS_4_26_3"])
def test_fft_model_shares_reconstruct_through_our_lagrange(native, name):
    ps = SETS[name]
    nat, p, n, k = ps.native(), ps.prime_modulus, ps.share_count, ps.secret_count
    need = ps.reconstruction_threshold()
    rng = random.Random(5)
    for trial in range(8):
        s = [rng.randrange(p) for _ in range(k)]
        r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
        shares = _model_share(ps, s, r)
        subsets = [list(range(n)), sorted(rng.sample(range(n), need)),
                   sorted(rng.sample(range(n), min(n, need + 1)))]
        for idx in subsets:
            ys = [shares[i] for i in idx]
            assert [v % p for v in nat.reconstruct(idx, ys)] == s       # our Lagrange path
            assert _model_reconstruct(ps, idx, ys) == s                 # the crate's interpolation
            lag = nat.lagrange_matrix(idx)                              # what the GPU applies
            rec = [sum(lag[j * len(idx) + i] * ys[i] for i in range(len(idx))) % p for j in range(k)]
            assert rec == s


def test_large_set_dropout_reconstruct(native):
    ps = PSS_155_728_100
    nat, p = ps.native(), ps.prime_modulus
    rng = random.Random(728)
    s = [rng.randrange(p) for _ in range(ps.secret_count)]
    r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
    shares = _model_share(ps, s, r)
    idx = sorted(rng.sample(range(ps.share_count), ps.reconstruction_threshold()))
    assert [v % p for v in nat.reconstruct(idx, [shares[i] for i in idx])] == s


def test_largest_set_reconstructs_from_all_and_from_survivors(native):
    """PSS_155_19682_100 through the barycentric Lagrange matrices: every clerk
    (node set = all 19,683rd roots of unity: the O(n) weight path), the bare
    threshold, and a large survivor set (generic O(n^2) weights)."""
    ps = PSS_155_19682_100
    nat, p, n = ps.native(), ps.prime_modulus, ps.share_count
    rng = random.Random(3)
    s = [rng.randrange(p) for _ in range(ps.secret_count)]
    r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
    shares = [v % p for v in nat.share(s, r)]
    for idx in (list(range(n)), sorted(rng.sample(range(n), ps.reconstruction_threshold())),
                [i for i in range(n) if i % 5]):
        assert [v % p for v in nat.reconstruct(idx, [shares[i] for i in idx])] == s


def test_reference_full_loop_vector(native):
    """full_loop.rs:57-64,148: two participants share [1,2,3,4] under PSS_4_8_3;
    the summed shares reconstruct to [2,4,6,8] (batches of 3, zero-padded)."""
    ps = PSS_4_8_3
    nat, p = ps.native(), ps.prime_modulus
    rng = random.Random(1)
    total = [[0] * ps.share_count for _ in range(2)]
    for _ in range(2):
        for b, batch in enumerate(([1, 2, 3], [4, 0, 0])):
            r = [rng.randrange(p - 1) for _ in range(ps.privacy_threshold_)]  # the crate draws [0, p-1)
            sh = _model_share(ps, batch, r)
            total[b] = [(a + x) % p for a, x in zip(total[b], sh)]
    out = []
    for b in range(2):
        out += [v % p for v in nat.reconstruct(list(range(ps.share_count)), total[b])]
    assert out[:4] == [2, 4, 6, 8]
