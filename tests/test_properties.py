"""Property-based tests (hypothesis) of the host engines and the wire codec."""
import base64

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from sda_amd import control as C

from helpers import varint_encode as py_varint_encode

I64 = st.integers(min_value=-(2 ** 63), max_value=2 ** 63 - 1)


@settings(max_examples=200, deadline=None)
@given(st.lists(I64, max_size=50))
def test_varint_roundtrip(native, values):
    enc = C.varint_encode(values)
    assert enc == py_varint_encode(values)
    assert C.varint_decode(enc) == values


@settings(max_examples=200, deadline=None)
@given(st.binary(max_size=200))
def test_base64_matches_stdlib(native, data):
    assert C.b64(data) == base64.b64encode(data).decode()
    assert C.unb64(C.b64(data)) == data


@settings(max_examples=50, deadline=None)
@given(st.text(max_size=40), st.integers(min_value=1, max_value=10 ** 6),
       st.integers(min_value=2, max_value=2 ** 31 - 1))
def test_aggregation_wire_roundtrip(native, title, dim, modulus):
    agg = C.aggregation(title, dim, modulus, C.new_id(), C.new_id(),
                        masking_scheme=C.masking_full(modulus),
                        committee_sharing_scheme=C.sharing_additive(3, modulus))
    assert C.canonicalize("Aggregation", agg) == agg


@settings(max_examples=40, deadline=None)
@given(st.lists(st.integers(min_value=-10 ** 6, max_value=10 ** 6), min_size=1, max_size=30),
       st.integers(min_value=2, max_value=9))
def test_additive_shares_sum_to_secret(native, secrets, n):
    m = 433
    shares = C.generate_shares(C.sharing_additive(n, m), secrets)
    assert [sum(col) % m for col in zip(*shares)] == [s % m for s in secrets]


@settings(max_examples=25, deadline=None)
@given(st.lists(st.integers(min_value=0, max_value=432), min_size=1, max_size=20),
       st.lists(st.integers(min_value=0, max_value=432), min_size=1, max_size=20),
       st.integers(min_value=0, max_value=7))
def test_packed_shamir_linear_with_any_single_dropout(native, a, b, drop):
    n = min(len(a), len(b))
    a, b = a[:n], b[:n]
    s = C.sharing_pss_4_8_3()
    sa, sb = C.generate_shares(s, a), C.generate_shares(s, b)
    summed = [[(x + y) % 433 for x, y in zip(u, v)] for u, v in zip(sa, sb)]
    indexed = [(i, summed[i]) for i in range(8) if i != drop]
    out = C.reconstruct_secrets(s, n, indexed)
    assert [v % 433 for v in out] == [(x + y) % 433 for x, y in zip(a, b)]


@settings(max_examples=30, deadline=None)
@given(st.lists(st.integers(min_value=0, max_value=432), min_size=1, max_size=40))
def test_sealed_shares_roundtrip(native, values):
    import json
    pk, sk = native.crypto.box_keypair()
    kp = json.dumps({"ek": C.sodium(pk), "dk": C.sodium(sk)})
    enc = native.control.encrypt_shares(json.dumps(C.sodium(pk)), values)
    assert native.control.decrypt_shares(kp, enc) == values
