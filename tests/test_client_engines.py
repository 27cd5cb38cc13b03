"""Client-side crypto engines (C++): masking, sharing, varints, sealed shares.

References: client/src/crypto/masking/{none,full,chacha}.rs,
client/src/crypto/sharing/{additive,packed_shamir,batched}.rs,
client/src/crypto/encryption/sodium.rs (varint framing + crypto_box_seal).
Python models in tests/helpers.py serve as the independent oracle.
"""
import random

import pytest

from sda_amd import control as C

from helpers import varint_decode as py_varint_decode
from helpers import varint_encode as py_varint_encode


@pytest.mark.parametrize("values", [[0], [-1], [1], [63, 64, -64, -65], [2 ** 31 - 1, -2 ** 31],
                                    [2 ** 62, -2 ** 62], list(range(-300, 300, 7))])
def test_varint_matches_model(native, values):
    enc = C.varint_encode(values)
    assert enc == py_varint_encode(values)
    assert C.varint_decode(enc) == values
    assert py_varint_decode(enc) == values


def test_varint_known_bytes(native):
    # zigzag: 0->0, -1->1, 1->2, 64->128 (two bytes)
    assert C.varint_encode([0, -1, 1, 64]) == bytes([0x00, 0x01, 0x02, 0x80, 0x01])


def test_varint_dangling_byte_rejected(native):
    with pytest.raises(Exception):
        C.varint_decode(bytes([0x80]))


@pytest.mark.parametrize("scheme", ["None", C.masking_full(433), C.masking_chacha(433, 50, 128)])
def test_mask_roundtrip(native, scheme):
    rng = random.Random(1)
    parts = [[rng.randrange(433) for _ in range(50)] for _ in range(5)]
    masks, masked = [], []
    for s in parts:
        mk, ms = C.mask_secrets(scheme, s)
        masks.append(mk)
        masked.append(ms)
    total_masked = [sum(col) % 433 for col in zip(*masked)]
    combined = C.combine_masks(scheme, masks)
    out = C.unmask(scheme, combined, total_masked)
    expect = [sum(col) % 433 for col in zip(*parts)]
    assert [v % 433 for v in out] == expect
    if scheme == "None":
        assert masks[0] == []


def test_additive_sharing(native):
    scheme = C.sharing_additive(5, 433)
    secrets = list(range(-20, 20))
    shares = C.generate_shares(scheme, secrets)
    assert len(shares) == 5 and all(len(s) == len(secrets) for s in shares)
    rec = [sum(col) % 433 for col in zip(*shares)]
    assert rec == [s % 433 for s in secrets]
    # combine (clerk side) is an element-wise sum
    comb = C.combine_shares(scheme, [shares[0], shares[1]])
    assert [c % 433 for c in comb] == [(a + b) % 433 for a, b in zip(shares[0], shares[1])]


@pytest.mark.parametrize("drop", [[], [2], [0], [7]])  # t+k = 7 of 8 needed
def test_packed_shamir_reconstruct_with_dropouts(native, drop):
    scheme = C.sharing_pss_4_8_3()
    rng = random.Random(7)
    secrets = [rng.randrange(433) for _ in range(10)]  # not a multiple of 3: padding
    shares = C.generate_shares(scheme, secrets)
    assert len(shares) == 8 and all(len(s) == 4 for s in shares)  # ceil(10/3) batches
    indexed = [(i, shares[i]) for i in range(8) if i not in drop]
    out = C.reconstruct_secrets(scheme, len(secrets), indexed)
    assert [v % 433 for v in out] == secrets


def test_packed_shamir_too_few_shares(native):
    scheme = C.sharing_pss_4_8_3()
    shares = C.generate_shares(scheme, [1, 2, 3])
    with pytest.raises(Exception):
        C.reconstruct_secrets(scheme, 3, [(i, shares[i]) for i in range(6)])  # needs 7


def test_packed_shamir_linear(native):
    scheme = C.sharing_pss_4_8_3()
    a, b = [5, 6, 7, 8], [100, 200, 300, 400]
    sa, sb = C.generate_shares(scheme, a), C.generate_shares(scheme, b)
    summed = [[(x + y) % 433 for x, y in zip(u, v)] for u, v in zip(sa, sb)]
    out = C.reconstruct_secrets(scheme, 4, list(enumerate(summed)))
    assert [v % 433 for v in out] == [(x + y) % 433 for x, y in zip(a, b)]


def test_sealed_shares_roundtrip(native):
    import json
    pk, sk = native.crypto.box_keypair()
    kp = {"ek": C.sodium(pk), "dk": C.sodium(sk)}
    kp = C.canonicalize("EncryptionKeypair", kp)
    vals = [3, -4, 432, 0, 2 ** 40]
    enc = json.loads(native.control.encrypt_shares(json.dumps(kp["ek"]), vals))
    assert list(enc) == ["Sodium"]
    assert len(C.unb64(enc["Sodium"])) == 48 + len(C.varint_encode(vals))
    dec = native.control.decrypt_shares(json.dumps(kp), json.dumps(enc))
    assert dec == vals
    # the host opener agrees with libsodium-format sealed boxes
    pt = native.crypto.box_seal_open(C.unb64(enc["Sodium"]), pk, sk)
    assert C.varint_decode(pt) == vals
