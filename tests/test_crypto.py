"""Known-answer and cross-implementation tests of the host crypto (CPU).

Oracles: published vectors (NaCl box test, RFC 7748, RFC 8032, RFC 8439, the
Salsa20 specification), Python's hashlib (SHA-512, BLAKE2b), independent Python
models (tests/helpers.py) and, where the image's OpenSSL 3 provides them, libcrypto
via ctypes (X25519, Ed25519, Poly1305, ChaCha20).
"""
import ctypes
import ctypes.util
import hashlib
import os

import pytest

from helpers import poly1305 as py_poly1305, salsa20_block as py_salsa20_block

H = bytes.fromhex


def test_sha512_constants_and_kat(native):
    c = native.crypto
    assert c.sha512_round_constant(0) == 0x428A2F98D728AE22
    assert c.sha512_round_constant(79) == 0x6C44198C4A475817
    assert c.sha512_iv(0) == 0x6A09E667F3BCC908
    for msg in [b"", b"abc", b"a" * 111, b"a" * 112, b"a" * 1000, os.urandom(777)]:
        assert c.sha512(msg) == hashlib.sha512(msg).digest()


@pytest.mark.parametrize("outlen", [1, 24, 32, 64])
def test_blake2b_vs_hashlib(native, outlen):
    for msg in [b"", b"abc", os.urandom(64), os.urandom(128), os.urandom(129), os.urandom(1000)]:
        assert native.crypto.blake2b(msg, outlen) == hashlib.blake2b(msg, digest_size=outlen).digest()
    key = os.urandom(32)
    msg = os.urandom(200)
    assert native.crypto.blake2b(msg, outlen, key) == hashlib.blake2b(msg, digest_size=outlen, key=key).digest()


def test_salsa20_spec_and_model(native):
    key = bytes(range(1, 17)) + bytes(range(201, 217))
    nonce = bytes(range(101, 109))
    ctr = int.from_bytes(bytes(range(109, 117)), "little")
    out = native.crypto.salsa20_block(key, nonce, ctr)
    assert list(out[:8]) == [69, 37, 68, 39, 41, 15, 107, 193]
    assert out == py_salsa20_block(key, nonce, ctr)
    for _ in range(5):
        k, n, c = os.urandom(32), os.urandom(8), int.from_bytes(os.urandom(8), "little")
        assert native.crypto.salsa20_block(k, n, c) == py_salsa20_block(k, n, c)


def test_nacl_box_vector(native):
    c = native.crypto
    alicesk = H("77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a")
    bobpk = H("de9edb7d7b7dc1b4d35b61c2ece435373f8343c85b78674dadfc7e146f882b4f")
    assert c.x25519_base(alicesk) == H("8520f0098930a754748b7ddcb43ef75a0dbf3a0d26381af4eba4a98eaa9b4e6a")
    shared, ok = c.x25519(alicesk, bobpk)
    assert ok and shared == H("4a5d9d5ba4ce2de1728e3bf480350f25e07e21c947d19e3376f09b3c1e161742")
    k = c.box_beforenm(bobpk, alicesk)
    assert k == H("1b27556473e985d462cd51197a9a46c76009549eac6474f206c4ee0844f68389")
    nonce = H("69696ee955b62b73cd62bda875fc73d68219e0036b7a0b37")
    m = H("be075fc53c81f2d5cf141316ebeb0c7b5228c52a4c62cbd44b66849b64244ffce5ecbaaf33bd751a1ac728d45e6c61296cdc3c01233561f41db66cce314adb310e3be8250c46f06dceea3a7fa1348057e2f6556ad6b1318a024a838f21af1fde048977eb48f59ffd4924ca1c60902e52f0a089bc76897040e082f937763848645e0705")
    expect = H("f3ffc7703f9400e52a7dfb4b3d3305d98e993b9f48681273c29650ba32fc76ce48332ea7164d96a4476fb8c531a1186ac0dfc17c98dce87b4da7f011ec48c97271d2c20f9b928fe2270d6fb863d51738b48eeee314a7cc8ab932164548e526ae90224368517acfeabd6bb3732bc0e9da99832b61ca01b6de56244a9e88d5f9b37973f622a43d14a6599b1f654cb45a74e355a5")
    assert c.secretbox_easy(m, nonce, k) == expect


def test_poly1305_rfc8439_and_model(native):
    key = H("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    assert native.crypto.poly1305(b"Cryptographic Forum Research Group", key) == H("a8061dc1305136c6c22b8baf0c0127a9")
    for n in [0, 1, 15, 16, 17, 63, 64, 1000]:
        k, m = os.urandom(32), os.urandom(n)
        assert native.crypto.poly1305(m, k) == py_poly1305(m, k)


def test_ed25519_rfc8032(native):
    c = native.crypto
    seed = H("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    pk, sk = c.ed25519_keypair_from_seed(seed)
    assert pk == H("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a")
    assert sk == seed + pk
    sig = c.ed25519_sign(b"", sk)
    assert sig == H("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert c.ed25519_verify(sig, b"", pk)
    # RFC 8032 test 2 (one-byte message)
    seed2 = H("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb")
    pk2, sk2 = c.ed25519_keypair_from_seed(seed2)
    assert pk2 == H("3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c")
    sig2 = c.ed25519_sign(H("72"), sk2)
    assert sig2 == H("92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00")
    assert c.ed25519_verify(sig2, H("72"), pk2)
    assert not c.ed25519_verify(sig2, H("73"), pk2)
    bad = bytearray(sig2)
    bad[40] ^= 1
    assert not c.ed25519_verify(bytes(bad), H("72"), pk2)


def test_sealed_box_roundtrip(native):
    c = native.crypto
    pk, sk = c.box_keypair()
    for n in [0, 1, 31, 32, 100, 5000]:
        m = os.urandom(n)
        ct = c.box_seal(m, pk)
        assert len(ct) == n + 48
        assert c.box_seal_open(ct, pk, sk) == m
        tampered = bytearray(ct)
        tampered[-1 if n else 40] ^= 1
        assert c.box_seal_open(bytes(tampered), pk, sk) is None
    # deterministic ephemeral key -> structure check: epk || mac || ct
    esk = os.urandom(32)
    ct = c.box_seal(b"hello", pk, esk)
    epk = c.x25519_base(esk)
    assert ct[:32] == epk
    nonce = c.seal_nonce(epk, pk)
    k = c.box_beforenm(pk, esk)
    assert ct[32:] == c.secretbox_easy(b"hello", nonce, k)


def test_chacharng_matches_chacha20_rfc(native):
    # rand-0.3 ChaChaRng with a zero seed == ChaCha20 keystream, zero key/nonce
    rng = native.crypto.ChaChaRng([0, 0, 0, 0])
    words = [rng.next_u32() for _ in range(4)]
    assert words == [0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653]
    # next_u64 = high word first
    rng = native.crypto.ChaChaRng([1, 2, 3, 4])
    a, b = rng.next_u32(), rng.next_u32()
    rng2 = native.crypto.ChaChaRng([1, 2, 3, 4])
    assert rng2.next_u64() == (a << 32) | b
    # gen_range is uniform-mod with rejection zone
    rng3 = native.crypto.ChaChaRng([7])
    rng4 = native.crypto.ChaChaRng([7])
    for _ in range(100):
        v = rng4.next_u64()
        assert rng3.gen_range(0, 433) == v % 433


# ------------------------------------------------------------ OpenSSL oracle
def _libcrypto():
    name = ctypes.util.find_library("crypto")
    if not name:
        return None
    try:
        return ctypes.CDLL(name)
    except OSError:
        return None


def _evp_raw_public(lib, nid, priv: bytes) -> bytes:
    lib.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
    lib.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.EVP_PKEY_get_raw_public_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
    lib.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
    key = lib.EVP_PKEY_new_raw_private_key(nid, None, priv, len(priv))
    assert key
    buf = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    assert lib.EVP_PKEY_get_raw_public_key(key, buf, ctypes.byref(n)) == 1
    lib.EVP_PKEY_free(key)
    return buf.raw[:n.value]


def test_openssl_oracle_x25519_ed25519(native):
    lib = _libcrypto()
    if lib is None:
        pytest.skip("libcrypto not available")
    NID_X25519, NID_ED25519 = 1034, 1087
    for _ in range(10):
        sk = os.urandom(32)
        assert native.crypto.x25519_base(sk) == _evp_raw_public(lib, NID_X25519, sk)
        seed = os.urandom(32)
        pk, _ = native.crypto.ed25519_keypair_from_seed(seed)
        assert pk == _evp_raw_public(lib, NID_ED25519, seed)


def test_x25519_comb_table_of_the_base_point_is_the_generated_one(native):
    """The host's fixed-base table builder (Montgomery u -> edwards25519 point, 32 x 8
    multiples, one inversion for all) on u = 9 gives the table the GPU's ephemeral
    public keys come from (csrc/kernels/ed25519_base.inc, written by
    scripts/gen_ed25519_base.py with plain integers)."""
    import os
    import re
    import struct

    blob, ok = native.crypto.x25519_comb_tables([bytes([9] + [0] * 31)])
    assert ok == [True]
    words = struct.unpack("<%dI" % (len(blob) // 4), blob)
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "kernels",
                       "ed25519_base.inc")
    ref = [int(x, 16) for x in re.findall(r"0x([0-9a-f]+)u", open(inc).read())]
    assert len(ref) == len(words) == 32 * 8 * 32
    for e in range(256):
        assert list(words[32 * e:32 * e + 30]) == ref[32 * e:32 * e + 30], e
        assert words[32 * e + 30] == 1  # the "has a table" mark


def test_x25519_comb_table_refuses_a_key_on_the_twist(native):
    # u = 2 is not the u-coordinate of a curve25519 point (it lies on the twist)
    blob, ok = native.crypto.x25519_comb_tables([bytes([2] + [0] * 31), native.crypto.box_keypair()[0]])
    assert ok == [False, True]
    assert blob[:32 * 8 * 32 * 4] == bytes(32 * 8 * 32 * 4)
