"""Pure-Python models used as independent oracles in tests."""
from __future__ import annotations


def zigzag(v: int) -> int:
    return (v << 1) ^ (v >> 63) if v < 0 else v << 1


def unzigzag(z: int) -> int:
    return (z >> 1) ^ -(z & 1)


def varint_encode(values) -> bytes:
    """integer-encoding `VarInt for i64` (zigzag + LEB128), reference sodium.rs:36-41."""
    out = bytearray()
    for v in values:
        z = zigzag(int(v)) & ((1 << 64) - 1)
        while True:
            b = z & 0x7F
            z >>= 7
            if z:
                out.append(b | 0x80)
            else:
                out.append(b)
                break
    return bytes(out)


def varint_decode(data: bytes) -> list[int]:
    out, z, shift = [], 0, 0
    for b in data:
        z |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            out.append(unzigzag(z))
            z, shift = 0, 0
    if shift:
        raise ValueError("dangling continuation byte")
    return out


# --- independent Salsa20 (spec model) ------------------------------------
def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def salsa20_core(inp: list[int]) -> list[int]:
    x = list(inp)
    for _ in range(10):
        for a, b, c, d in ((0, 4, 8, 12), (5, 9, 13, 1), (10, 14, 2, 6), (15, 3, 7, 11)):
            x[b] ^= _rotl((x[a] + x[d]) & 0xFFFFFFFF, 7)
            x[c] ^= _rotl((x[b] + x[a]) & 0xFFFFFFFF, 9)
            x[d] ^= _rotl((x[c] + x[b]) & 0xFFFFFFFF, 13)
            x[a] ^= _rotl((x[d] + x[c]) & 0xFFFFFFFF, 18)
        for a, b, c, d in ((0, 1, 2, 3), (5, 6, 7, 4), (10, 11, 8, 9), (15, 12, 13, 14)):
            x[b] ^= _rotl((x[a] + x[d]) & 0xFFFFFFFF, 7)
            x[c] ^= _rotl((x[b] + x[a]) & 0xFFFFFFFF, 9)
            x[d] ^= _rotl((x[c] + x[b]) & 0xFFFFFFFF, 13)
            x[a] ^= _rotl((x[d] + x[c]) & 0xFFFFFFFF, 18)
    return [(x[i] + inp[i]) & 0xFFFFFFFF for i in range(16)]


def salsa20_block(key: bytes, nonce: bytes, ctr: int) -> bytes:
    w = lambda b, i: int.from_bytes(b[4 * i:4 * i + 4], "little")  # noqa: E731
    c = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    n16 = nonce + ctr.to_bytes(8, "little")
    inp = [c[0], w(key, 0), w(key, 1), w(key, 2), w(key, 3), c[1], w(n16, 0), w(n16, 1),
           w(n16, 2), w(n16, 3), c[2], w(key, 4), w(key, 5), w(key, 6), w(key, 7), c[3]]
    return b"".join(v.to_bytes(4, "little") for v in salsa20_core(inp))


# --- independent Poly1305 (RFC 8439 big-integer model) --------------------
def poly1305(msg: bytes, key: bytes) -> bytes:
    r = int.from_bytes(key[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    s = int.from_bytes(key[16:32], "little")
    p = (1 << 130) - 5
    acc = 0
    for i in range(0, len(msg), 16):
        blk = msg[i:i + 16] + b"\x01"
        acc = (acc + int.from_bytes(blk, "little")) * r % p
    return ((acc + s) & ((1 << 128) - 1)).to_bytes(16, "little")


# --- tss 0.2 packed Shamir model (FFT construction) ----------
def fft2_inverse(a, omega, p):
    n = len(a)
    inv_omega = pow(omega, p - 2, p)
    res = fft2(a, inv_omega, p)
    ninv = pow(n, p - 2, p)
    return [x * ninv % p for x in res]


def fft2(a, omega, p):
    n = len(a)
    if n == 1:
        return [a[0] % p]
    ev = fft2(a[0::2], omega * omega % p, p)
    od = fft2(a[1::2], omega * omega % p, p)
    out = [0] * n
    w = 1
    for i in range(n // 2):
        t = w * od[i] % p
        out[i] = (ev[i] + t) % p
        out[i + n // 2] = (ev[i] - t) % p
        w = w * omega % p
    return out


def dft(a, omega, p):
    n = len(a)
    return [sum(a[j] * pow(omega, i * j, p) for j in range(n)) % p for i in range(n)]


def tss_share(secrets, randomness, t, n, k, p, ws, wn):
    values = [0] + list(secrets) + list(randomness)
    assert len(values) == t + k + 1
    coeffs = fft2_inverse(values, ws, p)
    coeffs += [0] * (n + 1 - len(coeffs))
    pts = dft(coeffs, wn, p)  # radix-3 FFT == DFT of size n+1
    assert pts[0] == 0
    return pts[1:]
