"""GPU kernel numerics: every HIP kernel against the host C++ oracle or a plain
PyTorch reference of the same op (run with -m gpu on an MI355X)."""
import os

import pytest
import torch

from helpers import varint_decode, varint_encode

pytestmark = pytest.mark.gpu


def _words_le(b: bytes):
    return [int.from_bytes(b[4 * i:4 * i + 4], "little", signed=True) for i in range(len(b) // 4)]


def _bytes_le(words):
    return b"".join((int(w) & 0xFFFFFFFF).to_bytes(4, "little") for w in words)


def test_x25519_matches_host(cuda, native):
    c = native.crypto
    N = 96
    sc = [os.urandom(32) for _ in range(N)]
    pts = [c.box_keypair()[0] for _ in range(N - 2)] + [bytes([9] + [0] * 31), os.urandom(32)]
    from sda_amd.ops import gpu as G
    out = G.x25519(torch.tensor([_words_le(s) for s in sc], dtype=torch.int32, device=cuda),
                   torch.tensor([_words_le(p) for p in pts], dtype=torch.int32, device=cuda))
    out = out.cpu().tolist()
    for i in range(N):
        assert _bytes_le(out[i]) == c.x25519(sc[i], pts[i])[0], i


def _keytable(native, cuda, count):
    from sda_amd.engine import KeyTable
    return KeyTable.generate(count, cuda)


def test_x25519_fixed_base_matches_ladder(cuda, native):
    """The edwards25519 fixed-base route to an ephemeral public key (64 table
    additions) against the ladder on u = 9 and against the host."""
    from sda_amd._native import gpu
    n = 300
    sc = torch.randint(-2 ** 31, 2 ** 31 - 1, (n, 8), dtype=torch.int32)
    sc[0] = 0
    sc[1] = -1
    sc[2] = 0x77777777
    sc[3] = 0x88888888 - (1 << 32)  # every digit at the carry border
    nine = torch.zeros(n, 8, dtype=torch.int32)
    nine[:, 0] = 9
    d_sc, d_pt = sc.to(cuda), nine.to(cuda)
    a = torch.empty(n, 8, dtype=torch.int32, device=cuda)
    b = torch.empty(n, 8, dtype=torch.int32, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    gpu().x25519(n, d_sc.data_ptr(), d_pt.data_ptr(), a.data_ptr(), st)
    gpu().x25519_base(n, d_sc.data_ptr(), b.data_ptr(), st)
    assert torch.equal(a, b)
    for j in (0, 1, 5):
        host = native.crypto.x25519_base(sc[j].numpy().tobytes())
        assert b[j].cpu().numpy().tobytes() == host


@pytest.mark.parametrize("many,tables", [(0, False), (1, False), (1, True)])
def test_seal_setup_forms_open_on_host(cuda, native, many, tables):
    """The key-agreement kernels of the seal side -- two lanes per message with two
    ladders; one lane with the fixed-base table for the public key and a ladder for the
    shared point; one lane with tables for both (the recipients' keys get their own,
    one of them a key on the twist that has none) -- give boxes the host opens."""
    from sda_amd._native import gpu
    from sda_amd.engine import KeyTable
    from sda_amd.ops.sealed import Arena, seal_data, seal_setup
    keys = _keytable(native, cuda, 2)
    if tables:
        assert keys.tables(10) is None and keys.tables(10 ** 6) is not None
        # a third recipient whose public key is on the twist (no edwards25519 point):
        # X25519 still works for it, through the ladder
        sk3 = os.urandom(32)
        keys = KeyTable.from_bytes(keys.pk_bytes + [bytes([2] + [0] * 31)], keys.sk_bytes + [sk3], cuda)
    M, L, m = 70, 300, 433
    nk = len(keys.pk_bytes)
    vals64 = torch.randint(0, m, (M, L), dtype=torch.int64)
    kidx = torch.tensor([j % nk for j in range(M)], dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    gpu().set_seal_many(many)
    try:
        arena = Arena.empty(M, L, m, cuda)
        ks = seal_setup(arena, kidx, keys.pks, os.urandom(32), 0, err,
                        pk_tables=keys.tables() if tables else None)
        seal_data(arena, ks, vals64.to(torch.int16).to(cuda), err)
        blobs = arena.to_blobs()
    finally:
        gpu().set_seal_many(-1)
    assert int(err.item()) == 0
    for j in range(M):
        if j % nk == 2:  # the twist key has no matching secret key: its boxes only have to be
            continue     # produced without an error (the ladder path beside the table path)
        pt = native.crypto.box_seal_open(blobs[j], keys.pk_bytes[j % nk], keys.sk_bytes[j % nk])
        assert pt is not None and varint_decode(pt) == vals64[j].tolist(), j


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("L,modulus", [(1, 433), (10, 433), (5000, 433), (20000, 433),
                                       (3000, 2 ** 31 - 1), (70000, 65521), (150001, 433),
                                       (40000, 2 ** 31 - 1), (25000, 5038849), (7, 746497),
                                       (8192, (1 << 27) - 39),
                                       # a message's last values (fewer than a lane's 32) are spread over
                                       # the lanes behind them: few such lanes left at a tile's end
                                       (8191, 433), (8145, 746497), (16382, 5038849),
                                       # ends of at most a wave's 2048 values go four to a workgroup
                                       (2048, 433), (2047, 746497), (2049, 433), (10240, 5038849)])
def test_gpu_seal_opens_on_host(cuda, native, monkeypatch, L, modulus, fused):
    """GPU-sealed boxes open on the host. `fused`: the tag's middle chunks computed
    inside the encode kernel (per tile, in LDS) instead of by a pass over the
    stored ciphertext -- both must give libsodium's tag."""
    from sda_amd.ops import gpu as G
    from sda_amd.ops import sealed
    from sda_amd.ops.sealed import seal
    monkeypatch.setattr(sealed, "FUSED_SEAL_MAC", fused)
    keys = _keytable(native, cuda, 2)
    M = 5
    vdt = G.value_dtype(modulus)
    vals64 = torch.randint(0, modulus, (M, L), dtype=torch.int64)
    vals = vals64.to(vdt).to(cuda) if vdt == torch.int16 else vals64.to(torch.int32).to(cuda)
    kidx = torch.tensor([j % 2 for j in range(M)], dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    arena = seal(vals, kidx, keys.pks, os.urandom(32), 0, err, modulus)
    blobs = arena.to_blobs()
    assert int(err.item()) == 0
    for j in range(M):
        pk, sk = keys.pk_bytes[j % 2], keys.sk_bytes[j % 2]
        pt = native.crypto.box_seal_open(blobs[j], pk, sk)
        assert pt is not None, f"host could not open GPU box {j}"
        assert varint_decode(pt) == vals64[j].tolist()


@pytest.mark.parametrize("L", [1, 7, 4096, 9000, 40000])
def test_host_seal_opens_on_gpu(cuda, native, L):
    """Host (libsodium-format) boxes, including Rust-style negative shares."""
    from sda_amd.ops.sealed import Arena, open_
    m = 433
    keys = _keytable(native, cuda, 1)
    M = 4
    rows = []
    blobs = []
    for j in range(M):
        row = [int(x) for x in torch.randint(-m + 1, m, (L,)).tolist()]
        rows.append([x % m for x in row])
        blobs.append(native.crypto.box_seal(varint_encode(row), keys.pk_bytes[0]))
    arena = Arena.from_blobs(blobs, L, m, cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    kidx = torch.zeros(M, dtype=torch.int32, device=cuda)
    out = open_(arena, kidx, keys.sks, keys.pks, err, out_dtype=torch.int32)
    assert int(err.item()) == 0
    assert out.cpu().tolist() == rows


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_mac_modes_seal_and_open(cuda, native, mode):
    """The three Poly1305 arrangements give libsodium's tags on both sides: every
    chunk by Horner (0), middle chunks on the matrix cores with the first / last
    chunk in a launch of their own (1, the default), or inside the chunk kernel (2).
    Lengths: one chunk, first + last only, and several middle chunks."""
    from sda_amd._native import gpu
    from sda_amd.ops.sealed import Arena, open_, seal
    m = 433
    keys = _keytable(native, cuda, 1)
    gpu().set_mac_mfma(mode)
    try:
        for L in (5, 9000, 12000, 60000):
            vals64 = torch.randint(0, m, (3, L), dtype=torch.int64)
            kidx = torch.zeros(3, dtype=torch.int32, device=cuda)
            err = torch.zeros(1, dtype=torch.int32, device=cuda)
            arena = seal(vals64.to(torch.int16).to(cuda), kidx, keys.pks, os.urandom(32), 0, err, m)
            blobs = arena.to_blobs()
            for j in range(3):
                pt = native.crypto.box_seal_open(blobs[j], keys.pk_bytes[0], keys.sk_bytes[0])
                assert pt is not None and varint_decode(pt) == vals64[j].tolist(), (mode, L, j)
            back = Arena.from_blobs(blobs, L, m, cuda)
            out = open_(back, kidx, keys.sks, keys.pks, err, out_dtype=torch.int32)
            assert int(err.item()) == 0, (mode, L)
            assert torch.equal(out.cpu().to(torch.int64), vals64), (mode, L)
    finally:
        gpu().set_mac_mfma(1)


def test_one_pass_mac_block_edges(cuda, native):
    """Boxes of at most four chunks take the one-pass MAC (a wave per message, lanes
    strided over the 16-byte blocks from the message's end): plaintext lengths
    around every edge of that layout -- partial and whole final blocks, one block
    short of / exactly / one past a round of 64 blocks and a group of four rounds,
    the longest short box and the first chunked one (an arena sized for two-byte
    codes switches at L = 32752, one built from the blobs at 65504 bytes) -- sealed on
    the GPU and opened on the host, and sealed on the host and opened on the GPU.
    One-byte codes, so a box of L values has L plaintext bytes."""
    from sda_amd.ops import gpu as G
    from sda_amd.ops.sealed import Arena, open_, seal
    m = 433
    keys = _keytable(native, cuda, 1)
    kidx = torch.zeros(2, dtype=torch.int32, device=cuda)
    for L in (1, 2, 15, 16, 17, 31, 32, 33, 1007, 1008, 1009, 1023, 1024, 1025, 4095, 4096, 4097, 4112, 8191,
              4064, 4065, 8160, 8161, 16352, 16353, 16368, 32752, 32753, 49120, 49121, 65504, 65505):
        vals64 = torch.randint(0, 64, (2, L), dtype=torch.int64)
        err = torch.zeros(1, dtype=torch.int32, device=cuda)
        arena = seal(vals64.to(torch.int16).to(cuda), kidx, keys.pks, os.urandom(32), 0, err, m)
        blobs = arena.to_blobs()
        assert int(err.item()) == 0
        for j in range(2):
            assert len(blobs[j]) == 48 + L
            pt = native.crypto.box_seal_open(blobs[j], keys.pk_bytes[0], keys.sk_bytes[0])
            assert pt is not None and varint_decode(pt) == vals64[j].tolist(), (L, j)
        host = [native.crypto.box_seal(varint_encode(vals64[j].tolist()), keys.pk_bytes[0])
                for j in range(2)]
        back = Arena.from_blobs(host, L, m, cuda)
        out = open_(back, kidx, keys.sks, keys.pks, err, out_dtype=torch.int32)
        assert int(err.item()) == 0, L
        assert torch.equal(out.cpu().to(torch.int64), vals64), L
        # a flipped bit anywhere fails the check: first, middle and last byte
        for pos in (48, 48 + L // 2, 48 + L - 1, 33):
            bad = bytearray(host[0])
            bad[pos] ^= 0x40
            e2 = torch.zeros(1, dtype=torch.int32, device=cuda)
            open_(Arena.from_blobs([bytes(bad), host[1]], L, m, cuda), kidx, keys.sks, keys.pks, e2)
            assert int(e2.item()) & 2, (L, pos)


def _open_sum_case(native, cuda, rows_, P, L, m, gen, stats=None):
    """Host-sealed boxes (row-major: message r*P + p) -> open_sum vs a plain sum."""
    from sda_amd.ops.sealed import Arena, open_setup, open_sum
    keys = _keytable(native, cuda, 1)
    vals, blobs = [], []
    for j in range(rows_ * P):
        row = gen(j)
        vals.append([x % m for x in row])
        blobs.append(native.crypto.box_seal(varint_encode(row), keys.pk_bytes[0]))
    arena = Arena.from_blobs(blobs, L, m, cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    kidx = torch.zeros(rows_ * P, dtype=torch.int32, device=cuda)
    ks = open_setup(arena, kidx, keys.sks, keys.pks, err)
    out = torch.empty(rows_, L, dtype=torch.int32, device=cuda)
    open_sum(arena, ks, err, rows=rows_, out=out, stats=stats)
    ref = torch.tensor(vals, dtype=torch.int64).view(rows_, P, L).sum(1) % m
    return int(err.item()), out.cpu().to(torch.int64), ref


@pytest.mark.parametrize("L", [1, 7, 6144, 6145, 20000, 40000])
def test_open_sum_matches_torch(cuda, native, L):
    """Fused decode + combine over participants whose varint streams drift
    apart (all-1-byte, all-2-byte and mixed rows, Rust-style negatives)."""
    m = 433

    def gen(j):
        kind = j % 4
        if kind == 0:
            return [0] * L                                         # 1-byte varints
        if kind == 1:
            return torch.randint(200, m, (L,)).tolist()            # 2-byte varints
        if kind == 2:
            return torch.randint(-m + 1, m, (L,)).tolist()         # negatives (additive.rs:47)
        return torch.randint(0, m, (L,)).tolist()
    e, out, ref = _open_sum_case(native, cuda, 3, 9, L, m, gen)
    assert e == 0
    assert torch.equal(out, ref)


@pytest.mark.parametrize("lean", [1, 0])
@pytest.mark.parametrize("L,m", [(1, 433), (7, 433), (553, 433), (6144, 433), (6145, 433),
                                 (20000, 433), (40000, 433), (30000, 8191), (9000, 64),
                                 (7, 5038849), (6145, 65521), (20000, 746497), (20000, 5038849),
                                 (30000, (1 << 27) - 39)])
def test_open_sum_canonical_streams(cuda, native, L, m, lean):
    """Canonical shares only (what our participants and any canonical encoder
    produce): the lean kernels (sums of zigzag codes, k_decode_sum_z for varints of
    up to two bytes, m <= 2^13, and of up to four, m <= 2^27) and the generic one
    (lean switched off) both equal the plain sum. Row kinds stress
    the range edges: all-1-byte, all-2-byte, alternating and random streams
    drift apart by up to 2x in bytes, so 1 KiB sub-chunk cuts split varints."""
    from sda_amd._native import gpu

    def gen(j):
        kind = j % 5
        if kind == 0:
            return [0] * L
        if kind == 1:
            return torch.randint(min(64, m - 1), m, (L,)).tolist()
        if kind == 2:  # values on both sides of every varint length border
            edge = [63, 64] if m <= 8192 else [63, 64, 8191, 8192, 1048575, 1048576]
            return [edge[(i + i // 7) % len(edge)] % m for i in range(L)]
        if kind == 3:
            return [(m - 1) if (i % 3) else 1 for i in range(L)]
        return torch.randint(0, m, (L,)).tolist()
    gpu().set_decode_lean(lean)
    stats = {}
    try:
        e, out, ref = _open_sum_case(native, cuda, 2, 11, L, m, gen, stats)
    finally:
        gpu().set_decode_lean(1)
    assert e == 0
    assert torch.equal(out, ref)
    # canonical streams stay on the lean kernels: nothing raised the fallback
    assert int(stats["redo"].item()) == 0


@pytest.mark.parametrize("swz", [0, 1])
@pytest.mark.parametrize("L,m,by_value", [(6145, 433, -1), (20000, 433, -1), (30000, 8191, -1),
                                          (20000, 746497, 0), (20000, 746497, 1),
                                          (20000, 5038849, 0), (20000, 5038849, 1),
                                          (7, 746497, 1), (6145, 5038849, 1)])
def test_open_sum_accumulator_layouts(cuda, native, L, m, swz, by_value):
    """The lean decode-sum kernels with plain and with padded (33-word) accumulator
    rows, each forced for every modulus, and for the long-code fields both the byte-wise
    and the value-wise kernel: all equal the plain sum and none falls back."""
    from sda_amd._native import gpu

    def gen(j):
        if j % 3 == 0:
            return torch.randint(min(64, m - 1), m, (L,)).tolist()
        if j % 3 == 1:
            return [(m - 1) if (i % 5) else 0 for i in range(L)]
        return torch.randint(0, m, (L,)).tolist()
    gpu().set_decode_swz(swz)
    gpu().set_decode_long(by_value)
    stats = {}
    try:
        e, out, ref = _open_sum_case(native, cuda, 2, 9, L, m, gen, stats)
    finally:
        gpu().set_decode_swz(-1)
        gpu().set_decode_long(-1)
    assert e == 0
    assert torch.equal(out, ref)
    assert int(stats["redo"].item()) == 0


def test_open_sum_foreign_encodings(cuda, native):
    """Non-canonical values (>= m, long varints up to 10 bytes) take the generic
    and slow decode paths inside the fused kernel; large modulus (u32 path)."""
    L = 9000

    def gen_small(j):
        row = torch.randint(0, 433, (L,)).tolist()
        for i in range(j, L, 97):
            row[i] = [433 * 5 + 7, -(2 ** 40) - 3, 2 ** 62 + 11, 70000][i % 4]
        return row
    e, out, ref = _open_sum_case(native, cuda, 2, 5, L, 433, gen_small)
    assert e == 0
    assert torch.equal(out, ref)

    big = 2 ** 31 - 1
    e, out, ref = _open_sum_case(native, cuda, 1, 6, L, big,
                                 lambda j: torch.randint(-big + 1, big, (L,)).tolist())
    assert e == 0
    assert torch.equal(out, ref)

    # mid-size fields (lean kernel for up to four bytes): a code one byte longer than
    # the field's canonical ones, a negative value, a five-byte code -> generic decoder
    for m, odd in ((65521, [2 ** 20 + 5]), (746497, [2 ** 20 + 5, -3]),
                   (5038849, [2 ** 27 + 9]), (5038849, [-(2 ** 22)])):
        def gen_mid(j, m=m, odd=odd):
            row = torch.randint(0, m, (L,)).tolist()
            for i in range(j + 1, L, 1013):
                row[i] = odd[i % len(odd)]
            return row
        from sda_amd._native import gpu
        for by_value in (0, 1):  # the byte-wise and the value-wise lean kernel both notice
            gpu().set_decode_long(by_value)
            stats = {}
            try:
                e, out, ref = _open_sum_case(native, cuda, 2, 5, L, m, gen_mid, stats)
            finally:
                gpu().set_decode_long(-1)
            assert e == 0, (m, odd)
            assert torch.equal(out, ref), (m, odd)
            assert int(stats["redo"].item()) != 0, (m, odd, by_value)


def test_open_sum_flags_wrong_length(cuda, native):
    from sda_amd.ops.sealed import Arena, open_setup, open_sum
    keys = _keytable(native, cuda, 1)
    L = 5000
    blobs = [native.crypto.box_seal(varint_encode(list(range(L - (j == 1)))), keys.pk_bytes[0])
             for j in range(3)]
    arena = Arena.from_blobs(blobs, L, 433, cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    ks = open_setup(arena, torch.zeros(3, dtype=torch.int32, device=cuda), keys.sks, keys.pks, err)
    open_sum(arena, ks, err, rows=1, out=torch.empty(L, dtype=torch.int32, device=cuda))
    assert int(err.item()) & 4


def test_tampered_box_is_rejected(cuda, native):
    from sda_amd.ops.sealed import Arena, open_
    keys = _keytable(native, cuda, 1)
    blob = bytearray(native.crypto.box_seal(varint_encode(list(range(100))), keys.pk_bytes[0]))
    blob[60] ^= 0x10
    arena = Arena.from_blobs([bytes(blob)], 100, 433, cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    open_(arena, torch.zeros(1, dtype=torch.int32, device=cuda), keys.sks, keys.pks, err)
    assert int(err.item()) & 2


def test_colsum_matches_torch(cuda):
    from sda_amd.ops import gpu as G
    for dt, m in [(torch.int16, 433), (torch.int32, 2 ** 31 - 1)]:
        x = torch.randint(0, m, (3, 50, 1003), dtype=torch.int64)
        out = torch.empty(3, 1003, dtype=torch.int32, device=cuda)
        G.colsum(x.to(dt).to(cuda) if dt == torch.int16 else x.to(torch.int32).to(cuda), m, out)
        assert torch.equal(out.cpu().to(torch.int64), x.sum(1) % m)


def test_chacha_mask_matches_rand03(cuda, native):
    from sda_amd.ops import gpu as G
    P, D, m = 3, 50, 433
    seeds = torch.randint(-2 ** 31, 2 ** 31, (P, 4), dtype=torch.int64).to(torch.int32)
    out = torch.empty(D, dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    G.chacha_mask_sum(seeds.to(cuda), D, m, out, err)
    exp = [0] * D
    for p in range(P):
        rng = native.crypto.ChaChaRng([int(w) & 0xFFFFFFFF for w in seeds[p].tolist()])
        for i in range(D):
            exp[i] = (exp[i] + rng.gen_range(0, m)) % m
    assert out.cpu().tolist() == exp
    assert int(err.item()) == 0


class _zone_cap:
    """rand-0.3 acceptance zone capped on the host model and the device kernels alike
    (test hook): rejections, at most 1e-10 per draw in production, become frequent."""

    def __init__(self, native, cap):
        self.native, self.cap = native, cap

    def __enter__(self):
        from sda_amd._native import gpu
        self.native.crypto.set_chacha_zone_cap(self.cap)
        gpu().set_chacha_zone_cap(self.cap)

    def __exit__(self, *exc):
        from sda_amd._native import gpu
        self.native.crypto.set_chacha_zone_cap(2 ** 64 - 1)
        gpu().set_chacha_zone_cap(2 ** 64 - 1)


def _host_masks(native, seeds, D, m):
    out = []
    for row in seeds.tolist():
        rng = native.crypto.ChaChaRng([int(w) & 0xFFFFFFFF for w in row])
        out.append([rng.gen_range(0, m) for _ in range(D)])
    return torch.tensor(out, dtype=torch.int64)


def _rejected_positions(native, seed_row, count, m, cap):
    zone = min(2 ** 64 - 1 - (2 ** 64 - 1) % m, cap - cap % m)
    rng = native.crypto.ChaChaRng([int(w) & 0xFFFFFFFF for w in seed_row])
    return [d for d in range(count) if rng.next_u64() >= zone]


@pytest.mark.parametrize("m,den", [(433, 16), (2 ** 31 - 1, 16), (433, 3)])
def test_chacha_mask_with_rejected_draws_matches_rand03(cuda, native, m, den):
    """rand 0.3 `gen_range` re-draws a rejected value, which shifts every later
    element of that participant's stream (client/src/crypto/masking/chacha.rs:36-39,
    67-72). With the acceptance zone capped so that about one draw in `den` is
    rejected, the device expansion -- recipient sum and participant masking -- must
    equal the host ChaChaRng element for element: rejections on a ChaCha block's
    last draw, on a 2048-draw chunk's last draw, several in one block."""
    from sda_amd.ops import gpu as G
    P, D = 5, 6001  # three chunks of draws, a ragged tail
    cap = 2 ** 64 - 2 ** 64 // den
    g = torch.Generator().manual_seed(den * 7 + m % 97)
    seeds = torch.randint(-2 ** 31, 2 ** 31, (P, 4), dtype=torch.int64, generator=g)
    # participant 0's seed: a stream whose draw 2047 (last of the first chunk) is rejected
    zone = cap - cap % m
    for s0 in range(4000):
        rng = native.crypto.ChaChaRng([s0])
        for _ in range(2047):
            rng.next_u64()
        if rng.next_u64() >= zone:
            seeds[0] = torch.tensor([s0, 0, 0, 0])
            break
    else:
        pytest.fail("no seed with a rejection on a chunk's last draw")
    seeds = seeds.to(torch.int32)
    rej = [_rejected_positions(native, row, D + D // 2, m, cap) for row in seeds.tolist()]
    assert 2047 in rej[0]
    assert any(d % 8 == 7 for r in rej for d in r)                      # a block's last draw
    assert any(a + 1 == b for r in rej for a, b in zip(r, r[1:]))       # two in a row
    with _zone_cap(native, cap):
        masks = _host_masks(native, seeds, D, m)
        err = torch.zeros(1, dtype=torch.int32, device=cuda)
        out = torch.empty(D, dtype=torch.int32, device=cuda)
        G.chacha_mask_sum(seeds.to(cuda), D, m, out, err)
        secrets = torch.randint(-m, m, (P, D), dtype=torch.int32, generator=g)
        masked = G.chacha_mask_apply(secrets.to(cuda), seeds.to(cuda), m, err)
        torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(out.cpu().to(torch.int64), masks.sum(0) % m)
    assert torch.equal(masked.cpu().to(torch.int64), (secrets.to(torch.int64) + masks) % m)
    # without the cap the same seeds expand without a rejection, to other values
    out2 = torch.empty(D, dtype=torch.int32, device=cuda)
    G.chacha_mask_sum(seeds.to(cuda), D, m, out2, err)
    assert torch.equal(out2.cpu().to(torch.int64), _host_masks(native, seeds, D, m).sum(0) % m)
    assert not torch.equal(out, out2)


def test_chacha_mask_reports_a_stream_that_runs_dry(cuda, native):
    """More than half of the draws rejected: the scanned range (2 D + 4096 draws)
    cannot hold D accepted ones; the error word says so instead of a wrong sum."""
    from sda_amd.ops import gpu as G
    P, D, m = 2, 9000, 433
    seeds = torch.tensor([[1, 2, 3, 4], [5, 6, 7, 8]], dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    out = torch.empty(D, dtype=torch.int32, device=cuda)
    with _zone_cap(native, 2 ** 62):  # three draws in four rejected
        G.chacha_mask_sum(seeds, D, m, out, err)
        torch.cuda.synchronize()
    assert int(err.item()) & 8


def test_round_with_chacha_masks_under_rejections(cuda, native):
    """A whole round whose participants and recipient both meet rejected draws."""
    from sda_amd.models.schemes import Additive, AggregationSpec, ChaChaMask
    with _zone_cap(native, 2 ** 64 - 2 ** 64 // 9):
        _round(cuda, AggregationSpec(5003, 433, Additive(3, 433), ChaChaMask(433, 5003)), 7)


def test_additive_shares_sum_to_secret(cuda):
    from sda_amd.ops import gpu as G
    P, D, n, m = 4, 5000, 3, 433
    secrets = torch.randint(-1000, 1000, (P, D), dtype=torch.int32, device=cuda)
    shares = torch.empty(n, P, D, dtype=torch.int16, device=cuda)
    cnt = torch.empty(n * P * G.tiles(D), dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    G.share_additive(secrets, n, m, shares, cnt, G.MASK_NONE, os.urandom(32), 0)
    s = shares.to(torch.int64).sum(0) % m
    assert torch.equal(s, torch.remainder(secrets.to(torch.int64), m))
    # random shares are spread over [0, m)
    r = shares[0].to(torch.int64).flatten()
    assert r.min() >= 0 and r.max() < m
    hist = torch.bincount(r, minlength=m).float()
    assert hist.std() / hist.mean() < 0.25
    # byte counts match the varint lengths
    exp = [len(varint_encode(shares[c, p].to(torch.int64).tolist())) for c in range(n) for p in range(P)]
    got = cnt.view(n * P, -1).sum(1).tolist()
    assert got == exp


def _round(cuda, spec, P, clerks=None):
    from sda_amd.engine import DeviceAggregator, reference_sum
    agg = DeviceAggregator(spec, cuda)
    secrets = torch.randint(0, spec.field_modulus, (P, spec.dimension), dtype=torch.int32,
                            device=cuda)
    res = agg.run_round(secrets, clerks=clerks)
    assert torch.equal(res.output, reference_sum(secrets, spec.field_modulus))
    return res


def test_unchecked_rounds_stay_two_deep(cuda):
    """Unchecked rounds (no host read-back) may be queued at most two ahead of the GPU:
    the host queues a round ten times faster than the GPU runs it, and every round in
    flight holds its own arenas. Outputs of all of them stay correct."""
    from sda_amd.engine import DeviceAggregator, reference_sum
    from sda_amd.models import AggregationSpec, Additive
    spec = AggregationSpec(20000, 433, Additive(3, 433))
    agg = DeviceAggregator(spec, cuda)
    secrets = torch.randint(0, 433, (16, 20000), dtype=torch.int32, device=cuda)
    ref = reference_sum(secrets, 433)
    outs = []
    for _ in range(9):
        res = agg.run_round(secrets, check=False)
        outs.append((res.output, res.err))
        assert len(agg._inflight) <= 2
        assert all(ev.query() for ev in list(agg._inflight)[:-2]) or len(agg._inflight) <= 2
    torch.cuda.synchronize()
    for out, err in outs:
        assert int(err.item()) == 0
        assert torch.equal(out, ref)


@pytest.mark.parametrize("name", ["additive", "fullmask", "chachamask", "pss", "pss_dropout"])
def test_unchecked_rounds_result_path_beside_the_next_round(cuda, name):
    """Unchecked rounds run their result path (clerks seal, recipient opens,
    reconstructs, unmasks) on a stream of their own and hand the tensors over at
    first read. Rounds over different inputs, read one round late (as the
    benchmarks do), read at once, and mixed with checked rounds, all give the
    plain sums; the overlap can be switched off and changes nothing."""
    from sda_amd.engine import DeviceAggregator, reference_sum
    from sda_amd.models import (PSS_4_8_3, Additive, AggregationSpec, ChaChaMask, FullMask,
                                pss_5_of_8)
    D, P, m = 30011, 12, 433
    clerks = None
    if name == "additive":
        spec = AggregationSpec(D, m, Additive(3, m))
    elif name == "fullmask":
        spec = AggregationSpec(D, m, Additive(3, m), FullMask(m))
    elif name == "chachamask":
        spec = AggregationSpec(D, m, Additive(3, m), ChaChaMask(m, D))
    elif name == "pss":
        spec = AggregationSpec(D, m, PSS_4_8_3)
    else:
        spec, clerks = AggregationSpec(D, m, pss_5_of_8()), [0, 2, 3, 5, 7]
    agg = DeviceAggregator(spec, cuda)
    xs = [torch.randint(0, m, (P, D), dtype=torch.int32, device=cuda) for _ in range(6)]
    refs = [reference_sum(x, m) for x in xs]
    # read one round late
    prev, got = None, []
    for x in xs:
        res = agg.run_round(x, clerks=clerks, check=False)
        assert res._ready is not None  # its result path went to the tail stream
        if prev is not None:
            got.append((prev.output, prev.err))
        prev = res
    got.append((prev.output, prev.err))
    assert prev._ready is None
    # a checked round right behind unchecked ones, then unchecked ones read at once
    chk = agg.run_round(xs[0], clerks=clerks)
    assert chk._ready is None and torch.equal(chk.output, refs[0])  # joined by its own check
    now = [agg.run_round(x, clerks=clerks, check=False).output.clone() for x in xs[:3]]
    agg.overlap_reveal = False
    off = agg.run_round(xs[1], clerks=clerks, check=False)
    assert off._ready is None
    torch.cuda.synchronize()
    for (out, err), ref in zip(got, refs):
        assert int(err.item()) == 0
        assert torch.equal(out, ref)
    for out, ref in zip(now, refs):
        assert torch.equal(out, ref)
    assert int(off.err.item()) == 0 and torch.equal(off.output, refs[1])
    # the engine's running OR over all of these rounds, and a round that must raise it
    assert int(agg.take_errors().item()) == 0
    agg.overlap_reveal = True
    agg.run_round(xs[2], clerks=clerks, check=False)
    agg.corrupt_next_round()
    agg.run_round(xs[3], clerks=clerks, check=False)
    agg.run_round(xs[4], clerks=clerks, check=False)
    assert int(agg.take_errors().item()) != 0
    assert int(agg.take_errors().item()) == 0  # taken: a fresh start


def test_round_additive(cuda):
    from sda_amd.models import AggregationSpec, Additive
    _round(cuda, AggregationSpec(10000, 433, Additive(3, 433)), 7)


def test_round_additive_fullmask(cuda):
    from sda_amd.models import AggregationSpec, Additive, FullMask
    _round(cuda, AggregationSpec(5000, 433, Additive(3, 433), FullMask(433)), 5)


def test_round_additive_chachamask(cuda):
    from sda_amd.models import AggregationSpec, Additive, ChaChaMask
    _round(cuda, AggregationSpec(5000, 433, Additive(3, 433), ChaChaMask(433, 5000)), 5)


def test_round_large_modulus(cuda):
    from sda_amd.models import AggregationSpec, Additive
    m = 2 ** 31 - 1
    _round(cuda, AggregationSpec(3000, m, Additive(5, m)), 4)


def test_round_pss_483(cuda):
    from sda_amd.models import AggregationSpec, PSS_4_8_3
    _round(cuda, AggregationSpec(10000, 433, PSS_4_8_3), 6)


def test_round_pss_dropout(cuda):
    from sda_amd.models import AggregationSpec, PSS_4_8_3, pss_5_of_8
    _round(cuda, AggregationSpec(3001, 433, PSS_4_8_3), 4, clerks=[0, 1, 2, 4, 5, 6, 7])
    _round(cuda, AggregationSpec(3001, 433, pss_5_of_8()), 4, clerks=[1, 3, 4, 6, 7])


def test_round_pss_fullmask(cuda):
    from sda_amd.models import AggregationSpec, PSS_4_8_3, FullMask
    _round(cuda, AggregationSpec(2000, 433, PSS_4_8_3, FullMask(433)), 3)


@pytest.mark.parametrize("M,T", [(7, 3), (5000, 3), (5000, 16), (4096, 1), (300, 700), (5000, 64), (5000, 65)])
def test_segscan_rows(cuda, native, M, T):
    """Row-wise exclusive scan: the workgroup-per-row kernel and the thread-per-row one
    (many short rows) against torch.cumsum; a row off its expected sum raises the error word."""
    from sda_amd.ops import gpu as G
    data = torch.randint(0, 1000, (M, T), dtype=torch.int32)
    data[:, -1] += 100_000 - data.sum(dim=1, dtype=torch.int32)  # every row sums to 100,000
    want = torch.cumsum(data, dim=1, dtype=torch.int64) - data
    d = data.to(cuda)
    totals = torch.empty(M, dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    G.segscan(d, totals, expect=100_000, err=err)
    assert torch.equal(d.cpu().to(torch.int64), want)
    assert torch.equal(totals.cpu(), torch.full((M,), 100_000, dtype=torch.int32))
    assert int(err.item()) == 0
    bad = data.clone()
    bad[M // 2, 0] += 1
    d = bad.to(cuda)
    G.segscan(d, totals, expect=100_000, err=err)
    assert int(err.item()) != 0
