"""Checked, tensor-level wrappers around the gfx950 kernels in ``_sda_gpu``.

Every wrapper validates device / dtype / shape / contiguity on the host before
launching (a kernel fed a wrong shape could fault the whole node), then passes
raw pointers plus the current HIP stream. All launches are asynchronous.
"""
from __future__ import annotations

import torch

from .._native import gpu as _gpu

TILE_VALUES = 4096
CHUNK_BYTES = 16384
SUB_BYTES = 1024                  # terminator-count granularity of the fused clerk path
SUB_PER_CHUNK = CHUNK_BYTES // SUB_BYTES
SUM_TILE = 6144                   # elements per decode-sum tile (k_decode_sum)
MSGKEY_BYTES = 80
POW_WORDS = 6560  # Poly1305 tables per message (k_poly_powers; kernels.hpp kPowWords)
POW_SHORT_WORDS = 320  # ... of the one-pass MAC of short messages (kPowShortWords)
SHORT_MAX_CHUNKS = 4   # messages of at most this many 16 KiB chunks take it (kShortMaxChunks)
SEAL_OVERHEAD = 48

MASK_NONE, MASK_FULL, MASK_CHACHA = 0, 1, 2


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _check(t: torch.Tensor, name: str, dtype=None, numel: int | None = None, min_numel: int | None = None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if dtype is not None and t.dtype not in (dtype if isinstance(dtype, tuple) else (dtype,)):
        raise TypeError(f"{name}: dtype {t.dtype} not in {dtype}")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: expected {numel} elements, got {t.numel()}")
    if min_numel is not None and t.numel() < min_numel:
        raise ValueError(f"{name}: expected at least {min_numel} elements, got {t.numel()}")


def value_dtype(modulus: int) -> torch.dtype:
    """u16 storage when every canonical value fits (m <= 65536), else u32 (int32 view)."""
    return torch.int16 if 0 < modulus <= 65536 else torch.int32


def value_bytes(dtype: torch.dtype) -> int:
    return {torch.uint8: 1, torch.int16: 2}.get(dtype, 4)


VALUE_DTYPES = (torch.uint8, torch.int16, torch.int32)


def varint_max_len(modulus: int) -> int:
    """Longest zigzag varint of a canonical value below `modulus` (0 = any u32)."""
    if modulus == 0:
        return 5
    z = 2 * (modulus - 1)
    n = 1
    while z >= 128:
        z >>= 7
        n += 1
    return n


def tiles(L: int) -> int:
    return (L + TILE_VALUES - 1) // TILE_VALUES


def chunks_for(max_pt: int) -> int:
    return (max_pt + 32 + CHUNK_BYTES - 1) // CHUNK_BYTES


def rng_words(key: bytes) -> list[int]:
    if len(key) != 32:
        raise ValueError("rng key must be 32 bytes")
    return [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]


# --------------------------------------------------------------- launches ----
def _gate_args(gate):
    """(tensor, value) dispatch token or None -> (pointer, value)."""
    if gate is None:
        return 0, 0
    t, v = gate
    _check(t, "gate", torch.int32, numel=1)
    return _ptr(t), int(v) & 0xFFFFFFFF


KEY_TABLE_WORDS = 32 * 8 * 32  # fixed-base table of one public key (kernels.hpp kKeyTableWords)


def seal_setup(M, rng_key, owner_base, key_idx, pks, ct, stride, keys, err, gate=None,
               pk_tables=None):
    """`pk_tables` (int32 [K][KEY_TABLE_WORDS], from the host's x25519_comb_tables): the
    public keys' fixed-base tables, which large launches use instead of the ladder."""
    _check(key_idx, "key_idx", torch.int32, numel=M)
    _check(pks, "pks", torch.int32)
    if pks.numel() % 8:
        raise ValueError("pks must be [K][8] words")
    if pk_tables is not None:
        _check(pk_tables, "pk_tables", torch.int32, numel=pks.numel() // 8 * KEY_TABLE_WORDS)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(err, "err", torch.int32, numel=1)
    if stride % 64:
        raise ValueError("stride must be a multiple of 64")
    _gpu().seal_setup(M, rng_words(rng_key), owner_base, _ptr(key_idx), _ptr(pks), _ptr(ct),
                      stride, _ptr(keys), _ptr(err), *_gate_args(gate),
                      0 if pk_tables is None else _ptr(pk_tables), _stream())


def open_setup(M, key_idx, sks, pks, ct, stride, keys, err, gate=None):
    _check(key_idx, "key_idx", torch.int32, numel=M)
    _check(sks, "sks", torch.int32)
    _check(pks, "pks", torch.int32, numel=sks.numel())
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(err, "err", torch.int32, numel=1)
    _gpu().open_setup(M, _ptr(key_idx), _ptr(sks), _ptr(pks), _ptr(ct), stride, _ptr(keys),
                      _ptr(err), *_gate_args(gate), _stream())


def gate_wait(gate, timeout_us: int = 3000):
    """On the current stream: wait (bounded) until a setup kernel launched with
    `gate` has been dispatched (see launch_gate_wait)."""
    ptr, val = _gate_args(gate)
    _gpu().gate_wait(ptr, val, int(timeout_us), _stream())


def x25519(scalars: torch.Tensor, points: torch.Tensor) -> torch.Tensor:
    _check(scalars, "scalars", torch.int32)
    _check(points, "points", torch.int32, numel=scalars.numel())
    if scalars.numel() % 8:
        raise ValueError("x25519 operands are [N][8] words")
    out = torch.empty_like(scalars)
    _gpu().x25519(scalars.numel() // 8, _ptr(scalars), _ptr(points), _ptr(out), _stream())
    return out


def share_additive(secrets, n, modulus, shares, cnt, mask_mode, rng_key, owner_base,
                   mask_out=None, mask_cnt=None):
    """Additive shares of `secrets` [P][D] (+ a full mask with MASK_FULL). ChaCha-masked
    participants mask first (:func:`chacha_mask_apply`) and share with MASK_NONE."""
    P, D = secrets.shape
    _check(secrets, "secrets", torch.int32)
    vb = value_bytes(shares.dtype)
    _check(shares, "shares", (torch.int16, torch.int32), numel=n * P * D)
    T = tiles(D)
    _check(cnt, "cnt", torch.int32, numel=n * P * T)
    if n < 2:
        raise ValueError("additive sharing needs at least 2 shares")
    if mask_mode not in (MASK_NONE, MASK_FULL):
        raise ValueError("share_additive: mask mode none or full")
    if mask_mode == MASK_FULL:  # the masks are stored like the shares
        _check(mask_out, "mask_out", shares.dtype, numel=P * D)
        _check(mask_cnt, "mask_cnt", torch.int32, numel=P * T)
    z = 0
    _gpu().share_additive(P, D, n, modulus, vb, _ptr(secrets), mask_mode,
                          rng_words(rng_key), owner_base, _ptr(shares), _ptr(cnt),
                          _ptr(mask_out) if mask_out is not None else z,
                          _ptr(mask_cnt) if mask_cnt is not None else z, _stream())


def mask_secrets(secrets, modulus, rng_key, owner_base, mask_out, mask_cnt) -> torch.Tensor:
    """Fully masked secrets (canonical int32 [P][D]) + the masks: the additive
    share kernel with a single share, whose only share is the masked secret."""
    P, D = secrets.shape
    _check(secrets, "secrets", torch.int32)
    _check(mask_out, "mask_out", torch.int32, numel=P * D)
    _check(mask_cnt, "mask_cnt", torch.int32, numel=P * tiles(D))
    masked = torch.empty(P, D, dtype=torch.int32, device=secrets.device)
    cnt = torch.empty(P * tiles(D), dtype=torch.int32, device=secrets.device)
    _gpu().share_additive(P, D, 1, modulus, 4, _ptr(secrets), MASK_FULL,
                          rng_words(rng_key), owner_base, _ptr(masked), _ptr(cnt),
                          _ptr(mask_out), _ptr(mask_cnt), _stream())
    return masked


def share_pss(secrets, n, k, t, prime, matrix, shares, cnt, mask_mode, rng_key, owner_base,
              mask_out=None):
    P, D = secrets.shape
    B = (D + k - 1) // k
    _check(secrets, "secrets", torch.int32)
    _check(matrix, "matrix", torch.int32, numel=n * (k + t))
    vb = value_bytes(shares.dtype)
    _check(shares, "shares", VALUE_DTYPES, numel=n * P * B)
    if shares.dtype == torch.uint8 and prime > 256:
        raise ValueError("u8 share storage needs a prime <= 256")
    _check(cnt, "cnt", torch.int32, numel=n * P * tiles(B))
    if mask_mode not in (MASK_NONE, MASK_FULL):
        raise ValueError("share_pss: mask mode none or full")
    if mask_mode == MASK_FULL:  # the masks are stored like the shares
        _check(mask_out, "mask_out", shares.dtype, numel=P * D)
    z = 0
    _gpu().share_pss(P, D, n, k, t, prime, vb, _ptr(secrets), _ptr(matrix), mask_mode,
                     rng_words(rng_key), owner_base, _ptr(shares), _ptr(cnt),
                     _ptr(mask_out) if mask_out is not None else z, z, _stream())


# ---- ChaCha masks (rand-0.3 ChaChaRng streams; chacha_mask.hip) ---------------------------
def chacha_seeds(P: int, seed_words: int, rng_key: bytes, owner_base: int, device) -> torch.Tensor:
    """Fresh per-participant mask seeds [P][seed_words] from the round's CSPRNG."""
    if not 1 <= seed_words <= 8:
        raise ValueError("seed_words must be 1..8")
    seeds = torch.empty(P, seed_words, dtype=torch.int32, device=device)
    _gpu().chacha_seeds(P, seed_words, rng_words(rng_key), owner_base, _ptr(seeds), _stream())
    return seeds


def chacha_mask_apply(secrets: torch.Tensor, seeds: torch.Tensor, modulus: int,
                      err: torch.Tensor) -> torch.Tensor:
    """masked[p][e] = (secrets[p][e] + mask_p[e]) mod m, mask_p = the rand-0.3
    `gen_range(0, m)` stream of seed p (chacha.rs:29-45), exact under rejected draws."""
    P, D = secrets.shape
    _check(secrets, "secrets", torch.int32)
    _check(seeds, "seeds", torch.int32)
    if seeds.dim() != 2 or seeds.shape[0] != P or not 1 <= seeds.shape[1] <= 8:
        raise ValueError("seeds must be [P][1..8] words")
    _check(err, "err", torch.int32, numel=1)
    masked = torch.empty_like(secrets)
    scratch = torch.empty(_gpu().chacha_scratch_words(P, D), dtype=torch.int32, device=secrets.device)
    _gpu().chacha_mask_apply(P, D, modulus, seeds.shape[1], _ptr(seeds), _ptr(secrets),
                             _ptr(masked), _ptr(scratch), _ptr(err), _stream())
    return masked


def count(vals: torch.Tensor, cnt: torch.Tensor):
    M, L = vals.shape
    _check(vals, "vals", VALUE_DTYPES)
    _check(cnt, "cnt", torch.int32, numel=M * tiles(L))
    _gpu().count(M, L, value_bytes(vals.dtype), _ptr(vals), _ptr(cnt), _stream())


def chacha_mask_sum(seeds: torch.Tensor, D: int, modulus: int, out: torch.Tensor, err):
    """out[e] = sum_p mask_p[e] mod m over the seeds [P][w] (chacha.rs:56-77), exact
    under rejected draws."""
    P, w = seeds.shape
    _check(seeds, "seeds", torch.int32)
    _check(out, "out", torch.int32, numel=D)
    _check(err, "err", torch.int32, numel=1)
    dev = seeds.device
    groups = _gpu().chacha_sum_groups(P, D)
    part = torch.empty(groups, D, dtype=torch.int32, device=dev)
    scratch = torch.empty(_gpu().chacha_scratch_words(P, D), dtype=torch.int32, device=dev)
    fix = torch.empty(D, dtype=torch.int64, device=dev)
    _gpu().chacha_mask_sum(P, D, modulus, w, _ptr(seeds), _ptr(out), _ptr(part), groups,
                           _ptr(scratch), _ptr(fix), _ptr(err), _stream())


def segscan(data: torch.Tensor, totals: torch.Tensor | None, expect: int | None = None,
            err: torch.Tensor | None = None):
    """Exclusive scan of every row of `data` [M][T] in place; `totals` [M] gets the
    row sums. With `expect` and `err`, a row that does not sum to `expect` sets
    the malformed bit of the error word."""
    M, T = data.shape
    _check(data, "data", torch.int32)
    if totals is not None:
        _check(totals, "totals", torch.int32, numel=M)
    e = 0
    if expect is not None:
        _check(err, "err", torch.int32, numel=1)
        e = _ptr(err)
    _gpu().segscan(M, T, _ptr(data), _ptr(totals) if totals is not None else 0,
                   int(expect or 0) & 0xFFFFFFFF, e, _stream())


def encode_encrypt(vals, tile_off, keys, ct, stride, mac=None, max_code_bytes=5):
    """Varint-encode + encrypt the rows of `vals` into the arena. `mac` =
    (pows, pt_len, partials, K) fuses the Poly1305 of the middle chunks into the
    pass (`partials` zeroed); :func:`mac_edges` and :func:`mac_final` complete
    the tag. `max_code_bytes`: :func:`varint_max_len` of the values' modulus (the
    bound the arena's slots are sized by); 32-bit values of at most 3 / 4 bytes
    run with a smaller LDS tile and more workgroups per CU."""
    M, L = vals.shape
    _check(vals, "vals", VALUE_DTYPES)
    _check(tile_off, "tile_off", torch.int32, numel=M * tiles(L))
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    pows = pt_len = partials = 0
    K = 0
    if mac is not None:
        t_pows, t_len, t_part, K = mac
        _check(t_pows, "pows", torch.int32, min_numel=M * POW_WORDS)
        _check(t_len, "pt_len", torch.int32, numel=M)
        _check(t_part, "partials", torch.int32, numel=M * K * 8)
        pows, pt_len, partials = _ptr(t_pows), _ptr(t_len), _ptr(t_part)
    _gpu().encode_encrypt(M, L, value_bytes(vals.dtype), _ptr(vals), _ptr(tile_off), _ptr(keys),
                          _ptr(ct), stride, pows, pt_len, partials, K, int(max_code_bytes), _stream())


def poly_powers(M, keys, pows, full=True):
    """Per-message Poly1305 tables (chunk factors for the Horner lanes; weight
    digits, row factors and pad-bit prefixes for the matrix-core rows). `full` =
    False: the Horner factors only, which is all that messages of at most two
    chunks (no middle chunk) ever read."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_WORDS)
    _gpu().poly_powers(M, _ptr(keys), _ptr(pows), 1 if full else 0, _stream())


def poly_powers_short(M, keys, pows):
    """r^1 .. r^64 per message: the table of :func:`mac_short`."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_SHORT_WORDS)
    _gpu().poly_powers_short(M, _ptr(keys), _ptr(pows), _stream())


def mac_short(M, keys, pows, ct, stride, pt_len, verify, ok=None, err=None):
    """Poly1305 of every message in one pass, a wave per message (meant for messages
    of at most SHORT_MAX_CHUNKS chunks): writes the tag into the slot header, or
    with `verify` compares it (`ok` [M] optional; a mismatch raises the MAC bit of
    `err`). Reads the ciphertext, so it goes ahead of :func:`decrypt_count`."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_SHORT_WORDS)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    _check(err, "err", torch.int32, numel=1)
    if ok is not None:
        _check(ok, "ok", torch.int32, numel=M)
    _gpu().mac_short(M, _ptr(keys), _ptr(pows), _ptr(ct), stride, _ptr(pt_len), 1 if verify else 0,
                     _ptr(ok) if ok is not None else 0, _ptr(err), _stream())


def decrypt_count(M, K, keys, ct, stride, pt_len, term_cnt=None, sub_cnt=None):
    """In-place decryption plus varint terminator counts (per 16 KiB chunk and/or
    per 1 KiB sub-chunk), without any MAC work: the second half of opening short
    messages, after :func:`mac_short` has read the ciphertext."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    if term_cnt is None and sub_cnt is None:
        raise ValueError("decrypt_count needs term_cnt and/or sub_cnt")
    if term_cnt is not None:
        _check(term_cnt, "term_cnt", torch.int32, numel=M * K)
    if sub_cnt is not None:
        _check(sub_cnt, "sub_cnt", torch.int32, numel=M * K * SUB_PER_CHUNK)
    _gpu().decrypt_count(M, K, _ptr(keys), _ptr(ct), stride, _ptr(pt_len),
                         _ptr(term_cnt) if term_cnt is not None else 0,
                         _ptr(sub_cnt) if sub_cnt is not None else 0, _stream())


def mac_edges(M, K, keys, pows, ct, stride, pt_len, partials):
    """Poly1305 partials of every message's first and last chunk (Horner)."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_WORDS)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    _check(partials, "partials", torch.int32, numel=M * K * 8)
    _gpu().mac_edges(M, K, _ptr(keys), _ptr(pows), _ptr(ct), stride, _ptr(pt_len), _ptr(partials),
                     _stream())


def mac_chunks(M, K, keys, pows, ct, stride, pt_len, partials, decrypt, term_cnt=None,
               sub_cnt=None):
    """Poly1305 chunk partials; with `decrypt`, in-place decryption plus varint
    terminator counts per 16 KiB chunk (`term_cnt` [M][K]) and/or per 1 KiB
    sub-chunk (`sub_cnt` [M][K * SUB_PER_CHUNK])."""
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_WORDS)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    _check(partials, "partials", torch.int32, numel=M * K * 8)
    if decrypt:
        if term_cnt is None and sub_cnt is None:
            raise ValueError("decrypt needs term_cnt and/or sub_cnt")
        if term_cnt is not None:
            _check(term_cnt, "term_cnt", torch.int32, numel=M * K)
        if sub_cnt is not None:
            _check(sub_cnt, "sub_cnt", torch.int32, numel=M * K * SUB_PER_CHUNK)
    _gpu().mac_chunks(M, K, _ptr(keys), _ptr(pows), _ptr(ct), stride, _ptr(pt_len), _ptr(partials),
                      1 if decrypt else 0, _ptr(term_cnt) if term_cnt is not None else 0,
                      _ptr(sub_cnt) if sub_cnt is not None else 0, _stream())


def mac_final(M, K, keys, pows, ct, stride, pt_len, partials, verify, ok=None, err=None):
    _check(keys, "keys", torch.uint8, min_numel=M * MSGKEY_BYTES)
    _check(pows, "pows", torch.int32, min_numel=M * POW_WORDS)
    _check(ct, "ct", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    _check(partials, "partials", torch.int32, numel=M * K * 8)
    _check(err, "err", torch.int32, numel=1)
    if ok is not None:
        _check(ok, "ok", torch.int32, numel=M)
    _gpu().mac_final(M, K, _ptr(keys), _ptr(pows), _ptr(ct), stride, _ptr(pt_len), _ptr(partials),
                     1 if verify else 0, _ptr(ok) if ok is not None else 0, _ptr(err), _stream())


def decode(M, K, L, modulus, pt, stride, pt_len, elem_start, vals, err):
    _check(vals, "vals", (torch.int16, torch.int32), numel=M * L)
    _check(elem_start, "elem_start", torch.int32, numel=M * K)
    _check(pt, "pt", torch.uint8, min_numel=M * stride)
    _gpu().decode(M, K, L, modulus, value_bytes(vals.dtype), _ptr(pt), stride, _ptr(pt_len),
                  _ptr(elem_start), _ptr(vals), _ptr(err), _stream())


def sum_tiles(L: int) -> int:
    return (L + SUM_TILE - 1) // SUM_TILE


def locate_tiles(pre: torch.Tensor, totals: torch.Tensor, L: int, tile_sub: torch.Tensor):
    """tile_sub[j][t] = the sub-chunk holding the terminator of element t*SUM_TILE
    of message j (end sentinel S past the message), from the exclusive
    sub-chunk ranks `pre` [M][S]."""
    M, S = pre.shape
    _check(pre, "pre", torch.int32)
    _check(totals, "totals", torch.int32, numel=M)
    _check(tile_sub, "tile_sub", torch.int32, numel=M * (sum_tiles(L) + 1))
    _gpu().locate_tiles(M, S, L, _ptr(pre), _ptr(totals), _ptr(tile_sub), _stream())


def decode_sum_wide(modulus: int) -> bool:
    """Moduli above 2^27 are summed in 64-bit accumulators (two words per slab entry)."""
    return modulus > 1 << 27


def decode_sum_group_limit(modulus: int) -> int:
    """Most participants one decode-sum accumulator may add up. u32 accumulators hold
    sums of zigzag codes of up to 14 bits (m <= 2^13: two-byte varints), 21 bits
    (2 (m - 1) < 2^21: three bytes) or 28 bits (m <= 2^27: four bytes); above that the
    accumulators are 64 bits wide and any group fits."""
    if decode_sum_wide(modulus):
        return 1 << 30
    if modulus <= 8192:
        per = 16383
    else:  # a longer code than the field's raises the fallback
        per = (1 << 21) - 1 if 2 * (modulus - 1) < 1 << 21 else (1 << 28) - 1
    return max(1, (2 ** 32 - 1) // max(1, per))


def decode_sum(rows: int, P: int, Pg: int, L: int, modulus: int, pt, stride, pt_len, pre,
               tile_sub, part, out, err, redo=None, acc=None):
    """out[r] = sum_p decode(message r*P + p) mod m (fused decode + combine); with
    `acc` (int64 [rows][L]) the sums are added to it instead and `out` may be None.

    `redo`: a zeroed int32 scratch word enabling the lean kernels (m <= 2^27)."""
    M = rows * P
    S = pre.shape[1]
    if modulus <= 0:
        raise ValueError("decode_sum needs a modulus")
    if Pg < 1 or Pg > decode_sum_group_limit(modulus):
        raise ValueError("decode_sum: the group's sums must fit the accumulators")
    if redo is not None:
        _check(redo, "redo", torch.int32, numel=1)
    groups = (P + Pg - 1) // Pg
    _check(pt, "pt", torch.uint8, min_numel=M * stride)
    _check(pt_len, "pt_len", torch.int32, numel=M)
    _check(pre, "pre", torch.int32, numel=M * S)
    _check(tile_sub, "tile_sub", torch.int32, numel=M * (sum_tiles(L) + 1))
    _check(part, "part", torch.int32, numel=groups * rows * L * (2 if decode_sum_wide(modulus) else 1))
    if acc is not None:
        _check(acc, "acc", torch.int64, numel=rows * L)
    else:
        _check(out, "out", torch.int32, numel=rows * L)
    _check(err, "err", torch.int32, numel=1)
    _gpu().decode_sum(rows, P, Pg, L, modulus, _ptr(pt), stride, _ptr(pt_len), S, _ptr(pre),
                      _ptr(tile_sub), _ptr(part), _ptr(out) if acc is None else 0,
                      _ptr(acc) if acc is not None else 0, _ptr(err),
                      _ptr(redo) if redo is not None else 0, _stream())


def colsum(vals: torch.Tensor, modulus: int, out: torch.Tensor):
    """out[g][l] = sum_r vals[g][r][l] mod m for vals [G][R][L]."""
    G, R, L = vals.shape
    _check(vals, "vals", (torch.int16, torch.int32))
    _check(out, "out", torch.int32, numel=G * L)
    _gpu().colsum(G, R, L, modulus, value_bytes(vals.dtype), _ptr(vals), _ptr(out), _stream())


def pss_reconstruct(ys: torch.Tensor, lag: torch.Tensor, k: int, D: int, prime: int,
                    out: torch.Tensor):
    nI, B = ys.shape
    _check(ys, "ys", torch.int32)
    _check(lag, "lag", torch.int32, numel=k * nI)
    _check(out, "out", torch.int32, numel=D)
    if B * k < D:
        raise ValueError("not enough batches for the dimension")
    _gpu().pss_reconstruct(B, k, nI, D, prime, _ptr(lag), _ptr(ys), _ptr(out), _stream())


def sub_mod(a: torch.Tensor, b: torch.Tensor, modulus: int, out: torch.Tensor):
    _check(a, "a", torch.int32)
    _check(b, "b", torch.int32, numel=a.numel())
    _check(out, "out", torch.int32, numel=a.numel())
    _gpu().sub_mod(a.numel(), modulus, _ptr(a), _ptr(b), _ptr(out), _stream())


# ---- packed Shamir on the matrix cores (int8 limbs; modgemm.hip) ----------------
def padded_k(K: int) -> int:
    return (K + 63) // 64 * 64


def limb_scheme(prime: int, Kp: int) -> tuple[int, int]:
    """(limbs, bits) of the GEMM operands for this field and (padded) K: 7-bit non-negative
    digits (3 limbs for p < 2^21, 4 for p < 2^28) or, for 2^21 <= p < 2^24 - 2^18 and
    K <= 4096, three signed base-256 digits of the balanced residue."""
    if not 2 <= prime < 2 ** 28:
        raise ValueError("modgemm: modulus must be in [2, 2^28)")
    return tuple(_gpu().limb_scheme(prime, Kp))


def limb_count(prime: int, Kp: int) -> int:
    return limb_scheme(prime, Kp)[0]


def limbs_of(values: torch.Tensor, Kp: int, prime: int) -> torch.Tensor:
    """Limb planes [L][rows][Kp] (int8) of a [rows][K] matrix of canonical field elements,
    in limb_scheme(prime, Kp)."""
    if prime < 16:
        raise ValueError("limbs_of takes the modulus (the limb count follows from it)")
    rows, K = values.shape
    limbs, bits = limb_scheme(prime, Kp)
    v = values.to(torch.int64)
    out = torch.zeros(limbs, rows, Kp, dtype=torch.int8, device=values.device)
    if bits == 7:
        for l in range(limbs):
            out[l, :, :K] = ((v >> (7 * l)) & 0x7F).to(torch.int8)
        return out
    v = torch.where(v > prime // 2, v - prime, v)  # balanced residue
    for l in range(limbs - 1):
        d = ((v & 0xFF) ^ 0x80) - 0x80  # low byte as int8
        out[l, :, :K] = d.to(torch.int8)
        v = (v - d) >> 8
    out[limbs - 1, :, :K] = v.to(torch.int8)
    return out


PANEL_MAX_K = 256  # the panel-resident GEMM kernel's longest (padded) K


def a_fragments(A_limbs: torch.Tensor) -> torch.Tensor:
    """A limbs [L][M][Kp] in the order the panel-resident GEMM kernel's waves load them
    (rows padded to a multiple of 64): pass as `a_frag` to :func:`modgemm_i8`."""
    _check(A_limbs, "A_limbs", torch.int8)
    L, M, Kp = A_limbs.shape
    out = torch.empty(_gpu().a_fragments_bytes(M, Kp, L), dtype=torch.int8, device=A_limbs.device)
    _gpu().a_fragments(M, Kp, L, _ptr(A_limbs), _ptr(out), _stream())
    return out


def modgemm_i8(A_limbs: torch.Tensor, B_limbs: torch.Tensor, prime: int, out: torch.Tensor,
               ldc_z: int, ldc_m: int, ldc_n: int, limit: int, cnt: torch.Tensor | None = None,
               a_frag: torch.Tensor | None = None):
    """out[z*ldc_z + m*ldc_m + n*ldc_n] = (A . B_z)[m][n] mod prime (A [L][M][Kp], B [L][Z][N][Kp]).

    `a_frag`: :func:`a_fragments` of A_limbs (made here when K is short and it is not
    given -- a caller that reuses A keeps it): the panel-resident kernel needs it.

    `cnt` (int32 [M * Z * tiles(N)], zeroed): the epilogue also adds up the varint
    bytes of what it writes, per (row m, batch z, 4096-column tile) -- :func:`count`
    of the output taken as M x Z messages of N values, without the extra pass."""
    _check(A_limbs, "A_limbs", torch.int8)
    _check(B_limbs, "B_limbs", torch.int8)
    L, M, Kp = A_limbs.shape
    Lb, Z, N, Kb = B_limbs.shape
    if Kb != Kp or Lb != L or L != limb_count(prime, Kp):
        raise ValueError("limb shape mismatch")
    vb = value_bytes(out.dtype)
    if out.dtype == torch.uint8 and prime > 256:
        raise ValueError("u8 output needs a prime <= 256")
    max_idx = (Z - 1) * ldc_z + (M - 1) * ldc_m + (N - 1) * ldc_n
    if min(limit, max_idx + 1) > out.numel():
        raise ValueError("output too small for the GEMM index map")
    if cnt is not None:
        _check(cnt, "cnt", torch.int32)
        if cnt.numel() < M * Z * tiles(N):
            raise ValueError("cnt too small")
    if a_frag is None and Kp <= PANEL_MAX_K:
        a_frag = a_fragments(A_limbs)
    if a_frag is not None:
        _check(a_frag, "a_frag", torch.int8)
        if a_frag.numel() != _gpu().a_fragments_bytes(M, Kp, L):
            raise ValueError("a_frag does not belong to A_limbs")
    _gpu().modgemm_i8(M, N, Kp, Z, L, prime, _ptr(A_limbs), 0 if a_frag is None else _ptr(a_frag),
                      _ptr(B_limbs), Z * N * Kp, vb,
                      _ptr(out), ldc_z, ldc_m, ldc_n, limit, 0 if cnt is None else _ptr(cnt),
                      _stream())


def pss_x_limbs(secrets: torch.Tensor, k: int, t: int, prime: int, rng_key: bytes,
                owner_base: int) -> torch.Tensor:
    P, D = secrets.shape
    _check(secrets, "secrets", torch.int32)
    B = (D + k - 1) // k
    Kp = padded_k(k + t)
    L = limb_count(prime, Kp)
    X = torch.empty(L, P, B, Kp, dtype=torch.int8, device=secrets.device)
    _gpu().pss_x_limbs(P, D, B, k, t, Kp, prime, _ptr(secrets), rng_words(rng_key), owner_base,
                       _ptr(X), _stream())
    return X


def limbs_t(Y: torch.Tensor, Kp: int, prime: int) -> torch.Tensor:
    """Limbs of Y [R][N] (int32 canonical field elements) transposed to [L][1][N][Kp]."""
    if prime < 16:
        raise ValueError("limbs_t takes the modulus (the limb count follows from it)")
    R, N = Y.shape
    _check(Y, "Y", torch.int32)
    out = torch.empty(limb_count(prime, Kp), 1, N, Kp, dtype=torch.int8, device=Y.device)
    _gpu().limbs_t(R, N, Kp, prime, _ptr(Y), _ptr(out), _stream())
    return out
