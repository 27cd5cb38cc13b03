"""Device aggregation engine: one full SDA round on a single MI355X.

Simulates P participants, an n-clerk committee and the recipient with the
exact cryptographic dataflow of the reference protocol:

  participate  (client/src/participate.rs:37-113)
      mask -> share -> per-clerk sealed boxes (+ sealed mask for the recipient)
  snapshot     (server/src/snapshot.rs:4-47)
      transpose P x n -> n x P : free, shares are written clerk-major
  clerk        (client/src/clerk.rs:63-107)
      open P boxes -> combine (sum mod m) -> seal the result for the recipient
  reveal       (client/src/receive.rs:80-157)
      open n results -> reconstruct (sum / Lagrange, any >= t+k clerks) ->
      unmask (sum of masks / ChaCha seed expansion) -> output in [0, m)

Every stage is a HIP kernel (csrc/kernels). Keys are real X25519 keypairs; the
per-round randomness is a fresh 256-bit key from OS entropy driving counter-mode
ChaCha20 streams (one per participant and purpose).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from ._native import native
from .models.schemes import Additive, AggregationSpec, ChaChaMask, FullMask, PackedShamir
from .ops import gpu as G
from .ops.sealed import Arena, open_, seal


class AggregationError(RuntimeError):
    pass


def _words(b: bytes) -> list[int]:
    return [int.from_bytes(b[4 * i:4 * i + 4], "little", signed=True) for i in range(len(b) // 4)]


@dataclass
class KeyTable:
    """X25519 keypairs: index 0..n-1 = clerks, index n = recipient."""

    pks: torch.Tensor  # int32 [K][8]
    sks: torch.Tensor  # int32 [K][8]
    pk_bytes: list = field(default_factory=list)
    sk_bytes: list = field(default_factory=list)

    @classmethod
    def generate(cls, count: int, device) -> "KeyTable":
        c = native().crypto
        pairs = [c.box_keypair() for _ in range(count)]
        pk = [p for p, _ in pairs]
        sk = [s for _, s in pairs]
        pks = torch.tensor([_words(p) for p in pk], dtype=torch.int32, device=device)
        sks = torch.tensor([_words(s) for s in sk], dtype=torch.int32, device=device)
        return cls(pks, sks, pk, sk)


@dataclass
class RoundResult:
    output: torch.Tensor          # int32 [D], canonical in [0, m)
    clerks_used: list
    stage_ms: dict


class DeviceAggregator:
    """Runs complete aggregation rounds for one :class:`AggregationSpec`."""

    def __init__(self, spec: AggregationSpec, device=None, keys: KeyTable | None = None,
                 time_stages: bool = False):
        self.spec = spec
        self.device = torch.device(device or "cuda")
        self.n = spec.n_clerks
        self.m = spec.field_modulus
        self.keys = keys or KeyTable.generate(self.n + 1, self.device)
        self.vdtype = G.value_dtype(self.m)
        self.time_stages = time_stages
        self._round = 0
        if isinstance(spec.sharing, PackedShamir):
            p = spec.sharing.native()
            p.validate()
            self._pss = p
            self._share_matrix = torch.tensor(p.share_matrix(), dtype=torch.int64).to(
                torch.int32).to(self.device)
        else:
            self._pss = None

    # ------------------------------------------------------------ helpers ----
    def _key_idx(self, values: Sequence[int]) -> torch.Tensor:
        return torch.tensor(list(values), dtype=torch.int32, device=self.device)

    def _mark(self, marks, name):
        if self.time_stages:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append((name, ev))

    # ---------------------------------------------------------- the round ----
    def participate(self, secrets: torch.Tensor, rng_key: bytes, owner_base: int, err):
        """Participant side for a wave of participants -> (clerk arena, mask arena)."""
        spec, n, m = self.spec, self.n, self.m
        P, D = secrets.shape
        B = spec.batches
        T = G.tiles(B)
        dev = self.device
        shares = torch.empty(n, P, B, dtype=self.vdtype, device=dev)
        cnt = torch.empty(n * P * T, dtype=torch.int32, device=dev)
        mask_mode = G.MASK_NONE
        mask_out = mask_cnt = seeds = None
        seed_words = 0
        if isinstance(spec.masking, FullMask):
            mask_mode = G.MASK_FULL
            mask_out = torch.empty(P, D, dtype=torch.int32, device=dev)
            mask_cnt = torch.empty(P * G.tiles(D), dtype=torch.int32, device=dev)
        elif isinstance(spec.masking, ChaChaMask):
            mask_mode = G.MASK_CHACHA
            seed_words = spec.masking.seed_words
            seeds = torch.empty(P, seed_words, dtype=torch.int32, device=dev)
        if self._pss is None:
            G.share_additive(secrets, n, m, shares, cnt, mask_mode, rng_key, owner_base,
                             mask_out=mask_out, mask_cnt=mask_cnt, seeds=seeds,
                             seed_words=seed_words, err=err)
        else:
            ps = spec.sharing
            G.share_pss(secrets, n, ps.secret_count, ps.privacy_threshold_, m,
                        self._share_matrix, shares, cnt, mask_mode, rng_key, owner_base,
                        mask_out=mask_out, seeds=seeds, seed_words=seed_words, err=err)
            mask_cnt = None  # recounted by seal()
        # clerk-major messages: j = c * P + p
        key_idx = torch.arange(n, dtype=torch.int32, device=dev).repeat_interleave(P)
        clerk_arena = seal(shares.view(n * P, B), key_idx, self.keys.pks, rng_key,
                           owner_base * 64, err, m, cnt=cnt)
        mask_arena = None
        rkey = self._key_idx([n] * P)
        if mask_mode == G.MASK_FULL:
            mask_arena = seal(mask_out, rkey, self.keys.pks, rng_key, owner_base * 64 + n * P,
                              err, m, cnt=mask_cnt)
        elif mask_mode == G.MASK_CHACHA:
            mask_arena = seal(seeds, rkey, self.keys.pks, rng_key, owner_base * 64 + (n + 1) * P,
                              err, 0)
        return clerk_arena, mask_arena

    def clerk(self, clerk_arena: Arena, P: int, rng_key: bytes, owner_base: int, err,
              clerks: Sequence[int] | None = None) -> tuple[Arena, list]:
        """All clerks: open their P boxes, combine, seal the sums for the recipient."""
        n, m, B = self.n, self.m, self.spec.batches
        dev = self.device
        clerks = list(range(n)) if clerks is None else list(clerks)
        # jobs of the participating clerks (contiguous per clerk)
        if clerks == list(range(n)):
            arena = clerk_arena
        else:  # clerk dropout: only the live clerks' jobs are opened
            parts = [clerk_arena.slice(c * P, P) for c in clerks]
            arena = Arena(len(clerks) * P, B, m, clerk_arena.stride, clerk_arena.K,
                          torch.cat([a.ct for a in parts]), torch.cat([a.pt_len for a in parts]))
        key_idx = torch.tensor(clerks, dtype=torch.int32, device=dev).repeat_interleave(P)
        vals = open_(arena, key_idx, self.keys.sks, self.keys.pks, err, out_dtype=self.vdtype)
        combined = torch.empty(len(clerks), B, dtype=torch.int32, device=dev)
        G.colsum(vals.view(len(clerks), P, B), m, combined)
        res_vals = combined if self.vdtype == torch.int32 else combined.to(self.vdtype)
        rkey = self._key_idx([n] * len(clerks))
        res_arena = seal(res_vals, rkey, self.keys.pks, rng_key, owner_base, err, m)
        return res_arena, clerks

    def reveal(self, res_arena: Arena, clerks: list, mask_arena: Arena | None, P: int, err):
        spec, n, m, D, B = self.spec, self.n, self.m, self.spec.dimension, self.spec.batches
        dev = self.device
        rk = self._key_idx([n] * res_arena.M)
        ys = open_(res_arena, rk, self.keys.sks, self.keys.pks, err, out_dtype=torch.int32)
        masked = torch.empty(D, dtype=torch.int32, device=dev)
        if self._pss is None:
            if len(clerks) != n:
                raise AggregationError("additive sharing needs every clerk's result")
            G.colsum(ys.view(1, n, B), m, masked)
        else:
            if len(clerks) < spec.sharing.reconstruction_threshold():
                raise AggregationError("Not enough shares to reconstruct")
            lag = torch.tensor(self._pss.lagrange_matrix(clerks), dtype=torch.int64).to(
                torch.int32).to(dev)
            G.pss_reconstruct(ys, lag, spec.sharing.secret_count, D, m, masked)
        if mask_arena is None:
            return masked
        mask_sum = torch.empty(D, dtype=torch.int32, device=dev)
        rkey = self._key_idx([n] * mask_arena.M)
        if isinstance(spec.masking, FullMask):
            masks = open_(mask_arena, rkey, self.keys.sks, self.keys.pks, err,
                          out_dtype=torch.int32)
            G.colsum(masks.view(1, P, D), m, mask_sum)
        else:
            seeds = open_(mask_arena, rkey, self.keys.sks, self.keys.pks, err,
                          out_dtype=torch.int32)
            G.chacha_mask_sum(seeds, D, m, mask_sum, err)
        out = torch.empty(D, dtype=torch.int32, device=dev)
        G.sub_mod(masked, mask_sum, m, out)
        return out

    def run_round(self, secrets: torch.Tensor, clerks: Sequence[int] | None = None,
                  check: bool = True) -> RoundResult:
        """One full round for participant vectors `secrets` [P][D] (int32, on device)."""
        if secrets.dim() != 2 or secrets.shape[1] != self.spec.dimension:
            raise ValueError("secrets must be [P][dimension]")
        if secrets.dtype != torch.int32 or secrets.device.type != "cuda":
            raise ValueError("secrets must be an int32 GPU tensor")
        secrets = secrets.contiguous()
        P = secrets.shape[0]
        rng_key = native().crypto.random_bytes(32)
        self._round += 1
        err = torch.zeros(1, dtype=torch.int32, device=self.device)
        marks: list = []
        self._mark(marks, "start")
        clerk_arena, mask_arena = self.participate(secrets, rng_key, 0, err)
        self._mark(marks, "participate")
        res_arena, used = self.clerk(clerk_arena, P, rng_key, 1 << 48, err, clerks)
        self._mark(marks, "clerk")
        out = self.reveal(res_arena, used, mask_arena, P, err)
        self._mark(marks, "reveal")
        stage_ms = {}
        if check or self.time_stages:
            e = int(err.item())
            if e:
                raise AggregationError(f"device error word 0x{e:x} ({describe_error(e)})")
            for (a, ea), (b, eb) in zip(marks, marks[1:]):
                stage_ms[b] = ea.elapsed_time(eb)
        return RoundResult(out, used, stage_ms)


def describe_error(e: int) -> str:
    names = []
    if e & 1:
        names.append("bad public key")
    if e & 2:
        names.append("MAC verification failed")
    if e & 4:
        names.append("malformed varint stream")
    if e & 8:
        names.append("ChaCha mask rejection (host fallback needed)")
    if e & 16:
        names.append("value out of range")
    return ", ".join(names) or "none"


def reference_sum(secrets: torch.Tensor, modulus: int) -> torch.Tensor:
    """Plain PyTorch int64 reference: sum over participants mod m in [0, m)."""
    return torch.remainder(secrets.to(torch.int64).sum(0), modulus).to(torch.int32)
