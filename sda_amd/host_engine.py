"""Host (CPU) aggregation engine: the reference dataflow on the C++ client engines.

Same round semantics and `run_round` interface as the device engine
(:class:`sda_amd.engine.DeviceAggregator`), but every step is the per-participant
client code path of the reference (client/src/participate.rs:37-113,
clerk.rs:63-107, receive.rs:80-157) executed by the C++ core: OS-RNG masks and
shares, zigzag varints, one sealed box per (participant, clerk). It is the
correctness oracle for the device engine, the CPU backend of
:class:`sda_amd.parallel.DistributedAggregator` (gloo tests), and the
reference-equivalent baseline.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import control as C
from ._native import native
from .models.schemes import AggregationSpec, PackedShamir


@dataclass
class HostKeys:
    """X25519 keypairs as raw bytes: index 0..n-1 = clerks, index n = recipient."""

    pks: list
    sks: list

    @classmethod
    def generate(cls, count: int) -> "HostKeys":
        pairs = [native().crypto.box_keypair() for _ in range(count)]
        return cls([p for p, _ in pairs], [s for _, s in pairs])

    def ek(self, i: int) -> str:
        return json.dumps(C.sodium(self.pks[i]))

    def keypair(self, i: int) -> str:
        return json.dumps({"ek": C.sodium(self.pks[i]), "dk": C.sodium(self.sks[i])})


@dataclass
class HostRoundResult:
    output: Optional[np.ndarray]
    clerks_used: list
    stage_ms: dict = field(default_factory=dict)


class HostAggregator:
    def __init__(self, spec: AggregationSpec, keys: HostKeys | None = None):
        self.spec = spec
        self.n = spec.n_clerks
        self.m = spec.field_modulus
        self.keys = keys or HostKeys.generate(self.n + 1)
        self._mask = json.dumps(spec.masking.to_wire())
        self._share = json.dumps(spec.sharing.to_wire())
        self._c = native().control

    def run_round(self, secrets, clerks: Sequence[int] | None = None, check: bool = True,
                  reducer=None, owner_base: int = 0, router=None) -> HostRoundResult:
        spec, n, m, c = self.spec, self.n, self.m, self._c
        secrets = np.asarray(secrets, dtype=np.int64)
        if secrets.ndim != 2 or secrets.shape[1] != spec.dimension:
            raise ValueError("secrets must be [P][dimension]")
        P, D = secrets.shape
        B = spec.batches
        live = list(range(n)) if clerks is None else sorted(set(int(x) for x in clerks))
        if len(live) < spec.sharing.reconstruction_threshold():
            raise C.errors.SdaError("Not enough shares to reconstruct")
        t = {"start": time.perf_counter()}

        # participants (participate.rs:37-113)
        boxes = []        # [P][n] sealed share vectors
        mask_boxes = []   # [P] sealed masks for the recipient
        for p in range(P):
            mask, masked = c.mask_secrets(self._mask, secrets[p].tolist())
            shares = c.generate_shares(self._share, masked)
            boxes.append([c.encrypt_shares(self.keys.ek(j), shares[j]) for j in range(n)])
            if spec.masking.has_mask():
                mask_boxes.append(c.encrypt_shares(self.keys.ek(n), mask))
        t["participate"] = time.perf_counter()

        # clerks: open this device's participants' boxes and combine (clerk.rs:63-107)
        # snapshot transpose: P x n -> n x P (locally, or routed to the clerks' ranks)
        inbox = (router.exchange_host(boxes) if router is not None
                 else [[boxes[p][j] for p in range(P)] for j in range(n)])
        combined = np.zeros((len(live), B), dtype=np.int64)
        for i, j in enumerate(live):
            kp = self.keys.keypair(j)
            acc = np.zeros(B, dtype=np.int64)
            for box in inbox[j]:
                acc += np.asarray(c.decrypt_shares(kp, box), dtype=np.int64)
            combined[i] = np.remainder(acc, m)
        mask_sum = None
        if spec.masking.has_mask():
            rk = self.keys.keypair(n)
            masks = [c.decrypt_shares(rk, mb) for mb in mask_boxes]
            mask_sum = np.remainder(np.asarray(c.combine_masks(self._mask, masks), dtype=np.int64), m)
        t["clerk"] = time.perf_counter()

        if reducer is not None:
            rows = len(live) + (1 if mask_sum is not None else 0)
            partials = np.zeros((rows, max(B, D)), dtype=np.int64)
            partials[:len(live), :B] = combined
            if mask_sum is not None:
                partials[len(live), :D] = mask_sum
            reduced = reducer(partials)
            t["reduce"] = time.perf_counter()
            if reduced is None:
                return HostRoundResult(None, live, _ms(t))
            reduced = np.remainder(np.asarray(reduced, dtype=np.int64), m)
            combined = reduced[:len(live), :B]
            if mask_sum is not None:
                mask_sum = reduced[len(live), :D]

        # clerks seal results for the recipient; recipient reconstructs + unmasks
        rkp = self.keys.keypair(n)
        indexed = []
        for i, j in enumerate(live):
            box = c.encrypt_shares(self.keys.ek(n), combined[i].tolist())
            indexed.append((j, c.decrypt_shares(rkp, box)))
        if isinstance(spec.sharing, PackedShamir):
            out = c.reconstruct_secrets(self._share, D, indexed)
        else:
            out = np.remainder(np.sum([np.asarray(v, dtype=np.int64) for _, v in indexed], 0), m)
            out = out.tolist()
        if mask_sum is not None:
            out = c.unmask(self._mask, mask_sum.tolist(), out)
        t["reveal"] = time.perf_counter()
        return HostRoundResult(np.remainder(np.asarray(out, dtype=np.int64), m), live, _ms(t))


def _ms(t: dict) -> dict:
    keys = list(t)
    return {b: (t[b] - t[a]) * 1e3 for a, b in zip(keys, keys[1:])}
