"""Host (CPU) aggregation engine: the reference dataflow on the C++ client engines.

Same round semantics as the device engine
(:class:`sda_amd.engine.DeviceAggregator`), but every step is the per-participant
client code path of the reference (client/src/participate.rs:37-113,
clerk.rs:63-107, receive.rs:80-157) executed by the C++ core: OS-RNG masks and
shares, zigzag varints, one sealed box per (participant, clerk). It is the
correctness oracle for the device engine, the CPU backend of
:class:`sda_amd.parallel.DistributedAggregator` (gloo tests), and the
reference-equivalent baseline.

The round is exposed both whole (:meth:`HostAggregator.run_round`) and as the
role steps the distributed engine composes (``participate`` -> ``clerk_combine``
-> ``seal_result`` -> ``reveal``); a step that needs a secret key this process
does not hold raises.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import control as C
from ._native import native
from .models.schemes import AggregationSpec, PackedShamir


@dataclass
class HostKeys:
    """X25519 keypairs as raw bytes: index 0..n-1 = clerks, index n = recipient.
    ``sks[i]`` is None where this process does not hold the secret key."""

    pks: list
    sks: list

    @classmethod
    def generate(cls, count: int) -> "HostKeys":
        pairs = [native().crypto.box_keypair() for _ in range(count)]
        return cls([p for p, _ in pairs], [s for _, s in pairs])

    def ek(self, i: int) -> str:
        return json.dumps(C.sodium(self.pks[i]))

    def keypair(self, i: int) -> str:
        if self.sks[i] is None:
            raise PermissionError(f"this process does not hold the secret key of party {i}")
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

    # ---- role steps -----------------------------------------------------------
    def live(self, clerks: Sequence[int] | None) -> List[int]:
        live = list(range(self.n)) if clerks is None else sorted(set(int(x) for x in clerks))
        if len(live) < self.spec.sharing.reconstruction_threshold():
            raise C.errors.SdaError("Not enough shares to reconstruct")
        return live

    def participate(self, secrets) -> Tuple[list, Optional[list]]:
        """participate.rs:37-113 for every row of `secrets`: (boxes [P][n] sealed
        for the clerks, mask boxes [P] sealed for the recipient or None)."""
        spec, n, c = self.spec, self.n, self._c
        secrets = np.asarray(secrets, dtype=np.int64)
        if secrets.ndim != 2 or secrets.shape[1] != spec.dimension:
            raise ValueError("secrets must be [P][dimension]")
        boxes, mask_boxes = [], []
        for p in range(secrets.shape[0]):
            mask, masked = c.mask_secrets(self._mask, secrets[p].tolist())
            shares = c.generate_shares(self._share, masked)
            boxes.append([c.encrypt_shares(self.keys.ek(j), shares[j]) for j in range(n)])
            if spec.masking.has_mask():
                mask_boxes.append(c.encrypt_shares(self.keys.ek(n), mask))
        return boxes, (mask_boxes if spec.masking.has_mask() else None)

    def clerk_combine(self, clerk: int, boxes: Sequence[str]) -> np.ndarray:
        """clerk.rs:79-86: open the boxes sealed for `clerk` and sum mod m."""
        kp = self.keys.keypair(clerk)
        acc = np.zeros(self.spec.batches, dtype=np.int64)
        for box in boxes:
            acc += np.asarray(self._c.decrypt_shares(kp, box), dtype=np.int64)
        return np.remainder(acc, self.m)

    def seal_result(self, combined: np.ndarray) -> str:
        """clerk.rs:99-100: the clerk's combined shares sealed for the recipient."""
        return self._c.encrypt_shares(self.keys.ek(self.n), np.asarray(combined).tolist())

    def reveal(self, results: Sequence[Tuple[int, str]], mask_boxes: Optional[Sequence[str]]):
        """receive.rs:102-152: open the clerks' results (committee index, box),
        reconstruct, open + combine the masks, unmask."""
        spec, c, m, D = self.spec, self._c, self.m, self.spec.dimension
        rkp = self.keys.keypair(self.n)
        if len(results) < spec.sharing.reconstruction_threshold():
            raise C.errors.SdaError("Not enough shares to reconstruct")
        indexed = [(j, c.decrypt_shares(rkp, box)) for j, box in results]
        if isinstance(spec.sharing, PackedShamir):
            out = c.reconstruct_secrets(self._share, D, indexed)
        else:
            out = np.remainder(np.sum([np.asarray(v, dtype=np.int64) for _, v in indexed], 0), m)
            out = out.tolist()
        if spec.masking.has_mask():
            masks = [c.decrypt_shares(rkp, mb) for mb in mask_boxes]
            mask_sum = np.remainder(np.asarray(c.combine_masks(self._mask, masks), dtype=np.int64), m)
            out = c.unmask(self._mask, mask_sum.tolist(), out)
        return np.remainder(np.asarray(out, dtype=np.int64), m)

    # ---- the whole round in one process ------------------------------------------
    def run_round(self, secrets, clerks: Sequence[int] | None = None, check: bool = True,
                  reducer=None, owner_base: int = 0) -> HostRoundResult:
        """One round. `reducer(partials) -> reduced | None` (the ``owner``
        multi-process layout): sums the per-clerk partial sums and the mask
        partial over processes onto the root."""
        spec, n, m = self.spec, self.n, self.m
        live = self.live(clerks)
        t = {"start": time.perf_counter()}
        boxes, mask_boxes = self.participate(secrets)
        P, D, B = len(boxes), spec.dimension, spec.batches
        t["participate"] = time.perf_counter()
        # snapshot transpose (snapshot.rs:11-27): P x n -> n x P
        combined = np.stack([self.clerk_combine(j, [boxes[p][j] for p in range(P)]) for j in live])
        t["clerk"] = time.perf_counter()
        if reducer is None:
            results = [(j, self.seal_result(combined[i])) for i, j in enumerate(live)]
            out = self.reveal(results, mask_boxes)
            t["reveal"] = time.perf_counter()
            return HostRoundResult(out, live, _ms(t))

        # owner layout: plaintext partials are summed across processes
        c = self._c
        mask_sum = None
        if mask_boxes is not None:
            rk = self.keys.keypair(n)
            masks = [c.decrypt_shares(rk, mb) for mb in mask_boxes]
            mask_sum = np.remainder(np.asarray(c.combine_masks(self._mask, masks), dtype=np.int64), m)
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
        results = [(j, self.seal_result(reduced[i, :B])) for i, j in enumerate(live)]
        rkp = self.keys.keypair(n)
        indexed = [(j, c.decrypt_shares(rkp, box)) for j, box in results]
        if isinstance(spec.sharing, PackedShamir):
            out = c.reconstruct_secrets(self._share, D, indexed)
        else:
            out = np.remainder(np.sum([np.asarray(v, dtype=np.int64) for _, v in indexed], 0), m).tolist()
        if mask_sum is not None:
            out = c.unmask(self._mask, reduced[len(live), :D].tolist(), out)
        t["reveal"] = time.perf_counter()
        return HostRoundResult(np.remainder(np.asarray(out, dtype=np.int64), m), live, _ms(t))


def _ms(t: dict) -> dict:
    keys = list(t)
    return {b: (t[b] - t[a]) * 1e3 for a, b in zip(keys, keys[1:])}
