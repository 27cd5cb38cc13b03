"""Participant-wave streaming with accumulator checkpoints.

Rounds too large to be resident -- the largest benchmark configuration is 10k participants x
125M dimensions, i.e. 5 TB of inputs and ~13 TB of packed-Shamir shares -- run
as waves of W participants through the device engine's participate+clerk
phase. Only the clerks' running sums (n x B) and the recipient's mask sum (D)
persist between waves; each wave's shares, arenas and decoded values are
recycled. The running sums are checkpointed every few waves so a stopped
run resumes where it stopped (the reference's durability is its
stores; on the GPU path it is these accumulators).

In a multi-GPU round each rank streams its own participant range, every wave's
sealed boxes travel to the clerks' ranks, and the clerks' sealed results go to
the recipient's rank once, at the end.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import torch

from .engine import AggregationError, DeviceAggregator, describe_error


@dataclass
class StreamResult:
    output: Optional[torch.Tensor]
    clerks_used: list
    waves: int
    resumed_from: int = 0
    stage_ms: dict = field(default_factory=dict)


class StreamingAggregator:
    def __init__(self, engine: DeviceAggregator, wave: int = 64,
                 checkpoint: Optional[str] = None, checkpoint_every: int = 8):
        if wave <= 0:
            raise ValueError("wave must be positive")
        self.engine = engine
        self.wave = wave
        self.checkpoint = checkpoint
        self.every = max(1, checkpoint_every)

    # ---- checkpoints ---------------------------------------------------------
    def _fingerprint(self, total: int, live, rows) -> str:
        spec = self.engine.spec
        return json.dumps({"dimension": spec.dimension, "modulus": spec.field_modulus,
                           "sharing": spec.sharing.to_wire(), "masking": spec.masking.to_wire(),
                           "participants": total, "wave": self.wave, "live": list(live),
                           "rows": list(rows)}, sort_keys=True)

    def _save(self, acc, mask_acc, next_wave: int, fp: str):
        from safetensors.torch import save_file

        tensors = {"acc": acc.cpu().contiguous()}
        if mask_acc is not None:
            tensors["mask"] = mask_acc.cpu().contiguous()
        tmp = self.checkpoint + ".tmp"
        save_file(tensors, tmp, metadata={"fingerprint": fp, "next_wave": str(next_wave)})
        os.replace(tmp, self.checkpoint)  # atomic: a crash leaves the previous checkpoint

    def _load(self, fp: str):
        if not self.checkpoint or not os.path.exists(self.checkpoint):
            return None
        from safetensors import safe_open

        with safe_open(self.checkpoint, framework="pt") as f:
            meta = f.metadata() or {}
            if meta.get("fingerprint") != fp:
                raise AggregationError("checkpoint belongs to a different aggregation")
            acc = f.get_tensor("acc")
            mask = f.get_tensor("mask") if "mask" in f.keys() else None
        return acc, mask, int(meta["next_wave"])

    # ---- the round -------------------------------------------------------------
    def run(self, total: int, make_wave: Callable[[int, int, int], torch.Tensor],
            clerks: Optional[Sequence[int]] = None, reducer=None, committee=None,
            owner_base: int = 0, resume: bool = True, stop_after: Optional[int] = None,
            check: bool = True) -> StreamResult:
        """Aggregate `total` participants delivered by ``make_wave(w, first, count)``.

        Multi-GPU: `committee` (a :class:`sda_amd.parallel.device_round.DeviceCommittee`)
        routes every wave's boxes to the clerks' ranks and gathers the sealed
        results at the end; `reducer` is the ``owner`` layout's plaintext
        reduce. This rank's running sums -- one row per clerk it accumulates
        for, plus on the recipient's rank the mask sum -- are what the
        checkpoints hold. `stop_after` ends the run after that many waves of
        this call (checkpoint kept) -- used to exercise resume.
        """
        eng = self.engine
        live = eng._live(clerks)
        B, D, dev = eng.spec.batches, eng.spec.dimension, eng.device
        waves = (total + self.wave - 1) // self.wave
        # accumulator rows: the live clerks (one GPU / owner) or this rank's hosted ones
        rows = list(live) if committee is None else [c for c in committee.hosted if c in live]
        fp = self._fingerprint(total, live, rows)
        acc = torch.zeros(len(rows), B, dtype=torch.int64, device=dev)
        has_mask = eng.spec.masking.has_mask()
        keeps_mask = has_mask and (committee is None or committee.comm.rank == committee.ROOT)
        mask_acc = torch.zeros(D, dtype=torch.int64, device=dev) if keeps_mask else None
        start = 0
        if resume:
            state = self._load(fp)
            if state is not None:
                acc.copy_(state[0])
                if mask_acc is not None:
                    mask_acc.copy_(state[1])
                start = state[2]
        err = eng.new_error_word()
        marks: list = []
        eng._mark(marks, "start")
        ctx = None
        rk = None  # recipient / result key agreement: queued behind the first wave's
        done = 0
        for w in range(start, waves):
            first = w * self.wave
            count = min(self.wave, total - first)
            x = make_wave(w, first, count)
            if committee is not None:
                part, mask_arena = committee.participate_exchange_clerk(
                    x, live, err, owner_base=owner_base + first)
                if ctx is None:
                    ctx = committee.begin(live, err)
                    ctx.mask_acc = mask_acc
                committee.ship_masks(ctx, mask_arena, err)
                for i, c in enumerate(rows):  # `part`: one row per clerk, this rank's are non-zero
                    acc[i] += part[c]
                mask_acc = ctx.mask_acc
            else:
                comb, msum = eng.participate_and_clerk(x, live, err, owner_base=owner_base + first)
                if rk is None:
                    rk = eng.prepare_reveal(live, err)
                acc += comb
                if mask_acc is not None:
                    mask_acc += msum
            done += 1
            eng.throttle()  # the host stays at most two waves ahead of the GPU
            last = w == waves - 1
            if self.checkpoint and ((w + 1) % self.every == 0 or last or
                                    (stop_after is not None and done >= stop_after)):
                self._check(err)  # never checkpoint state built on a failed wave
                self._save(acc, mask_acc, w + 1, fp)
            if stop_after is not None and done >= stop_after and not last:
                return StreamResult(None, live, done, start)
        eng._mark(marks, "waves")
        m = eng.m
        if committee is not None:
            if ctx is None:  # resumed past the last wave
                ctx = committee.begin(live, err)
                ctx.mask_acc = mask_acc
            full = torch.zeros(eng.n, B, dtype=torch.int64, device=dev)
            for i, c in enumerate(rows):
                full[c] = acc[i]
            out, used = committee.finish(ctx, full, err, marks)
            if check:
                self._check(err)
            res = StreamResult(out, used, done, start)
        else:
            combined = torch.remainder(acc, m).to(torch.int32)
            mask_sum = torch.remainder(mask_acc, m).to(torch.int32) if mask_acc is not None else None
            if reducer is not None:
                combined, mask_sum = eng.reduce_partials(combined, mask_sum, reducer, marks)
                if combined is None:
                    self._check(err)
                    return StreamResult(None, live, done, start)
            out = eng.reveal(combined, mask_sum, live, err, marks=marks, keys=rk)
            if check:
                self._check(err)
            res = StreamResult(out, live, done, start)
        if eng.time_stages:
            torch.cuda.synchronize()
            for (a, ea), (b, eb) in zip(marks, marks[1:]):
                res.stage_ms[b] = ea.elapsed_time(eb)
        return res

    @staticmethod
    def _check(err):
        e = int(err.item())
        if e:
            raise AggregationError(f"device error word 0x{e:x} ({describe_error(e)})")
