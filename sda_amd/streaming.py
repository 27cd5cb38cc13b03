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
import queue
import threading
import time
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
    err: Optional[torch.Tensor] = None   # the run's device error word (int32 [1])
    wave: int = 0                        # participants per wave
    plan: Optional[dict] = None          # the planner's account when it chose the wave
    checkpoint: Optional[dict] = None    # checkpoints written and what they cost the stream


class _CheckpointWriter:
    """Checkpoints off the wave loop: the running sums are copied to pinned host
    memory on a side stream (behind an event on the compute stream, so the GPU keeps
    working on the next wave), and a thread waits for the copy, checks the error
    word that travelled with it -- state built on a failed wave is never written --
    and writes the file. The wave loop only queues; it blocks when a third
    checkpoint is requested while two are still being written."""

    def __init__(self, path: str, device):
        self.path, self.device = path, device
        self.stream = torch.cuda.Stream(device=device)  # default priority
        self.free: "queue.Queue" = queue.Queue()
        self.jobs: "queue.Queue" = queue.Queue()
        self.failure: Optional[str] = None
        self.written = 0
        self.host_ms = 0.0      # time the wave loop spent queuing checkpoints
        self.write_ms = 0.0     # time the writer thread spent copying out + writing
        self._bufs = 0
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _buffers(self, acc, mask_acc):
        try:
            return self.free.get_nowait()
        except queue.Empty:
            if self._bufs >= 2:
                return self.free.get()  # both in use: wait for the writer
        self._bufs += 1
        return {"acc": torch.empty(acc.shape, dtype=acc.dtype, pin_memory=True),
                "mask": (torch.empty(mask_acc.shape, dtype=mask_acc.dtype, pin_memory=True)
                         if mask_acc is not None else None),
                "err": torch.empty(1, dtype=torch.int32, pin_memory=True)}

    def save(self, acc, mask_acc, err, next_wave: int, fingerprint: str):
        t0 = time.perf_counter()
        if self.failure:
            raise AggregationError(self.failure)
        buf = self._buffers(acc, mask_acc)
        main = torch.cuda.current_stream(self.device)
        # a snapshot on the device first: the next wave adds to `acc` while the copy runs
        snap = acc.clone()
        msnap = mask_acc.clone() if mask_acc is not None else None
        esnap = err.clone()
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            buf["acc"].copy_(snap, non_blocking=True)
            if msnap is not None:
                buf["mask"].copy_(msnap, non_blocking=True)
            buf["err"].copy_(esnap, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        for t in (snap, msnap, esnap):
            if t is not None:
                t.record_stream(self.stream)
        self.jobs.put((buf, done, next_wave, fingerprint))
        self.host_ms += (time.perf_counter() - t0) * 1e3

    def _run(self):
        from safetensors.torch import save_file

        while True:
            job = self.jobs.get()
            if job is None:
                return
            buf, done, next_wave, fp = job
            t0 = time.perf_counter()
            try:
                done.synchronize()
                e = int(buf["err"][0])
                if e:
                    self.failure = f"device error word 0x{e:x} ({describe_error(e)})"
                else:
                    tensors = {"acc": buf["acc"]}
                    if buf["mask"] is not None:
                        tensors["mask"] = buf["mask"]
                    tmp = self.path + ".tmp"
                    save_file(tensors, tmp, metadata={"fingerprint": fp, "next_wave": str(next_wave)})
                    os.replace(tmp, self.path)  # atomic: a crash leaves the previous checkpoint
                    self.written += 1
            except Exception as ex:  # noqa: BLE001 - reported on the wave loop
                self.failure = f"checkpoint writer: {type(ex).__name__}: {ex}"
            self.write_ms += (time.perf_counter() - t0) * 1e3
            self.free.put(buf)
            self.jobs.task_done()

    def close(self):
        """Wait for the queued checkpoints; raises what the writer met."""
        self.jobs.join()
        self.jobs.put(None)
        self.thread.join()
        if self.failure:
            raise AggregationError(self.failure)

    def report(self) -> dict:
        return {"written": self.written, "wave_loop_ms": self.host_ms, "writer_thread_ms": self.write_ms}


class StreamingAggregator:
    def __init__(self, engine: DeviceAggregator, wave: Optional[int] = None,
                 checkpoint: Optional[str] = None, checkpoint_every: int = 8):
        """`wave`: participants per wave; None = as many as the planner fits into the
        device's free memory (:mod:`sda_amd.planner`)."""
        if wave is not None and wave <= 0:
            raise ValueError("wave must be positive")
        self.engine = engine
        self.wave = wave
        self.plan = None
        self.checkpoint = checkpoint
        self.every = max(1, checkpoint_every)

    # ---- checkpoints ---------------------------------------------------------
    def _fingerprint(self, total: int, live, rows) -> str:
        spec = self.engine.spec
        return json.dumps({"dimension": spec.dimension, "modulus": spec.field_modulus,
                           "sharing": spec.sharing.to_wire(), "masking": spec.masking.to_wire(),
                           "participants": total, "wave": self.wave, "live": list(live),
                           "rows": list(rows)}, sort_keys=True)

    def _stored_wave(self) -> Optional[int]:
        if not self.checkpoint or not os.path.exists(self.checkpoint):
            return None
        from safetensors import safe_open

        with safe_open(self.checkpoint, framework="pt") as f:
            meta = f.metadata() or {}
        try:
            return int(json.loads(meta.get("fingerprint", "{}")).get("wave") or 0) or None
        except (ValueError, TypeError):
            return None

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
        if self.wave is None:
            stored = self._stored_wave() if resume else None
            if stored:
                self.wave = stored  # a resumed run keeps the wave size its checkpoint was cut at
            else:
                # waves are produced on the fly: each wave's input is priced in
                self.plan = eng.plan(total, input_resident=False)
                self.wave = self.plan.wave
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
        writer = _CheckpointWriter(self.checkpoint, dev) if self.checkpoint else None
        try:
            return self._waves(total, make_wave, live, rows, fp, acc, mask_acc, start, waves, err,
                               marks, ctx, rk, done, writer, reducer, committee, owner_base,
                               stop_after, check)
        finally:
            if writer is not None and writer.thread.is_alive():
                writer.jobs.put(None)  # an exception in the loop: let the thread go

    def _waves(self, total, make_wave, live, rows, fp, acc, mask_acc, start, waves, err, marks, ctx,
               rk, done, writer, reducer, committee, owner_base, stop_after, check):
        eng = self.engine
        B, D, dev = eng.spec.batches, eng.spec.dimension, eng.device

        def result(out, used):
            return StreamResult(out, used, done, start, err=err, wave=self.wave,
                                plan=self.plan.as_dict() if self.plan is not None else None,
                                checkpoint=writer.report() if writer is not None else None)

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
                for lo, hi in self._pieces(x.shape[0]):
                    comb, msum = self._wave_piece(x[lo:hi], live, err, owner_base + first + lo)
                    acc += comb
                    if mask_acc is not None:
                        mask_acc += msum
                if rk is None:
                    rk = eng.prepare_reveal(live, err)
            done += 1
            eng.throttle()  # the host stays at most two waves ahead of the GPU
            last = w == waves - 1
            if writer is not None and ((w + 1) % self.every == 0 or last or
                                       (stop_after is not None and done >= stop_after)):
                # queued, not waited for: the error word travels with the snapshot and
                # the writer drops a checkpoint built on a failed wave
                writer.save(acc, mask_acc, err, w + 1, fp)
            if stop_after is not None and done >= stop_after and not last:
                if writer is not None:
                    writer.close()
                return result(None, live)
        eng._mark(marks, "waves")
        if writer is not None:
            writer.close()
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
            res = result(out, used)
        else:
            combined = torch.remainder(acc, m).to(torch.int32)
            mask_sum = torch.remainder(mask_acc, m).to(torch.int32) if mask_acc is not None else None
            if reducer is not None:
                combined, mask_sum = eng.reduce_partials(combined, mask_sum, reducer, marks)
                if combined is None:
                    if check:
                        self._check(err)
                    return result(None, live)
            out = eng.reveal(combined, mask_sum, live, err, marks=marks, keys=rk)
            if check:
                self._check(err)
            res = result(out, live)
        if eng.time_stages:
            torch.cuda.synchronize()
            for (a, ea), (b, eb) in zip(marks, marks[1:]):
                res.stage_ms[b] = ea.elapsed_time(eb)
        return res

    def _pieces(self, count: int):
        """Participant ranges a wave is run in: one, unless an earlier wave ran out of
        memory and was cut (`_split`)."""
        parts = getattr(self, "_split", 1)
        return [(count * i // parts, count * (i + 1) // parts) for i in range(parts)
                if count * (i + 1) // parts > count * i // parts]

    def _wave_piece(self, x, live, err, owner_base):
        """participate + clerk for one piece; a piece that does not fit (the planner's
        byte model is an estimate) is retried in halves, and later waves start cut."""
        eng = self.engine
        try:
            return eng.participate_and_clerk(x, live, err, owner_base=owner_base)
        except torch.cuda.OutOfMemoryError:
            if x.shape[0] < 2:
                raise
            torch.cuda.synchronize(eng.device)
            torch.cuda.empty_cache()
            self._split = getattr(self, "_split", 1) * 2
            h = x.shape[0] // 2
            c1, m1 = self._wave_piece(x[:h], live, err, owner_base)
            c2, m2 = self._wave_piece(x[h:], live, err, owner_base + h)
            return c1 + c2, (m1 + m2 if m1 is not None else None)

    @staticmethod
    def _check(err):
        e = int(err.item())
        if e:
            raise AggregationError(f"device error word 0x{e:x} ({describe_error(e)})")
