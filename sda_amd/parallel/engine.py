"""Distributed aggregation: one process per GPU, torch.distributed over RCCL/xGMI.

``committee`` (default, the protocol's trust model). Every rank owns a shard
of the participants and seals their boxes for every clerk. The snapshot
transpose (server/src/snapshot.rs:4-47) is a uniform all-to-all of sealed boxes
over xGMI (parallel/routing.py): rank r plays the clerks of its piece of the
clerk axis and holds *only their* secret keys; with at least as many ranks as
clerks no rank ever sees two clerks' shares of one participant. A clerk that
spans several ranks sums its hosts' partial sums on its lead rank -- plaintext
partials never leave the clerk's own ranks -- and the lead seals the combined
shares for the recipient (client/src/clerk.rs:99-100). Rank 0, the only holder
of the recipient key, gathers the sealed results that arrive before the
deadline, reconstructs from any >= t + k of them (server/src/server.rs:119-120,
client/src/receive.rs:127-144), opens the participants' mask boxes and unmasks.

``owner`` (an explicit, *non-private upper bound*): every rank runs its
participants' whole pipeline locally, including the clerks' open + combine of
its own boxes, and the plaintext per-clerk partial sums are summed onto rank 0
with one RCCL reduce. Every rank holds every key. Sealed boxes never cross
xGMI; it measures what the all-to-all costs, it is not the protocol.

Failure model (committee): a clerk rank that dies after the exchange simply
never posts its result flag; the recipient proceeds at the deadline with the
results it has, or raises "Not enough clerk results" below the reconstruction
threshold. Collectives carry the process group's timeout, so a rank that loses
a peer mid-transfer exits non-zero instead of hanging.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from ..models.schemes import AggregationSpec
from .comm import Comm
from .router import RowRouter, gather_rows_to
from .liveness import partial_stage, result_stage
from .routing import hosted_clerks, hosts, lead, plan

ROOT = 0


def _owner_base(rank: int) -> int:
    # RNG stream ids are purpose<<56 | owner: give every rank a disjoint owner range
    return rank << 40


class DistributedAggregator:
    """Multi-process round runner over a device or host engine.

    ``engine="device"``: :class:`sda_amd.engine.DeviceAggregator` on
    ``cuda:LOCAL_RANK`` (the MI355X path). ``engine="host"``:
    :class:`sda_amd.host_engine.HostAggregator` (CPU; gloo tests).

    `deadline_s` bounds the wait for clerk results; `fault_hook(stage, rank)`
    is called at the stage boundaries ("before_partials", "before_results") and,
    on the host engines, between the result rendezvous and the transfer it
    decided ("before_result_transfer") -- the fault-injection points of the tests.
    `strict_liveness` (device engine): a rank posts its liveness flags only once its
    GPU has finished the work in front of the stage (see DeviceCommittee).
    """

    def __init__(self, spec: AggregationSpec, engine: str = "device", device=None, group=None,
                 time_stages: bool = False, layout: str = "committee", waves: int = 4,
                 force_pipeline: bool = False, fault_tolerant: bool = True,
                 deadline_s: float = 60.0, fault_hook=None, pss_backend: str = "auto",
                 strict_liveness: bool = False,
                 loopback: bool = False, max_op_bytes: int = 1 << 30):
        if layout not in ("committee", "owner"):
            raise ValueError("layout must be 'committee' or 'owner'")
        if engine not in ("device", "host"):
            raise ValueError("engine must be 'device' or 'host'")
        self.spec = spec
        self.comm = Comm(group, deadline_s=deadline_s, loopback=loopback,
                         max_op_bytes=max_op_bytes)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.kind, self.layout = engine, layout
        self.fault_tolerant, self.fault_hook = fault_tolerant, fault_hook
        self.stream = None
        n = spec.n_clerks
        self.hosted = hosted_clerks(self.rank, self.world, n) if layout == "committee" \
            else list(range(n))
        pk, sk = self._keys(n)
        if engine == "device":
            from ..engine import DeviceAggregator, KeyTable

            if device is None:
                device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
            self.engine = DeviceAggregator(spec, device=device,
                                           keys=KeyTable.from_bytes(pk, sk, device),
                                           time_stages=time_stages, pss_backend=pss_backend)
            self._committee = None
            # the round's kernels go on a stream that does not share a hardware
            # queue with RCCL's transfer stream (committee layout: the exchange of
            # wave w must run beside the sealing of wave w + 1)
            if layout == "committee" and self.comm.device_native and \
                    (self.world > 1 or loopback):
                with torch.cuda.device(device):
                    self.stream = self.comm.pick_compute_stream(device)
            if layout == "committee":
                from .device_round import DeviceCommittee

                self._committee = DeviceCommittee(self.engine, self.comm, waves=waves,
                                                  force_pipeline=force_pipeline,
                                                  fault_tolerant=fault_tolerant,
                                                  fault_hook=fault_hook)
                self._committee.strict_liveness = strict_liveness
        else:
            from ..host_engine import HostAggregator, HostKeys

            self.engine = HostAggregator(spec, keys=HostKeys(pk, sk))
        # int32 reduction is exact when the sum of `world` values < m fits
        self._narrow = self.world * (spec.field_modulus - 1) < 2 ** 31
        self._rid = 0

    def set_waves(self, waves) -> None:
        """Participant waves the committee exchange is pipelined over: a count, or
        "taper" (small first and last waves; see DeviceCommittee.set_waves). Takes
        effect at the next round; every rank must use the same value."""
        cm = getattr(self, "_committee", None)
        if cm is not None:
            cm.set_waves(waves)

    # ---- key custody -----------------------------------------------------------
    def _keys(self, n: int):
        """(pk[n+1], sk[n+1]) as bytes; sk[i] is None where this rank must not
        hold it. Committee: clerk c's keypair is generated by its lead and the
        secret key goes point to point to the clerk's other hosts only; the
        recipient's is generated on rank 0 and never leaves it. Public keys are
        broadcast. Owner layout: everything from rank 0 to every rank."""
        from .._native import native

        comm, W, me = self.comm, self.world, self.rank
        gen = native().crypto.box_keypair
        pk, sk = [None] * (n + 1), [None] * (n + 1)
        if self.layout == "owner":
            for i in range(n + 1):
                pair = gen() if me == ROOT else (None, None)
                pk[i] = comm.broadcast_bytes(pair[0], 32, src=ROOT)
                sk[i] = comm.broadcast_bytes(pair[1], 32, src=ROOT)
            return pk, sk
        sends, recvs, want = [], [], []
        for c in range(n):
            hs = hosts(c, W, n)
            mine = gen() if me == hs[0] else (None, None)
            pk[c] = comm.broadcast_bytes(mine[0], 32, src=hs[0])
            if me == hs[0]:
                sk[c] = mine[1]
                for r in hs[1:]:
                    sends.append((r, mine[1]))
                    comm.note("key", "send", r, c, 32)
            elif me in hs:
                recvs.append((hs[0], 32))
                want.append(c)
                comm.note("key", "recv", hs[0], c, 32)
        for c, b in zip(want, comm.exchange_bytes(sends, recvs)):
            sk[c] = b
        mine = gen() if me == ROOT else (None, None)
        pk[n] = comm.broadcast_bytes(mine[0], 32, src=ROOT)
        sk[n] = mine[1]
        return pk, sk

    # ---- owner layout ---------------------------------------------------------
    def _reduce(self, partials):
        """Sum the per-clerk (+ mask) partial rows over ranks onto rank 0."""
        if isinstance(partials, np.ndarray):
            wire = partials.astype(np.int32) if self._narrow else partials
            self.comm.note("plain-partial", "send", ROOT, -1, wire.nbytes)
            out = self.comm.reduce_sum(wire)
            return None if out is None else out.astype(np.int64)
        wire = partials.to(torch.int32) if self._narrow else partials
        self.comm.note("plain-partial", "send", ROOT, -1, wire.numel() * wire.element_size())
        out = self.comm.reduce_sum(wire)
        return None if out is None else out.to(torch.int64)

    # ---- rounds -----------------------------------------------------------------
    def run_round(self, secrets_local, clerks: Optional[Sequence[int]] = None,
                  check: bool = True):
        """One round over every rank's participants; rank 0 gets the output.

        Every rank must hold the same number of participants (the plan cuts
        every source's boxes alike).
        """
        if self.layout == "owner":
            return self.engine.run_round(secrets_local, clerks=clerks, check=check,
                                         reducer=self._reduce, owner_base=_owner_base(self.rank))
        if self.kind == "host":
            return self._host_round(secrets_local, clerks)
        if self.stream is None:
            return self._committee_round(secrets_local, clerks, check)
        # on the probed compute stream, ordered after and before the caller's stream
        caller = torch.cuda.current_stream(self.engine.device)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            res = self._committee_round(secrets_local, clerks, check)
        caller.wait_stream(self.stream)
        for t in (res.output, res.err):
            if t is not None:
                t.record_stream(caller)
        return res

    def _committee_round(self, secrets_local, clerks, check):
        from ..engine import RoundResult

        eng, cm = self.engine, self._committee
        live = eng._live(clerks)
        err = eng.new_error_word()
        marks: list = []
        eng._mark(marks, "start")
        acc, mask_arena = cm.participate_exchange_clerk(
            secrets_local, live, err, owner_base=_owner_base(self.rank), marks=marks)
        # the result path's key agreement queues on the side stream BEHIND the
        # participants' and clerks' (needed last; ahead of them it delayed the
        # first encrypt by two X25519 ladders)
        ctx = cm.begin(live, err)
        cm.ship_masks(ctx, mask_arena, err)
        out, used = cm.finish(ctx, acc, err, marks=marks)
        return eng._finish(err, marks, check, RoundResult(out, used, {}))

    def run_streamed(self, total_local: int, make_wave, wave: Optional[int] = None,
                     clerks: Optional[Sequence[int]] = None, checkpoint: Optional[str] = None,
                     checkpoint_every: int = 8, resume: bool = True):
        """Stream this rank's `total_local` participants in waves (device engine).

        Every rank must stream the same number of participants with the same
        wave size (None: the smallest of the ranks' planned waves). Checkpoints are
        per rank: pass a rank-specific path.
        """
        if self.kind != "device":
            raise ValueError("streaming runs on the device engine")
        from ..streaming import StreamingAggregator

        if wave is None:
            # every rank must cut its participants alike: agree on the smallest plan
            mine = self.engine.plan(total_local, input_resident=False).wave
            wave = max(1, int(-self.comm.all_reduce_max(-float(mine))))
        st = StreamingAggregator(self.engine, wave=wave, checkpoint=checkpoint,
                                 checkpoint_every=checkpoint_every)
        if self.layout == "owner":
            return st.run(total_local, make_wave, clerks=clerks, reducer=self._reduce,
                          owner_base=_owner_base(self.rank), resume=resume)
        if self.stream is None:
            return st.run(total_local, make_wave, clerks=clerks, committee=self._committee,
                          owner_base=_owner_base(self.rank), resume=resume)
        caller = torch.cuda.current_stream(self.engine.device)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            res = st.run(total_local, make_wave, clerks=clerks, committee=self._committee,
                         owner_base=_owner_base(self.rank), resume=resume)
        caller.wait_stream(self.stream)
        if res.output is not None:
            res.output.record_stream(caller)
        return res

    # ---- committee round on the host engines (CPU, gloo) ----------------------------
    def _hook(self, stage: str):
        if self.fault_hook is not None:
            self.fault_hook(stage, self.rank)

    def _host_round(self, secrets, clerks):
        """The committee dataflow of :mod:`device_round` with the reference's
        per-participant client code (C++ core) in place of the kernels. Sealed
        boxes travel as length-prefixed rows of a fixed stride."""
        from ..host_engine import HostRoundResult

        eng, comm = self.engine, self.comm
        spec, n, m = self.spec, eng.n, eng.m
        W, me = self.world, self.rank
        B = spec.batches
        live = eng.live(clerks)
        self._rid += 1
        topic = f"h{self._rid}"
        ft = self.fault_tolerant and W > 1
        secrets = np.asarray(secrets, dtype=np.int64)
        P = secrets.shape[0]
        boxes, mask_boxes = eng.participate(secrets)

        # ---- snapshot transpose: clerk-major rows -> the clerks' ranks
        stride = _row_stride(max(B, spec.dimension))
        pl = plan(me, W, n, P)
        arena = _pack_rows([boxes[p][c] for c in range(n) for p in range(P)], stride)
        inbox = torch.zeros(pl.inbox_rows, stride, dtype=torch.uint8)
        comm.exchange(*RowRouter(comm, pl).ops([(arena, inbox)], kind="box"))
        # masks travel with the participations (snapshot.rs:32-43): every rank's
        # participants' mask boxes -> the recipient
        masks_in = None
        if mask_boxes is not None:
            src = _pack_rows(mask_boxes, stride)
            masks_in = torch.zeros(W * P, stride, dtype=torch.uint8) if me == ROOT else None
            comm.exchange(*gather_rows_to(comm, ROOT, [(src, masks_in)], P, kind="mask"))

        # ---- clerks: open + combine per hosted segment
        partial = {}
        for i, s in enumerate(pl.segments):
            if s.clerk in live:
                first, rows = pl.segment_rows(i)
                partial[s.clerk] = eng.clerk_combine(s.clerk, _unpack_rows(inbox[first:first + rows]))

        # ---- clerk-internal: co-hosts' partial sums -> the lead
        self._hook("before_partials")
        complete, go = partial_stage(comm, topic, live, n, ft)
        sends, recvs, inbound = [], [], {}
        for c in live:
            hs = hosts(c, W, n)
            if me not in hs:
                continue
            mine = torch.from_numpy(partial.get(c, np.zeros(B, dtype=np.int64)).astype(np.int64))
            if c in complete:
                inbound[c] = [mine]
                for r in hs[1:]:
                    buf = torch.empty(B, dtype=torch.int64)
                    recvs.append((r, buf))
                    inbound[c].append(buf)
                    comm.note("partial", "recv", r, c, buf.numel() * 8)
            elif c in go:
                sends.append((hs[0], mine))
                comm.note("partial", "send", hs[0], c, mine.numel() * 8)
        comm.exchange(sends, recvs)

        # ---- results: the lead seals the clerk's combined shares for the recipient
        sealed = {}
        for c in sorted(complete):
            tot = np.remainder(sum(t.numpy() for t in inbound[c]), m)
            sealed[c] = eng.seal_result(tot)
        self._hook("before_results")
        arrived = result_stage(comm, topic, live, n, ft, sealed, ROOT)
        # (a rank lost from here on has already been counted in: the recipient's
        # receive from it fails when the backend notices, not at the rendezvous)
        self._hook("before_result_transfer")
        need = spec.sharing.reconstruction_threshold()
        enough = len(arrived) >= need
        res_in = torch.zeros(len(live), stride, dtype=torch.uint8) if me == ROOT else None
        sends, recvs = [], []
        if enough:
            for i, c in enumerate(live):
                if c not in arrived:
                    continue
                ld = lead(c, W, n)
                if ld == me:
                    row = _pack_rows([sealed[c]], stride)
                    if me == ROOT:
                        res_in[i:i + 1].copy_(row)
                    else:
                        sends.append((ROOT, row))
                        comm.note("result", "send", ROOT, c, stride)
                elif me == ROOT:
                    recvs.append((ld, res_in[i:i + 1]))
                    comm.note("result", "recv", ld, c, stride)
        comm.exchange(sends, recvs)

        if me != ROOT:
            return HostRoundResult(None, arrived)
        if not enough:
            from .. import control as C

            raise C.errors.SdaError(
                f"Not enough clerk results to reconstruct: {len(arrived)} of {len(live)} arrived, "
                f"{need} needed")
        blobs = _unpack_rows(res_in)
        results = [(c, blobs[live.index(c)]) for c in arrived]
        out = eng.reveal(results, _unpack_rows(masks_in) if masks_in is not None else None)
        return HostRoundResult(out, arrived)


# ---- host rows: u32 length | Encryption JSON | padding ---------------------------------
def _row_stride(L: int) -> int:
    blob = 48 + 10 * L                      # sealed box over <= 10-byte varints
    text = 16 + (blob + 2) // 3 * 4         # {"Sodium":"<base64>"}
    return (4 + text + 7) // 8 * 8


def _pack_rows(items, stride: int) -> torch.Tensor:
    out = np.zeros((len(items), stride), dtype=np.uint8)
    for i, s in enumerate(items):
        b = s.encode()
        if 4 + len(b) > stride:
            raise ValueError("sealed box larger than the row stride")
        out[i, :4] = np.frombuffer(len(b).to_bytes(4, "little"), dtype=np.uint8)
        out[i, 4:4 + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return torch.from_numpy(out)


def _unpack_rows(rows: torch.Tensor):
    arr = rows.numpy()
    out = []
    for i in range(arr.shape[0]):
        ln = int.from_bytes(arr[i, :4].tobytes(), "little")
        out.append(arr[i, 4:4 + ln].tobytes().decode())
    return out
