"""The committee round on the device engine: one process per MI355X, sealed
boxes routed to the ranks that play the clerks over RCCL/xGMI.

Dataflow per rank (reference roles in brackets):

  participants  mask + share + seal P x n boxes              [participate.rs:37-113]
  exchange      the snapshot transpose as a uniform all-to-all of sealed boxes
                (parallel/routing.py), pipelined over participant waves so
                wave w travels while wave w+1 is being sealed   [snapshot.rs:11-27]
  clerks        open + combine the inbox, per hosted clerk      [clerk.rs:79-86]
  clerk-internal a clerk that spans several ranks sums its hosts' partial sums
                on its lead rank (plaintext never leaves the clerk's own ranks)
  results       the lead seals the clerk's combined shares for the recipient
                and sends that one box to rank 0                [clerk.rs:99-100]
  recipient     rank 0 opens the results that arrived (>= t + k), reconstructs,
                opens the participants' mask boxes and unmasks  [receive.rs:80-157]

X25519 is latency-bound (one ladder per lane, ~1 ms however few messages), so
key agreement happens once per round on the side stream: the participants' seal
keys for every wave at once, the 32-byte ephemeral-key headers travel ahead of
the data over the same plan, and the clerks (and the recipient, for the result
boxes) derive their open keys while the waves are still being sealed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch

from .._native import native
from ..engine import AggregationError, DeviceAggregator
from ..models.schemes import ChaChaMask, FullMask
from ..ops import gpu as G
from ..ops.sealed import Arena, KeySet, open_setup, open_sum, seal_data, seal_setup
from .comm import Comm
from .router import RowRouter, gather_rows_to
from .liveness import partial_stage, result_stage
from .routing import hosted_clerks, hosts, lead, plan


def _header_arena(hdr: torch.Tensor, K: int) -> Arena:
    """32-byte ephemeral public keys [M][32] viewed as an arena of bare headers
    (all that key agreement reads). `K`: chunks per slot of the arena the boxes
    themselves live in -- it decides whether the derived key set carries the
    complete Poly1305 tables, so that they are made here, beside the bulk work,
    and not again on the consuming stream."""
    return Arena(hdr.shape[0], 0, 0, 32, K, hdr.view(-1), None)


@dataclass
class RoundContext:
    """Per-round state created ahead of the data (result-box key agreement)."""
    rid: int
    live: List[int]
    led: List[int]                      # live clerks this rank leads
    res_arena: Optional[Arena] = None   # this rank's led clerks' result boxes
    ks_res: Optional[KeySet] = None
    res_in: Optional[Arena] = None      # root: one row per live clerk
    ko_res: Optional[KeySet] = None
    ev: Optional[torch.cuda.Event] = None
    mask_acc: Optional[torch.Tensor] = None  # root: running mask sum (int64 [D])
    stats: dict = field(default_factory=dict)


class DeviceCommittee:
    ROOT = 0  # the recipient's rank

    def __init__(self, engine: DeviceAggregator, comm: Comm, waves: int = 4,
                 force_pipeline: bool = False, fault_tolerant: bool = True, fault_hook=None):
        self.engine, self.comm = engine, comm
        self.set_waves(waves)
        self.force_pipeline = force_pipeline
        self.fault_tolerant = fault_tolerant
        self.fault_hook = fault_hook
        # Liveness flags say "my host reached this stage"; with strict_liveness they say
        # "my GPU finished the work in front of this stage": the host waits for its stream
        # before it posts, so a rank that dies while that work is still running is left
        # out by its peers instead of being waited for. Costs the host its lead over the
        # GPU once per guarded stage (rounds no longer queue ahead); off by default.
        self.strict_liveness = False
        # the clerks' key agreement queued behind the first wave's share kernel (True) or
        # beside it (False: as early as possible)
        self.open_keys_behind_share = True
        n, W, me = engine.n, comm.world, comm.rank
        self.hosted = hosted_clerks(me, W, n)
        self.led = [c for c in self.hosted if lead(c, W, n) == me]
        for c in self.hosted:
            if not engine.keys.holds(c):
                raise ValueError(f"rank {me} plays clerk {c} but does not hold its secret key")
        if me == self.ROOT and not engine.keys.holds(n):
            raise ValueError("the recipient's rank does not hold the recipient key")
        self._rid = 0
        # int32 sums of `world` values below m are exact when they fit
        self._narrow = W * (engine.m - 1) < 2 ** 31

    # ------------------------------------------------------------------ waves ----
    TAPER = (1, 3, 4, 4, 3, 1)  # sixteenths of the participants per wave

    def set_waves(self, waves) -> None:
        """`waves`: a count (equal waves) or "taper": six waves of 1/16, 3/16, 4/16,
        4/16, 3/16, 1/16 of the participants -- when the exchange is what bounds the
        round, its critical path is the first wave's seal + all transfers + the last
        wave's open, so small first and last waves shorten it without the small
        grids of many equal waves."""
        if waves == "taper":
            self.waves = "taper"
        else:
            self.waves = max(1, int(waves))

    def wave_bounds(self, P: int, pipelined: bool):
        """Participant ranges [lo, hi) of the waves (the same on every rank)."""
        if not pipelined:
            return [(0, P)]
        if self.waves == "taper":
            cuts, acc = [0], 0
            for f in self.TAPER:
                acc += f
                cuts.append(P * acc // 16)
            bounds = list(zip(cuts, cuts[1:]))
        else:
            nw = min(self.waves, P)
            bounds = [(P * w // nw, P * (w + 1) // nw) for w in range(nw)]
        return [(lo, hi) for lo, hi in bounds if hi > lo]

    # ------------------------------------------------------------------ begin ----
    def begin(self, live, err) -> RoundContext:
        """Result-path key agreement ahead of the data: every lead derives the
        seal keys of its clerks' result boxes and sends the 32-byte headers to
        the recipient, which derives the matching open keys -- all on the side
        stream, hidden behind the round's bulk work."""
        eng, comm = self.engine, self.comm
        n, m, B, dev = eng.n, eng.m, eng.spec.batches, eng.device
        me, root = comm.rank, self.ROOT
        self._rid += 1
        ctx = RoundContext(self._rid, list(live), [c for c in self.led if c in live])
        main, side = torch.cuda.current_stream(dev), eng._side_stream()
        rng_key = native().crypto.random_bytes(32)
        pks, sks = eng.keys.pks, eng.keys.sks
        # Nothing here waits for the main stream: called after the round's bulk
        # work has been queued, it must run beside it, not behind it (`err` was
        # initialised before the participants' setup, which this stream already
        # ordered itself after).
        with torch.cuda.stream(side):
            hdr = None
            if ctx.led:
                k = len(ctx.led)
                ctx.res_arena = Arena.empty(k, B, m, dev)
                kidx = torch.full((k,), n, dtype=torch.int32, device=dev)
                ctx.ks_res = seal_setup(ctx.res_arena, kidx, pks, rng_key, 0, err).with_powers()
                hdr = ctx.res_arena.ct.view(k, ctx.res_arena.stride)[:, :32].contiguous()
            sends, recvs = [], []
            hdr_in = None
            if me == root:
                hdr_in = torch.zeros(len(live), 32, dtype=torch.uint8, device=dev)
            loop = comm.loopback
            for i, c in enumerate(live):
                ld = lead(c, comm.world, n)
                if ld == me:
                    row = hdr[ctx.led.index(c):ctx.led.index(c) + 1]
                    if me == root and not loop:
                        hdr_in[i:i + 1].copy_(row)
                    else:
                        sends.append((root, row))
                        comm.note("hdr", "send", root, c, 32)
                if me == root and (ld != me or loop):
                    recvs.append((ld, hdr_in[i:i + 1]))
                    comm.note("hdr", "recv", ld, c, 32)
            h = comm.exchange_async(sends, recvs)
            h.wait()
            if me == root:
                ctx.res_in = Arena.empty(len(live), B, m, dev)
                kidx_r = torch.full((len(live),), n, dtype=torch.int32, device=dev)
                ctx.ko_res = open_setup(_header_arena(hdr_in, ctx.res_in.K), kidx_r, sks, pks, err)
                if comm.world == 1 and ctx.led == list(live) and not loop:
                    ctx.res_in = ctx.res_arena  # one rank: the results are opened where they were sealed
            ctx.ev = torch.cuda.Event()
            ctx.ev.record(side)
        for t in (ctx.ks_res, ctx.ko_res):
            if t is not None:
                t.record_stream(main)
        for a in (ctx.res_arena, ctx.res_in):
            if a is not None:
                a.ct.record_stream(main)
                a.pt_len.record_stream(main)
        return ctx

    def _kidx_inbox(self, key, plans) -> torch.Tensor:
        """Clerk index of every inbox row (which secret key opens it), cached per shape."""
        cache = self.__dict__.setdefault("_kidx_cache", {})
        if key not in cache:
            W = self.comm.world
            idx = [torch.full((W * s.count,), s.clerk, dtype=torch.int32)
                   for pl in plans for s in pl.segments]
            cache[key] = (torch.cat(idx) if idx else torch.zeros(0, dtype=torch.int32)).to(
                self.engine.device)
        return cache[key]

    # ------------------------------------------- participants + exchange + clerks ----
    def participate_exchange_clerk(self, secrets: torch.Tensor, live, err, owner_base: int = 0,
                                   marks=None):
        """Returns (acc, mask_arena): acc[c] = int64 [B] sum of clerk c's shares
        over the boxes this rank opened (zero for clerks it does not play),
        mask_arena = this rank's participants' mask boxes sealed for the
        recipient (or None)."""
        eng, comm = self.engine, self.comm
        spec, n, m = eng.spec, eng.n, eng.m
        W, me = comm.world, comm.rank
        marks = [] if marks is None else marks
        if secrets.dim() != 2 or secrets.shape[1] != spec.dimension:
            raise ValueError("secrets must be [P][dimension]")
        if secrets.dtype != torch.int32 or secrets.device.type != "cuda":
            raise ValueError("secrets must be an int32 GPU tensor")
        secrets = secrets.contiguous()
        P, D = secrets.shape
        B, dev = spec.batches, eng.device
        bounds = self.wave_bounds(P, W > 1 or self.force_pipeline)
        plans = [plan(me, W, n, hi - lo) for lo, hi in bounds]
        routers = [RowRouter(comm, pl) for pl in plans]
        in_base, rows_in = [], 0
        for pl in plans:
            in_base.append(rows_in)
            rows_in += pl.inbox_rows
        rng_key = native().crypto.random_bytes(32)
        eng._round += 1
        main, side = torch.cuda.current_stream(dev), eng._side_stream()
        pks, sks = eng.keys.pks, eng.keys.sks

        # wave-blocked clerk-major arena: wave w's n * P_w slots are contiguous
        arena = Arena.empty(n * P, B, m, dev)
        alias = W == 1 and not comm.loopback  # one rank: the inbox is the arena, nothing moves
        kidx_send = torch.cat([eng._kidx_clerk(hi - lo) for lo, hi in bounds])
        if alias:
            inbox, kidx_in = arena, kidx_send
        else:
            inbox = Arena(rows_in, B, m, arena.stride, arena.K,
                          torch.empty(rows_in * arena.stride, dtype=torch.uint8, device=dev),
                          torch.empty(rows_in, dtype=torch.int32, device=dev))
            kidx_in = self._kidx_inbox(tuple(bounds), plans)
        mask_arena = None
        if isinstance(spec.masking, FullMask):
            mask_arena = Arena.empty(P, D, m, dev)
        elif isinstance(spec.masking, ChaChaMask):
            mask_arena = Arena.empty(P, spec.masking.seed_words, 0, dev)
        kidx_rcpt = torch.full((P,), n, dtype=torch.int32, device=dev)

        gate = eng._gate_token()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ks = seal_setup(arena, kidx_send, pks, rng_key, 0, err, gate=gate,
                            pk_tables=eng.keys.tables(arena.M)).with_powers()
            ks_mask = None
            if mask_arena is not None:
                ks_mask = seal_setup(mask_arena, kidx_rcpt, pks, rng_key, n * P, err).with_powers()
            ev_seal = torch.cuda.Event()
            ev_seal.record(side)

        opened = {}

        def open_keys():
            # The ephemeral-key headers ahead of the data, then the clerks' open keys.
            # Queued behind the first wave's share kernel, not beside it: beside it the
            # ladder waves take register space from the share grid (a one-wave round's
            # share kernel ran 2.96 ms instead of 2.40).
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if alias:
                    ko = open_setup(arena, kidx_in, sks, pks, err)
                else:
                    hdr = arena.ct.view(arena.M, arena.stride)[:, :32].contiguous()
                    hdr_in = torch.empty(rows_in, 32, dtype=torch.uint8, device=dev)
                    sends, recvs = [], []
                    for (lo, hi), r, base in zip(bounds, routers, in_base):
                        s_, r_ = r.ops([(hdr, hdr_in)], src_base=n * lo, dst_base=base, kind="hdr")
                        sends += s_
                        recvs += r_
                    h = comm.exchange_async(sends, recvs)
                    h.wait()
                    ko = open_setup(_header_arena(hdr_in, arena.K), kidx_in, sks, pks, err)
                ev = torch.cuda.Event()
                ev.record(side)
            ko.record_stream(main)
            opened["ko"], opened["ev"] = ko, ev

        # caching-allocator stream bookkeeping: side-allocated keys are consumed on
        # main, main-allocated buffers are touched on side
        for t in (ks, ks_mask):
            if t is not None:
                t.record_stream(main)
        for t in (arena.ct, kidx_send, kidx_in, kidx_rcpt) + \
                ((mask_arena.ct,) if mask_arena is not None else ()):
            t.record_stream(side)
        eng._mark(marks, "keys")

        # running sums of the hosted clerks' shares: one int64 row per clerk (waves of
        # sums below m never overflow), rows of clerks this rank does not play stay zero
        acc = torch.zeros(n, B, dtype=torch.int64, device=dev)
        src2d = arena.ct.view(arena.M, arena.stride)
        dst2d = inbox.ct.view(inbox.M, inbox.stride)
        src_len, dst_len = arena.pt_len.view(-1, 1), inbox.pt_len.view(-1, 1)

        def finish(w, handle):
            handle.wait()
            ko = opened["ko"]
            main.wait_event(opened["ev"])
            pl, base = plans[w], in_base[w]
            segs = [(i, s) for i, s in enumerate(pl.segments) if s.count and s.clerk in live]
            if not segs:
                return
            counts = {s.count for _, s in segs}
            contiguous = [i for i, _ in segs] == list(range(segs[0][0], segs[0][0] + len(segs)))
            if len(counts) == 1 and contiguous:
                # equal segments side by side: one launch, a row per clerk
                first, _ = pl.segment_rows(segs[0][0])
                rows = len(segs) * W * segs[0][1].count
                c0 = segs[0][1].clerk  # side-by-side segments are mostly consecutive clerks
                if [s.clerk for _, s in segs] == list(range(c0, c0 + len(segs))):
                    # the sums go straight into the clerks' running rows
                    open_sum(inbox.slice(base + first, rows), ko.slice(base + first, rows), err,
                             rows=len(segs), out=None, acc=acc[c0:c0 + len(segs)])
                else:
                    out = torch.empty(len(segs), B, dtype=torch.int32, device=dev)
                    open_sum(inbox.slice(base + first, rows), ko.slice(base + first, rows), err,
                             rows=len(segs), out=out)
                    for j, (_, s) in enumerate(segs):
                        acc[s.clerk] += out[j]
            else:
                for i, s in segs:
                    first, rows = pl.segment_rows(i)
                    open_sum(inbox.slice(base + first, rows), ko.slice(base + first, rows), err,
                             rows=1, out=None, acc=acc[s.clerk])

        pending = None
        if not self.open_keys_behind_share:
            open_keys()
        G.gate_wait(gate)
        for w, (lo, hi) in enumerate(bounds):
            Pw = hi - lo
            shares, cnt, mvals, mcnt = eng._share(secrets[lo:hi], rng_key, owner_base + lo, err)
            if w == 0:  # the first wave's shares overlap the whole-round seal setup
                if self.open_keys_behind_share:
                    open_keys()
                main.wait_event(ev_seal)
            box = arena.slice(n * lo, n * Pw)
            seal_data(box, ks.slice(n * lo, n * Pw), shares.view(n * Pw, B), err, cnt)
            del shares
            eng._inject_corruption(box)
            if mask_arena is not None:
                seal_data(mask_arena.slice(lo, Pw), ks_mask.slice(lo, Pw), mvals, err, mcnt)
            if alias:
                handle = _Done()
            else:
                sends, recvs = routers[w].ops([(src2d, dst2d), (src_len, dst_len)],
                                              src_base=n * lo, dst_base=in_base[w], kind="box")
                handle = comm.exchange_async(sends, recvs)
            if pending is not None:
                finish(*pending)
            pending = (w, handle)
        eng._mark(marks, "participate")
        finish(*pending)
        eng._mark(marks, "clerk")
        return acc, mask_arena

    # ------------------------------------------------------------------ masks ----
    def ship_masks(self, ctx: RoundContext, mask_arena: Optional[Arena], err):
        """Every rank's participants' mask boxes travel to the recipient's rank,
        which opens them and adds the masks (full.rs:37-52) or the re-expanded
        ChaCha seeds (chacha.rs:56-77) to its running mask sum."""
        if mask_arena is None:
            return
        eng, comm = self.engine, self.comm
        W, me, root, dev = comm.world, comm.rank, self.ROOT, eng.device
        P = mask_arena.M
        if W == 1 and not comm.loopback:
            box = mask_arena
        else:
            box = None
            dst2d = dst_len = None
            if me == root:
                box = Arena(W * P, mask_arena.L, mask_arena.modulus, mask_arena.stride, mask_arena.K,
                            torch.empty(W * P * mask_arena.stride, dtype=torch.uint8, device=dev),
                            torch.empty(W * P, dtype=torch.int32, device=dev))
                dst2d, dst_len = box.ct.view(W * P, box.stride), box.pt_len.view(-1, 1)
            sends, recvs = gather_rows_to(
                comm, root, [(mask_arena.ct.view(P, mask_arena.stride), dst2d),
                             (mask_arena.pt_len.view(-1, 1), dst_len)], P, kind="mask")
            comm.exchange_async(sends, recvs).wait()
        if me != root:
            return
        kidx = torch.full((box.M,), eng.n, dtype=torch.int32, device=dev)
        ko = open_setup(box, kidx, eng.keys.sks, eng.keys.pks, err)
        msum = eng._open_masks(box, ko, err).to(torch.int64)
        ctx.mask_acc = msum if ctx.mask_acc is None else ctx.mask_acc + msum

    # ----------------------------------------------------------------- finish ----
    def _hook(self, stage: str):
        if self.fault_hook is not None:
            self.fault_hook(stage, self.comm.rank)

    def finish(self, ctx: RoundContext, acc: torch.Tensor, err, marks=None):
        """Clerk-internal reduce, sealed results to the recipient, reveal.
        Returns (output or None, clerks_used)."""
        eng, comm = self.engine, self.comm
        n, m, B, dev = eng.n, eng.m, eng.spec.batches, eng.device
        W, me, root, live = comm.world, comm.rank, self.ROOT, ctx.live
        topic = f"r{ctx.rid}"
        ft = self.fault_tolerant and W > 1
        wire_dtype = torch.int32 if self._narrow else torch.int64
        rem = torch.remainder(acc, m)  # [n][B] int64, canonical
        wire = rem if wire_dtype == torch.int64 or W == 1 else rem.to(wire_dtype)

        # ---- clerk-internal: co-hosts' partial sums -> the clerk's lead
        self._hook("before_partials")
        if ft and self.strict_liveness:
            torch.cuda.current_stream(dev).synchronize()
        complete, go = partial_stage(comm, topic, live, n, ft)
        sends, recvs, inbound = [], [], {}
        for c in live:
            hs = hosts(c, W, n)
            if me not in hs:
                continue
            if c in complete:
                inbound[c] = []
                for r in hs[1:]:
                    buf = torch.empty(B, dtype=wire_dtype, device=dev)
                    recvs.append((r, buf))
                    inbound[c].append(buf)
                    comm.note("partial", "recv", r, c, buf.numel() * buf.element_size())
            elif c in go:
                t = wire[c]
                sends.append((hs[0], t))
                comm.note("partial", "send", hs[0], c, t.numel() * t.element_size())
        comm.exchange_async(sends, recvs).wait()
        if marks is not None:
            eng._mark(marks, "partials")

        # ---- results: each lead seals its clerks' combined shares for the recipient
        torch.cuda.current_stream(dev).wait_event(ctx.ev)
        led_ok = [c for c in ctx.led if c in complete]
        if ctx.led:
            lo, hi = ctx.led[0], ctx.led[-1] + 1
            if led_ok == ctx.led and not any(inbound[c] for c in led_ok) and \
                    ctx.led == list(range(lo, hi)):
                combined = rem[lo:hi].to(torch.int32)  # no co-hosts: the sums are this rank's own
            else:
                combined = torch.zeros(len(ctx.led), B, dtype=torch.int32, device=dev)
                for c in led_ok:
                    tot = rem[c]
                    for buf in inbound[c]:
                        tot = tot + buf
                    combined[ctx.led.index(c)] = torch.remainder(tot, m).to(torch.int32)
            eng.seal_results(ctx.res_arena, ctx.ks_res, combined, err)
        self._hook("before_results")
        if ft and self.strict_liveness:
            torch.cuda.current_stream(dev).synchronize()
        arrived = result_stage(comm, topic, live, n, ft, led_ok, root)
        need = eng.spec.sharing.reconstruction_threshold()
        enough = len(arrived) >= need
        sends, recvs = [], []
        if enough:
            for i, c in enumerate(live):
                if c not in arrived:
                    continue
                ld = lead(c, W, n)
                loop = comm.loopback
                if ld == me:
                    k = ctx.led.index(c)
                    src = ctx.res_arena.ct.view(-1, ctx.res_arena.stride)[k:k + 1]
                    srcl = ctx.res_arena.pt_len.view(-1, 1)[k:k + 1]
                    if me == root and not loop:
                        if ctx.res_in is not ctx.res_arena:
                            ctx.res_in.ct.view(-1, ctx.res_in.stride)[i:i + 1].copy_(src)
                            ctx.res_in.pt_len.view(-1, 1)[i:i + 1].copy_(srcl)
                    else:
                        sends += [(root, src), (root, srcl)]
                        comm.note("result", "send", root, c, src.numel())
                if me == root and (ld != me or loop):
                    recvs += [(ld, ctx.res_in.ct.view(-1, ctx.res_in.stride)[i:i + 1]),
                              (ld, ctx.res_in.pt_len.view(-1, 1)[i:i + 1])]
                    comm.note("result", "recv", ld, c, ctx.res_in.stride)
        comm.exchange_async(sends, recvs).wait()
        if marks is not None:
            eng._mark(marks, "results")
        if me != root:
            return None, arrived
        if not enough:
            raise AggregationError(
                f"Not enough clerk results to reconstruct: {len(arrived)} of {len(live)} arrived, "
                f"{need} needed")
        mask_sum = None
        if ctx.mask_acc is not None:
            mask_sum = torch.remainder(ctx.mask_acc, m).to(torch.int32)
        rows = [live.index(c) for c in arrived]
        out = eng.open_results(ctx.res_in, ctx.ko_res, arrived, err, mask_sum, rows=rows)
        if marks is not None:
            eng._mark(marks, "reveal")
        return out, arrived


class _Done:
    def wait(self):
        pass
