"""Collectives, point-to-point transfers and the liveness rendezvous of the
distributed engines.

With the ``nccl`` backend (RCCL on ROCm, over xGMI) tensors stay on the GPU.
With ``gloo`` (CPU tests, or several ranks sharing one GPU) device tensors are
staged through host memory with synchronous copies, so the same engine code
runs on both.

Every payload that leaves a rank is recorded in ``Comm.audit`` as
``(kind, direction, peer, clerk, nbytes)``: tests assert from it that plaintext
partial sums only ever travel between hosts of the same clerk, and the bench
reports the bytes a rank puts on xGMI per round.

The rendezvous (``arrive`` / ``decide`` / ``decision``) is the reference's
result polling (client/src/receive.rs:86-96, server/src/server.rs:104-129: a
snapshot is ready once enough clerking results were posted) on the process
group's key-value store: a clerk that has reached the result stage posts a
flag, the recipient waits for the flags up to a deadline and publishes which
clerks it will read, and only those send. A clerk whose process died never
posts, so no rank ever waits on a transfer from a dead peer.
"""
from __future__ import annotations

import time
from datetime import timedelta
from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


class Comm:
    _instances = 0  # per process: every rank constructs its Comm objects in the same order

    def __init__(self, group=None, deadline_s: float = 60.0, loopback: bool = False,
                 max_op_bytes: int = 1 << 30):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device_native = self.backend == "nccl"
        self.deadline_s = float(deadline_s)
        self.audit: List[tuple] = []
        self.rendezvous_s = 0.0  # host time spent in the store rendezvous (arrive / decide / decision)
        self._store = None
        # Rendezvous keys live under a per-instance prefix: round counters restart
        # at 1 in every engine, and a second engine on the same process group must
        # not read the first one's flags and decisions.
        Comm._instances += 1
        self._nonce = Comm._instances
        self._garbage: List[tuple] = []  # (delete-after time, keys) of decisions this rank published
        # Loopback: a rank's own piece of an exchange is sent to itself through the
        # backend's send/recv instead of being copied locally. It makes the
        # point-to-point path (grouped isend/irecv, the transfer stream's ordering
        # against the compute streams) run on a single rank.
        self.loopback = bool(loopback)
        # Largest single send/recv: longer transfers are cut into runs of whole rows
        # (both sides cut alike, the shapes agree), which also keeps every op's byte
        # count far below 2^31.
        self.max_op_bytes = int(max_op_bytes)
        self.compute_stream_probe = None  # outcome of pick_compute_stream, for reports

    # -- accounting -------------------------------------------------------------
    def note(self, kind: str, direction: str, peer: int, clerk: int, nbytes: int):
        self.audit.append((kind, direction, peer, clerk, int(nbytes)))

    def bytes_sent(self, kinds: Optional[Iterable[str]] = None) -> int:
        ks = None if kinds is None else set(kinds)
        return sum(n for k, d, p, _, n in self.audit
                   if d == "send" and p != self.rank and (ks is None or k in ks))

    def reset_audit(self):
        self.audit = []

    # -- staging helpers ------------------------------------------------------
    def _to_wire(self, t):
        if isinstance(t, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(t)), "numpy", None
        if t.is_cuda and not self.device_native:
            return t.cpu(), "cuda", t.device  # synchronous copy: gloo only sees host memory
        return t, "torch", None

    @staticmethod
    def _from_wire(w, kind, device):
        if kind == "numpy":
            return w.numpy()
        if kind == "cuda":
            return w.to(device)
        return w

    def _wire_device(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.device_native else "cpu"

    # -- collectives ------------------------------------------------------------
    def barrier(self):
        if self.device_native:
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    def broadcast(self, t, src: int = 0):
        w, kind, dev = self._to_wire(t)
        dist.broadcast(w, src=src, group=self.group)
        return self._from_wire(w, kind, dev)

    def broadcast_bytes(self, data: Optional[bytes], nbytes: int, src: int = 0) -> bytes:
        """Public data (e.g. a public key) from `src` to everyone."""
        buf = torch.zeros(nbytes, dtype=torch.uint8)
        if self.rank == src:
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).clone()
        buf = buf.to(self._wire_device())
        dist.broadcast(buf, src=src, group=self.group)
        return bytes(buf.cpu().numpy().tobytes())

    def reduce_sum(self, t, dst: int = 0):
        """Sum over ranks; the result on `dst`, None elsewhere."""
        w, kind, dev = self._to_wire(t)
        w = w.contiguous()
        dist.reduce(w, dst=dst, op=dist.ReduceOp.SUM, group=self.group)
        return self._from_wire(w, kind, dev) if self.rank == dst else None

    def all_reduce_max(self, value: float) -> float:
        t = torch.tensor([value], dtype=torch.float64, device=self._wire_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def all_reduce_or(self, value: int) -> int:
        """Bitwise OR of a 32-bit word over ranks (RCCL has no BOR: one MAX per bit)."""
        bits = torch.tensor([(int(value) >> i) & 1 for i in range(32)], dtype=torch.int32,
                            device=self._wire_device())
        dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=self.group)
        return sum(int(b) << i for i, b in enumerate(bits.cpu().tolist()))

    def all_gather_object(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    # -- point to point -----------------------------------------------------------
    def exchange_async(self, sends, recvs):
        """Start a point-to-point exchange; returns a handle with ``wait()``.

        `sends` / `recvs` are lists of (peer, tensor); transfers between one
        pair of ranks are matched in list order; peer == self appears only in
        loopback mode (callers otherwise copy locally). With RCCL the operations are one grouped launch
        on the communicator's stream (every xGMI link busy at once), which
        first waits for work already queued on the current stream; the caller
        keeps queuing compute and calls ``wait()`` (the current stream then
        waits for the transfer) right before consuming the receives. With gloo
        the exchange completes before returning.
        """
        if not sends and not recvs:
            return _Done()
        if not self.device_native:
            self._exchange_host(sends, recvs)
            return _Done()
        sends = [(p, c) for p, t in sends for c in self._cut(t.contiguous())]
        recvs = [(p, c) for p, t in recvs for c in self._cut(t)]
        ops = [dist.P2POp(dist.isend, t, p, group=self.group) for p, t in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=self.group) for p, t in recvs]
        return _Pending(dist.batch_isend_irecv(ops), [t for _, t in sends])

    def _cut(self, t: torch.Tensor):
        """`t` as runs of whole leading-dimension rows of at most max_op_bytes each."""
        nbytes = t.numel() * t.element_size()
        if nbytes <= self.max_op_bytes or t.dim() == 0 or t.shape[0] <= 1:
            return [t]
        if not t.is_contiguous():
            raise ValueError("exchange: receive buffers must be contiguous")
        row = nbytes // t.shape[0]
        step = max(1, self.max_op_bytes // max(1, row))
        return [t[i:i + step] for i in range(0, t.shape[0], step)]

    def exchange(self, sends, recvs):
        self.exchange_async(sends, recvs).wait()

    def pick_compute_stream(self, device, tries: int = 8, spin_us: int = 1500):
        """A stream whose kernels run *beside* the backend's transfers.

        HIP multiplexes a process's streams onto few hardware queues (4 by
        default) and two streams on one queue serialise. RCCL launches its
        transfer kernels on a stream of its own; if that stream shares a queue
        with the stream the round's kernels are queued on, every wave's exchange
        runs behind the next wave's compute instead of beside it (seen in a
        kernel trace: transfer kernels and compute kernels on one queue id, back
        to back). Candidates are probed: the candidate runs a bounded spin (a
        gate the host never posts), the backend carries a small send/recv of
        this rank to itself, issued from another stream; a candidate whose spin
        is still running when the transfer has finished sits on another queue.
        Every rank probes for itself (the transfer is local), no rank waits for
        another. Falls back to the current stream on any failure: correct,
        only without the overlap."""
        dev = torch.device(device)
        cur = torch.cuda.current_stream(dev)
        if not self.device_native:
            return cur
        try:
            from ..ops import gpu as G

            gate = torch.zeros(1, dtype=torch.int32, device=dev)
            src = torch.zeros(4 << 20, dtype=torch.uint8, device=dev)
            dst = torch.empty_like(src)
            issue = torch.cuda.Stream(device=dev)
            cand = cur
            with torch.cuda.device(dev):
                for _ in range(tries):
                    cand = torch.cuda.Stream(device=dev)
                    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    torch.cuda.synchronize(dev)
                    with torch.cuda.stream(cand):
                        e0.record(cand)
                        G.gate_wait((gate, 1), timeout_us=spin_us)  # never posted: ends at the limit
                        e2.record(cand)
                    with torch.cuda.stream(issue):
                        ops = [dist.P2POp(dist.isend, src, self.rank, group=self.group),
                               dist.P2POp(dist.irecv, dst, self.rank, group=self.group)]
                        for w in dist.batch_isend_irecv(ops):
                            w.wait()
                        e1.record(issue)
                    torch.cuda.synchronize(dev)
                    if e0.elapsed_time(e1) < 0.6 * e0.elapsed_time(e2):
                        self.compute_stream_probe = "beside the transfers"
                        return cand
            self.compute_stream_probe = "no candidate ran beside the transfers"
            return cand
        except Exception as e:  # noqa: BLE001 - the probe is an optimisation only
            self.compute_stream_probe = f"probe failed: {type(e).__name__}"
            return cur

    def _exchange_host(self, sends, recvs):
        # gloo has no pair from a rank to itself: loopback transfers are matched in
        # list order here (RCCL carries them as real send/recv pairs)
        own_s = [t for p, t in sends if p == self.rank]
        own_r = [t for p, t in recvs if p == self.rank]
        if len(own_s) != len(own_r):
            raise RuntimeError("loopback: unmatched transfers to self")
        for src, dst in zip(own_s, own_r):
            dst.copy_(src)
        sends = [(p, t) for p, t in sends if p != self.rank]
        recvs = [(p, t) for p, t in recvs if p != self.rank]
        host_sends = [(p, t.contiguous().cpu() if t.is_cuda else t.contiguous()) for p, t in sends]
        host_recvs = [(p, torch.empty(t.shape, dtype=t.dtype) if (t.is_cuda or not t.is_contiguous())
                       else t, t) for p, t in recvs]
        ops = [dist.P2POp(dist.isend, t, p, group=self.group) for p, t in host_sends]
        ops += [dist.P2POp(dist.irecv, h, p, group=self.group) for p, h, _ in host_recvs]
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        for _, h, t in host_recvs:
            if h is not t:
                t.copy_(h)

    def exchange_bytes(self, sends: Sequence[tuple], recvs: Sequence[tuple]) -> List[bytes]:
        """Small byte strings point to point: `sends` = [(peer, bytes)], `recvs` =
        [(peer, nbytes)]; returns the received strings in `recvs` order."""
        dev = self._wire_device()
        st = [(p, torch.frombuffer(bytearray(b), dtype=torch.uint8).clone().to(dev)) for p, b in sends]
        rt = [(p, torch.empty(n, dtype=torch.uint8, device=dev)) for p, n in recvs]
        self.exchange(st, rt)
        return [bytes(t.cpu().numpy().tobytes()) for _, t in rt]

    def send_object(self, obj, peer: int):
        """Host objects (CPU engines): blocking pickled send."""
        dist.send_object_list([obj], dst=peer, group=self.group)

    def recv_object(self, peer: int):
        out = [None]
        dist.recv_object_list(out, src=peer, group=self.group)
        return out[0]

    # -- liveness rendezvous on the process group's store -------------------------
    @property
    def store(self):
        if self._store is None:
            from torch.distributed.distributed_c10d import _get_default_store

            self._store = dist.PrefixStore(f"sda{self._nonce}", _get_default_store())
        return self._store

    def arrive(self, topic: str, who) -> None:
        """Post "`who` reached `topic`" (non-blocking)."""
        t0 = time.perf_counter()
        self.store.set(f"{topic}/at/{who}", b"1")
        self.rendezvous_s += time.perf_counter() - t0

    def decide(self, topic: str, expected: Sequence, deadline_s: Optional[float] = None,
               all_or_nothing: bool = False, also: Sequence = ()) -> List:
        """Collect arrivals: returns the members of `expected` that arrived -- as
        soon as all have, else at the deadline -- and publishes them (plus
        `also`, members the decider vouches for itself) for :meth:`decision`.
        With `all_or_nothing` an incomplete set is published as empty."""
        expected = list(expected)
        t0 = time.perf_counter()
        deadline = time.monotonic() + (self.deadline_s if deadline_s is None else deadline_s)
        keys = {w: f"{topic}/at/{w}" for w in expected}
        live = expected
        if expected:
            try:
                self.store.wait(list(keys.values()),
                                timedelta(seconds=max(0.001, deadline - time.monotonic())))
            except Exception:  # noqa: BLE001 - the store raises on timeout
                live = [w for w in expected if self.store.check([keys[w]])]
        if all_or_nothing and len(live) < len(expected):
            live = []
        pub = [str(w) for w in live] + [str(w) for w in also]
        self.store.set(f"{topic}/live", ",".join(pub).encode() or b"-")
        self._collect(list(keys.values()) + [f"{topic}/live"])
        self.rendezvous_s += time.perf_counter() - t0
        return live

    def _collect(self, keys: List[str]) -> None:
        """Delete the keys of decisions that every reader has given up on or read by
        now (a reader waits at most 3 deadlines + 2 s), so the store does not grow by
        O(clerks) keys per round."""
        now = time.monotonic()
        self._garbage.append((now + 4 * self.deadline_s + 10, keys))
        while self._garbage and self._garbage[0][0] < now:
            for k in self._garbage.pop(0)[1]:
                try:
                    self.store.delete_key(k)
                except Exception:  # noqa: BLE001 - a store without delete support only grows
                    self._garbage.clear()
                    return

    def decision(self, topic: str, deadline_s: Optional[float] = None) -> List[str]:
        """The published outcome of :meth:`decide`. Blocks until it is there; a
        decider that never publishes (its process died) counts as "nobody"."""
        t = self.deadline_s if deadline_s is None else deadline_s
        t0 = time.perf_counter()
        try:
            # the decider itself may wait a full deadline for stragglers first
            self.store.wait([f"{topic}/live"], timedelta(seconds=2 * t + 2))
            v = self.store.get(f"{topic}/live").decode()
        except Exception:  # noqa: BLE001 - the store raises on timeout
            return []
        finally:
            self.rendezvous_s += time.perf_counter() - t0
        return [] if v == "-" else v.split(",")


class _Done:
    def wait(self):
        pass


class _Pending:
    def __init__(self, works, keep):
        self.works = works
        self.keep = keep  # send buffers must outlive the transfer

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
        self.keep = []
