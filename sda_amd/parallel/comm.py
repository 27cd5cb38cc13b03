"""Collectives for the aggregation engines.

With the ``nccl`` backend (RCCL on ROCm, over xGMI) tensors stay on the GPU.
With ``gloo`` (CPU tests, or several ranks sharing one GPU) device tensors are
staged through host memory, so the same engine code runs on both.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device_native = self.backend == "nccl"

    # -- staging helpers ------------------------------------------------------
    def _to_wire(self, t):
        if isinstance(t, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(t)), "numpy", None
        if t.is_cuda and not self.device_native:
            return t.cpu(), "cuda", t.device
        return t, "torch", None

    @staticmethod
    def _from_wire(w, kind, device):
        if kind == "numpy":
            return w.numpy()
        if kind == "cuda":
            return w.to(device)
        return w

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

    def reduce_sum(self, t, dst: int = 0):
        """Sum over ranks; the result on `dst`, None elsewhere."""
        w, kind, dev = self._to_wire(t)
        w = w.contiguous()
        dist.reduce(w, dst=dst, op=dist.ReduceOp.SUM, group=self.group)
        return self._from_wire(w, kind, dev) if self.rank == dst else None

    def all_reduce_max(self, value: float) -> float:
        dev = torch.device("cuda", torch.cuda.current_device()) if self.device_native else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def all_to_all_equal(self, out: torch.Tensor, inp: torch.Tensor):
        """Equal-split all-to-all of a flat buffer (rank r gets block r of every rank)."""
        w_in, kind, dev = self._to_wire(inp)
        if kind == "cuda":
            w_out = torch.empty_like(w_in)
            dist.all_to_all_single(w_out, w_in, group=self.group)
            out.copy_(w_out.to(dev))
        else:
            dist.all_to_all_single(out, w_in, group=self.group)
        return out

    def exchange_async(self, sends, recvs):
        """Start a point-to-point exchange; returns a handle with ``wait()``.

        With RCCL the grouped send/recv runs on the communicator's stream,
        which first waits for work already queued on the current stream; the
        caller keeps queuing compute and calls ``wait()`` (the current stream
        then waits for the transfer) right before consuming the receives. With
        gloo the exchange completes before returning.
        """
        if not self.device_native or (not sends and not recvs):
            self.exchange(sends, recvs)
            return _Done()
        ops = [dist.P2POp(dist.isend, t.contiguous(), p, group=self.group) for p, t in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=self.group) for p, t in recvs]
        return _Pending(dist.batch_isend_irecv(ops), [t for _, t in sends])

    def exchange(self, sends, recvs):
        """Point-to-point exchange: `sends` / `recvs` are lists of (peer, tensor).

        Transfers to/from the same peer are matched in list order; peer ==
        self must not appear (callers copy locally). With RCCL the operations
        are one grouped launch (every xGMI link busy at once); with gloo the
        device tensors are staged through host buffers.
        """
        if not sends and not recvs:
            return
        if self.device_native:
            ops = [dist.P2POp(dist.isend, t.contiguous(), p, group=self.group) for p, t in sends]
            ops += [dist.P2POp(dist.irecv, t, p, group=self.group) for p, t in recvs]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            return
        host_sends = [(p, t.contiguous().cpu() if t.is_cuda else t.contiguous()) for p, t in sends]
        host_recvs = [(p, torch.empty(t.shape, dtype=t.dtype) if t.is_cuda else t, t)
                      for p, t in recvs]
        ops = [dist.P2POp(dist.isend, t, p, group=self.group) for p, t in host_sends]
        ops += [dist.P2POp(dist.irecv, h, p, group=self.group) for p, h, _ in host_recvs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for _, h, t in host_recvs:
            if h is not t:
                t.copy_(h)

    def all_gather_object(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out


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
