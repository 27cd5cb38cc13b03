"""Committee routers: move sealed boxes from participant shards to clerk shards.

Device: ciphertext arenas (fixed-stride slots) travel as contiguous byte ranges
with their plaintext lengths -- grouped RCCL send/recv, no size pre-exchange
needed because the slot stride is fixed by (dimension, modulus). Host: lists of
wire-format `Encryption` objects (gloo tests).
"""
from __future__ import annotations

import torch

from .comm import Comm
from .routing import plan


class CommitteeRouter:
    def __init__(self, comm: Comm, n: int, P: int):
        self.comm, self.n, self.P = comm, n, P
        self.sends, self.recvs = plan(comm.rank, comm.world, n, P)
        self.bytes_sent = 0

    # ---- device arenas --------------------------------------------------------
    def exchange(self, arena):
        """Clerk-major arena [n*P] of this rank's participants -> inbox [n*P]."""
        inbox, handle = self.exchange_async(arena)
        handle.wait()
        return inbox

    def exchange_async(self, arena):
        """Start the exchange; returns (inbox, handle): ``handle.wait()`` before
        reading the inbox (the send arena must stay alive until then)."""
        from ..ops.sealed import Arena

        P, st, me = self.P, arena.stride, self.comm.rank
        if arena.M != self.n * P:
            raise ValueError("arena does not match the routing plan")
        inbox = Arena(arena.M, arena.L, arena.modulus, st, arena.K,
                      torch.empty_like(arena.ct), torch.empty_like(arena.pt_len))

        def rng(t):
            a, b = t.clerk * P + t.lo, t.clerk * P + t.hi
            return slice(a * st, b * st), slice(a, b)

        sends, recvs, sent = [], [], 0
        for t in self.sends:
            bs, ls = rng(t)
            if t.peer == me:
                inbox.ct[bs].copy_(arena.ct[bs])
                inbox.pt_len[ls].copy_(arena.pt_len[ls])
            else:
                sends += [(t.peer, arena.ct[bs]), (t.peer, arena.pt_len[ls])]
                sent += (bs.stop - bs.start)
        for t in self.recvs:
            if t.peer == me:
                continue
            bs, ls = rng(t)
            recvs += [(t.peer, inbox.ct[bs]), (t.peer, inbox.pt_len[ls])]
        handle = self.comm.exchange_async(sends, recvs)
        self.bytes_sent = sent
        return inbox, handle

    # ---- host lists -------------------------------------------------------------
    def exchange_host(self, boxes):
        """boxes[p][c] (this rank's participants) -> inbox[c][p'] (P per clerk)."""
        outgoing = {}
        for t in self.sends:
            outgoing.setdefault(t.peer, []).append(
                (t.clerk, t.lo, t.hi, [boxes[p][t.clerk] for p in range(t.lo, t.hi)]))
        everyone = self.comm.all_gather_object(outgoing)
        inbox = [[None] * self.P for _ in range(self.n)]
        for src, out in enumerate(everyone):
            for c, lo, hi, items in out.get(self.comm.rank, []):
                inbox[c][lo:hi] = items
        return inbox
