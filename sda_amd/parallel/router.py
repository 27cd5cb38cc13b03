"""Committee routers: move sealed boxes from participant shards to clerk shards.

Device: ciphertext arenas (fixed-stride slots) travel as contiguous byte ranges
with their plaintext lengths -- grouped RCCL send/recv, no size pre-exchange
needed because the slot stride is fixed by (dimension, modulus). The same plan
moves just the 32-byte ephemeral-key headers ahead of the data, so the clerks'
key agreement can run while the participants are still sealing. Host: lists
of wire-format `Encryption` objects (gloo tests).
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

    # ---- generic row exchange ----------------------------------------------------
    def row_ops(self, src, dst, base: int = 0, extra=()):
        """Point-to-point ops moving rows of a clerk-major block of n*P rows.

        `src` / `dst`: [M][R] tensors (M >= base + n*P); rows [base, base+n*P)
        hold this rank's block (clerk c's participants at base + c*P ...).
        `extra`: further (src, dst) row tensors moved alongside (e.g. lengths).
        Local transfers are copied directly. Returns (sends, recvs, bytes_sent).
        """
        P, me = self.P, self.comm.rank
        pairs = [(src, dst)] + list(extra)
        sends, recvs, sent = [], [], 0

        def rows(t):
            return slice(base + t.clerk * P + t.lo, base + t.clerk * P + t.hi)

        for t in self.sends:
            r = rows(t)
            for s, d in pairs:
                if t.peer == me:
                    d[r].copy_(s[r])
                else:
                    sends.append((t.peer, s[r]))
            if t.peer != me:
                sent += src[r].numel() * src.element_size()
        for t in self.recvs:
            if t.peer == me:
                continue
            r = rows(t)
            for _, d in pairs:
                recvs.append((t.peer, d[r]))
        return sends, recvs, sent

    # ---- device arenas --------------------------------------------------------
    def exchange(self, arena):
        """Clerk-major arena [n*P] of this rank's participants -> inbox [n*P]."""
        inbox, handle = self.exchange_async(arena)
        handle.wait()
        return inbox

    def exchange_async(self, arena, inbox=None):
        """Start the exchange; returns (inbox, handle): ``handle.wait()`` before
        reading the inbox (the send arena must stay alive until then)."""
        from ..ops.sealed import Arena

        if arena.M != self.n * self.P:
            raise ValueError("arena does not match the routing plan")
        if inbox is None:
            inbox = Arena(arena.M, arena.L, arena.modulus, arena.stride, arena.K,
                          torch.empty_like(arena.ct), torch.empty_like(arena.pt_len))
        elif inbox.M != arena.M or inbox.stride != arena.stride:
            raise ValueError("inbox does not match the arena")
        src = arena.ct.view(arena.M, arena.stride)
        dst = inbox.ct.view(inbox.M, inbox.stride)
        sends, recvs, sent = self.row_ops(
            src, dst, extra=[(arena.pt_len.view(-1, 1), inbox.pt_len.view(-1, 1))])
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
