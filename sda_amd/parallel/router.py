"""Row movers: carry fixed-stride rows between ranks along a committee plan.

Sealed boxes live in fixed-stride slots (the device ciphertext arena, or the
host engines' length-prefixed rows), so the snapshot transpose needs no size
pre-exchange: a transfer is a contiguous run of rows on both sides. The same
plan moves the 32-byte ephemeral-key headers ahead of the data, so the clerks'
key agreement overlaps the participants' sealing.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import torch

from .comm import Comm
from .routing import Plan


class RowRouter:
    def __init__(self, comm: Comm, plan: Plan):
        if plan.rank != comm.rank or plan.world != comm.world:
            raise ValueError("plan does not belong to this rank")
        self.comm, self.plan = comm, plan

    def ops(self, pairs: Sequence[Tuple[torch.Tensor, torch.Tensor]], src_base: int = 0,
            dst_base: int = 0, kind: str = "box"):
        """Point-to-point ops moving the plan's rows of every (src, dst) pair.

        `src`: [>= src_base + n*P][R] clerk-major rows of this rank's
        participants; `dst`: [>= dst_base + inbox_rows][R] inbox rows. Rows
        that stay on this rank are copied directly (on the current stream).
        Returns (sends, recvs) for :meth:`Comm.exchange_async`.
        """
        me = self.comm.rank
        loop = self.comm.loopback  # the own piece travels like any other
        sends, recvs = [], []
        for t in self.plan.sends:
            if t.count == 0:
                continue
            s = slice(src_base + t.src_row, src_base + t.src_row + t.count)
            if t.peer == me and not loop:
                d = slice(dst_base + t.dst_row, dst_base + t.dst_row + t.count)
                for src, dst in pairs:
                    if dst.data_ptr() != src.data_ptr() or s != d:
                        dst[d].copy_(src[s])
                continue
            for src, _ in pairs:
                rows = src[s]
                sends.append((t.peer, rows))
                self.comm.note(kind, "send", t.peer, t.clerk, rows.numel() * rows.element_size())
        for t in self.plan.recvs:
            if t.count == 0 or (t.peer == me and not loop):
                continue
            d = slice(dst_base + t.dst_row, dst_base + t.dst_row + t.count)
            for _, dst in pairs:
                rows = dst[d]
                recvs.append((t.peer, rows))
                self.comm.note(kind, "recv", t.peer, t.clerk, rows.numel() * rows.element_size())
        return sends, recvs


def gather_rows_to(comm: Comm, root: int, pairs: Iterable[Tuple[torch.Tensor, torch.Tensor]],
                   rows_per_rank: int, kind: str, senders: Sequence[int] | None = None):
    """Every rank in `senders` (default: all) sends its `rows_per_rank` rows of
    each `src` to `root`, which places rank r's at rows [r * rows_per_rank, ...)
    of `dst`. Returns (sends, recvs)."""
    me = comm.rank
    loop = comm.loopback
    senders = list(range(comm.world)) if senders is None else list(senders)
    sends, recvs = [], []
    for src, dst in pairs:
        if me in senders:
            if me == root and not loop:
                dst[me * rows_per_rank:(me + 1) * rows_per_rank].copy_(src[:rows_per_rank])
            else:
                rows = src[:rows_per_rank]
                sends.append((root, rows))
                comm.note(kind, "send", root, -1, rows.numel() * rows.element_size())
        if me == root:
            for r in senders:
                if r != root or loop:
                    rows = dst[r * rows_per_rank:(r + 1) * rows_per_rank]
                    recvs.append((r, rows))
                    comm.note(kind, "recv", r, -1, rows.numel() * rows.element_size())
    return sends, recvs
