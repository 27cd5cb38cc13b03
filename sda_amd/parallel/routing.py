"""Committee plan: which rank plays which clerk for which participants.

This is the reference's snapshot transpose (server/src/snapshot.rs:4-47,
server/src/stores.rs:86-101: participations P x n -> clerk jobs n x P) as an
on-node all-to-all over xGMI, plus the clerk -> recipient result path
(client/src/clerk.rs:99-100, client/src/receive.rs:127-138).

Every source rank s holds, clerk-major, the sealed boxes of its P participants
for all n clerks: a *line* of n * P slots, slot c * P + p = participant p's box
for clerk c. The line is cut into `world` equal pieces and piece r goes to rank
r -- from every source alike, so the exchange is a uniform all-to-all (every
xGMI link of the fully connected node carries the same n * P / world boxes,
the self piece stays local). A piece is at most two *segments* when n <=
world: the tail of one clerk's slots and the head of the next one's.

    world 8, n 3, P 1000: pieces of 375 slots
      rank 0: clerk 0 [0, 375)      rank 2: clerk 0 [750, 1000) + clerk 1 [0, 125)
      rank 1: clerk 0 [375, 750)    rank 3: clerk 1 [125, 500)   ...

Properties (tests/test_routing.py):
  * coverage   every box is received exactly once;
  * balance    every rank opens world * (n * P / world) = n * P boxes, the
               one-GPU clerk load, whatever world and n;
  * custody    rank r needs only the secret keys of the clerks in its piece
               (``hosts``): one or two clerks when n <= world;
  * privacy    when n <= world the participant ranges of a rank's two
               segments are disjoint, so no rank ever holds two clerks' shares
               of one participant (with n > world a rank necessarily plays
               several whole clerks, as the single GPU does);
  * leads      clerk c's lowest host (``lead``) collects its co-hosts' partial
               sums, seals the combined shares for the recipient and sends that
               one box to the recipient's rank.

A rank's inbox is segment-major, source-major inside a segment: segment i
starts at ``offsets[i]`` and holds ``world * (hi - lo)`` boxes, source s's at
``offsets[i] + s * (hi - lo)`` -- so one clerk's boxes are contiguous and the
open + combine kernels see a [rows][boxes] shape as on one GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from typing import List, Tuple


@dataclass(frozen=True)
class Segment:
    clerk: int
    lo: int   # participant range [lo, hi) within every source's P participants
    hi: int

    @property
    def count(self) -> int:
        return self.hi - self.lo


@dataclass(frozen=True)
class Transfer:
    peer: int      # destination (for sends) or source (for receives)
    clerk: int
    src_row: int   # first row in the source's clerk-major arena (c * P + lo)
    dst_row: int   # first row in the destination's inbox
    count: int


def piece(rank: int, world: int, n: int, P: int) -> List[Segment]:
    """The segments of rank `rank`'s piece of every source's line."""
    total = n * P
    a, b = rank * total // world, (rank + 1) * total // world
    segs: List[Segment] = []
    x = a
    while x < b:
        c = x // P
        hi = min(P, b - c * P)
        segs.append(Segment(c, x - c * P, hi))
        x = c * P + hi
    return segs


def hosts(clerk: int, world: int, n: int) -> List[int]:
    """Ranks that play (a slice of) `clerk`, independent of P: the ranks whose
    share [r n / world, (r + 1) n / world) of the clerk axis overlaps [c, c + 1)."""
    return [r for r in range(world) if clerk * world < (r + 1) * n and r * n < (clerk + 1) * world]


def lead(clerk: int, world: int, n: int) -> int:
    return hosts(clerk, world, n)[0]


def hosted_clerks(rank: int, world: int, n: int) -> List[int]:
    return [c for c in range(n) if rank in hosts(c, world, n)]


@dataclass(frozen=True)
class Plan:
    """Rank `rank`'s view of the exchange of P-participant shards."""
    rank: int
    world: int
    n: int
    P: int
    segments: Tuple[Segment, ...]   # this rank's inbox segments
    offsets: Tuple[int, ...]        # first inbox row of each segment
    inbox_rows: int
    sends: Tuple[Transfer, ...]
    recvs: Tuple[Transfer, ...]

    def segment_rows(self, i: int) -> Tuple[int, int]:
        """(first inbox row, row count) of segment i."""
        return self.offsets[i], self.world * self.segments[i].count


@lru_cache(maxsize=256)
def plan(rank: int, world: int, n: int, P: int) -> Plan:
    def layout(r):
        segs = piece(r, world, n, P)
        offs, o = [], 0
        for s in segs:
            offs.append(o)
            o += world * s.count
        return segs, offs, o

    segs, offs, rows = layout(rank)
    sends: List[Transfer] = []
    for d in range(world):
        dsegs, doffs, _ = layout(d)
        for s, o in zip(dsegs, doffs):
            sends.append(Transfer(d, s.clerk, s.clerk * P + s.lo, o + rank * s.count, s.count))
    recvs: List[Transfer] = []
    for src in range(world):
        for s, o in zip(segs, offs):
            recvs.append(Transfer(src, s.clerk, s.clerk * P + s.lo, o + src * s.count, s.count))
    return Plan(rank, world, n, P, tuple(segs), tuple(offs), rows, tuple(sends), tuple(recvs))
