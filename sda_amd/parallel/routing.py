"""Committee routing: where each participant shard's sealed boxes go.

This is the reference's snapshot transpose (server/src/snapshot.rs:4-47,
server/src/stores.rs:86-101: participations P x n -> clerk jobs n x P) as an
on-node data movement plan over xGMI.

Source rank s holds, clerk-major, the sealed boxes of its P participants for
every clerk c. With N ranks and n clerks:

* N - 1 >= n (the normal case): the other N - 1 ranks, at offsets
  k = 0..N-2 (rank s+1+k), are split into n groups by k mod n; clerk c's P
  boxes are cut into |group c| contiguous parts, part j going to the j-th rank
  of group c. Properties (tests/test_routing.py):
    - privacy: a rank never receives two clerks' shares of the same
      participant, nor its own participants' boxes;
    - balance: every rank receives exactly P boxes per clerk (n * P in all, the
      single-GPU clerk load), whatever N and n;
    - bandwidth: the traffic spreads over all N - 1 peers (xGMI links), about
      n * P / (N - 1) boxes per link.
* N - 1 < n (too few ranks to keep clerks apart): clerk c's whole piece goes to
  rank s+1+c mod N (possibly s itself). Balance still holds.

Every rank's inbox is clerk-major with exactly P slots per clerk, so the open +
combine kernels see the same [n][P][B] shape as on one GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple


@dataclass(frozen=True)
class Transfer:
    peer: int     # destination (for sends) or source (for receives)
    clerk: int
    lo: int       # participant range [lo, hi) within the clerk's P slots
    hi: int

    @property
    def count(self) -> int:
        return self.hi - self.lo


def destinations(src: int, world: int, n: int) -> List[List[int]]:
    """Per clerk, the ordered destination ranks of source `src`'s boxes."""
    if world - 1 >= n:
        groups: List[List[int]] = [[] for _ in range(n)]
        for k in range(world - 1):
            groups[k % n].append((src + 1 + k) % world)
        return groups
    return [[(src + 1 + c) % world] for c in range(n)]


def parts(P: int, g: int) -> List[Tuple[int, int]]:
    return [(P * j // g, P * (j + 1) // g) for j in range(g)]


def plan(rank: int, world: int, n: int, P: int) -> Tuple[List[Transfer], List[Transfer]]:
    """(sends, receives) of `rank`; every rank has the same P."""
    sends: List[Transfer] = []
    for c, group in enumerate(destinations(rank, world, n)):
        for d, (lo, hi) in zip(group, parts(P, len(group))):
            if hi > lo:
                sends.append(Transfer(d, c, lo, hi))
    recvs: List[Transfer] = []
    for s in range(world):
        for c, group in enumerate(destinations(s, world, n)):
            for d, (lo, hi) in zip(group, parts(P, len(group))):
                if d == rank and hi > lo:
                    recvs.append(Transfer(s, c, lo, hi))
    return sends, recvs
