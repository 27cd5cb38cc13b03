"""Committee routing plan properties (sda_amd/parallel/routing.py)."""
import itertools

import pytest

from sda_amd.parallel.routing import destinations, plan


CASES = [(w, n, P) for w in (1, 2, 3, 4, 8) for n in (2, 3, 5, 8) for P in (1, 7, 1000)]


@pytest.mark.parametrize("world,n,P", CASES)
def test_plan_coverage_and_balance(world, n, P):
    plans = [plan(r, world, n, P) for r in range(world)]
    # sends and receives match pairwise
    sent = sorted((r, t.peer, t.clerk, t.lo, t.hi) for r, (s, _) in enumerate(plans) for t in s)
    recv = sorted((t.peer, r, t.clerk, t.lo, t.hi) for r, (_, rv) in enumerate(plans) for t in rv)
    assert sent == recv
    for r, (sends, recvs) in enumerate(plans):
        # every source's P boxes of every clerk are sent exactly once
        for c in range(n):
            covered = sorted((t.lo, t.hi) for t in sends if t.clerk == c)
            assert covered[0][0] == 0 and covered[-1][1] == P
            assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
        # balance: each clerk region of the inbox is exactly [0, P)
        for c in range(n):
            got = sorted((t.lo, t.hi) for t in recvs if t.clerk == c)
            assert got[0][0] == 0 and got[-1][1] == P
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


@pytest.mark.parametrize("world,n", [(w, n) for w in (4, 5, 8, 16) for n in (2, 3, 5, 7) if w - 1 >= n])
def test_plan_privacy(world, n):
    for s in range(world):
        groups = destinations(s, world, n)
        flat = list(itertools.chain(*groups))
        assert s not in flat                      # never back to the participants' own GPU
        assert len(flat) == len(set(flat))        # one clerk per destination per source
        assert sorted(flat) == sorted(set(range(world)) - {s})  # all links used


def test_eight_gpus_three_clerks_link_load():
    # config 2 weak-scaled to 8 GPUs: at most ceil(P/2) boxes per link
    P = 1000
    sends, _ = plan(0, 8, 3, P)
    per_peer = {}
    for t in sends:
        per_peer[t.peer] = per_peer.get(t.peer, 0) + t.count
    assert len(per_peer) == 7 and max(per_peer.values()) <= 500
