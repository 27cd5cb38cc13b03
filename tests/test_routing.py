"""Committee plan properties (CPU): the snapshot transpose as a uniform all-to-all.

The reference transposes participations P x n into clerk jobs n x P
(server/src/snapshot.rs:11-27, server/src/stores.rs:86-101); the plan must
deliver every box exactly once, keep the clerks' load balanced, and keep two
clerks' shares of one participant off the same rank whenever there are at least
as many ranks as clerks.
"""
import itertools

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from sda_amd.parallel.routing import hosted_clerks, hosts, lead, piece, plan

CASES = [(1, 3, 7), (2, 3, 5), (3, 3, 4), (4, 3, 5), (8, 3, 1000), (8, 8, 125), (4, 8, 6),
         (3, 8, 5), (8, 26, 3), (5, 2, 9), (7, 3, 1), (8, 3, 2)]


def _deliveries(world, n, P):
    """{(dst, inbox_row): (src, clerk, participant)} from every rank's sends."""
    got = {}
    for s in range(world):
        for t in plan(s, world, n, P).sends:
            for i in range(t.count):
                key = (t.peer, t.dst_row + i)
                assert key not in got, "two boxes land on one inbox row"
                got[key] = (s, t.clerk, t.src_row - t.clerk * P + i)
    return got


@pytest.mark.parametrize("world,n,P", CASES)
def test_every_box_delivered_once_and_sends_match_recvs(world, n, P):
    got = _deliveries(world, n, P)
    assert sorted(got.values()) == sorted(itertools.product(range(world), range(n), range(P)))
    # receives mirror the sends exactly
    for r in range(world):
        pl = plan(r, world, n, P)
        mine = sorted((t.peer, t.clerk, t.src_row, t.dst_row, t.count) for t in pl.recvs if t.count)
        theirs = sorted((s, t.clerk, t.src_row, t.dst_row, t.count)
                        for s in range(world) for t in plan(s, world, n, P).sends
                        if t.peer == r and t.count)
        assert mine == theirs
        rows = sorted(row for (d, row) in got if d == r)
        assert rows == list(range(pl.inbox_rows))  # the inbox is dense


@pytest.mark.parametrize("world,n,P", CASES)
def test_balance_and_uniform_links(world, n, P):
    total = n * P
    for r in range(world):
        pl = plan(r, world, n, P)
        per_source = sum(s.count for s in pl.segments)
        assert per_source in (total // world, -(-total // world))
        assert pl.inbox_rows == world * per_source
        # every source sends this rank the same number of boxes: a uniform all-to-all
        by_src = {}
        for t in pl.recvs:
            by_src[t.peer] = by_src.get(t.peer, 0) + t.count
        assert set(by_src.values()) == ({per_source} if per_source else set())


@pytest.mark.parametrize("world,n,P", CASES)
def test_custody_and_privacy(world, n, P):
    got = _deliveries(world, n, P)
    for r in range(world):
        segs = piece(r, world, n, P)
        # a rank only receives boxes of clerks it is a host of
        assert {s.clerk for s in segs} <= set(hosted_clerks(r, world, n))
        seen = {}
        for (d, _), (src, c, p) in got.items():
            if d == r:
                seen.setdefault((src, p), set()).add(c)
        if n <= world:
            assert len(hosted_clerks(r, world, n)) <= 2
            # no rank ever holds two clerks' shares of one participant
            assert all(len(cs) == 1 for cs in seen.values())
    for c in range(n):
        hs = hosts(c, world, n)
        assert hs and lead(c, world, n) == hs[0] and hs == sorted(hs)
        # the hosts' segments partition the clerk's P slots
        cover = sorted((s.lo, s.hi) for r in hs for s in piece(r, world, n, P) if s.clerk == c)
        flat = [x for lo, hi in cover for x in range(lo, hi)]
        assert flat == list(range(P))


def test_single_rank_inbox_is_the_arena():
    pl = plan(0, 1, 3, 10)
    assert [(s.clerk, s.lo, s.hi) for s in pl.segments] == [(0, 0, 10), (1, 0, 10), (2, 0, 10)]
    assert all(t.src_row == t.dst_row for t in pl.sends)


def test_eight_ranks_eight_clerks_is_one_clerk_per_rank():
    for r in range(8):
        assert hosted_clerks(r, 8, 8) == [r]
        assert [(s.clerk, s.lo, s.hi) for s in piece(r, 8, 8, 125)] == [(r, 0, 125)]


@settings(max_examples=60, deadline=None)
@given(st.integers(1, 9), st.integers(2, 12), st.integers(1, 40))
def test_plan_properties_random(world, n, P):
    got = _deliveries(world, n, P)
    assert len(got) == world * n * P
    for c in range(n):
        assert hosts(c, world, n)


@pytest.mark.parametrize("waves", [1, 2, 4, 8, "taper"])
@pytest.mark.parametrize("P", [1, 5, 16, 24, 250, 1000])
def test_wave_bounds_cover_the_participants(waves, P):
    """The pipelined committee round cuts a rank's participants into waves (equal
    ones, or the tapered schedule with small first and last waves): consecutive,
    non-empty ranges that cover [0, P) -- every rank derives the same cut."""
    import types

    from sda_amd.parallel.device_round import DeviceCommittee

    me = types.SimpleNamespace(waves=waves, TAPER=DeviceCommittee.TAPER)
    bounds = DeviceCommittee.wave_bounds(me, P, True)
    assert bounds[0][0] == 0 and bounds[-1][1] == P
    assert all(hi > lo for lo, hi in bounds)
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    assert len(bounds) <= (6 if waves == "taper" else waves)
    assert DeviceCommittee.wave_bounds(me, P, False) == [(0, P)]
    if waves == "taper" and P >= 16:
        sizes = [hi - lo for lo, hi in bounds]
        assert sizes[0] <= sizes[2] and sizes[-1] <= sizes[-3]


def test_decode_group_size_rule():
    """Participant groups of the clerk's decode + sum: the u32 accumulators' limit is
    never exceeded, groups cover all participants, the headline shape gets ~10k blocks,
    per-clerk opens keep at least 40 participants per block, and small waves still get
    ~4k blocks."""
    from sda_amd.ops.gpu import decode_sum_group_limit
    from sda_amd.ops.sealed import decode_group_size
    for P in (1, 2, 7, 39, 40, 125, 250, 1000, 10000):
        for tr in (1, 2, 163, 489, 815, 1304, 20346 * 8):
            for m in (2, 433, 8191, 65521, 746497, 5038849, (1 << 27) - 39, 2 ** 31 - 1):
                lim = decode_sum_group_limit(m)
                pg = decode_group_size(P, tr, lim)
                assert 1 <= pg <= min(P, lim) or (pg == 1 and P >= 1)
                groups = -(-P // pg)
                assert groups * pg >= P
    lim = decode_sum_group_limit(433)
    assert 9000 <= -(-1000 // decode_group_size(1000, 489, lim)) * 489 <= 11000   # headline
    assert decode_group_size(1000, 163, lim) >= 38                                  # one clerk's row
    assert -(-125 // decode_group_size(125, 489, lim)) * 489 >= 4096                # an 8-wave slice
    # code lengths decide the limit on the lean path
    assert decode_sum_group_limit(433) == (2 ** 32 - 1) // 16383
    assert decode_sum_group_limit(746497) == (2 ** 32 - 1) // (2 ** 21 - 1)
    assert decode_sum_group_limit(5038849) == (2 ** 32 - 1) // (2 ** 28 - 1)
    # above 2^27 the accumulators are 64 bits wide: the group size is the block-count rule's
    assert decode_sum_group_limit(2 ** 31 - 1) >= 10000
    assert decode_group_size(1000, 489, decode_sum_group_limit(2 ** 31 - 1)) == \
        decode_group_size(1000, 489, lim)
