"""Who is still there: the two rendezvous points of a committee round.

A round loses nothing it can do without: a clerk whose process died after the
exchange never posts a flag, so nobody waits on a transfer from it. This is the
reference's tolerance (server/src/server.rs:119-120: a snapshot is ready with
>= reconstruction_threshold results; client/src/receive.rs:127-144: reveal
uses the results that exist) on the process group's key-value store.

Ordering rule that keeps one dead rank from cascading into time-outs elsewhere:
every rank first posts *all* its own flags (non-blocking), then takes the
decisions it owns (bounded by one common deadline), and only then reads other
ranks' decisions. A lead that spent a full deadline waiting for a dead co-host
still reaches the result rendezvous in time because that one allows two.
"""
from __future__ import annotations

import time
from typing import Iterable, List, Sequence, Set, Tuple

from .comm import Comm
from .routing import hosts, lead


def partial_stage(comm: Comm, topic: str, live: Sequence[int], n: int,
                  enabled: bool) -> Tuple[Set[int], Set[int]]:
    """Clerk-internal reduce: returns (complete, go).

    `complete`: the clerks this rank leads whose every co-host is alive (the
    lead receives one partial sum from each). `go`: the clerks this rank
    co-hosts whose lead will read its partial sum."""
    me, W = comm.rank, comm.world
    led, cohosted = [], []
    for c in live:
        hs = hosts(c, W, n)
        if me == hs[0]:
            led.append((c, hs[1:]))
        elif me in hs:
            cohosted.append(c)
    if not enabled or W == 1:
        return {c for c, _ in led}, set(cohosted)
    for c in cohosted:
        comm.arrive(f"{topic}/c{c}", me)
    t_end = time.monotonic() + comm.deadline_s
    complete = set()
    for c, others in led:
        if others:
            got = comm.decide(f"{topic}/c{c}", others, all_or_nothing=True,
                              deadline_s=max(0.05, t_end - time.monotonic()))
            if len(got) < len(others):
                continue
        complete.add(c)
    go = {c for c in cohosted if str(me) in comm.decision(f"{topic}/c{c}")}
    return complete, go


def result_stage(comm: Comm, topic: str, live: Sequence[int], n: int, enabled: bool,
                 ready: Iterable[int], root: int) -> List[int]:
    """Sealed results -> recipient: `ready` are the clerks this rank leads and
    has a sealed result for. Returns the clerks (in `live` order) whose results
    the recipient will read -- the same list on every rank that is alive."""
    me, W = comm.rank, comm.world
    ready = list(ready)
    if not enabled or W == 1:
        return list(live)
    if me == root:
        remote = [c for c in live if lead(c, W, n) != root]
        got = set(comm.decide(f"{topic}/res", remote, also=ready,
                              deadline_s=2 * comm.deadline_s + 1)) | set(ready)
    else:
        for c in ready:
            comm.arrive(f"{topic}/res", c)
        got = set(int(x) for x in comm.decision(f"{topic}/res", deadline_s=3 * comm.deadline_s + 2))
    return [c for c in live if c in got]
