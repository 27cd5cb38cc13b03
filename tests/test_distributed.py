"""Multi-process aggregation over torch.distributed (CPU, gloo).

The same DistributedAggregator that runs one rank per MI355X over RCCL is run
here with the host engine on gloo: per-rank key custody, per-rank participant
shards, the all-to-all of sealed boxes, the clerk-internal partial reduce, the
sealed results gathered on rank 0, the recipient stage. Rank 0 checks the output
against the plain sum of every rank's inputs; every rank reports its transfer
audit so the tests can assert what travelled where.

Reference behaviour covered: snapshot transpose (server/src/snapshot.rs:11-27),
clerk result sealing (client/src/clerk.rs:79-100), reveal from the results that
exist (client/src/receive.rs:127-144, server/src/server.rs:119-120).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sda_amd.models.schemes import (PSS_4_8_3, Additive, AggregationSpec, ChaChaMask, FullMask,
                                    pss_5_of_8)
from sda_amd.parallel.routing import hosted_clerks, hosts


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spec(name, D):
    if name == "additive":
        return AggregationSpec(D, 433, Additive(3, 433))
    if name == "fullmask":
        return AggregationSpec(D, 433, Additive(3, 433), FullMask(433))
    if name == "chachamask":
        return AggregationSpec(D, 433, Additive(3, 433), ChaChaMask(433, D))
    if name == "pss":
        return AggregationSpec(D, 433, PSS_4_8_3)
    if name == "pssmask":
        return AggregationSpec(D, 433, PSS_4_8_3, FullMask(433))
    if name == "pss5of8":
        return AggregationSpec(D, 433, pss_5_of_8())
    if name == "bigmod":
        return AggregationSpec(D, 2 ** 31 - 1, Additive(4, 2 ** 31 - 1))
    raise ValueError(name)


def _inputs(rank, P, D, m):
    rng = np.random.default_rng(1234 + rank)
    return rng.integers(0, m, size=(P, D), dtype=np.int64)


def _exit_after(q, msg):
    """Report and leave without any teardown (the queue's feeder thread must
    have flushed before the process image goes away)."""
    q.put(msg)
    q.close()
    q.join_thread()
    os._exit(0)


def _worker(rank, world, port, name, P, D, clerks, layout, die, die_stage, q):
    import datetime

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=120))
        from sda_amd.parallel import DistributedAggregator

        def hook(stage, r):
            if stage == die_stage and r in die:
                # the process is gone: no result flag, no further traffic
                _exit_after(q, ("died", rank))

        spec = _spec(name, D)
        agg = DistributedAggregator(spec, engine="host", layout=layout, deadline_s=4.0,
                                    fault_hook=hook if die else None)
        held = [i for i, s in enumerate(agg.engine.keys.sks) if s is not None]
        agg.comm.reset_audit()
        try:
            res = agg.run_round(_inputs(rank, P, D, spec.field_modulus), clerks=clerks)
        except Exception as e:  # noqa: BLE001
            q.put(("raised", rank, f"{type(e).__name__}: {e}"))
            if rank == 0:
                # rank 0 also serves the rendezvous store: let the survivors finish
                # their round against it before this process goes away
                import time

                time.sleep(14)
            _exit_after(q, ("bye", rank))
        info = {"rank": rank, "held": held, "audit": list(agg.comm.audit),
                "used": list(res.clerks_used)}
        if rank == 0:
            expect = sum(_inputs(r, P, D, spec.field_modulus).sum(0) for r in range(world))
            expect = np.remainder(expect, spec.field_modulus)
            info["ok"] = bool(np.array_equal(res.output, expect))
        else:
            info["ok"] = res.output is None
        if die:
            _exit_after(q, ("ok", rank, info))  # peers are gone: no collective teardown
        q.put(("ok", rank, info))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", rank, f"rank {rank}: {type(e).__name__}: {e}"))


def _run(world, name, P=3, D=17, clerks=None, layout="committee", die=(),
         die_stage="before_results"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, name, P, D, clerks, layout, tuple(die), die_stage, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = []
    while len([r for r in results if r[0] != "bye"]) < world:
        results.append(q.get(timeout=300))
    for p in procs:
        p.join(timeout=60)
    return [r for r in results if r[0] != "bye"]


def _check_ok(results, world):
    errs = [r for r in results if r[0] in ("err", "raised")]
    assert not errs, errs
    infos = {r[1]: r[2] for r in results if r[0] == "ok"}
    assert len(infos) == world and all(i["ok"] for i in infos.values()), results
    return infos


def _check_custody(infos, world, n):
    """Key custody and plaintext confinement of the committee layout."""
    for r, info in infos.items():
        mine = hosted_clerks(r, world, n)
        # exactly the hosted clerks' secret keys; the recipient's only on rank 0
        assert info["held"] == mine + ([n] if r == 0 else []), (r, info["held"], mine)
        for kind, direction, peer, clerk, nbytes in info["audit"]:
            assert kind in ("box", "mask", "partial", "result", "hdr"), kind
            if kind == "partial":
                # plaintext partial sums stay among the hosts of that clerk, towards its lead
                assert clerk in mine and peer in hosts(clerk, world, n), (r, peer, clerk)
                if direction == "recv":
                    assert hosts(clerk, world, n)[0] == r
            if kind == "box" and direction == "recv":
                assert clerk in mine  # sealed boxes only reach ranks that play the clerk
            if kind in ("result", "mask") and direction == "send":
                assert peer == 0  # sealed results / masks go to the recipient's rank


@pytest.mark.parametrize("layout", ["committee", "owner"])
@pytest.mark.parametrize("name", ["additive", "fullmask", "chachamask", "pss", "bigmod"])
def test_distributed_two_ranks(native, name, layout):
    infos = _check_ok(_run(2, name, layout=layout), 2)
    if layout == "committee":
        _check_custody(infos, 2, _spec(name, 17).n_clerks)


@pytest.mark.parametrize("layout", ["committee", "owner"])
def test_distributed_three_ranks_pss_dropout_by_argument(native, layout):
    _check_ok(_run(3, "pss5of8", P=2, D=10, clerks=[0, 2, 3, 5, 7], layout=layout), 3)


@pytest.mark.parametrize("world,name", [(4, "additive"), (4, "pssmask"), (8, "additive"),
                                        (8, "pss"), (8, "fullmask")])
def test_committee_custody_world_4_and_8(native, world, name):
    """n = 3 (clerks spanning several ranks, two-clerk ranks) and n = 8 (one
    clerk per rank at world 8, two per rank at world 4)."""
    infos = _check_ok(_run(world, name, P=4, D=11), world)
    n = _spec(name, 11).n_clerks
    _check_custody(infos, world, n)
    if n < world:  # some clerk spans several ranks: its partials were reduced on its lead
        assert any(k == "partial" for i in infos.values() for k, *_ in i["audit"])
    else:
        assert not any(k == "partial" for i in infos.values() for k, *_ in i["audit"])


def test_clerk_rank_dies_before_the_gather(native):
    """World 8, PSS_4_8_3 (t + k = 7 of 8): one clerk's process exits after the
    exchange without posting its result; the recipient reconstructs from the 7
    that arrived."""
    results = _run(8, "pss", P=2, D=10, die=(5,))
    assert ("died", 5) in results
    ok = {r[1]: r[2] for r in results if r[0] == "ok"}
    assert not [r for r in results if r[0] in ("err", "raised")], results
    assert sorted(ok) == [0, 1, 2, 3, 4, 6, 7]
    assert ok[0]["ok"] and ok[0]["used"] == [0, 1, 2, 3, 4, 6, 7]


def test_too_many_clerk_ranks_die(native):
    """Two of eight clerks lost leaves 6 < t + k = 7 results: a clear error on
    the recipient, no hang anywhere."""
    results = _run(8, "pss", P=2, D=10, die=(3, 6))
    raised = [r for r in results if r[0] == "raised"]
    assert len(raised) == 1 and raised[0][1] == 0, results
    assert "Not enough clerk results" in raised[0][2] and "6 of 8" in raised[0][2]
    assert sorted(r[1] for r in results if r[0] == "ok") == [1, 2, 4, 5, 7]


@pytest.mark.parametrize("stage", ["before_partials", "before_results"])
def test_host_of_a_spanning_clerk_dies(native, stage):
    """With n = 3 < world = 4 every clerk spans two ranks. Rank 1 (co-host of
    clerk 0, lead of clerk 1) dies: the clerks it took part in lose their
    results; additive sharing needs all three, so the round fails cleanly on
    the recipient -- and nobody hangs on the dead rank."""
    results = _run(4, "additive", P=4, D=9, die=(1,), die_stage=stage)
    assert ("died", 1) in results
    raised = [r for r in results if r[0] == "raised"]
    assert len(raised) == 1 and raised[0][1] == 0 and "Not enough clerk results" in raised[0][2]
    assert sorted(r[1] for r in results if r[0] == "ok") == [2, 3]


def test_clerk_rank_dies_between_the_rendezvous_and_its_transfer(native):
    """The window the rendezvous cannot close: rank 5 posts its result flag, is
    counted in by the recipient, and exits before its sealed result has left.
    The recipient's receive from it must fail -- a raised error and a process
    that ends, not a hang -- and ranks that have nothing to do with rank 5
    finish their round."""
    import time

    t0 = time.monotonic()
    results = _run(8, "pss", P=2, D=10, die=(5,), die_stage="before_result_transfer")
    assert time.monotonic() - t0 < 110  # below the workers' 120 s process-group timeout
    assert ("died", 5) in results
    raised = [r for r in results if r[0] == "raised"]
    assert [r[1] for r in raised] == [0], results
    assert "Not enough clerk results" not in raised[0][2]  # a transport error, not a decision
    assert sorted(r[1] for r in results if r[0] == "ok") == [1, 2, 3, 4, 6, 7]


def test_host_engine_single_process(native):
    from sda_amd.host_engine import HostAggregator

    for name in ["additive", "fullmask", "chachamask", "pss"]:
        spec = _spec(name, 11)
        x = _inputs(0, 4, 11, 433)
        res = HostAggregator(spec).run_round(x)
        assert np.array_equal(res.output, np.remainder(x.sum(0), 433)), name
