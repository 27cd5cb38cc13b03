"""Multi-process aggregation over torch.distributed (CPU, gloo).

The same DistributedAggregator that runs one rank per MI355X over RCCL is run
here with the host engine on gloo: key broadcast from rank 0, per-rank
participant shards, bucketed reduce of clerk partials, recipient stage on
rank 0. Rank 0 checks the output against the plain sum of every rank's inputs.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sda_amd.models.schemes import (PSS_4_8_3, Additive, AggregationSpec, ChaChaMask, FullMask,
                                    pss_5_of_8)


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
    if name == "pss5of8":
        return AggregationSpec(D, 433, pss_5_of_8())
    if name == "bigmod":
        return AggregationSpec(D, 2 ** 31 - 1, Additive(4, 2 ** 31 - 1))
    raise ValueError(name)


def _inputs(rank, P, D, m):
    rng = np.random.default_rng(1234 + rank)
    return rng.integers(0, m, size=(P, D), dtype=np.int64)


def _worker(rank, world, port, name, P, D, clerks, layout, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from sda_amd.parallel import DistributedAggregator

        spec = _spec(name, D)
        agg = DistributedAggregator(spec, engine="host", layout=layout)
        res = agg.run_round(_inputs(rank, P, D, spec.field_modulus), clerks=clerks)
        if rank == 0:
            expect = sum(_inputs(r, P, D, spec.field_modulus).sum(0) for r in range(world))
            expect = np.remainder(expect, spec.field_modulus)
            q.put(("ok", bool(np.array_equal(res.output, expect))))
        else:
            q.put(("ok", res.output is None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", f"rank {rank}: {type(e).__name__}: {e}"))


def _run(world, name, P=3, D=17, clerks=None, layout="committee"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, P, D, clerks, layout, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs
    assert all(r[1] for r in results), results


@pytest.mark.parametrize("layout", ["committee", "owner"])
@pytest.mark.parametrize("name", ["additive", "fullmask", "chachamask", "pss", "bigmod"])
def test_distributed_two_ranks(native, name, layout):
    _run(2, name, layout=layout)


@pytest.mark.parametrize("layout", ["committee", "owner"])
def test_distributed_three_ranks_pss_dropout(native, layout):
    _run(3, "pss5of8", P=2, D=10, clerks=[0, 2, 3, 5, 7], layout=layout)


def test_distributed_four_ranks_committee_spread(native):
    # N - 1 >= n: boxes split over every peer, one clerk per (source, destination)
    _run(4, "fullmask", P=5, D=9)


def test_host_engine_single_process(native):
    from sda_amd.host_engine import HostAggregator

    for name in ["additive", "fullmask", "chachamask", "pss"]:
        spec = _spec(name, 11)
        x = _inputs(0, 4, 11, 433)
        res = HostAggregator(spec).run_round(x)
        assert np.array_equal(res.output, np.remainder(x.sum(0), 433)), name
