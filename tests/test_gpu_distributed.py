"""Distributed device engine on one GPU: two ranks share cuda:0 over gloo
(device tensors staged through host memory). Exercises the same
DistributedAggregator + DeviceAggregator code that runs one rank per MI355X
over RCCL; rank 0 compares with the plain PyTorch sum of both ranks' inputs.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, layout, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from sda_amd.models.schemes import PSS_4_8_3, Additive, AggregationSpec, FullMask
        from sda_amd.parallel import DistributedAggregator

        D, P, m = 5000, 6, 433
        spec = {"fullmask": AggregationSpec(D, m, Additive(3, m), FullMask(m)),
                "additive2": AggregationSpec(D, m, Additive(2, m)),
                "pss": AggregationSpec(D, m, PSS_4_8_3)}[name]
        agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", 0),
                                    layout="committee" if layout == "stream" else layout)

        def inputs(r):
            g = torch.Generator().manual_seed(99 + r)
            return torch.randint(0, m, (P, D), dtype=torch.int32, generator=g)

        if layout == "stream":
            # streamed committee round: waves of 4, pipelined exchange inside each wave
            res = agg.run_streamed(P, lambda w, first, count: inputs(rank)[first:first + count].cuda(),
                                   wave=4)
        else:
            res = agg.run_round(inputs(rank).cuda())
        if rank == 0:
            ref = torch.remainder(sum(inputs(r).to(torch.int64).sum(0) for r in range(world)), m)
            q.put(("ok", bool(torch.equal(res.output.cpu().to(torch.int64), ref))))
        else:
            q.put(("ok", res.output is None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", f"rank {rank}: {type(e).__name__}: {e}"))


@pytest.mark.parametrize("world,name,layout", [(2, "fullmask", "committee"),
                                               (2, "pss", "committee"),
                                               (2, "fullmask", "owner"),
                                               (3, "additive2", "committee"),
                                               (3, "fullmask", "stream")])
def test_distributed_device_ranks_one_gpu(cuda, world, name, layout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, layout, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r[1] for r in results if r[0] == "err"]
    assert not errs, errs
    assert all(r[1] for r in results), results


@pytest.mark.parametrize("layout", ["committee", "owner"])
def test_bench_over_rccl_single_rank(cuda, layout):
    """bench.py's distributed path on the real backend: torchrun, one rank,
    `nccl` (RCCL) process group, the pipelined committee exchange (every
    transfer is rank-local at world size 1) and the RCCL reduce / all-reduce /
    barrier calls. bench.py checks the aggregate against the reference sum in
    its first warmup round and exits non-zero on a mismatch."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "1", "--force-dist", "--layout", layout,
           "--steps", "2", "--warmup", "1", "--participants", "48", "--dim", "100000"]
    out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
