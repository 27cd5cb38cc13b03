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
        from sda_amd.models.schemes import (PSS_4_8_3, Additive, AggregationSpec, ChaChaMask,
                                            FullMask)
        from sda_amd.parallel import DistributedAggregator

        D, P, m = 5000, 6, 433
        if name == "bigmod":
            m = 2 ** 31 - 1
        spec = {"fullmask": AggregationSpec(D, m, Additive(3, m), FullMask(m)),
                "additive2": AggregationSpec(D, m, Additive(2, m)),
                "chacha": AggregationSpec(D, m, Additive(3, m), ChaChaMask(m, D)),
                "bigmod": AggregationSpec(D, m, Additive(4, m), FullMask(m)),
                "pss": AggregationSpec(D, m, PSS_4_8_3)}[name]
        agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", 0),
                                    layout="owner" if layout == "owner" else "committee",
                                    waves=3, force_pipeline=True, deadline_s=30.0,
                                    strict_liveness=layout == "strict")
        # key custody: only the hosted clerks' secret keys (+ the recipient's on rank 0)
        if layout != "owner":
            from sda_amd.parallel.routing import hosted_clerks

            held = [i for i in range(spec.n_clerks + 1) if agg.engine.keys.holds(i)]
            want = hosted_clerks(rank, world, spec.n_clerks) + ([spec.n_clerks] if rank == 0 else [])
            assert held == want, (held, want)

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
            assert res.output is not None
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
                                               (4, "chacha", "committee"),
                                               # sums of waves of values below m = 2^31 - 1
                                               # must not wrap (pipelined waves, world 1 and 2)
                                               (1, "bigmod", "committee"),
                                               (2, "bigmod", "committee"),
                                               (3, "fullmask", "stream"),
                                               # liveness flags posted only once the GPU has
                                               # finished the work in front of the stage
                                               (2, "pss", "strict"), (3, "additive2", "strict")])
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
    assert line["hbm_high_water_bytes"] > 0 and line["xgmi"]["bytes_sent_per_rank_per_round"] == 0
    assert ("committee" in line["config"]["parallelism"]) == (layout == "committee")
    assert ("non-private upper bound" in line["config"]["parallelism"]) == (layout == "owner")


@pytest.mark.parametrize("dist", [False, True])
def test_bench_fails_on_a_corrupted_box_in_a_timed_step(cuda, dist):
    """A flipped ciphertext bit in a timed (unchecked) step must fail the run:
    the error words of all timed steps are OR-ed on device and read once."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tail = ["--gpus", "1", "--steps", "3", "--warmup", "1", "--participants", "24", "--dim",
            "60000", "--corrupt-step", "1"]
    if dist:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(root, "bench.py"), "--force-dist"] + tail
    else:
        cmd = [sys.executable, os.path.join(root, "bench.py")] + tail
    out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert out.returncode != 0
    assert "MAC verification failed" in out.stderr, out.stderr[-2000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_bench_loopback_over_rccl(cuda):
    """One rank, `nccl` group, loopback: the rank's own piece of the header
    exchange (side stream), of every wave's box exchange and of the result path
    travels through grouped RCCL isend/irecv to itself, so the point-to-point path
    and its stream ordering against the compute streams run on a one-GPU machine.
    The process-group timeout is short: a self send/recv that RCCL cannot match
    fails the test instead of hanging it."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--force-dist",
           "--loopback", "--waves", "3", "--dist-timeout", "60", "--steps", "2", "--warmup", "1",
           "--participants", "48", "--dim", "100000", "--check"]
    out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and "loopback" in line["config"]["parallelism"]


def _loopback_worker(port, name, q):
    import datetime

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                                timeout=datetime.timedelta(seconds=60))
        from sda_amd.models.schemes import PSS_4_8_3, Additive, AggregationSpec, FullMask
        from sda_amd.parallel import DistributedAggregator

        D, P, m = 5000, 12, 433
        spec = {"fullmask": AggregationSpec(D, m, Additive(3, m), FullMask(m)),
                "pss": AggregationSpec(D, m, PSS_4_8_3)}[name]
        agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", 0),
                                    waves=3, force_pipeline=True, deadline_s=15.0, loopback=True)
        x = torch.randint(0, m, (P, D), dtype=torch.int32, device="cuda")
        ok = True
        for _ in range(3):  # several rounds: send buffers and events are recycled
            res = agg.run_round(x)
            ok = ok and bool(torch.equal(res.output.cpu().to(torch.int64),
                                         torch.remainder(x.cpu().to(torch.int64).sum(0), m)))
        sent = sorted({k for k, d, *_ in agg.comm.audit if d == "send"})
        q.put(("ok", ok, sent))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", f"{type(e).__name__}: {e}", []))


@pytest.mark.parametrize("name", ["fullmask", "pss"])
def test_loopback_rounds_with_masks_and_pss_over_rccl(cuda, name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_loopback_worker, args=(_free_port(), name, q))
    p.start()
    kind, ok, sent = q.get(timeout=200)
    p.join(timeout=60)
    assert kind == "ok" and ok, (kind, ok)
    # everything that would cross xGMI went through send/recv: headers, boxes, results
    assert {"hdr", "box", "result"} <= set(sent), sent
    if name == "fullmask":
        assert "mask" in sent
