#!/usr/bin/env python3
"""Runs the BASELINE.json configs and prints one JSON line each (rank 0).

  --config 1  CLI plumbing: sdad + sda walkthrough, 3 x 10-dim, m=433, additive-3
              (expected reveal 0 2 2 4 4 6 6 8 8 10)
  --config 2  1k x 1M, additive-3 on the GPU(s)                 (= bench.py)
  --config 3  1k x 1M per GPU, Packed Shamir k=3 n=8 (PSS_4_8_3), committee layout
  --config 4  10k x 125M (GPT-2-small gradient), PSS_4_8_3 (8 clerks), streamed in
              participant waves with accumulator checkpoints
  --config 5  1k x 1M per GPU, packed Shamir 5-of-8 (t=2, k=3) with 3 clerks dropped

Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench_configs.py --config 3
Scaled-down runs: --participants / --dim override the per-rank sizes.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

# RCCL (one stream per P2P peer) + the engine's side stream need more than the
# default 4 hardware queues per process, or streams get multiplexed onto one
# queue and serialise (measured: +6 ms per round). Must precede HIP init.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--participants", type=int, default=None, help="per rank")
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--wave", type=int, default=None, help="participants per wave (config 4)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--layout", default="committee", choices=["committee", "owner"])
    ap.add_argument("--checkpoint", default=None, help="config 4 accumulator checkpoint path")
    ap.add_argument("--check", action="store_true", help="verify against a plain sum")
    return ap.parse_args()


def emit(d):
    print(json.dumps(d), flush=True)


def config1():
    """The reference README walkthrough through our binaries (CPU)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from sda_amd._native import bin_path

    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as tmp:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        srv = subprocess.Popen([bin_path("sdad"), "--jfs", f"{tmp}/server", "httpd", "-b",
                                f"127.0.0.1:{port}"], stdout=subprocess.PIPE, text=True)
        srv.stdout.readline()
        url = f"http://127.0.0.1:{port}"

        def sda(ident, *a):
            r = subprocess.run([bin_path("sda"), "-s", url, "-i", f"{tmp}/agent/{ident}", *a],
                               capture_output=True, text=True, timeout=60)
            if r.returncode:
                raise SystemExit(r.stderr)
            return r.stdout
        try:
            for i in ["recipient", "clerk-1", "clerk-2", "clerk-3"]:
                sda(i, "agent", "create")
                sda(i, "agent", "keys", "create")
            for i in ["part-1", "part-2", "part-3"]:
                sda(i, "agent", "create")
            key = sda("recipient", "agent", "keys", "show").split()[0]
            agg = "ad3142d8-9a83-4f40-a64a-a8c90b701bde"
            sda("recipient", "aggregations", "create", "--id", agg, "aggro", "10", "433", key, "3")
            sda("recipient", "aggregations", "begin", agg)
            sda("part-1", "participate", agg, *"0 1 2 3 4 5 6 7 8 9".split())
            sda("part-2", "participate", agg, *"0 0 0 0 0 0 0 0 0 0".split())
            sda("part-3", "participate", agg, *"0 1 0 1 0 1 0 1 0 1".split())
            sda("recipient", "aggregations", "end", agg)
            for i in ["recipient", "clerk-1", "clerk-2", "clerk-3"]:
                sda(i, "clerk", "--once")
            out = sda("recipient", "aggregations", "reveal", agg)
        finally:
            srv.terminate()
            srv.wait(timeout=10)
    vals = [int(v) for v in out.split("values: [")[1].split("]")[0].split(",")]
    emit({"config": 1, "output": vals, "expected": [0, 2, 2, 4, 4, 6, 6, 8, 8, 10],
          "correct": vals == [0, 2, 2, 4, 4, 6, 6, 8, 8, 10],
          "seconds": time.perf_counter() - t0})


def gpu_configs(args):
    import torch
    import torch.distributed as dist

    from sda_amd.engine import DeviceAggregator
    from sda_amd.models import PSS_4_8_3, Additive, AggregationSpec, pss_5_of_8

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    c = args.config
    m = 433
    P = args.participants or (10000 // world if c == 4 else 1000)
    D = args.dim or (125_000_000 if c == 4 else 1_000_000)
    sharing = {2: Additive(3, m), 3: PSS_4_8_3, 4: PSS_4_8_3, 5: pss_5_of_8(m)}[c]
    spec = AggregationSpec(D, m, sharing)
    clerks = [0, 2, 3, 5, 7] if c == 5 else None  # config 5: clerks 1, 4, 6 dropped

    if world > 1:
        from sda_amd.parallel import DistributedAggregator

        agg = DistributedAggregator(spec, engine="device", device=dev, layout=args.layout)
        eng = agg.engine
    else:
        agg, eng = None, DeviceAggregator(spec, device=dev)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            agg.comm.barrier()

    def gen(seed, count):
        g = torch.Generator(device=dev).manual_seed(seed)
        return torch.randint(0, m, (count, D), dtype=torch.int32, device=dev, generator=g)

    ok = None
    if c == 4:
        wave = args.wave or 32
        ck = (args.checkpoint + f".rank{rank}") if args.checkpoint else None

        def make(w, first, count):
            return gen(1000 * (rank + 1) + w, count)
        sync()
        t0 = time.perf_counter()
        if world > 1:
            res = agg.run_streamed(P, make, wave=wave, checkpoint=ck)
        else:
            from sda_amd.streaming import StreamingAggregator

            res = StreamingAggregator(eng, wave=wave, checkpoint=ck).run(P, make)
        sync()
        secs = time.perf_counter() - t0
        if world > 1:
            secs = agg.comm.all_reduce_max(secs)
        if args.check and world == 1:
            ref = torch.zeros(D, dtype=torch.int64, device=dev)
            for w in range((P + wave - 1) // wave):
                ref += make(w, w * wave, min(wave, P - w * wave)).to(torch.int64).sum(0)
            ok = bool(torch.equal(res.output, torch.remainder(ref, m).to(torch.int32)))
        steps, ms = 1, secs * 1e3
    else:
        x = gen(1234 + rank, P)

        def step():
            if world > 1:
                return agg.run_round(x, clerks=clerks)
            return eng.run_round(x, clerks=clerks)
        for _ in range(args.warmup):
            res = step()
        if args.check:
            local_sum = x.to(torch.int64).sum(0)
            tot = agg.comm.reduce_sum(local_sum) if world > 1 else local_sum
            if rank == 0:
                ok = bool(torch.equal(res.output, torch.remainder(tot, m).to(torch.int32)))
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = step()
        sync()
        secs = time.perf_counter() - t0
        if world > 1:
            secs = agg.comm.all_reduce_max(secs)
        steps, ms = args.steps, secs / args.steps * 1e3
    if rank == 0:
        emit({"config": c, "metric": "aggregated secret-shared elements/sec", "unit": "elements/s",
              "value": P * world * D / (ms / 1e3), "ms_per_round": ms, "steps": steps,
              "n_gpus": world, "participants": P * world, "dimension": D,
              "sharing": spec.sharing.to_wire(), "clerks_used": clerks or list(range(spec.n_clerks)),
              "layout": args.layout if world > 1 else "single GPU",
              "wave": args.wave or 32 if c == 4 else None, "correct": ok})
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.config == 1:
        config1()
    else:
        gpu_configs(args)


if __name__ == "__main__":
    main()
