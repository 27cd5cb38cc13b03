#!/usr/bin/env python3
"""Runs the benchmark configurations (sda_amd/models/configs.py) and prints one
JSON line each (rank 0).

  --config 1  CLI plumbing: sdad + sda walkthrough, 3 x 10-dim, m=433, additive-3
              (expected reveal 0 2 2 4 4 6 6 8 8 10)
  --config 2  1k x 1M, additive-3 on the GPU(s)                 (= bench.py)
  --config 3  1k x 1M per GPU, Packed Shamir k=3 n=8 (PSS_4_8_3), committee layout
  --config 4  10k x 125M (GPT-2-small gradient), PSS_4_8_3 (8 clerks), streamed in
              participant waves with accumulator checkpoints
  --config 5  1k x 1M per GPU, packed Shamir 5-of-8 (t=2, k=3) with 3 clerks dropped
  --config 6  1k x 1M, the reference's PSS_155_728_100 (728 clerks) on the int8-limb
              MFMA GEMM
  --config 7  config 5 over a prime below 256 (u8 share storage)
  --config 8  16 x 1M per GPU, the reference's PSS_155_19682_100 (19,682 clerks)
  --config 9  config 2 with a full mask (masks sealed for the recipient)
  --config 10 config 2 with a ChaCha mask (rand-0.3 seed expansion on both sides)
  --config 11 config 10 over m = 2^31 - 1

Multi-GPU: python bench_configs.py --config 3 --gpus N   (starts its own N ranks), or
           python -m torch.distributed.run --nproc-per-node N bench_configs.py --config 3 --gpus N
Scaled-down runs: --participants / --dim override the per-rank sizes;
--pss-backend valu|mfma forces the packed-Shamir kernel family.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True, choices=list(range(1, 12)))
    ap.add_argument("--gpus", type=int, default=0,
                    help="ranks (one per GPU). > 1 from a plain command line: the script starts "
                         "them itself through torch.distributed.run. 0 = whatever the launcher "
                         "started (1 from a plain command line)")
    ap.add_argument("--pss-backend", default=None, choices=["auto", "valu", "mfma"])
    ap.add_argument("--participants", type=int, default=None, help="per rank")
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--wave", type=int, default=None,
                    help="participants per wave of a streamed configuration (default: what the "
                         "HBM planner fits into the free device memory)")
    ap.add_argument("--checkpoint-every", type=int, default=8, help="waves between checkpoints")
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
    from sda_amd.models.configs import bench_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus and args.gpus != world:
        raise SystemExit(f"bench_configs.py: --gpus {args.gpus} but the launcher started {world}")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import datetime

        dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=600))
    c = args.config
    cfg = bench_config(c)
    P = args.participants or (cfg.participants // world if cfg.streamed else cfg.participants)
    D = args.dim or cfg.dimension
    spec = cfg.spec(D)
    m = spec.field_modulus
    clerks = list(cfg.clerks) if cfg.clerks is not None else None
    backend = args.pss_backend or cfg.pss_backend

    if world > 1:
        from sda_amd.parallel import DistributedAggregator

        agg = DistributedAggregator(spec, engine="device", device=dev, layout=args.layout,
                                    pss_backend=backend)
        eng = agg.engine
    else:
        agg, eng = None, DeviceAggregator(spec, device=dev, pss_backend=backend)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            agg.comm.barrier()

    free_at_start = eng.free_bytes()

    def gen(seed, count):
        g = torch.Generator(device=dev).manual_seed(seed)
        return torch.randint(0, m, (count, D), dtype=torch.int32, device=dev, generator=g)

    ok = None
    stream_info = None
    if cfg.streamed:
        wave = args.wave  # None: the planner sizes the waves from the free HBM
        ck = (args.checkpoint + f".rank{rank}") if args.checkpoint else None

        def make(w, first, count):
            return gen(1000 * (rank + 1) + w, count)
        sync()
        t0 = time.perf_counter()
        if world > 1:
            res = agg.run_streamed(P, make, wave=wave, checkpoint=ck,
                                   checkpoint_every=args.checkpoint_every)
        else:
            from sda_amd.streaming import StreamingAggregator

            res = StreamingAggregator(eng, wave=wave, checkpoint=ck,
                                      checkpoint_every=args.checkpoint_every).run(P, make)
        sync()
        secs = time.perf_counter() - t0
        wave = res.wave
        stream_info = {"plan": res.plan, "checkpoint": res.checkpoint}
        if world > 1:
            secs = agg.comm.all_reduce_max(secs)
        if args.check:
            ref = torch.zeros(D, dtype=torch.int64, device=dev)
            for w in range((P + wave - 1) // wave):
                ref += make(w, w * wave, min(wave, P - w * wave)).to(torch.int64).sum(0)
            if world > 1:  # every rank's participants: the plain sums reduced to rank 0
                ref = agg.comm.reduce_sum(ref)
            if rank == 0:
                ok = bool(torch.equal(res.output, torch.remainder(ref, m).to(torch.int32)))
        steps, ms = 1, secs * 1e3
    else:
        x = gen(1234 + rank, P)

        def step(check):
            if world > 1:
                return agg.run_round(x, clerks=clerks, check=check)
            return eng.run_round(x, clerks=clerks, check=check)
        # warm-up: checked rounds (at least one, so every kernel's code object is loaded
        # and there is an output to verify), plus the timed loop's own device ops
        err_total = torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(max(1, args.warmup)):
            res = step(True)
            err_total |= res.err
        if args.check:
            local_sum = x.to(torch.int64).sum(0)
            tot = agg.comm.reduce_sum(local_sum) if world > 1 else local_sum
            if rank == 0:
                ok = bool(torch.equal(res.output, torch.remainder(tot, m).to(torch.int32)))
        # ... and unchecked ones, queued two deep like the timed rounds: the second round
        # in flight needs its own set of arenas, allocated here and not in the timed loop
        for _ in range(3 if args.steps > 1 else 0):
            step(False)
        err_total.zero_()
        err_total |= eng.take_errors()  # (the warm-up's words count too)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res = step(False)        # no host synchronisation inside the timed loop: the
        err_total |= eng.take_errors()  # engine ORs the rounds' error words on the device
        sync()
        secs = time.perf_counter() - t0
        e = int(err_total.item())
        if world > 1:
            secs = agg.comm.all_reduce_max(secs)
            e = agg.comm.all_reduce_or(e)
        if e:
            from sda_amd.engine import describe_error

            raise SystemExit(f"bench_configs: device error word 0x{e:x} in the timed steps "
                             f"({describe_error(e)})")
        steps, ms = args.steps, secs / args.steps * 1e3
    if rank == 0:
        emit({"config": c, "name": cfg.name, "what": cfg.what,
              "metric": "aggregated secret-shared elements/sec", "unit": "elements/s",
              "value": P * world * D / (ms / 1e3), "ms_per_round": ms, "steps": steps,
              "n_gpus": world, "participants": P * world, "dimension": D,
              "sharing": spec.sharing.to_wire(), "masking": spec.masking.to_wire(),
              "clerks_used": clerks or f"all {spec.n_clerks}",
              "pss_backend": ("mfma" if eng._pss_mfma else "valu") if eng._pss is not None else None,
              "share_storage": str(eng.vdtype).replace("torch.", ""),
              "layout": args.layout if world > 1 else "single GPU",
              "hbm_high_water_bytes": torch.cuda.max_memory_allocated(),
              "hbm_reserved_bytes": torch.cuda.max_memory_reserved(),
              "hbm_free_bytes_at_start": free_at_start,
              "plan": (stream_info or {}).get("plan") if cfg.streamed else eng.plan(P).as_dict(),
              "checkpoint": (stream_info or {}).get("checkpoint"),
              "wave": wave if cfg.streamed else None, "correct": ok})
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.config == 1:
        config1()
        return
    from sda_amd.utils.launch import self_launch, wants_self_launch

    if wants_self_launch(args.gpus):
        # N ranks asked for from a plain command line: child processes, started before
        # this one has imported torch or touched a GPU
        sys.exit(self_launch(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    gpu_configs(args)


if __name__ == "__main__":
    main()
