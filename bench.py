#!/usr/bin/env python3
"""Headline benchmark: aggregated secret-shared elements/sec.

BASELINE.json metric: "aggregated secret-shared elements/sec (1M-dim vec, 1k
participants, 3 clerks)" -- config 2: 1000 participants x 1,000,000-dim vectors,
3-way additive sharing mod 433, no mask, libsodium-compatible sealed boxes.

One *step* is a complete SDA round, end to end on device: participants mask +
share + seal (X25519 / XSalsa20-Poly1305) their vectors for every clerk, shares
are routed to the clerks, every clerk verifies + decrypts + decodes + combines
its P boxes and seals the sum for the recipient, the recipient opens the n
results, reconstructs and unmasks. elements/s = participants x dimension / step
time (whole job: summed over all ranks).

Scaling is *weak*: each rank hosts `--participants` (default 1000) participants,
so N ranks aggregate N x 1000 x 1M elements per step. With N > 1 the round runs
through sda_amd.parallel.DistributedAggregator. Default layout `owner`: every
GPU hosts a slice of each of the n clerks (a clerk is one organisation whose job
spans the node), so a GPU opens the boxes its own participants sealed -- the
same per-GPU trust boundary as the one-GPU round -- and the clerks' partial sums
plus mask partials are reduced to rank 0, the recipient, in one RCCL bucket:
N x the one-GPU work, (n+1) x D integers over xGMI per round.
`--layout committee` routes every sealed box over xGMI to ranks playing the
clerks (no rank holding two clerks' shares of a participant): the snapshot
transpose as grouped RCCL send/recv, 5.5 GB out of every rank per round, which
a point-to-point xGMI link cannot move in one round's compute time at N=2.

Launch: python bench.py --gpus 1 --steps 5 --warmup 2
        python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
            --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "aggregated secret-shared elements/sec (1M-dim vec, 1k participants, 3 clerks)"
# Reference-equivalent single-threaded CPU implementation, measured here (the
# reference publishes no numbers): `sda_cpu_bench --participants 4
# --dim 1000000` -> 1.16e6 elements/s (OS-RNG draw per share value, sealed box
# per (participant, clerk), element-wise combine), same 3-clerk mod-433 config.
BASELINE_ELEMS_PER_S = 1.16e6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--participants", type=int, default=1000, help="participants per rank")
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--clerks", type=int, default=3)
    ap.add_argument("--modulus", type=int, default=433)
    ap.add_argument("--check", action="store_true", help="verify the output every step")
    ap.add_argument("--stages", action="store_true", help="print per-stage times (rank 0)")
    ap.add_argument("--layout", default="owner", choices=["committee", "owner"],
                    help="committee: boxes routed to the clerks' GPUs (protocol trust model); "
                         "owner: each GPU hosts a slice of every clerk and opens its own "
                         "participants' boxes (default)")
    ap.add_argument("--waves", type=int, default=4,
                    help="committee layout: participant waves the exchange is pipelined over")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed engine even on one rank (measures its overhead)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="override GPU_MAX_HW_QUEUES (0 = leave the process default)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI; gloo only to rehearse several ranks on one GPU")
    return ap.parse_args()


def main():
    args = parse()
    if args.hw_queues > 0:  # must precede HIP init
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("bench.py: launch with torch.distributed.run for --gpus > 1", file=sys.stderr)
            sys.exit(2)
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dist_mode = world > 1 or args.force_dist
    if dist_mode:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")

    from sda_amd.models.schemes import Additive, AggregationSpec, NoMask

    spec = AggregationSpec(args.dim, args.modulus, Additive(args.clerks, args.modulus), NoMask(),
                           title="bench")
    P = args.participants
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    secrets = torch.randint(0, args.modulus, (P, args.dim), dtype=torch.int32, device="cuda",
                            generator=gen)

    if not dist_mode:
        from sda_amd.engine import DeviceAggregator, reference_sum

        agg = DeviceAggregator(spec, time_stages=args.stages)

        def step(check):
            res = agg.run_round(secrets, check=check)
            return res

        expected = reference_sum(secrets, args.modulus) if args.check else None
    else:
        from sda_amd.parallel.engine import DistributedAggregator

        agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", dev_index),
                                    time_stages=args.stages, layout=args.layout,
                                    waves=args.waves, force_pipeline=args.force_dist)

        def step(check):
            return agg.run_round(secrets, check=check)

        expected = None
        # the global reference sum, reduced to rank 0, validates the first warmup round
        local = agg.comm.reduce_sum(secrets.to(torch.int64).sum(0), dst=0)
        global_ref = torch.remainder(local, args.modulus).to(torch.int32) if rank == 0 else None

    # warmup (also validates the result once)
    for i in range(args.warmup):
        res = step(check=True)
        if i == 0 and not dist_mode:
            ref = reference_sum(secrets, args.modulus)
            if not torch.equal(res.output, ref):
                raise SystemExit("bench: device aggregation does not match the reference sum")
        if i == 0 and dist_mode and rank == 0:
            if not torch.equal(res.output, global_ref):
                raise SystemExit("bench: distributed aggregation does not match the reference sum")
    if dist_mode:
        agg.comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step(check=args.check)
        if expected is not None and not torch.equal(res.output, expected):
            raise SystemExit("bench: mismatch")
    torch.cuda.synchronize()
    if dist_mode:
        agg.comm.barrier()
    elapsed = time.perf_counter() - t0
    if dist_mode:
        elapsed = agg.comm.all_reduce_max(elapsed)
    ms = elapsed / args.steps * 1e3
    total_elems = P * world * args.dim
    value = total_elems / (ms / 1e3)
    if rank == 0:
        if args.stages and getattr(res, "stage_ms", None):
            print(json.dumps({"stage_ms": res.stage_ms}), file=sys.stderr)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "elements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_ELEMS_PER_S) if BASELINE_ELEMS_PER_S else None,
            "dtype": "int32 (field elements mod 433; no floating point in this workload)",
            "data": "synthetic uniform random participant vectors in [0, 433)",
            "config": {
                "model": f"SDA round: additive-{args.clerks} sharing, mod {args.modulus}, no mask, "
                         "libsodium sealed boxes (X25519+XSalsa20-Poly1305), zigzag varint",
                "global_batch": P * world,
                "seq_len": args.dim,
                "participants_per_gpu": P,
                "dimension": args.dim,
                "clerks": args.clerks,
                "parallelism": (f"dp{world} participants x committee-sharded clerks: sealed "
                                "boxes routed over xGMI (grouped RCCL send/recv), clerk partials "
                                "reduced to rank 0" if args.layout == "committee" else
                                f"dp{world} participants, every GPU hosting a slice of each clerk: clerk "
                                "partials + mask partials reduced to rank 0 over RCCL")
                               if world > 1 else "single GPU",
            },
        }
        print(json.dumps(line), flush=True)
    if dist_mode:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
