#!/usr/bin/env python3
"""Headline benchmark: aggregated secret-shared elements/sec.

BASELINE.json metric: "aggregated secret-shared elements/sec (1M-dim vec, 1k
participants, 3 clerks)" -- config 2: 1000 participants x 1,000,000-dim vectors,
3-way additive sharing mod 433, no mask, libsodium-compatible sealed boxes.

One *step* is a complete SDA round, end to end on device: participants mask +
share + seal (X25519 / XSalsa20-Poly1305) their vectors for every clerk, shares
are routed to the clerks, every clerk verifies + decrypts + decodes + combines
its boxes and seals the sum for the recipient, the recipient opens the n
results, reconstructs and unmasks. elements/s = participants x dimension / step
time (whole job: summed over all ranks). Every step draws fresh keys and
randomness; nothing is cached between steps.

Scaling is *weak*: each rank hosts `--participants` (default 1000) participants,
so N ranks aggregate N x 1000 x 1M elements per step. With N > 1 the round runs
through sda_amd.parallel.DistributedAggregator in its `committee` layout, the
protocol's trust model: every sealed box crosses xGMI to a rank that plays its
clerk (a uniform all-to-all, ~5.5 GB out of every rank per round at the default
size), each rank holds only its own clerks' secret keys, clerks' combined
shares reach rank 0 -- the recipient -- sealed. `--layout owner` is an explicit
non-private upper bound (each GPU opens its own participants' boxes and the
plaintext partial sums are reduced): it shows what the all-to-all costs.

Launch: python bench.py                                   (1 GPU, 20 timed rounds after 5)
        python bench.py --gpus N --steps K --warmup W      (starts its own N ranks)
        python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
            --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` with N > 1 and no rendezvous environment starts the N ranks itself: the
parent process runs `python -m torch.distributed.run` as a child before it has
imported torch or touched a GPU, relays rank 0's JSON line and exits with the
launcher's return code.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

# the host driver of the GPU boxes only supports dmabuf IPC (RCCL peer buffers)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "aggregated secret-shared elements/sec (1M-dim vec, 1k participants, 3 clerks)"
# The reference publishes no numbers (BASELINE.json "published": {}), so the
# denominators are reference-equivalent CPU implementations measured here with
# `sda_cpu_bench` on the same 3-clerk mod-433 1M-dim config:
#   strongest point  -- 8 threads, buffered ChaCha20 RNG:          1.41e7 elements/s
#   reference-style  -- 1 thread, one OS-RNG draw per share value: 1.16e6 elements/s
BASELINE_ELEMS_PER_S = 1.41e7
BASELINE_REFERENCE_STYLE = 1.16e6

# Roofline of the round on one MI355X: the ARX cores are pure 32-bit VALU work that
# no fusion removes -- XSalsa20 over every ciphertext byte twice (seal + open) and the
# ChaCha20 share RNG -- at ~1000 lane-ops per 64-byte block against 256 CUs x 64
# lanes x 2.4 GHz = 3.93e13 lane-ops/s.
VALU_LANE_OPS_PER_S = 256 * 64 * 2.4e9
ARX_OPS_PER_BLOCK = 1000.0


def arx_floor_ms(P: int, D: int, n: int, m: int) -> float:
    def vlen(v):
        z, k = 2 * v, 1
        while z >= 128:
            z >>= 7
            k += 1
        return k
    avg_len = sum(vlen(v) for v in range(m)) / m
    salsa_blocks = 2 * (P * n * D * avg_len) / 64.0
    draws_per_word = 3 if m ** 3 < 2 ** 32 else (2 if m <= 65536 else 1)
    chacha_blocks = P * D * (n - 1) / (16.0 * draws_per_word)
    return (salsa_blocks + chacha_blocks) * ARX_OPS_PER_BLOCK / VALU_LANE_OPS_PER_S * 1e3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5,
                    help="untimed rounds first; fewer than ~4 leave the card's clocks still "
                         "rising when the clock starts (the first rounds after idling run "
                         "14.6, 12.8, 12.5 ms)")
    ap.add_argument("--participants", type=int, default=1000, help="participants per rank")
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--clerks", type=int, default=3)
    ap.add_argument("--modulus", type=int, default=433)
    ap.add_argument("--check", action="store_true",
                    help="compare the output with the plain sum every step")
    ap.add_argument("--stages", action="store_true", help="print per-stage times (rank 0)")
    ap.add_argument("--layout", default="committee", choices=["committee", "owner"],
                    help="N > 1. committee (default): sealed boxes routed to the clerks' GPUs, "
                         "per-rank key custody, sealed results to rank 0. owner: non-private "
                         "upper bound, each GPU opens its own participants' boxes")
    ap.add_argument("--waves", type=lambda v: v if v == "taper" else int(v), default=0,
                    help="committee layout: participant waves the exchange is pipelined over. "
                         "A count, or 'taper' (six waves of 1/16, 3/16, 4/16, 4/16, 3/16, 1/16 of the "
                         "participants). 0 (default): with N > 1, 1 / 2 / 4 / 8 / taper are timed for "
                         "three untimed rounds each before the warm-up and the fastest is used "
                         "(more waves start the all-to-all earlier and shorten the exposed last "
                         "wave, fewer waves keep the grids large -- one wave exposes the whole "
                         "exchange but costs a rank 0.4 ms less compute than four: which wins "
                         "depends on the xGMI rate RCCL reaches); 4 on a single rank")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed engine even on one rank (measures its overhead)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI; gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--engine", default="device", choices=["device", "host"],
                    help="device = the HIP kernels on cuda:LOCAL_RANK. host = the C++ client "
                         "engines on the CPU over gloo: a rehearsal of the launch, exchange and "
                         "result paths on a machine without GPUs (use small --participants / "
                         "--dim); its numbers are not the benchmark")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="process-group timeout in seconds: a rank that loses a peer exits non-zero")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="override GPU_MAX_HW_QUEUES for this process (A/B measurements); 0 = leave "
                         "the environment's value, which is also what measured fastest")
    ap.add_argument("--loopback", action="store_true",
                    help="with --force-dist on one rank: the rank's own piece of every exchange "
                         "(ephemeral-key headers, sealed boxes, result boxes) goes through an RCCL "
                         "send/recv to itself instead of a local copy, so the point-to-point path "
                         "and its stream ordering run on a one-GPU machine")
    ap.add_argument("--p2p-chunk-mb", type=int, default=1024,
                    help="largest single RCCL send/recv; longer transfers are cut into runs of "
                         "whole boxes")
    ap.add_argument("--corrupt-step", type=int, default=-1,
                    help="fault injection: flip a ciphertext bit in this timed step (the run must fail)")
    return ap.parse_args()


def launcher_env(args):
    """(world, rank, local_rank) from the launcher's environment; a plain command
    line that wants the distributed engine on one rank gets a rendezvous of its own."""
    if (args.force_dist or args.engine == "host") and "MASTER_ADDR" not in os.environ:
        from sda_amd.utils.launch import free_port

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
                          WORLD_SIZE="1", LOCAL_RANK="0")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)",
              file=sys.stderr)
        sys.exit(2)
    return world, rank, local_rank


def host_rehearsal(args):
    """The N-rank committee round on the CPU engines over gloo: same launcher,
    same plan, same exchange / partial / result stages as the device run, with
    the reference's per-participant client code in place of the kernels."""
    import numpy as np
    import torch.distributed as dist

    from sda_amd.models.schemes import Additive, AggregationSpec, NoMask
    from sda_amd.parallel.engine import DistributedAggregator

    world, rank, _ = launcher_env(args)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))
    spec = AggregationSpec(args.dim, args.modulus, Additive(args.clerks, args.modulus), NoMask(),
                           title="bench")
    P, m = args.participants, args.modulus
    agg = DistributedAggregator(spec, engine="host", layout=args.layout,
                                deadline_s=min(60.0, args.dist_timeout / 4),
                                loopback=args.loopback)
    comm = agg.comm
    secrets = np.random.default_rng(1234 + rank).integers(0, m, size=(P, args.dim), dtype=np.int64)
    total = comm.reduce_sum(secrets.sum(0), dst=0)
    expected = np.remainder(total, m) if rank == 0 else None

    def verify(res, what):
        if rank == 0 and not np.array_equal(res.output, expected):
            raise SystemExit(f"bench: {what}: aggregate does not match the reference sum")

    for i in range(args.warmup):
        verify(agg.run_round(secrets), f"warmup round {i}")
    comm.reset_audit()
    comm.barrier()
    t0 = time.perf_counter()
    res = None
    for i in range(args.steps):
        res = agg.run_round(secrets)
        verify(res, f"step {i}")
    comm.barrier()
    elapsed = comm.all_reduce_max(time.perf_counter() - t0)
    ms = elapsed / max(1, args.steps) * 1e3
    sent = comm.bytes_sent() / max(1, args.steps)
    if rank == 0:
        value = P * world * args.dim / (ms / 1e3)
        print(json.dumps({
            "metric": METRIC, "value": value, "unit": "elements/s", "n_gpus": 0, "ranks": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int64 (host engines)", "data": "synthetic uniform random participant vectors",
            "rehearsal": "CPU engines over gloo: exercises the launcher and the committee "
                         "dataflow, not the benchmark",
            "xgmi": {"bytes_sent_per_rank_per_round": sent, "rank": rank},
            "config": {"model": f"SDA round: additive-{args.clerks} sharing, mod {m}, host engines",
                       "global_batch": P * world, "seq_len": args.dim,
                       "parallelism": f"dp{world} committee over gloo (CPU)"}}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    from sda_amd.utils.launch import self_launch, wants_self_launch

    if wants_self_launch(args.gpus):
        # asked for N ranks from a plain command line: start them as child processes
        # (this parent has not imported torch and never touches a GPU)
        sys.exit(self_launch(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    if args.engine == "host":
        return host_rehearsal(args)
    if args.hw_queues > 0:  # must precede HIP init
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))
    import torch
    import torch.distributed as dist

    world, rank, local_rank = launcher_env(args)
    if args.loopback and not (args.force_dist and world == 1):
        print("bench.py: --loopback needs --force-dist on one rank", file=sys.stderr)
        sys.exit(2)
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dist_mode = world > 1 or args.force_dist
    if dist_mode:
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index),
                                    timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)

    from sda_amd.engine import reference_sum
    from sda_amd.models.schemes import Additive, AggregationSpec, NoMask

    spec = AggregationSpec(args.dim, args.modulus, Additive(args.clerks, args.modulus), NoMask(),
                           title="bench")
    P = args.participants
    waves, wave_tuning = 1, {}
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    secrets = torch.randint(0, args.modulus, (P, args.dim), dtype=torch.int32, device="cuda",
                            generator=gen)

    if not dist_mode:
        from sda_amd.engine import DeviceAggregator

        agg = DeviceAggregator(spec, time_stages=args.stages)
        engine, comm = agg, None
        expected = reference_sum(secrets, args.modulus)
    else:
        from sda_amd.parallel.engine import DistributedAggregator

        waves = args.waves if args.waves else 4
        agg = DistributedAggregator(spec, engine="device", device=torch.device("cuda", dev_index),
                                    time_stages=args.stages, layout=args.layout,
                                    waves=waves, force_pipeline=args.force_dist,
                                    deadline_s=min(60.0, args.dist_timeout / 4),
                                    loopback=args.loopback,
                                    max_op_bytes=args.p2p_chunk_mb << 20)
        engine, comm = agg.engine, agg.comm
        if not args.waves and world > 1 and args.layout == "committee":
            # untimed: pick the pipeline depth on this node's measured exchange rate
            # (every rank takes the same decision: the times are max-reduced)
            for w in (1, 2, 4, 8, "taper"):
                agg.set_waves(w)
                agg.run_round(secrets, check=True)
                best = float("inf")
                for _ in range(2):  # the faster of two runs: one slow run must not decide
                    comm.barrier()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(3):  # in a row, as in the timed loop (a single round
                        agg.run_round(secrets, check=False)  # behind a synchronisation mostly
                    torch.cuda.synchronize()                 # measures the clocks coming back)
                    best = min(best, comm.all_reduce_max(time.perf_counter() - t0) / 3)
                wave_tuning[w] = best * 1e3
            waves = min(wave_tuning, key=wave_tuning.get)
            agg.set_waves(waves)
        # the global reference sum, reduced to rank 0
        total = comm.reduce_sum(secrets.to(torch.int64).sum(0), dst=0)
        expected = torch.remainder(total, args.modulus).to(torch.int32) if rank == 0 else None

    def verify(res, what):
        if rank == 0 and not torch.equal(res.output, expected):
            raise SystemExit(f"bench: {what}: aggregate does not match the reference sum")

    # warmup: rounds queued exactly as the timed ones are -- unchecked, two in flight --
    # and checked (device error word + output) after the clock has stopped. Three things
    # are being warmed. The first use of an op in a process loads its code object, which
    # on a machine that has not run the program before reads it from disk (tens of ms,
    # measured: a first process timed 17 ms rounds, every later one 13.6). A second round
    # in flight needs a second set of arenas, and rounds read back one by one left that
    # allocation to the timed loop. And the card's clocks: a few milliseconds without
    # work (the host reading a result back) and the next round takes 14.6 ms instead of
    # 12.4, the one after it 12.8 (scripts/exp_round_steps.py) -- so nothing is read
    # back between the last warm-up round and the timed region: the synchronisation
    # in front of the clock ends with the card still at its working clocks.
    err_total = torch.zeros(1, dtype=torch.int32, device="cuda")

    def device_verdict(r):
        # a round's error word and "output differs" as device values, no read-back
        wrong = (r.output != expected).any() if rank == 0 else None
        return r.err.clone(), wrong

    warm, prev = [], None
    for _ in range(args.warmup):
        r = agg.run_round(secrets, check=False)
        if prev is not None:  # one round late: reading a result waits for its result path
            warm.append(device_verdict(prev))
        prev = r
    if prev is not None:
        warm.append(device_verdict(prev))
    del prev
    err_total |= err_total  # (the timed region's own ops, used once)
    if dist_mode:
        comm.reset_audit()
        comm.barrier()
    err_total.zero_()
    engine.take_errors()  # the warm-up's words: each is checked below, after the clock
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    res = None
    host_s = 0.0  # host time spent queuing rounds (no synchronisation inside the loop)
    if dist_mode:
        comm.rendezvous_s = 0.0
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.corrupt_step:
            engine.corrupt_next_round()
        th = time.perf_counter()
        res = agg.run_round(secrets, check=args.check)
        host_s += time.perf_counter() - th
        if args.check:
            verify(res, f"step {i}")
    # the error words of the timed rounds are OR-ed on the device by the engine (on the
    # stream each round's result path ends on, beside the next round's first kernels)
    # and read once, after the clock stops
    err_total |= engine.take_errors()
    torch.cuda.synchronize()
    if dist_mode:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    # integrity of the timed region: any MAC / varint / key / range failure in any
    # step on any rank fails the run, and the last round's output must be right
    e = int(err_total.item())
    if dist_mode:
        e = comm.all_reduce_or(e)
        elapsed = comm.all_reduce_max(elapsed)
    if e:
        from sda_amd.engine import describe_error

        raise SystemExit(f"bench: device error word 0x{e:x} in the timed steps ({describe_error(e)})")
    if res is not None:
        verify(res, "last timed round")
    for i, (w_err, w_wrong) in enumerate(warm):  # the warm-up rounds: each one's verdict
        e = int(w_err.item())
        if dist_mode:
            e = comm.all_reduce_or(e)
        if e:
            from sda_amd.engine import describe_error

            raise SystemExit(f"bench: warmup round {i}: device error word 0x{e:x} ({describe_error(e)})")
        if w_wrong is not None and bool(w_wrong.item()):
            raise SystemExit(f"bench: warmup round {i}: aggregate does not match the reference sum")
    ms = elapsed / max(1, args.steps) * 1e3
    total_elems = P * world * args.dim
    value = total_elems / (ms / 1e3)
    hbm_peak = torch.cuda.max_memory_allocated()
    xgmi = None
    if dist_mode:
        hbm_peak = int(comm.all_reduce_max(float(hbm_peak)))
        kinds = {}
        for kind, direction, peer, _, nbytes in comm.audit:
            if direction == "send" and peer != rank:
                kinds[kind] = kinds.get(kind, 0) + nbytes
        per_round = {k: v / max(1, args.steps) for k, v in kinds.items()}
        xgmi = {"bytes_sent_per_rank_per_round": sum(per_round.values()),
                "by_kind": per_round, "rank": rank}
    if rank == 0:
        if args.stages and getattr(res, "stage_ms", None):
            print(json.dumps({"stage_ms": res.stage_ms}), file=sys.stderr)
        if not dist_mode:
            parallelism = "single GPU"
        elif args.layout == "committee":
            parallelism = (f"dp{world} participants x committee-sharded clerks: all-to-all of "
                           f"sealed boxes over xGMI (grouped RCCL send/recv, {waves} waves), "
                           "per-rank key custody, sealed clerk results gathered on rank 0")
            if world == 1 and args.loopback:
                parallelism += (" [one rank, loopback: its own piece travels through RCCL "
                                "send/recv to itself; nothing crosses xGMI]")
            elif world == 1:
                parallelism += " [distributed engine on one rank: nothing crosses xGMI]"
        else:
            parallelism = (f"dp{world} owner (non-private upper bound): every GPU opens its own "
                           "participants' boxes, plaintext clerk partials reduced to rank 0")
        floor = arx_floor_ms(P, args.dim, args.clerks, args.modulus)
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
            "vs_baseline": value / BASELINE_ELEMS_PER_S,
            "baseline": {"elements_per_s": BASELINE_ELEMS_PER_S,
                         "what": "reference-equivalent CPU implementation measured here (8 threads, "
                                 "buffered ChaCha20 RNG); the reference publishes no numbers",
                         "vs_reference_style_single_thread": value / BASELINE_REFERENCE_STYLE},
            "roofline_fraction": floor / ms,
            "roofline": {"arx_valu_floor_ms_per_gpu": floor,
                         "model": "XSalsa20 over the ciphertext twice + ChaCha20 share RNG at 1000 "
                                  "lane-ops per 64 B block, 3.93e13 int32 lane-ops/s"},
            "dtype": "int32 (field elements mod 433; no floating point in this workload)",
            "data": "synthetic uniform random participant vectors in [0, 433)",
            "hbm_high_water_bytes": hbm_peak,
            "hbm_reserved_bytes": torch.cuda.max_memory_reserved(),
            "xgmi": xgmi,
            "host_ms_per_step": {"queuing_rounds": host_s / max(1, args.steps) * 1e3,
                                 "of_which_store_rendezvous": (comm.rendezvous_s / max(1, args.steps) * 1e3
                                                               if dist_mode else 0.0),
                                 "note": "rank 0's host time inside run_round; the GPU runs behind "
                                         "it, so it only bounds the step when it exceeds ms_per_step"},
            "pipeline_waves": waves if dist_mode else None,
            "compute_stream_vs_rccl": comm.compute_stream_probe if dist_mode else None,
            "pipeline_wave_tuning_ms": {str(k): v for k, v in wave_tuning.items()} or None,
            "timed_steps_verified": "device error word of every timed step (OR-ed on the device by "
                                    "the engine over steps, and over ranks) + last round's output vs "
                                    "the plain sum; every warm-up round's error word and output too, "
                                    "read after the clock stopped",
            "round_pipelining": (None if dist_mode else
                                 "each round complete; a round's result path (clerks seal their "
                                 "sums, recipient opens + reconstructs) runs on a third stream "
                                 "beside the next round's first kernels; at most two rounds in flight"),
            "config": {
                "model": f"SDA round: additive-{args.clerks} sharing, mod {args.modulus}, no mask, "
                         "libsodium sealed boxes (X25519+XSalsa20-Poly1305), zigzag varint",
                "global_batch": P * world,
                "seq_len": args.dim,
                "participants_per_gpu": P,
                "dimension": args.dim,
                "clerks": args.clerks,
                "parallelism": parallelism,
            },
        }
        print(json.dumps(line), flush=True)
    if dist_mode:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
