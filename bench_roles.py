#!/usr/bin/env python3
"""The protocol roles over REST, host engines against the GPU backend.

What `sda clerk` / `sda aggregations reveal` / `sda participate-file` really
cost for a large aggregation: P participations of D-dimensional vectors are
uploaded to a loopback `HttpServer` (JFS store), the recipient snapshots, and
then the same-sized clerking jobs are processed by a clerk on the host engines
(single-threaded C++, the reference's loop: client/src/clerk.rs:63-107) and by
a clerk on the GPU backend (`libsda_device.so`); the recipient reveals on both.
Every number includes the wire work of the role: the HTTP transfer, JSON
parsing and base64 of the job (`fetch`), the cryptography (`process`) and the
result upload (`post`).

  python bench_roles.py                      # P = 1000, D = 100,000, 3 clerks, mod 433
  python bench_roles.py --participants 200 --dim 20000 --mask full

Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--participants", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=100_000)
    ap.add_argument("--modulus", type=int, default=433)
    ap.add_argument("--clerks", type=int, default=3)
    ap.add_argument("--mask", default="none", choices=["none", "full", "chacha"])
    ap.add_argument("--sharing", default="add", choices=["add", "pss483"])
    ap.add_argument("--store", default="memory", choices=["memory", "jfs", "document"])
    ap.add_argument("--cpu-participants", type=int, default=8,
                    help="participations also produced by the host engines, for the rate")
    ap.add_argument("--no-gpu", action="store_true", help="host engines only (no GPU in reach)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np

    from sda_amd import control as C

    P, D, m = args.participants, args.dim, args.modulus
    tmp = tempfile.TemporaryDirectory()
    server = {"memory": C.memory_server, "jfs": lambda: C.jfs_server(tmp.name + "/jfs"),
              "document": lambda: C.document_server(tmp.name + "/doc")}[args.store]()
    http = C.HttpServer(server, threads=8).start()
    svc = C.http_client(http.root, C.FileStore(tmp.name + "/tokens"))
    gpu = None if args.no_gpu else "gpu"

    def client(name, device=None):
        return C.SdaClient.create(C.FileStore(f"{tmp.name}/ks/{name}"), svc, upload=False,
                                  device=device)

    out = {"bench": "protocol roles over REST", "participants": P, "dimension": D, "modulus": m,
           "mask": args.mask, "sharing": args.sharing, "store": args.store}
    try:
        sharing = C.sharing_additive(args.clerks, m) if args.sharing == "add" else C.sharing_pss_4_8_3()
        n = C.share_count(sharing)
        masking = {"none": "None", "full": C.masking_full(m),
                   "chacha": C.masking_chacha(m, D, 128)}[args.mask]

        def one_round(tag, role_device):
            """A whole aggregation with its clerks and recipient on `role_device`."""
            recipient = client(f"{tag}-recipient", role_device)
            rkey = recipient.new_encryption_key()
            recipient.upload_agent()
            recipient.upload_encryption_key(rkey)
            agg = C.aggregation(tag, D, m, recipient.id, rkey, masking_scheme=masking,
                                committee_sharing_scheme=sharing)
            recipient.upload_aggregation(agg)
            return recipient, agg

        # One server, one aggregation: the committee holds CPU clerks and GPU clerks,
        # whose jobs are the same size (every clerk gets one box per participation).
        recipient, agg = one_round("bench", gpu)
        clerks = []
        for i in range(n):
            dev = gpu if (i % 2 == 1 or n == 1) else None  # odd committee slots on the GPU
            cl = client(f"clerk{i}", dev)
            k = cl.new_encryption_key()
            cl.upload_agent()
            cl.upload_encryption_key(k)
            clerks.append(cl)
        recipient.begin_aggregation(agg["id"])
        committee = svc.get_committee(recipient.agent, agg["id"])
        by_id = {c.id: c for c in clerks + [recipient]}
        order = [by_id[c] for c, _ in committee["clerks_and_keys"]]

        rng = np.random.default_rng(7)
        vectors = rng.integers(0, m, size=(P, D), dtype=np.int64)
        expect = np.remainder(vectors.sum(0), m)

        # ---- participants
        bulk = client("bulk", gpu)
        bulk.upload_agent()
        ncpu = min(args.cpu_participants, P)
        t0 = time.perf_counter()
        bulk.use_host()
        for i in range(ncpu):
            bulk.participate_many(vectors[i:i + 1], agg["id"])
        cpu_part_s = (time.perf_counter() - t0) / max(1, ncpu)
        if gpu:
            bulk.use_device(gpu)
        t0 = time.perf_counter()
        if P > ncpu:
            bulk.participate_many(vectors[ncpu:], agg["id"])
        rest_part_s = (time.perf_counter() - t0) / max(1, P - ncpu)
        out["participate"] = {
            "host_engine_s_per_participation": cpu_part_s,
            ("gpu_backend" if gpu else "host_engine_rest") + "_s_per_participation": rest_part_s,
            "gpu_backend_stage_ms_last_wave": bulk.device_timings() if gpu else None,
            "note": "seal + JSON/base64 encode + HTTP upload + server store, per participation"}

        # ---- snapshot (the server's transpose into one job per clerk)
        t0 = time.perf_counter()
        recipient.end_aggregation(agg["id"])
        out["snapshot_s"] = time.perf_counter() - t0

        # ---- clerks
        jobs = []
        for cl in order:
            t0 = time.perf_counter()
            did = cl.clerk_once()
            dt = time.perf_counter() - t0
            assert did
            jobs.append({"backend": "gpu" if cl.device else "cpu", "total_s": dt,
                         "role_ms": cl.role_timings(),
                         "device_ms": cl.device_timings() if cl.device else None})
        out["clerk_jobs"] = jobs
        cpu_jobs = [j for j in jobs if j["backend"] == "cpu"]
        gpu_jobs = [j for j in jobs if j["backend"] == "gpu"]
        box_bytes = len(C.unb64(svc.get_snapshot_result(
            recipient.agent, agg["id"], svc.get_aggregation_status(
                recipient.agent, agg["id"])["snapshots"][0]["id"])["clerk_encryptions"][0]
            ["encryption"]["Sodium"]))
        out["job_payload_bytes"] = P * box_bytes
        if cpu_jobs and gpu_jobs:
            c, g = cpu_jobs[0], gpu_jobs[-1]
            out["clerk_job_summary"] = {
                "cpu_total_s": c["total_s"], "gpu_total_s": g["total_s"],
                "speedup_total": c["total_s"] / g["total_s"],
                "cpu_process_ms": c["role_ms"]["process"], "gpu_process_ms": g["role_ms"]["process"],
                "speedup_process": c["role_ms"]["process"] / g["role_ms"]["process"],
                "fetch_ms_cpu_gpu": [c["role_ms"]["fetch"], g["role_ms"]["fetch"]],
                "gpu_kernels_ms": g["device_ms"].get("gpu")}

        # ---- recipient: reveal on its backend, then on the other one
        reveals = {}
        for label in (["gpu", "cpu"] if gpu else ["cpu"]):
            if label == "cpu":
                recipient.use_host()
            t0 = time.perf_counter()
            modulus, values = recipient.reveal_aggregation(agg["id"])
            reveals[label] = {"total_s": time.perf_counter() - t0, "role_ms": recipient.role_timings(),
                              "device_ms": recipient.device_timings() if label == "gpu" else None}
            ok = bool(np.array_equal(np.remainder(np.asarray(values, dtype=np.int64), m), expect))
            reveals[label]["correct"] = ok
            if not ok:
                raise SystemExit(f"bench_roles: {label} reveal does not match the plain sum")
        out["reveal"] = reveals
        out["correct"] = True
    finally:
        http.stop()
        tmp.cleanup()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
