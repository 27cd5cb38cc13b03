#!/usr/bin/env python3
"""Control plane at scale: P participations of D values through `sdad` over loopback.

The reference's service test runs 100 participants and 3 clerks with two-byte
fake payloads (integration-tests/tests/service.rs:28-126) and reports no
timings. This bench drives the real REST path with real sealed boxes: a `sdad`
process (JFS or document store on disk), P participations uploaded by `--clients`
concurrent REST clients, the snapshot (the server-side transpose P x n -> n x P,
server/src/snapshot.rs:11-27), one clerk job fetched and answered per clerk, and
the reveal. CPU only; no GPU is touched.

  python bench_rest.py                          # P = 1000, D = 10,000, both stores
  python bench_rest.py --stores jfs --participants 200

Prints one JSON line per store.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--participants", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=10_000)
    ap.add_argument("--modulus", type=int, default=433)
    ap.add_argument("--clerks", type=int, default=3)
    ap.add_argument("--clients", type=int, default=8, help="concurrent uploading clients")
    ap.add_argument("--stores", default="jfs,document")
    return ap.parse_args()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def codec_rates(C):
    """JSON + base64 of a clerking-job-shaped document, MB/s of JSON text."""
    blob = os.urandom(20_000)
    job = {"id": C.new_id(), "clerk": C.new_id(), "aggregation": C.new_id(), "snapshot": C.new_id(),
           "encryptions": [{"Sodium": C.b64(blob)} for _ in range(500)]}
    text = json.dumps(job, separators=(",", ":"))
    c = C._c()
    out = {"document_bytes": len(text)}
    t0 = time.perf_counter()
    for _ in range(5):
        c.canonicalize("ClerkingJob", text)     # parse + from_json + to_json + dump
    out["full_codec_round_trip_mb_s"] = 5 * len(text) / 1e6 / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(20):
        c.scan_clerking_job(text)               # the zero-copy view
    out["view_scan_mb_s"] = 20 * len(text) / 1e6 / (time.perf_counter() - t0)
    b64 = C.b64(blob * 50)
    t0 = time.perf_counter()
    for _ in range(20):
        c.base64_decode(b64)
    out["base64_decode_mb_s"] = 20 * len(b64) / 1e6 / (time.perf_counter() - t0)
    return out


def run_store(args, store, C, np):
    from sda_amd._native import bin_path

    P, D, m, n = args.participants, args.dim, args.modulus, args.clerks
    tmp = tempfile.TemporaryDirectory()
    port = free_port()
    flag = "--jfs" if store == "jfs" else "--document"
    srv = subprocess.Popen([bin_path("sdad"), flag, f"{tmp.name}/server", "--max-body-mb", "2048",
                            "httpd", "-b", f"127.0.0.1:{port}"], stdout=subprocess.PIPE, text=True)
    out = {"bench": "control plane over REST", "store": store, "participants": P, "dimension": D,
           "clerks": n, "uploading_clients": args.clients}
    try:
        srv.stdout.readline()
        url = f"http://127.0.0.1:{port}/"

        def client(name):
            ks = C.FileStore(f"{tmp.name}/ks/{name}")
            svc = C.http_client(url, C.FileStore(f"{tmp.name}/tok/{name}"))
            return C.SdaClient.create(ks, svc, upload=False), svc

        recipient, svc = client("recipient")
        rkey = recipient.new_encryption_key()
        recipient.upload_agent()
        recipient.upload_encryption_key(rkey)
        agg = C.aggregation("bench", D, m, recipient.id, rkey,
                            committee_sharing_scheme=C.sharing_additive(n, m))
        recipient.upload_aggregation(agg)
        clerks = []
        for i in range(n):
            cl, _ = client(f"clerk{i}")
            k = cl.new_encryption_key()
            cl.upload_agent()
            cl.upload_encryption_key(k)
            clerks.append(cl)
        recipient.begin_aggregation(agg["id"])
        committee = svc.get_committee(recipient.agent, agg["id"])
        by_id = {c.id: c for c in clerks + [recipient]}
        order = [by_id[c] for c, _ in committee["clerks_and_keys"]]

        # ---- participations: sealed once (host engines), uploaded by concurrent clients
        rng = np.random.default_rng(11)
        vectors = rng.integers(0, m, size=(P, D), dtype=np.int64)
        expect = np.remainder(vectors.sum(0), m)
        workers = []
        for w in range(args.clients):
            p, _ = client(f"part{w}")
            p.upload_agent()
            workers.append(p)
        t0 = time.perf_counter()
        sealed = [[] for _ in workers]

        def seal(w):
            for i in range(w, P, len(workers)):
                sealed[w].append(workers[w].new_participation(vectors[i].tolist(), agg["id"]))
        th = [threading.Thread(target=seal, args=(w,)) for w in range(len(workers))]
        [t.start() for t in th]
        [t.join() for t in th]
        out["seal_s"] = time.perf_counter() - t0
        body_bytes = len(json.dumps(sealed[0][0], separators=(",", ":")))
        t0 = time.perf_counter()

        def upload(w):
            for p in sealed[w]:
                workers[w].upload_participation(p)
        th = [threading.Thread(target=upload, args=(w,)) for w in range(len(workers))]
        [t.start() for t in th]
        [t.join() for t in th]
        dt = time.perf_counter() - t0
        out["upload"] = {"seconds": dt, "participations_per_s": P / dt,
                         "body_bytes": body_bytes, "mb_per_s": P * body_bytes / 1e6 / dt}

        # ---- status (count over the store), snapshot (the transpose), status again
        t0 = time.perf_counter()
        for _ in range(20):
            st = svc.get_aggregation_status(recipient.agent, agg["id"])
        out["status_ms"] = (time.perf_counter() - t0) / 20 * 1e3
        assert st["number_of_participations"] == P
        t0 = time.perf_counter()
        recipient.end_aggregation(agg["id"])
        out["snapshot_s"] = time.perf_counter() - t0

        # ---- clerk jobs
        jobs = []
        for cl in order:
            t0 = time.perf_counter()
            assert cl.clerk_once()
            jobs.append({"total_s": time.perf_counter() - t0, "role_ms": cl.role_timings()})
        job_bytes = P * (48 + 2 * D)  # approximate payload
        out["clerk_jobs"] = jobs
        out["job_fetch_mb_per_s"] = job_bytes * 4 / 3 / 1e6 / (jobs[0]["role_ms"]["fetch"] / 1e3)

        # ---- reveal
        t0 = time.perf_counter()
        modulus, values = recipient.reveal_aggregation(agg["id"])
        out["reveal_s"] = time.perf_counter() - t0
        out["correct"] = bool(np.array_equal(np.remainder(np.asarray(values, dtype=np.int64), m), expect))
        if not out["correct"]:
            raise SystemExit("bench_rest: the revealed aggregate does not match the plain sum")
    finally:
        srv.terminate()
        srv.wait(timeout=20)
        tmp.cleanup()
    return out


def main():
    args = parse()
    import numpy as np

    from sda_amd import control as C

    codec = codec_rates(C)
    for store in args.stores.split(","):
        res = run_store(args, store.strip(), C, np)
        res["codec"] = codec
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
