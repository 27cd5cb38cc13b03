"""The protocol roles with their bulk cryptography on the GPU backend
(`libsda_device.so`), over the real service path.

The reference's full-loop scenarios (integration-tests/tests/full_loop.rs:29-150:
recipient + clerks + participants, `[1,2,3,4]` twice -> `[2,4,6,8]`, variants
simple / full mask / ChaCha mask / packed Shamir) run through a loopback REST
server with the roles split between GPU and CPU agents in both directions: what
a GPU clerk posts must open on the CPU recipient and the other way round, i.e.
the wire format is the contract. Larger randomised rounds compare against the
plain sum; a clerk job is also processed by both backends from the same wire
`ClerkingJob` and the two sealed results must open to the same vector.

Roles: client/src/clerk.rs:25-37,63-107, client/src/receive.rs:80-157,
client/src/participate.rs:37-113.
"""
import json
import random
import subprocess

import pytest

from sda_amd import control as C
from sda_amd._native import bin_path

pytestmark = pytest.mark.gpu

SCHEMES = {
    "simple": dict(),
    "fullmask": dict(masking="full"),
    "chachamask": dict(masking="chacha"),
    "packedshamir": dict(sharing=C.sharing_pss_4_8_3()),
    "packedshamir_fullmask": dict(sharing=C.sharing_pss_4_8_3(), masking="full"),
}


def _agg(recipient, rkey, D, m, sharing=None, masking=None):
    mk = {"full": C.masking_full(m), "chacha": C.masking_chacha(m, D, 128)}.get(masking, "None")
    return C.aggregation("foo", D, m, recipient.id, rkey, masking_scheme=mk,
                         committee_sharing_scheme=sharing or C.sharing_additive(3, m))


def _client(tmp_path, name, service, device=None):
    ks = C.FileStore(str(tmp_path / "keystores" / name))
    return C.SdaClient.create(ks, service, upload=False, device=device)


import contextlib


@contextlib.contextmanager
def _rest_service(path):
    """A fresh JFS server behind a loopback REST server; yields the REST client."""
    server = C.jfs_server(str(path / "jfs"))
    http = C.HttpServer(server).start()
    try:
        yield C.http_client(http.root, C.FileStore(str(path / "tokens")))
    finally:
        http.stop()


@pytest.fixture
def rest(tmp_path, native, cuda):
    with _rest_service(tmp_path) as svc:
        yield svc


def _run_loop(tmp_path, service, kw, D, m, vectors, gpu_roles, drop_clerks=0):
    """gpu_roles: subset of {"recipient", "clerk", "participant"} that runs on the GPU."""
    dev = lambda role: "gpu" if role in gpu_roles else None  # noqa: E731
    recipient = _client(tmp_path, "recipient", service, dev("recipient"))
    rkey = recipient.new_encryption_key()
    recipient.upload_agent()
    recipient.upload_encryption_key(rkey)
    agg = _agg(recipient, rkey, D, m, **kw)
    recipient.upload_aggregation(agg)
    n = C.share_count(agg["committee_sharing_scheme"])
    clerks = [_client(tmp_path, f"clerk{i}", service, dev("clerk")) for i in range(n)]
    for cl in clerks:
        k = cl.new_encryption_key()
        cl.upload_agent()
        cl.upload_encryption_key(k)
    recipient.begin_aggregation(agg["id"])
    if "participant" in gpu_roles:
        # one bulk agent contributes every vector (a participation each)
        p = _client(tmp_path, "bulk", service, "gpu")
        p.upload_agent()
        p.participate_many(vectors, agg["id"])
    else:
        for i, v in enumerate(vectors):
            p = _client(tmp_path, f"part{i}", service)
            p.upload_agent()
            p.participate(v, agg["id"])
    recipient.end_aggregation(agg["id"])
    committee = service.get_committee(recipient.agent, agg["id"])
    order = [c for c, _ in committee["clerks_and_keys"]]
    by_id = {cl.id: cl for cl in clerks + [recipient]}  # any key holder may be drafted
    for idx, cid in enumerate(order):
        if idx < drop_clerks:
            continue  # this clerk never answers
        by_id[cid].run_chores(-1)
    modulus, values = recipient.reveal_aggregation(agg["id"])
    return C.SdaClient.positive(modulus, values)


@pytest.mark.parametrize("variant", list(SCHEMES))
@pytest.mark.parametrize("gpu_roles", [("clerk", "recipient"), ("participant",),
                                       ("clerk", "recipient", "participant")])
def test_full_loop_roles_on_gpu(rest, tmp_path, variant, gpu_roles):
    out = _run_loop(tmp_path, rest, SCHEMES[variant], 4, 433, [[1, 2, 3, 4], [1, 2, 3, 4]],
                    set(gpu_roles))
    assert out == [2, 4, 6, 8]


@pytest.mark.parametrize("gpu_roles", [("clerk", "recipient"), ("participant",)])
def test_packed_shamir_with_a_dropped_clerk(rest, tmp_path, gpu_roles):
    """PSS_4_8_3 reconstructs from t + k = 7 of 8 results (server/src/server.rs:119-120,
    client/src/receive.rs:127-144): the first committee member never clerks."""
    out = _run_loop(tmp_path, rest, SCHEMES["packedshamir"], 10, 433,
                    [[i % 7 for i in range(10)], [3] * 10, [432] * 10], set(gpu_roles), drop_clerks=1)
    assert out == [(i % 7 + 3 + 432) % 433 for i in range(10)]


@pytest.mark.parametrize("variant,D,m,P", [("simple", 20000, 433, 37),
                                           ("fullmask", 9000, 65521, 11),
                                           ("chachamask", 5000, 433, 9),
                                           ("packedshamir", 10001, 433, 23),
                                           ("simple", 3000, 2 ** 31 - 1, 5)])
def test_random_rounds_mixed_backends(native, cuda, tmp_path, variant, D, m, P):
    rng = random.Random(D + P)
    vectors = [[rng.randrange(m) for _ in range(D)] for _ in range(P)]
    expect = [sum(col) % m for col in zip(*vectors)]
    # CPU participants -> GPU clerks -> GPU recipient
    with _rest_service(tmp_path / "a") as svc:
        assert _run_loop(tmp_path / "a", svc, SCHEMES[variant], D, m, vectors,
                         {"clerk", "recipient"}) == expect
    # GPU participants -> CPU clerks -> CPU recipient (a server of its own: the
    # committee is drafted from every agent that has uploaded a key)
    with _rest_service(tmp_path / "b") as svc:
        assert _run_loop(tmp_path / "b", svc, SCHEMES[variant], D, m, vectors,
                         {"participant"}) == expect


def test_clerk_job_gpu_equals_cpu(tmp_path, native, cuda):
    """One wire ClerkingJob through both backends: the two sealed results are
    different ciphertexts of the same combined shares."""
    server = C.memory_server()
    recipient = _client(tmp_path, "recipient", server)
    rkey = recipient.new_encryption_key()
    recipient.upload_agent()
    recipient.upload_encryption_key(rkey)
    D, m = 7000, 433
    agg = _agg(recipient, rkey, D, m)
    recipient.upload_aggregation(agg)
    clerks = [_client(tmp_path, f"clerk{i}", server) for i in range(3)]
    for cl in clerks:
        k = cl.new_encryption_key()
        cl.upload_agent()
        cl.upload_encryption_key(k)
    recipient.begin_aggregation(agg["id"])
    rng = random.Random(5)
    for i in range(6):
        p = _client(tmp_path, f"part{i}", server)
        p.upload_agent()
        p.participate([rng.randrange(m) for _ in range(D)], agg["id"])
    recipient.end_aggregation(agg["id"])
    # the committee is drafted from every key holder (the recipient has a key too):
    # take a clerk that was
    drafted = [c for c, _ in server.get_committee(recipient.agent, agg["id"])["clerks_and_keys"]]
    cl = next(c for c in clerks if c.id in drafted)
    job = server.get_clerking_job(cl.agent, cl.id)
    assert job is not None and len(job["encryptions"]) == 6
    cpu = cl.process_clerking_job(job)
    cl.use_device("gpu")
    assert "gfx950" in cl.device
    gpu = cl.process_clerking_job(job)
    assert cl.device_timings()["gpu"] > 0
    assert cpu["encryption"] != gpu["encryption"]  # fresh ephemeral keys
    kp = recipient.keystore.get(rkey)
    opened = [C._c().decrypt_shares(kp, json.dumps(r["encryption"])) for r in (cpu, gpu)]
    assert [v % m for v in opened[0]] == [v % m for v in opened[1]]
    # a tampered box fails the job on the GPU as it does on the CPU
    bad = json.loads(json.dumps(job))
    raw = bytearray(C.unb64(bad["encryptions"][2]["Sodium"]))
    raw[60] ^= 1
    bad["encryptions"][2]["Sodium"] = C.b64(bytes(raw))
    with pytest.raises(Exception, match="decryption failure"):
        cl.process_clerking_job(bad)
    cl.use_host()
    with pytest.raises(Exception, match="decryption failure"):
        cl.process_clerking_job(bad)


def test_aggregations_the_device_does_not_take_stay_on_the_host(native):
    big = C.aggregation("x", 4, 2 ** 40, C.new_id(), C.new_id(),
                        committee_sharing_scheme=C.sharing_additive(3, 2 ** 40))
    assert "31 bits" in C._c().Client.device_unsupported(json.dumps(big))
    ok = C.aggregation("x", 4, 433, C.new_id(), C.new_id())
    assert C._c().Client.device_unsupported(json.dumps(ok)) == ""


def test_cli_walkthrough_with_gpu_agents(tmp_path, native, cuda):
    """README walkthrough (docs/simple-cli-example.sh) with `--device gpu` on the
    clerks, the recipient and one bulk participant; expected 0 2 2 4 4 6 6 8 8 10."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = subprocess.Popen([bin_path("sdad"), "--jfs", str(tmp_path / "server"), "httpd", "-b",
                            f"127.0.0.1:{port}"], stdout=subprocess.PIPE, text=True)
    try:
        srv.stdout.readline()
        url = f"http://127.0.0.1:{port}"

        def sda(ident, *a, gpu=False):
            cmd = [bin_path("sda"), "-s", url, "-i", str(tmp_path / "agent" / ident)]
            if gpu:
                cmd += ["--device", "gpu"]
            r = subprocess.run(cmd + list(a), capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            return r.stdout

        for i in ["recipient", "clerk-1", "clerk-2", "clerk-3"]:
            sda(i, "agent", "create")
            sda(i, "agent", "keys", "create")
        sda("bulk", "agent", "create")
        key = sda("recipient", "agent", "keys", "show").split()[0]
        agg = "ad3142d8-9a83-4f40-a64a-a8c90b701bde"
        sda("recipient", "aggregations", "create", "--id", agg, "aggro", "10", "433", key, "3")
        sda("recipient", "aggregations", "begin", agg)
        vec = tmp_path / "vectors.txt"
        vec.write_text("0 1 2 3 4 5 6 7 8 9\n0 0 0 0 0 0 0 0 0 0\n0 1 0 1 0 1 0 1 0 1\n")
        sda("bulk", "participate-file", agg, str(vec), gpu=True)
        sda("recipient", "aggregations", "end", agg)
        for i in ["recipient", "clerk-1", "clerk-2", "clerk-3"]:
            sda(i, "clerk", "--once", gpu=True)
        out = sda("recipient", "aggregations", "reveal", agg, gpu=True)
    finally:
        srv.terminate()
        srv.wait(timeout=10)
    vals = [int(v) for v in out.split("values: [")[1].split("]")[0].split(",")]
    assert vals == [0, 2, 2, 4, 4, 6, 6, 8, 8, 10]
