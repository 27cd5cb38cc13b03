"""Control-plane integration tests (CPU): server workflow + ACL over every store
backend, in-process and over the REST transport.

Mirrors the reference's integration suite (integration-tests/tests/crud.rs,
service.rs, full_loop.rs; harness integration-tests/src/lib.rs:86-187): the same
scenarios run against the in-process server and against an HTTP client talking
to a loopback REST server, for the memory, JSON-file (JFS) and document
(Mongo data model) stores.
"""
import pytest

from sda_amd import control as C

BACKENDS = ["memory", "jfs", "document", "http-jfs", "http-document"]


class Ctx:
    def __init__(self, server, service, http=None):
        self.server = server
        self.service = service
        self.http = http


def _make_server(kind, tmp_path):
    if kind.endswith("memory"):
        return C.memory_server()
    if kind.endswith("jfs"):
        return C.jfs_server(str(tmp_path / "jfs"))
    return C.document_server(str(tmp_path / "doc"))


@pytest.fixture(params=BACKENDS)
def ctx(request, tmp_path, native):
    kind = request.param
    server = _make_server(kind, tmp_path)
    if kind.startswith("http"):
        http = C.HttpServer(server).start()
        try:
            yield Ctx(server, C.http_client(http.root, C.FileStore(str(tmp_path / "tokens"))), http)
        finally:
            http.stop()
    else:
        yield Ctx(server, server)


def new_full_agent(service):
    ag = C.fake_agent()
    service.create_agent(ag, ag)
    key = C.fake_key_for(ag)
    service.create_encryption_key(ag, key)
    return ag, key


def small_aggregation(recipient, recipient_key, **kw):
    return C.aggregation("foo", 4, 13, recipient, recipient_key,
                         committee_sharing_scheme=C.sharing_additive(3, 13), **kw)


# ---- crud.rs ----------------------------------------------------------------------
def test_ping(ctx):
    assert ctx.server.ping() == {"running": True}
    assert ctx.service.ping() == {"running": True}


def test_agent_crud(ctx):
    alice = C.fake_agent()
    ctx.service.create_agent(alice, alice)
    assert ctx.service.get_agent(alice, alice["id"]) == alice
    assert ctx.service.get_agent(alice, C.new_id()) is None


def test_profile_crud(ctx):
    alice = C.fake_agent()
    ctx.service.create_agent(alice, alice)
    assert ctx.service.get_profile(alice, alice["id"]) is None
    prof = {"owner": alice["id"], "name": "alice", "twitter_id": None, "keybase_id": None,
            "website": None}
    ctx.service.upsert_profile(alice, prof)
    assert ctx.service.get_profile(alice, alice["id"]) == prof
    prof2 = dict(prof, name="still alice")
    ctx.service.upsert_profile(alice, prof2)
    assert ctx.service.get_profile(alice, alice["id"]) == prof2


def test_profile_acl(ctx):
    alice, bob = C.fake_agent(), C.fake_agent()
    ctx.service.create_agent(bob, bob)
    fake = {"owner": alice["id"], "name": "bob", "twitter_id": None, "keybase_id": None,
            "website": None}
    with pytest.raises(C.errors.PermissionDenied):
        ctx.service.upsert_profile(bob, fake)


def test_encryption_key_crud(ctx):
    alice, bob = C.fake_agent(), C.fake_agent()
    ctx.service.create_agent(alice, alice)
    ctx.service.create_agent(bob, bob)
    key = C.fake_key_for(alice)
    ctx.service.create_encryption_key(alice, key)
    assert ctx.service.get_encryption_key(bob, key["body"]["id"]) == key


def test_auth_tokens_crud(ctx):
    alice = C.fake_agent()
    tok = {"id": alice["id"], "body": "tok"}
    with pytest.raises(C.errors.InvalidCredentials):
        ctx.server.check_auth_token(tok)
    ctx.server.create_agent(alice, alice)
    ctx.server.upsert_auth_token(tok)
    assert ctx.server.check_auth_token(tok) == alice
    tok2 = {"id": alice["id"], "body": "token"}
    with pytest.raises(C.errors.InvalidCredentials):
        ctx.server.check_auth_token(tok2)
    ctx.server.upsert_auth_token(tok2)
    ctx.server.check_auth_token(tok2)
    with pytest.raises(C.errors.InvalidCredentials):
        ctx.server.check_auth_token(tok)
    ctx.server.delete_auth_token(alice["id"])
    for t in (tok, tok2):
        with pytest.raises(C.errors.InvalidCredentials):
            ctx.server.check_auth_token(t)


def test_aggregation_crud(ctx):
    alice, alice_key = new_full_agent(ctx.service)
    assert ctx.service.list_aggregations(alice) == []
    agg = small_aggregation(alice["id"], alice_key["body"]["id"])
    ctx.service.create_aggregation(alice, agg)
    assert len(ctx.service.list_aggregations(alice, "bar")) == 0
    assert len(ctx.service.list_aggregations(alice, "foo")) == 1
    assert len(ctx.service.list_aggregations(alice, "oo")) == 1
    assert len(ctx.service.list_aggregations(alice, None, C.new_id())) == 0
    assert len(ctx.service.list_aggregations(alice, None, alice["id"])) == 1
    assert ctx.service.get_aggregation(alice, agg["id"]) == agg
    ctx.service.delete_aggregation(alice, agg["id"])
    assert ctx.service.get_aggregation(alice, agg["id"]) is None
    assert ctx.service.list_aggregations(alice) == []


def test_recipient_only_operations(ctx):
    alice, alice_key = new_full_agent(ctx.service)
    mallory, _ = new_full_agent(ctx.service)
    agg = small_aggregation(alice["id"], alice_key["body"]["id"])
    # creating an aggregation for someone else is refused
    with pytest.raises(C.errors.PermissionDenied):
        ctx.service.create_aggregation(mallory, agg)
    ctx.service.create_aggregation(alice, agg)
    for op in (lambda: ctx.service.delete_aggregation(mallory, agg["id"]),
               lambda: ctx.service.suggest_committee(mallory, agg["id"]),
               lambda: ctx.service.get_aggregation_status(mallory, agg["id"]),
               lambda: ctx.service.create_snapshot(mallory, C.snapshot(agg["id"]))):
        with pytest.raises(C.errors.PermissionDenied):
            op()


# ---- service.rs: full mocked loop (20 agents, 100 participants, 3 clerks) -------------
def test_full_mocked_loop(ctx):
    agents = [new_full_agent(ctx.service) for _ in range(20)]
    alice, alice_key = agents[0]
    agg = small_aggregation(alice["id"], alice_key["body"]["id"])
    ctx.service.create_aggregation(alice, agg)
    candidates = ctx.service.suggest_committee(alice, agg["id"])
    assert len(candidates) == len(agents)
    clerks = candidates[:C.share_count(agg["committee_sharing_scheme"])]
    committee = C.committee(agg["id"], [(c["id"], c["keys"][0]) for c in clerks])
    ctx.service.create_committee(alice, committee)
    assert ctx.service.get_committee(alice, agg["id"]) == committee

    participants = [new_full_agent(ctx.service) for _ in range(100)]
    for pi, (p, _) in enumerate(participants):
        ctx.service.create_participation(p, {
            "id": C.new_id(), "participant": p["id"], "aggregation": agg["id"],
            "recipient_encryption": None,
            "clerk_encryptions": [[c["id"], C.sodium(bytes([ci, pi]))]
                                  for ci, c in enumerate(clerks)]})

    status = ctx.service.get_aggregation_status(alice, agg["id"])
    assert status["aggregation"] == agg["id"]
    assert status["number_of_participations"] == len(participants)
    assert status["snapshots"] == []
    snap = C.snapshot(agg["id"])
    ctx.service.create_snapshot(alice, snap)
    status = ctx.service.get_aggregation_status(alice, agg["id"])
    assert status["snapshots"] == [{"id": snap["id"], "number_of_clerking_results": 0,
                                    "result_ready": False}]

    by_id = {a["id"]: a for a, _ in agents}
    for ci, c in enumerate(clerks):
        agent = by_id[c["id"]]
        job = ctx.service.get_clerking_job(agent, c["id"])
        assert job["snapshot"] == snap["id"]
        assert len(job["encryptions"]) == len(participants)
        for e in job["encryptions"]:
            assert C.unb64(e["Sodium"])[0] == ci
        ctx.service.create_clerking_result(agent, {"job": job["id"], "clerk": c["id"],
                                                   "encryption": C.sodium(bytes([ci]))})

    status = ctx.service.get_aggregation_status(alice, agg["id"])
    assert status["snapshots"] == [{"id": snap["id"], "number_of_clerking_results": len(clerks),
                                    "result_ready": True}]
    for c in clerks:
        assert ctx.service.get_clerking_job(by_id[c["id"]], c["id"]) is None

    result = ctx.service.get_snapshot_result(alice, agg["id"], snap["id"])
    assert len(result["clerk_encryptions"]) == 3
    for ci, c in enumerate(clerks):
        enc = [x for x in result["clerk_encryptions"] if x["clerk"] == c["id"]][0]
        assert C.unb64(enc["encryption"]["Sodium"]) == bytes([ci])


def test_clerk_acl(ctx):
    """Only the clerk itself may poll its queue (server.rs ACL). Over REST the
    route carries no clerk id (GET /v1/aggregations/any/jobs): a non-clerk
    caller just sees its own, empty, queue."""
    agents = [new_full_agent(ctx.service) for _ in range(5)]
    alice, alice_key = agents[0]
    agg = small_aggregation(alice["id"], alice_key["body"]["id"])
    ctx.service.create_aggregation(alice, agg)
    clerk_ids = [a["id"] for a, _ in agents[1:4]]
    ctx.service.create_committee(alice, C.committee(
        agg["id"], [(a["id"], k["body"]["id"]) for a, k in agents[1:4]]))
    outsider = agents[4][0]
    if ctx.http is None:
        with pytest.raises(C.errors.PermissionDenied):
            ctx.service.get_clerking_job(outsider, clerk_ids[0])
    else:
        assert ctx.service.get_clerking_job(outsider, clerk_ids[0]) is None


# ---- full_loop.rs: real crypto through the SdaClient roles ------------------------------
AGG_SCHEMES = {
    "simple": dict(),
    "fullmask": dict(masking_scheme=C.masking_full(433)),
    "chachamask": dict(masking_scheme=C.masking_chacha(433, 4, 128)),
    "packedshamir": dict(committee_sharing_scheme=C.sharing_pss_4_8_3()),
}


def _client(tmp_path, name, service):
    ks = C.FileStore(str(tmp_path / "keystores" / name))
    agent = C.SdaClient.create(ks, service, upload=False)
    return agent


@pytest.mark.parametrize("variant", list(AGG_SCHEMES))
def test_full_loop(ctx, tmp_path, variant):
    kw = AGG_SCHEMES[variant]
    recipient = _client(tmp_path, "recipient", ctx.service)
    rkey = recipient.new_encryption_key()
    recipient.upload_agent()
    recipient.upload_encryption_key(rkey)
    agg = C.aggregation("foo", 4, 433, recipient.id, rkey,
                        masking_scheme=kw.get("masking_scheme", "None"),
                        committee_sharing_scheme=kw.get("committee_sharing_scheme",
                                                        C.sharing_additive(3, 433)))
    recipient.upload_aggregation(agg)

    clerks = [_client(tmp_path, f"clerk{i}", ctx.service) for i in range(8)]
    for cl in clerks:
        k = cl.new_encryption_key()
        cl.upload_agent()
        cl.upload_encryption_key(k)
    recipient.begin_aggregation(agg["id"])

    participants = [_client(tmp_path, f"part{i}", ctx.service) for i in range(2)]
    for p in participants:
        p.upload_agent()
        p.participate([1, 2, 3, 4], agg["id"])

    recipient.end_aggregation(agg["id"])
    status = ctx.service.get_aggregation_status(recipient.agent, agg["id"])
    assert status["number_of_participations"] == 2
    assert len(status["snapshots"]) == 1
    assert status["snapshots"][0]["number_of_clerking_results"] == 0
    assert status["snapshots"][0]["result_ready"] is False

    recipient.run_chores(-1)
    for cl in clerks:
        cl.run_chores(-1)

    status = ctx.service.get_aggregation_status(recipient.agent, agg["id"])
    snap = status["snapshots"][0]
    assert snap["number_of_clerking_results"] == C.share_count(agg["committee_sharing_scheme"])
    assert snap["result_ready"] is True

    modulus, values = recipient.reveal_aggregation(agg["id"])
    assert C.SdaClient.positive(modulus, values) == [2, 4, 6, 8]
