"""REST router semantics, wire-format shape and on-disk layouts (CPU).

References: server-http/src/lib.rs:131-315 (routes, status mapping, Basic auth,
`Resource-not-found` header), client-http/src/client.rs:43-102 (status -> result
mapping), protocol/src/*.rs serde shapes, server/src/jfs_stores/*
(directory layout), client-store/src/file.rs (keystore layout).
"""
import base64
import http.client
import json
import os

import pytest

from sda_amd import control as C


def basic(agent_id, token):
    return "Basic " + base64.b64encode(f"{agent_id}:{token}".encode()).decode()


@pytest.fixture
def server(native):
    return C.memory_server()


def register(server, agent, token="secret-token"):
    st, hdrs, body = C.http_handle(server, "POST", "/v1/agents/me",
                                   {"Authorization": basic(agent["id"], token)}, json.dumps(agent))
    return st


# ---- router --------------------------------------------------------------------------
def test_ping_route(server):
    st, hdrs, body = C.http_handle(server, "GET", "/v1/ping")
    assert st == 200 and json.loads(body) == {"running": True}


def test_unknown_route_is_bare_404(server):
    st, hdrs, _ = C.http_handle(server, "GET", "/v2/nothing")
    assert st == 404 and "Resource-not-found" not in hdrs
    st, hdrs, _ = C.http_handle(server, "GET", "/v1/agents/me/what/ever")
    assert st == 404 and "Resource-not-found" not in hdrs


def test_missing_resource_is_flagged_404(server):
    a = C.fake_agent()
    assert register(server, a) == 201
    st, hdrs, _ = C.http_handle(server, "GET", f"/v1/agents/{C.new_id()}",
                                {"Authorization": basic(a["id"], "secret-token")})
    assert st == 404 and hdrs.get("Resource-not-found") == "true"


def test_auth_required_and_checked(server):
    a = C.fake_agent()
    st, _, _ = C.http_handle(server, "GET", f"/v1/agents/{a['id']}")
    assert st == 401  # no Authorization header
    assert register(server, a) == 201
    st, _, _ = C.http_handle(server, "GET", f"/v1/agents/{a['id']}",
                             {"Authorization": basic(a["id"], "wrong")})
    assert st == 401
    st, _, body = C.http_handle(server, "GET", f"/v1/agents/{a['id']}",
                                {"Authorization": basic(a["id"], "secret-token")})
    assert st == 200 and json.loads(body) == a


def test_trust_on_first_use_cannot_be_stolen(server):
    a = C.fake_agent()
    assert register(server, a, "first") == 201
    assert register(server, a, "first") == 201      # idempotent re-registration
    assert register(server, a, "attacker") == 401   # a second token is refused
    st, _, _ = C.http_handle(server, "GET", f"/v1/agents/{a['id']}",
                             {"Authorization": basic(a["id"], "first")})
    assert st == 200


def test_inconsistent_agent_id_rejected(server):
    a = C.fake_agent()
    st, _, _ = C.http_handle(server, "POST", "/v1/agents/me",
                             {"Authorization": basic(C.new_id(), "t")}, json.dumps(a))
    assert st == 400


def test_bad_body_and_bad_uuid_are_400(server):
    a = C.fake_agent()
    register(server, a)
    auth = {"Authorization": basic(a["id"], "secret-token")}
    st, _, _ = C.http_handle(server, "POST", "/v1/aggregations", auth, "{not json")
    assert st == 400
    st, _, _ = C.http_handle(server, "POST", "/v1/aggregations", auth, "")
    assert st == 400
    st, _, _ = C.http_handle(server, "GET", "/v1/aggregations/not-a-uuid", auth)
    assert st == 400


def test_permission_denied_is_403(server):
    a, b = C.fake_agent(), C.fake_agent()
    register(server, a)
    register(server, b, "b-token")
    prof = {"owner": a["id"], "name": "x", "twitter_id": None, "keybase_id": None, "website": None}
    st, _, _ = C.http_handle(server, "POST", "/v1/agents/me/profile",
                             {"Authorization": basic(b["id"], "b-token")}, json.dumps(prof))
    assert st == 403


def test_list_aggregations_query(server):
    a = C.fake_agent()
    register(server, a)
    auth = {"Authorization": basic(a["id"], "secret-token")}
    agg = C.aggregation("hello world", 4, 13, a["id"], C.new_id())
    st, _, _ = C.http_handle(server, "POST", "/v1/aggregations", auth, json.dumps(agg))
    assert st == 201
    st, _, body = C.http_handle(server, "GET", "/v1/aggregations?title=lo%20wo", auth)
    assert st == 200 and json.loads(body) == [agg["id"]]
    st, _, body = C.http_handle(server, "GET", f"/v1/aggregations?recipient={C.new_id()}", auth)
    assert json.loads(body) == []


def test_parse_basic_auth(native):
    tok = json.loads(C._c().parse_basic_auth(basic("2b1b6b4c-0b87-4b9e-9f70-7d2e2c0d3a11", "a:b")))
    assert tok == {"id": "2b1b6b4c-0b87-4b9e-9f70-7d2e2c0d3a11", "body": "a:b"}
    for bad in ["", "Bearer x", "Basic !!!", "Basic " + base64.b64encode(b"nocolon").decode()]:
        with pytest.raises(C.errors.SdaError):
            C._c().parse_basic_auth(bad)


# ---- real sockets: keep-alive and chunked bodies --------------------------------------
def test_socket_keepalive_and_chunked(server):
    with C.HttpServer(server) as h:
        conn = http.client.HTTPConnection("127.0.0.1", h.port, timeout=10)
        for _ in range(3):  # several requests over one connection
            conn.request("GET", "/v1/ping")
            r = conn.getresponse()
            assert r.status == 200 and json.loads(r.read()) == {"running": True}
        a = C.fake_agent()
        body = json.dumps(a).encode()

        def chunks():
            for i in range(0, len(body), 7):
                yield body[i:i + 7]
        conn.request("POST", "/v1/agents/me", body=chunks(), encode_chunked=True,
                     headers={"Authorization": basic(a["id"], "tok"),
                              "Transfer-Encoding": "chunked"})
        r = conn.getresponse()
        r.read()
        assert r.status == 201
        conn.request("GET", f"/v1/agents/{a['id']}", headers={"Authorization": basic(a["id"], "tok")})
        r = conn.getresponse()
        assert r.status == 200 and json.loads(r.read()) == a
        conn.close()


def test_http_client_concurrent(server):
    """Many client threads against one server (worker pool, keep-alive)."""
    import threading
    with C.HttpServer(server, threads=4) as h:
        errors = []

        def worker():
            try:
                cli = C.http_client(h.root)
                a = C.fake_agent()
                cli.create_agent(a, a)
                for _ in range(10):
                    assert cli.get_agent(a, a["id"]) == a
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        ts = [threading.Thread(target=worker) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors


# ---- wire format ------------------------------------------------------------------------
def test_wire_shapes(native):
    a = C.fake_agent()
    assert set(a) == {"id", "verification_key"}
    assert C.canonicalize("Agent", a) == a
    agg = C.aggregation("t", 4, 433, a["id"], C.new_id(), masking_scheme=C.masking_chacha(433, 4),
                        committee_sharing_scheme=C.sharing_pss_4_8_3())
    can = C.canonicalize("Aggregation", agg)
    assert can == agg
    assert list(can) == ["id", "title", "vector_dimension", "modulus", "recipient", "recipient_key",
                         "masking_scheme", "committee_sharing_scheme",
                         "recipient_encryption_scheme", "committee_encryption_scheme"]
    assert can["masking_scheme"] == {"ChaCha": {"modulus": 433, "dimension": 4, "seed_bitsize": 128}}
    assert can["committee_sharing_scheme"]["PackedShamir"]["omega_shares"] == 150
    assert C.canonicalize("LinearMaskingScheme", "None") == "None"
    assert C.canonicalize("LinearMaskingScheme", {"Full": {"modulus": 7}}) == {"Full": {"modulus": 7}}
    assert C.canonicalize("AdditiveEncryptionScheme", "Sodium") == "Sodium"
    prof = C.canonicalize("Profile", {"owner": a["id"]})
    assert prof == {"owner": a["id"], "name": None, "twitter_id": None, "keybase_id": None,
                    "website": None}
    with pytest.raises(Exception):
        C.canonicalize("LinearMaskingScheme", {"Nope": {}})
    with pytest.raises(Exception):
        C.canonicalize("Agent", {"id": "zzz", "verification_key": a["verification_key"]})


def test_byte_array_lengths_enforced(native):
    a = C.fake_agent()
    bad = dict(a, verification_key={"id": C.new_id(), "body": C.sodium(bytes(31))})
    with pytest.raises(Exception):
        C.canonicalize("Agent", bad)
    enc = C.sodium(bytes(range(100)))  # Encryption is variable-length
    assert C.canonicalize("Encryption", enc) == enc


def test_base64_roundtrip(native):
    for n in range(0, 70):
        data = os.urandom(n)
        assert C.unb64(C.b64(data)) == data
        assert C.b64(data) == base64.b64encode(data).decode()


# ---- on-disk layouts ----------------------------------------------------------------
def test_jfs_layout(tmp_path, native):
    srv = C.jfs_server(str(tmp_path / "srv"))
    a, k = C.fake_agent(), None
    srv.create_agent(a, a)
    k = C.fake_key_for(a)
    srv.create_encryption_key(a, k)
    srv.upsert_profile(a, {"owner": a["id"], "name": "n"})
    agg = C.aggregation("t", 4, 13, a["id"], k["body"]["id"])
    srv.create_aggregation(a, agg)
    root = tmp_path / "srv"
    assert (root / "agents" / "agents" / f"{a['id']}.json").exists()
    assert (root / "agents" / "profiles" / f"{a['id']}.json").exists()
    assert (root / "agents" / "encryption_keys" / f"{k['body']['id']}.json").exists()
    assert (root / "agg" / "aggregations" / f"{agg['id']}.json").exists()
    # files hold the wire JSON
    assert json.loads((root / "agents" / "agents" / f"{a['id']}.json").read_text()) == a
    # persistence: a new server over the same directory sees the data
    srv2 = C.jfs_server(str(root))
    assert srv2.get_aggregation(a, agg["id"]) == agg


def test_document_store_persists(tmp_path, native):
    srv = C.document_server(str(tmp_path / "doc"))
    a = C.fake_agent()
    srv.create_agent(a, a)
    agg = C.aggregation("persist", 4, 13, a["id"], C.new_id())
    srv.create_aggregation(a, agg)
    srv2 = C.document_server(str(tmp_path / "doc"))
    assert srv2.get_agent(a, a["id"]) == a
    assert srv2.list_aggregations(a, "pers") == [agg["id"]]


def test_create_is_idempotent_but_not_overwriting(native):
    srv = C.memory_server()
    a = C.fake_agent()
    srv.create_agent(a, a)
    srv.create_agent(a, a)  # same content: fine
    other = dict(a, verification_key={"id": C.new_id(), "body": C.sodium(bytes(32))})
    with pytest.raises(C.errors.SdaError):
        srv.create_agent(other, other)


def test_client_filestore(tmp_path, native):
    ks = C.FileStore(str(tmp_path / "ks"))
    tok = ks.auth_token()
    assert len(tok) == 32 and tok.isalnum()
    assert ks.auth_token() == tok  # stable
    ks.put("thing", json.dumps({"x": 1}))
    assert json.loads(ks.get("thing")) == {"x": 1}
    ks.define_alias("agent", "thing")
    assert ks.resolve_alias("agent") == "thing"
    assert (tmp_path / "ks" / "thing.json").exists()
    assert (tmp_path / "ks" / "alias_agent.json").exists()
    assert ks.get("missing") is None


# ---- bulk downloads: response text and zero-copy views ---------------------------------
def new_full_agent(service):
    ag = C.fake_agent()
    service.create_agent(ag, ag)
    key = C.fake_key_for(ag)
    service.create_encryption_key(ag, key)
    return ag, key


def _bulk_fixture(service, masked):
    """A snapshotted aggregation with 5 fake participations; returns
    (recipient agent, aggregation, clerks)."""
    import os as _os

    recipient, rkey = new_full_agent(service)
    kw = dict(masking_scheme=C.masking_full(13)) if masked else {}
    agg = C.aggregation("bulk", 4, 13, recipient["id"], rkey["body"]["id"],
                        committee_sharing_scheme=C.sharing_additive(3, 13), **kw)
    service.create_aggregation(recipient, agg)
    clerks = [new_full_agent(service) for _ in range(3)]
    service.create_committee(recipient, C.committee(
        agg["id"], [(a["id"], k["body"]["id"]) for a, k in clerks]))
    for i in range(5):
        part, _ = new_full_agent(service)
        service.create_participation(part, {
            "id": C.new_id(), "participant": part["id"], "aggregation": agg["id"],
            "recipient_encryption": C.sodium(_os.urandom(70)) if masked else None,
            "clerk_encryptions": [[a["id"], C.sodium(_os.urandom(50 + i))] for a, _ in clerks]})
    service.create_snapshot(recipient, C.snapshot(agg["id"]))
    return recipient, agg, clerks


@pytest.mark.parametrize("kind", ["memory", "jfs", "document", "http-jfs"])
@pytest.mark.parametrize("masked", [False, True])
def test_bulk_downloads_as_text_equal_the_struct_forms(native, tmp_path, kind, masked):
    """`get_clerking_job_json` / `get_snapshot_result_json` carry the same
    document as the struct forms (ClerkingJob protocol/src/resources.rs:127-139,
    SnapshotResult :178-188), and the views locate every box in the text."""
    server = {"memory": C.memory_server, "jfs": lambda: C.jfs_server(str(tmp_path / "j")),
              "document": lambda: C.document_server(str(tmp_path / "d")),
              "http-jfs": lambda: C.jfs_server(str(tmp_path / "hj"))}[kind]()
    http = C.HttpServer(server).start() if kind.startswith("http") else None
    try:
        service = C.http_client(http.root, C.MemoryStore()) if http else server
        recipient, agg, clerks = _bulk_fixture(service, masked)
        clerk = clerks[1][0]
        job = service.get_clerking_job(clerk, clerk["id"])
        text = service.handle.get_clerking_job_json(json.dumps(clerk), clerk["id"])
        assert json.loads(text) == job
        head, spans = C._c().scan_clerking_job(text)
        assert json.loads(head) == dict(job, encryptions=[])
        assert [text[o:o + n] for o, n in spans] == [e["Sodium"] for e in job["encryptions"]]
        # results + masks
        for a, _ in clerks:
            j = service.get_clerking_job(a, a["id"])
            service.create_clerking_result(a, {"job": j["id"], "clerk": a["id"],
                                               "encryption": C.sodium(b"r" * 60)})
        snap = service.get_aggregation_status(recipient, agg["id"])["snapshots"][0]["id"]
        res = service.get_snapshot_result(recipient, agg["id"], snap)
        rtext = service.handle.get_snapshot_result_json(json.dumps(recipient), agg["id"], snap)
        assert json.loads(rtext) == res
        sid, count, results, has_masks, masks = C._c().scan_snapshot_result(rtext)
        assert sid == snap and count == 5 and has_masks == masked
        assert [(j, c, rtext[o:o + n]) for j, c, o, n in results] == \
            [(r["job"], r["clerk"], r["encryption"]["Sodium"]) for r in res["clerk_encryptions"]]
        assert [rtext[o:o + n] for o, n in masks] == \
            [e["Sodium"] for e in (res["recipient_encryptions"] or [])]
        # the ACLs of the struct forms hold for the text forms
        stranger, _ = new_full_agent(service)
        with pytest.raises(C.errors.PermissionDenied):
            service.handle.get_snapshot_result_json(json.dumps(stranger), agg["id"], snap)
    finally:
        if http:
            http.stop()


def test_views_accept_whitespace_and_reject_what_they_cannot_locate(native):
    scan = C._c().scan_clerking_job
    ids = {k: C.new_id() for k in ("id", "clerk", "aggregation", "snapshot")}
    plain = json.dumps(dict(ids, encryptions=[{"Sodium": "QUJD"}, {"Sodium": ""}]))
    head, spans = scan(plain)
    assert json.loads(head)["clerk"] == ids["clerk"] and [n for _, n in spans] == [4, 0]
    pretty = json.dumps(dict(ids, encryptions=[{"Sodium": "QUJD"}]), indent=2)
    assert scan(pretty) is not None
    reordered = json.dumps(dict(encryptions=[{"Sodium": "QUJD"}], **ids))
    assert scan(reordered) is not None
    # outside the plain shape: the caller falls back to the full codec
    assert scan(plain.replace("QUJD", "QU\\u004aD")) is None      # an escape inside a payload
    assert scan(json.dumps(dict(ids, encryptions=[{"Other": "QUJD"}]))) is None
    assert scan(json.dumps(ids)) is None                           # a field is missing
    assert scan(plain + "x") is None and scan(plain[:-1]) is None
    assert scan(json.dumps(dict(ids, extra=1, encryptions=[]))) is None
