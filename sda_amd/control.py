"""SDA control plane: servers, stores, REST transport and client roles.

Python face of the C++ runtime (``csrc/src/{server,stores_kv,stores_doc,http,
client}.cc``, bound in ``csrc/python/control_bindings.cc``). Protocol objects
are plain dicts in the reference's serde JSON wire form (protocol/src/*.rs), so
what a test builds here is byte-for-byte what crosses the REST API.

Reference seams:
  * ``Service``           protocol/src/methods.rs  -- the SdaService trait object
  * ``memory_server`` / ``jfs_server``   server/src/lib.rs:34-45
  * ``document_server``   server-store-mongodb/src/lib.rs:64-84 (same data model,
                          embedded document collections instead of a MongoDB)
  * ``HttpServer``        server-http/src/lib.rs (+ server-cli/src/lib.rs httpd)
  * ``http_client``       client-http/src/client.rs
  * ``SdaClient``         client/src/lib.rs + participate/clerk/receive/maintenance
  * ``FileStore`` / ``MemoryStore``   client-store/src/file.rs
"""
from __future__ import annotations

import json
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

from ._native import native

Obj = Dict[str, Any]


def _c():
    return native().control


def _enc(obj: Any) -> str:
    return json.dumps(obj, separators=(",", ":"))


def _dec(text: Optional[str]) -> Optional[Obj]:
    return None if text is None else json.loads(text)


# ---- errors (protocol/src/lib.rs:21-41) --------------------------------------
def _exc(name: str):
    return getattr(_c(), name)


class _Errors:
    def __getattr__(self, name):
        return _exc(name)


errors = _Errors()  # errors.SdaError / PermissionDenied / InvalidCredentials / Invalid


def new_id() -> str:
    """A random v4 UUID (the reference's ``Id::random()``)."""
    return _c().new_id()


def canonicalize(type_name: str, obj: Any) -> Obj:
    """Round-trip ``obj`` through the C++ wire codec (validates and normalises)."""
    return json.loads(_c().canonicalize(type_name, _enc(obj)))


def b64(data: bytes) -> str:
    return _c().base64_encode(data)


def unb64(text: str) -> bytes:
    return _c().base64_decode(text)


# ---- scheme / object constructors -----------------------------------------------
def masking_none() -> Any:
    return "None"


def masking_full(modulus: int) -> Obj:
    return {"Full": {"modulus": modulus}}


def masking_chacha(modulus: int, dimension: int, seed_bitsize: int = 128) -> Obj:
    return {"ChaCha": {"modulus": modulus, "dimension": dimension, "seed_bitsize": seed_bitsize}}


def sharing_additive(share_count: int, modulus: int) -> Obj:
    return {"Additive": {"share_count": share_count, "modulus": modulus}}


def sharing_packed_shamir(secret_count: int, share_count: int, privacy_threshold: int,
                          prime_modulus: int, omega_secrets: int, omega_shares: int) -> Obj:
    return {"PackedShamir": {"secret_count": secret_count, "share_count": share_count,
                             "privacy_threshold": privacy_threshold,
                             "prime_modulus": prime_modulus, "omega_secrets": omega_secrets,
                             "omega_shares": omega_shares}}


# The reference's named parameter sets (protocol/src/crypto.rs presets, tss-0.2).
PSS_4_8_3 = dict(secret_count=3, share_count=8, privacy_threshold=4, prime_modulus=433,
                 omega_secrets=354, omega_shares=150)


def sharing_pss_4_8_3() -> Obj:
    return sharing_packed_shamir(**PSS_4_8_3)


def aggregation(title: str, vector_dimension: int, modulus: int, recipient: str,
                recipient_key: str, masking_scheme: Any = "None",
                committee_sharing_scheme: Optional[Obj] = None,
                id: Optional[str] = None) -> Obj:
    """An ``Aggregation`` dict (protocol/src/aggregations.rs:9-34)."""
    return {
        "id": id or new_id(),
        "title": title,
        "vector_dimension": vector_dimension,
        "modulus": modulus,
        "recipient": recipient,
        "recipient_key": recipient_key,
        "masking_scheme": masking_scheme,
        "committee_sharing_scheme": committee_sharing_scheme or sharing_additive(3, modulus),
        "recipient_encryption_scheme": "Sodium",
        "committee_encryption_scheme": "Sodium",
    }


def committee(aggregation_id: str, clerks_and_keys: Iterable[Tuple[str, str]]) -> Obj:
    return {"aggregation": aggregation_id,
            "clerks_and_keys": [[c, k] for c, k in clerks_and_keys]}


def snapshot(aggregation_id: str, id: Optional[str] = None) -> Obj:
    return {"id": id or new_id(), "aggregation": aggregation_id}


def sodium(data: bytes) -> Obj:
    """``Encryption::Sodium(bytes)`` / key bodies."""
    return {"Sodium": b64(data)}


def fake_agent() -> Obj:
    """An agent with an all-zero verification key (integration-tests/src/lib.rs new_agent)."""
    return {"id": new_id(),
            "verification_key": {"id": new_id(), "body": sodium(bytes(32))}}


def fake_key_for(agent: Obj) -> Obj:
    """A SignedEncryptionKey with zero key/signature (new_key_for_agent)."""
    return {"signature": sodium(bytes(64)), "signer": agent["id"],
            "body": {"id": new_id(), "body": sodium(bytes(32))}}


def share_count(scheme: Obj) -> int:
    """``output_size()`` of a sharing scheme (number of clerks)."""
    (kind, p), = scheme.items()
    return p["share_count"]


# ---- service -------------------------------------------------------------------
class Service:
    """An ``SdaService`` (in-process server or REST client) speaking dicts."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    def ping(self) -> Obj:
        return json.loads(self._h.ping())

    # agents (SdaAgentService)
    def create_agent(self, caller: Obj, agent: Obj) -> None:
        self._h.create_agent(_enc(caller), _enc(agent))

    def get_agent(self, caller: Obj, agent_id: str) -> Optional[Obj]:
        return _dec(self._h.get_agent(_enc(caller), agent_id))

    def upsert_profile(self, caller: Obj, profile: Obj) -> None:
        self._h.upsert_profile(_enc(caller), _enc(profile))

    def get_profile(self, caller: Obj, owner: str) -> Optional[Obj]:
        return _dec(self._h.get_profile(_enc(caller), owner))

    def create_encryption_key(self, caller: Obj, key: Obj) -> None:
        self._h.create_encryption_key(_enc(caller), _enc(key))

    def get_encryption_key(self, caller: Obj, key_id: str) -> Optional[Obj]:
        return _dec(self._h.get_encryption_key(_enc(caller), key_id))

    # aggregations
    def list_aggregations(self, caller: Obj, filter: Optional[str] = None,
                          recipient: Optional[str] = None) -> List[str]:
        return list(self._h.list_aggregations(_enc(caller), filter, recipient))

    def get_aggregation(self, caller: Obj, aggregation_id: str) -> Optional[Obj]:
        return _dec(self._h.get_aggregation(_enc(caller), aggregation_id))

    def get_committee(self, caller: Obj, aggregation_id: str) -> Optional[Obj]:
        return _dec(self._h.get_committee(_enc(caller), aggregation_id))

    # participation / clerking
    def create_participation(self, caller: Obj, participation: Obj) -> None:
        self._h.create_participation(_enc(caller), _enc(participation))

    def get_clerking_job(self, caller: Obj, clerk: str) -> Optional[Obj]:
        return _dec(self._h.get_clerking_job(_enc(caller), clerk))

    def create_clerking_result(self, caller: Obj, result: Obj) -> None:
        self._h.create_clerking_result(_enc(caller), _enc(result))

    # recipient
    def create_aggregation(self, caller: Obj, agg: Obj) -> None:
        self._h.create_aggregation(_enc(caller), _enc(agg))

    def delete_aggregation(self, caller: Obj, aggregation_id: str) -> None:
        self._h.delete_aggregation(_enc(caller), aggregation_id)

    def suggest_committee(self, caller: Obj, aggregation_id: str) -> List[Obj]:
        return [json.loads(t) for t in self._h.suggest_committee(_enc(caller), aggregation_id)]

    def create_committee(self, caller: Obj, committee: Obj) -> None:
        self._h.create_committee(_enc(caller), _enc(committee))

    def get_aggregation_status(self, caller: Obj, aggregation_id: str) -> Optional[Obj]:
        return _dec(self._h.get_aggregation_status(_enc(caller), aggregation_id))

    def create_snapshot(self, caller: Obj, snap: Obj) -> None:
        self._h.create_snapshot(_enc(caller), _enc(snap))

    def get_snapshot_result(self, caller: Obj, aggregation_id: str,
                            snapshot_id: str) -> Optional[Obj]:
        return _dec(self._h.get_snapshot_result(_enc(caller), aggregation_id, snapshot_id))


class ServerService(Service):
    """The in-process server: service + server-side auth-token helpers."""

    def upsert_auth_token(self, token: Obj) -> None:
        self._h.upsert_auth_token(_enc(token))

    def check_auth_token(self, token: Obj) -> Obj:
        return json.loads(self._h.check_auth_token(_enc(token)))

    def delete_auth_token(self, agent_id: str) -> None:
        self._h.delete_auth_token(agent_id)

    def poll_clerking_job(self, clerk: str) -> Optional[Obj]:
        return _dec(self._h.poll_clerking_job(clerk))


def memory_server() -> ServerService:
    return ServerService(_c().memory_server())


def jfs_server(directory: str) -> ServerService:
    return ServerService(_c().jfs_server(str(directory)))


def document_server(directory: str) -> ServerService:
    return ServerService(_c().document_server(str(directory)))


def FileStore(directory: str):
    return _c().FileStore(str(directory))


def MemoryStore():
    return _c().MemoryStore()


def http_client(server_root: str, token_store=None) -> Service:
    return Service(_c().http_client(server_root, token_store or MemoryStore()))


class HttpServer:
    """The REST server over an in-process ``ServerService``; a context manager."""

    def __init__(self, server: ServerService, bind: str = "127.0.0.1:0", threads: int = 8):
        self._srv = _c().HttpServer(server.handle, threads)
        self._bind = bind
        self.port: Optional[int] = None

    def start(self) -> "HttpServer":
        self.port = self._srv.start(self._bind)
        return self

    def stop(self) -> None:
        self._srv.stop()

    @property
    def root(self) -> str:
        return f"http://127.0.0.1:{self.port}/"

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def http_handle(server: ServerService, method: str, target: str,
                headers: Optional[Dict[str, str]] = None, body: bytes | str = b""):
    """Route one request through the REST handler without a socket."""
    if isinstance(body, bytes):
        body = body.decode()
    return _c().http_handle(server.handle, method, target, headers or {}, body)


# ---- client roles ------------------------------------------------------------------
class SdaClient:
    """Agent roles over any ``Service`` (client/src/lib.rs:28-47)."""

    def __init__(self, agent: Obj, keystore, service: Service, device: Optional[str] = None):
        """`device`: None / "cpu" = the host engines; "gpu" or "gpu:N" = the roles'
        bulk cryptography (clerk jobs, reveal, bulk participation) on MI355X N
        through ``libsda_device.so`` (raises if the library or a GPU is missing)."""
        self.service = service
        self.keystore = keystore
        self._h = _c().Client(_enc(agent), keystore, service.handle)
        if device not in (None, "", "cpu", "host"):
            self.use_device(device)

    def use_device(self, device: str = "gpu", library: str = "") -> str:
        """Switch the roles to the GPU backend; returns its description."""
        kind, _, index = device.partition(":")
        if kind != "gpu":
            raise ValueError("device must be 'cpu', 'gpu' or 'gpu:N'")
        return self._h.use_device(library, int(index or 0))

    def use_host(self) -> None:
        self._h.use_host()

    @property
    def device(self) -> Optional[str]:
        return self._h.device

    def device_timings(self) -> Dict[str, float]:
        """Milliseconds of the last GPU role call's stages."""
        return dict(self._h.device_timings())

    @classmethod
    def create(cls, keystore, service: Service, upload: bool = True,
               encryption_key: bool = True, device: Optional[str] = None) -> "SdaClient":
        """new_agent + (optionally) upload_agent + new/upload encryption key."""
        agent = json.loads(_c().Client.new_agent(keystore))
        cl = cls(agent, keystore, service, device=device)
        if upload:
            cl.upload_agent()
            if encryption_key:
                cl.upload_encryption_key(cl.new_encryption_key())
        return cl

    @property
    def agent(self) -> Obj:
        return json.loads(self._h.agent)

    @property
    def id(self) -> str:
        return self.agent["id"]

    # maintenance
    def upload_agent(self) -> None:
        self._h.upload_agent()

    def new_encryption_key(self) -> str:
        return self._h.new_encryption_key()

    def upload_encryption_key(self, key_id: str) -> None:
        self._h.upload_encryption_key(key_id)

    def sign_export(self, key_id: str) -> Optional[Obj]:
        return _dec(self._h.sign_export(key_id))

    # participating
    def new_participation(self, values: Sequence[int], aggregation_id: str) -> Obj:
        return json.loads(self._h.new_participation(list(values), aggregation_id))

    def upload_participation(self, participation: Obj) -> None:
        self._h.upload_participation(_enc(participation))

    def participate(self, values: Sequence[int], aggregation_id: str) -> None:
        self._h.participate(list(values), aggregation_id)

    def new_participations(self, vectors: Sequence[Sequence[int]], aggregation_id: str) -> List[Obj]:
        """One participation per input vector, sealed in bulk (on the GPU backend
        when one is set)."""
        return [json.loads(t) for t in
                self._h.new_participations([list(v) for v in vectors], aggregation_id)]

    def participate_many(self, vectors, aggregation_id: str) -> None:
        """`vectors`: a sequence of integer sequences, or a [P][D] numpy array."""
        if hasattr(vectors, "ndim"):
            self._h.participate_array(vectors, aggregation_id)
        else:
            self._h.participate_many([list(v) for v in vectors], aggregation_id)

    def role_timings(self) -> Dict[str, float]:
        """Milliseconds of the last clerk_once / reveal_aggregation: fetch (service
        calls: HTTP, JSON, base64), process (the cryptography), post."""
        return dict(self._h.role_timings())

    # clerking
    def clerk_once(self) -> bool:
        return self._h.clerk_once()

    def run_chores(self, max_iterations: int = -1) -> None:
        self._h.run_chores(max_iterations)

    def process_clerking_job(self, job: Obj) -> Obj:
        return json.loads(self._h.process_clerking_job(_enc(job)))

    # receiving
    def upload_aggregation(self, agg: Obj) -> None:
        self._h.upload_aggregation(_enc(agg))

    def begin_aggregation(self, aggregation_id: str) -> None:
        self._h.begin_aggregation(aggregation_id)

    def end_aggregation(self, aggregation_id: str) -> None:
        self._h.end_aggregation(aggregation_id)

    def reveal_aggregation(self, aggregation_id: str) -> Tuple[int, List[int]]:
        """(modulus, values) -- RecipientOutput (receive.rs:8-21)."""
        m, vals = self._h.reveal_aggregation(aggregation_id)
        return m, list(vals)

    @staticmethod
    def positive(modulus: int, values: Sequence[int]) -> List[int]:
        """RecipientOutput::positive -- map into [0, modulus)."""
        return [v % modulus for v in values]


# ---- client-side crypto engines (client/src/crypto/*) ---------------------------
def mask_secrets(scheme: Any, secrets: Sequence[int]):
    return _c().mask_secrets(_enc(scheme), list(secrets))


def combine_masks(scheme: Any, masks: Sequence[Sequence[int]]):
    return _c().combine_masks(_enc(scheme), [list(m) for m in masks])


def unmask(scheme: Any, mask: Sequence[int], masked: Sequence[int]):
    return _c().unmask(_enc(scheme), list(mask), list(masked))


def generate_shares(scheme: Obj, secrets: Sequence[int]):
    return _c().generate_shares(_enc(scheme), list(secrets))


def combine_shares(scheme: Obj, shares: Sequence[Sequence[int]]):
    return _c().combine_shares(_enc(scheme), [list(s) for s in shares])


def reconstruct_secrets(scheme: Obj, dimension: int, indexed: Sequence[Tuple[int, Sequence[int]]]):
    return _c().reconstruct_secrets(_enc(scheme), dimension, [(i, list(v)) for i, v in indexed])


def varint_encode(values: Sequence[int]) -> bytes:
    return _c().varint_encode(list(values))


def varint_decode(data: bytes) -> List[int]:
    return _c().varint_decode(data)
