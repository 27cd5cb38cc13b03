"""CLI end-to-end: the reference walkthrough (README.md:20-160,
docs/simple-cli-example.sh) with our `sdad` + `sda` binaries.

Recipient + 3 clerks with keys, 3 participants, aggregation of 10 values mod 433
shared 3 ways; expected reveal `0 2 2 4 4 6 6 8 8 10`.
"""
import os
import re
import signal
import socket
import subprocess

import pytest

from sda_amd._native import bin_path


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def sdad(tmp_path, native):
    exe = bin_path("sdad")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} missing: run `make host`")
    port = _free_port()
    proc = subprocess.Popen([exe, "--jfs", str(tmp_path / "server"), "httpd", "-b",
                             f"127.0.0.1:{port}"], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)
    line = proc.stdout.readline()  # "listening on port N" once bound
    assert "listening" in line, proc.stderr.read()
    try:
        yield f"http://127.0.0.1:{port}"
    finally:
        proc.send_signal(signal.SIGTERM)
        try:
            proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()


def _sda(server, ident, *args, check=True):
    r = subprocess.run([bin_path("sda"), "-s", server, "-i", str(ident), *args],
                       capture_output=True, text=True, timeout=60)
    if check:
        assert r.returncode == 0, f"sda {' '.join(args)} failed: {r.stderr}"
    return r


@pytest.mark.parametrize("mask,sharing,clerks", [("none", "add", 3), ("full", "add", 3),
                                                  ("chacha", "add", 3), ("none", "shamir", 8)])
def test_cli_walkthrough(sdad, tmp_path, mask, sharing, clerks):
    agents = tmp_path / "agent"
    names = ["recipient"] + [f"clerk-{i}" for i in range(1, clerks + 1)]
    for n in names:
        _sda(sdad, agents / n, "agent", "create")
        _sda(sdad, agents / n, "agent", "keys", "create")
    for n in ("part-1", "part-2", "part-3"):
        _sda(sdad, agents / n, "agent", "create")
    _sda(sdad, agents / "recipient", "ping")

    aggid = "ad3142d8-9a83-4f40-a64a-a8c90b701bde"
    keys = [f[:-5] for f in os.listdir(agents / "recipient" / "keys")
            if f.endswith(".json") and '"ek"' in (agents / "recipient" / "keys" / f).read_text()]
    assert len(keys) == 1
    _sda(sdad, agents / "recipient", "aggregations", "create", "--id", aggid, "aggro", "10", "433",
         keys[0], str(clerks), "--mask", mask, "--sharing", sharing)
    _sda(sdad, agents / "recipient", "aggregations", "begin", aggid)

    _sda(sdad, agents / "part-1", "participate", aggid, *"0 1 2 3 4 5 6 7 8 9".split())
    _sda(sdad, agents / "part-2", "participate", aggid, *"0 0 0 0 0 0 0 0 0 0".split())
    _sda(sdad, agents / "part-3", "participate", aggid, *"0 1 0 1 0 1 0 1 0 1".split())

    _sda(sdad, agents / "recipient", "aggregations", "end", aggid)
    for n in names:
        _sda(sdad, agents / n, "clerk", "--once")

    out = _sda(sdad, agents / "recipient", "aggregations", "reveal", aggid).stdout
    m = re.search(r"values: \[([^\]]*)\]", out)
    assert m, out
    assert [int(x) for x in m.group(1).split(",")] == [0, 2, 2, 4, 4, 6, 6, 8, 8, 10]


def test_cli_errors(sdad, tmp_path):
    r = _sda(sdad, tmp_path / "nobody", "participate", "ad3142d8-9a83-4f40-a64a-a8c90b701bde", "1",
             check=False)
    assert r.returncode == 1 and "Agent is needed" in r.stderr
    r = _sda("http://127.0.0.1:1", tmp_path / "x", "ping", check=False)
    assert r.returncode == 1
    r = subprocess.run([bin_path("sda"), "bogus"], capture_output=True, text=True, timeout=30)
    assert r.returncode != 0


def test_agent_create_is_idempotent(sdad, tmp_path):
    ident = tmp_path / "a"
    _sda(sdad, ident, "agent", "create")
    first = _sda(sdad, ident, "agent", "show").stdout
    r = _sda(sdad, ident, "agent", "create")
    assert "existing agent" in r.stderr
    assert _sda(sdad, ident, "agent", "show").stdout == first
    # keys show lists what keys create made
    kid = _sda(sdad, ident, "agent", "keys", "create").stdout.strip()
    assert kid in _sda(sdad, ident, "agent", "keys", "show").stdout.split()


# ---- hostile HTTP input against the real daemon ------------------------------------
def _raw(server, payload: bytes, read=True) -> bytes:
    import socket

    host, port = server[len("http://"):].split(":")
    with socket.create_connection((host, int(port)), timeout=10) as s:
        s.sendall(payload)
        if not read:
            return b""
        s.settimeout(10)
        chunks = []
        try:
            while True:
                b = s.recv(65536)
                if not b:
                    break
                chunks.append(b)
        except OSError:
            pass
        return b"".join(chunks)


def _ping_ok(server):
    rep = _raw(server, b"GET /v1/ping HTTP/1.1\r\nConnection: close\r\n\r\n")
    return rep.startswith(b"HTTP/1.1 200") and b'{"running":true}' in rep


@pytest.mark.parametrize("payload,status", [
    (b"POST /v1/agents/me HTTP/1.1\r\nContent-Length: abc\r\n\r\n", b"400"),
    (b"POST /v1/agents/me HTTP/1.1\r\nContent-Length: -1\r\n\r\n", b"400"),
    (b"POST /v1/agents/me HTTP/1.1\r\nContent-Length: 99999999999999999999999\r\n\r\n", b"400"),
    (b"GET /v1/ping?a=%zz HTTP/1.1\r\n\r\n", b"400"),
    (b"GET /v1/ping?a=%4 HTTP/1.1\r\n\r\n", b"400"),
    (b"POST /v1/agents/me HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n", b"400"),
    (b"POST /v1/agents/me HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nffffffffffffffff\r\n", b"413"),
    (b"POST /v1/agents/me HTTP/1.1\r\nContent-Length: 999999999999\r\n\r\n", b"413"),
    (b"\r\n\r\n", b"400"),
])
def test_daemon_survives_malformed_requests(sdad, payload, status):
    """Unauthenticated garbage is answered (400 / 413), never fatal: the
    reference server answers such requests with an error too (rouille;
    server-http/src/lib.rs:105-122)."""
    rep = _raw(sdad, payload)
    assert rep.startswith(b"HTTP/1.1 " + status), rep[:200]
    assert _ping_ok(sdad)


def test_daemon_enforces_body_budget(tmp_path, native):
    """--max-body-mb bounds request bodies before they are buffered."""
    exe = bin_path("sdad")
    port = _free_port()
    proc = subprocess.Popen([exe, "--memory", "httpd", "-b", f"127.0.0.1:{port}",
                             "--max-body-mb", "1"], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)
    try:
        assert "listening" in proc.stdout.readline()
        server = f"http://127.0.0.1:{port}"
        rep = _raw(server, b"POST /v1/agents/me HTTP/1.1\r\nContent-Length: 2000000\r\n\r\n")
        assert rep.startswith(b"HTTP/1.1 413"), rep[:200]
        # chunked: the declared chunk alone exceeds the budget
        rep = _raw(server, b"POST /v1/agents/me HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n"
                           b"200000\r\n")
        assert rep.startswith(b"HTTP/1.1 413"), rep[:200]
        assert _ping_ok(server)
    finally:
        proc.send_signal(signal.SIGTERM)
        try:
            proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()


@pytest.mark.parametrize("args", [[], ["--mask", "full", "--sharing", "shamir", "--clerks", "8"]])
def test_walkthrough_script(native, args):
    """docs/cli-walkthrough.sh: the reference's docs/simple-cli-example.sh for these
    binaries, which -- unlike that script -- fails unless the revealed sum is right."""
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "docs",
                          "cli-walkthrough.sh")
    r = subprocess.run(["bash", script, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "values: [0, 2, 2, 4, 4, 6, 6, 8, 8, 10]" in r.stdout
    assert r.stdout.strip().splitlines()[-1].startswith("walkthrough ok")
