"""Starting N ranks from a plain command line, the loopback exchange, and
rendezvous isolation between engines on one process group (CPU, gloo).

`python bench.py --gpus N` is how the scaling runs are started: with no
rendezvous environment the script must start its own N workers as child
processes and relay rank 0's JSON line and the return code. The CPU rehearsal
(`--engine host`) runs the same launcher and the same committee dataflow
(reference: server/src/snapshot.rs:11-27 transpose, client/src/clerk.rs:79-100,
client/src/receive.rs:127-144) on the C++ client engines over gloo.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, script), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_wants_self_launch_only_outside_a_launcher():
    from sda_amd.utils.launch import wants_self_launch

    assert wants_self_launch(2, environ={})
    assert not wants_self_launch(1, environ={})
    assert not wants_self_launch(2, environ={"WORLD_SIZE": "2", "RANK": "0"})


def test_launch_module_does_not_import_torch():
    code = ("import sys; import sda_amd.utils.launch; "
            "sys.exit(1 if 'torch' in sys.modules else 0)")
    assert subprocess.run([sys.executable, "-c", code], cwd=ROOT).returncode == 0


@pytest.mark.parametrize("world", [2, 3])
def test_bench_starts_its_own_ranks(native, world):
    out = _run("bench.py", "--gpus", str(world), "--engine", "host", "--participants", "4",
               "--dim", "60", "--steps", "1", "--warmup", "1")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = _json_lines(out)
    assert len(lines) == 1, out.stdout  # one line, from rank 0
    line = lines[0]
    assert line["ranks"] == world and line["value"] > 0
    assert line["config"]["global_batch"] == 4 * world
    assert line["xgmi"]["bytes_sent_per_rank_per_round"] > 0  # sealed boxes crossed ranks


def test_launcher_relays_a_failing_rank(tmp_path):
    """A worker that exits non-zero fails the parent too (the return code a
    caller of `bench.py --gpus N` sees)."""
    from sda_amd.utils.launch import self_launch

    script = tmp_path / "worker.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert self_launch(str(script), [], 2, timeout=120) != 0
    script.write_text("import os\nassert os.environ['WORLD_SIZE'] == '2'\n")
    assert self_launch(str(script), [], 2, timeout=120) == 0


def test_bench_rejects_a_launcher_of_another_size(native):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--engine",
                          "host"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "launcher started 1" in out.stderr


def test_loopback_round_on_one_rank(native):
    """World 1 with loopback: the rank's own piece of every exchange goes through
    the exchange path (matched send/recv pairs) instead of a local copy."""
    out = _run("bench.py", "--gpus", "1", "--engine", "host", "--loopback", "--participants", "5",
               "--dim", "40", "--steps", "1", "--warmup", "1")
    assert out.returncode == 0, out.stderr[-3000:]
    assert _json_lines(out)[0]["ranks"] == 1


def _two_engines(rank, world, port, q):
    import datetime

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        from sda_amd.models.schemes import PSS_4_8_3, AggregationSpec
        from sda_amd.parallel import DistributedAggregator

        spec = AggregationSpec(9, 433, PSS_4_8_3)
        ok = []
        prefixes = []
        for inst in range(2):
            agg = DistributedAggregator(spec, engine="host", deadline_s=4.0)
            prefixes.append(agg.comm._nonce)
            x = np.random.default_rng(7 * inst + rank).integers(0, 433, size=(2, 9), dtype=np.int64)
            res = agg.run_round(x)
            tot = agg.comm.reduce_sum(x.sum(0))
            if rank == 0:
                ok.append(bool(np.array_equal(res.output, np.remainder(tot, 433))))
            # the first engine's round-1 flags must be invisible to the second engine
            if inst == 1 and rank == 0:
                ok.append(not agg.comm.store.check(["r2/res/live"]))
        q.put(("ok", rank, ok, prefixes))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", rank, f"{type(e).__name__}: {e}", []))


def test_two_engines_on_one_process_group_do_not_share_rendezvous_keys(native):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_engines, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    assert all(r[0] == "ok" for r in results), results
    for r in results:
        assert all(r[2]), results
        assert r[3][0] != r[3][1]  # a prefix per engine instance
