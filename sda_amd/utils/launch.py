"""Start the per-GPU worker processes of a benchmark from a plain command line.

``python bench.py --gpus N`` with no rendezvous environment is the caller
asking for N ranks: the script starts them as *fresh child processes* through
``python -m torch.distributed.run`` (one rank per GPU, rendezvous on 127.0.0.1)
and relays their output and return code. The parent never initialises the GPU
and never replaces itself with another program (the machines this runs on
refuse an exec from a process that has touched the GPU): it only waits.

Nothing here imports torch.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Optional, Sequence


def wants_self_launch(gpus: int, environ=None) -> bool:
    """True when `gpus` > 1 ranks were asked for and this process is not already one
    of them (torch.distributed.run exports WORLD_SIZE / RANK to its workers)."""
    env = os.environ if environ is None else environ
    return gpus > 1 and "WORLD_SIZE" not in env and "RANK" not in env


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(script: str, argv: Sequence[str], nproc: int, port: Optional[int] = None,
                timeout: Optional[float] = None) -> int:
    """Run `script argv` as `nproc` ranks under torch.distributed.run; stdout and
    stderr pass through (rank 0 prints the result line). Returns the launcher's
    return code: non-zero if any rank failed."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
           "--master-port", str(port or free_port()), script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL peer buffers need dmabuf IPC here
    env.setdefault("OMP_NUM_THREADS", "1")
    proc = subprocess.Popen(cmd, env=env)
    try:
        return proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        proc.terminate()
        try:
            proc.wait(timeout=20)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
        return 124
    except KeyboardInterrupt:
        proc.terminate()
        proc.wait()
        return 130
