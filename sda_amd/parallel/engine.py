"""Distributed aggregation: one process per GPU, torch.distributed over RCCL/xGMI.

Two layouts.

``committee`` (default, the protocol's trust model): every rank owns a shard of
the participants and seals their boxes for every clerk; the snapshot transpose
is a grouped RCCL send/recv that routes each clerk's boxes to ranks playing that
clerk (parallel/routing.py: no rank sees two clerks' shares of a participant,
every rank opens exactly n * P boxes, traffic spread over all xGMI peers);
ranks open + combine their inbox per clerk; the per-clerk partial sums (clerk
internal) and the mask partials are reduced to rank 0, the recipient.

``owner`` (upper bound, *not* privacy-preserving across GPUs): every rank owns a shard of the participants
and runs their whole pipeline locally -- mask, share, seal one box per clerk,
and the clerks' open + combine over *its* boxes. A clerk's combine is a sum
over participants, so each rank holds per-clerk partial sums; one bucketed
``reduce`` (all clerk rows + the mask row, int32 when ``world * m < 2^31``)
brings them to rank 0, which plays the recipient (re-seal, open, reconstruct,
unmask). Sealed boxes never cross xGMI: the only inter-GPU traffic per round is
``(n_clerks + mask) * D`` integers, independent of the participant count,
which keeps a point-to-point xGMI ring far from the bottleneck.

The clerk and recipient keypairs are generated on rank 0 and broadcast (a
clerk is one organisation whose job happens to run on several GPUs).

Reference context: participation routing and the snapshot transpose
(server/src/snapshot.rs:4-47) are what this replaces; the clerk combine is
client/src/clerk.rs:63-107, the recipient's reveal client/src/receive.rs:80-157.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from ..models.schemes import AggregationSpec
from .comm import Comm


def _owner_base(rank: int) -> int:
    # RNG stream ids are purpose<<56 | owner: give every rank a disjoint owner range
    return rank << 40


class DistributedAggregator:
    """Multi-process round runner over a device or host engine.

    ``engine="device"``: :class:`sda_amd.engine.DeviceAggregator` on
    ``cuda:LOCAL_RANK`` (the MI355X path). ``engine="host"``:
    :class:`sda_amd.host_engine.HostAggregator` (CPU; gloo tests).
    """

    def __init__(self, spec: AggregationSpec, engine: str = "device", device=None, group=None,
                 time_stages: bool = False, layout: str = "committee", waves: int = 4,
                 force_pipeline: bool = False):
        self.spec = spec
        self.comm = Comm(group)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.kind = engine
        n = spec.n_clerks
        keybuf = self._shared_keys(n + 1)
        if engine == "device":
            from ..engine import DeviceAggregator, KeyTable, _words

            if device is None:
                device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
            pk = [bytes(keybuf[i, :32].tolist()) for i in range(n + 1)]
            sk = [bytes(keybuf[i, 32:].tolist()) for i in range(n + 1)]
            keys = KeyTable(torch.tensor([_words(b) for b in pk], dtype=torch.int32, device=device),
                            torch.tensor([_words(b) for b in sk], dtype=torch.int32, device=device),
                            pk, sk)
            self.engine = DeviceAggregator(spec, device=device, keys=keys, time_stages=time_stages)
        elif engine == "host":
            from ..host_engine import HostAggregator, HostKeys

            keys = HostKeys([bytes(keybuf[i, :32].tolist()) for i in range(n + 1)],
                            [bytes(keybuf[i, 32:].tolist()) for i in range(n + 1)])
            self.engine = HostAggregator(spec, keys=keys)
        else:
            raise ValueError("engine must be 'device' or 'host'")
        # int32 reduction is exact when the sum of `world` values < m fits
        self._narrow = self.world * (spec.field_modulus - 1) < 2 ** 31
        if layout not in ("committee", "owner"):
            raise ValueError("layout must be 'committee' or 'owner'")
        self.layout = layout
        self.waves = max(1, waves)  # committee layout: exchange pipelined over participant waves
        self.force_pipeline = force_pipeline  # pipeline even on one rank (overhead measurement)
        self._routers = {}

    def _shared_keys(self, count: int) -> np.ndarray:
        from .._native import native

        buf = np.zeros((count, 64), dtype=np.uint8)
        if self.rank == 0:
            for i in range(count):
                pk, sk = native().crypto.box_keypair()
                buf[i, :32] = np.frombuffer(pk, dtype=np.uint8)
                buf[i, 32:] = np.frombuffer(sk, dtype=np.uint8)
        t = torch.from_numpy(buf)
        if self.comm.device_native:
            t = t.to(torch.device("cuda", torch.cuda.current_device()))
        t = self.comm.broadcast(t, src=0)
        return t.cpu().numpy() if isinstance(t, torch.Tensor) else t

    def _reduce(self, partials):
        """Sum the per-clerk (+ mask) partial rows over ranks onto rank 0."""
        if isinstance(partials, np.ndarray):
            wire = partials.astype(np.int32) if self._narrow else partials
            out = self.comm.reduce_sum(wire)
            return None if out is None else out.astype(np.int64)
        wire = partials.to(torch.int32) if self._narrow else partials
        out = self.comm.reduce_sum(wire)
        return None if out is None else out.to(torch.int64)

    def router(self, P):
        """Committee router for waves of P participants (P=None: any router,
        for plan-independent transfers through the communicator)."""
        if self.layout != "committee":
            return None
        if P is None:
            from types import SimpleNamespace

            return SimpleNamespace(comm=self.comm)
        if P not in self._routers:
            from .router import CommitteeRouter

            self._routers[P] = CommitteeRouter(self.comm, self.spec.n_clerks, P)
        return self._routers[P]

    def run_round(self, secrets_local, clerks: Optional[Sequence[int]] = None,
                  check: bool = True):
        """One round over every rank's participants; rank 0 gets the output.

        Every rank must hold the same number of participants (the routing
        plan cuts each clerk's P boxes into fixed parts).
        """
        P = int(secrets_local.shape[0])
        if self.kind == "device" and self.layout == "committee" and (self.world > 1 or
                                                                      self.force_pipeline):
            return self.engine.run_round(secrets_local, clerks=clerks, check=check,
                                         reducer=self._reduce, owner_base=_owner_base(self.rank),
                                         router_for=self.router, waves=min(self.waves, P))
        return self.engine.run_round(secrets_local, clerks=clerks, check=check,
                                     reducer=self._reduce, owner_base=_owner_base(self.rank),
                                     router=self.router(P))

    def run_streamed(self, total_local: int, make_wave, wave: int = 64,
                     clerks: Optional[Sequence[int]] = None, checkpoint: Optional[str] = None,
                     checkpoint_every: int = 8, resume: bool = True):
        """Stream this rank's `total_local` participants in waves (device engine).

        Every rank must stream the same number of participants with the same
        wave size (the routing plan is per wave size). Checkpoints are per
        rank: pass a rank-specific path.
        """
        if self.kind != "device":
            raise ValueError("streaming runs on the device engine")
        from ..streaming import StreamingAggregator

        st = StreamingAggregator(self.engine, wave=wave, checkpoint=checkpoint,
                                 checkpoint_every=checkpoint_every)
        return st.run(total_local, make_wave, clerks=clerks, reducer=self._reduce,
                      router_for=self.router if self.layout == "committee" else None,
                      owner_base=_owner_base(self.rank), resume=resume)
