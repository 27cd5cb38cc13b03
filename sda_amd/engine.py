"""Device aggregation engine: one full SDA round on a single MI355X.

Simulates P participants, an n-clerk committee and the recipient with the
exact cryptographic dataflow of the reference protocol:

  participate  (client/src/participate.rs:37-113)
      mask -> share -> per-clerk sealed boxes (+ sealed mask for the recipient)
  snapshot     (server/src/snapshot.rs:4-47)
      transpose P x n -> n x P : free, shares are written clerk-major
  clerk        (client/src/clerk.rs:63-107)
      open P boxes -> combine (sum mod m) -> seal the result for the recipient
  reveal       (client/src/receive.rs:80-157)
      open n results -> reconstruct (sum / Lagrange, any >= t+k clerks) ->
      unmask (sum of masks / ChaCha seed expansion) -> output in [0, m)

Every stage is a HIP kernel (csrc/kernels). Keys are real X25519 keypairs; the
per-round randomness is a fresh 256-bit key from OS entropy driving counter-mode
ChaCha20 streams (one per participant and purpose).
"""
from __future__ import annotations

import collections
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from ._native import native
from .models.schemes import Additive, AggregationSpec, ChaChaMask, FullMask, PackedShamir
from .ops import gpu as G
from .ops.sealed import (Arena, KeySet, open_, open_data, open_setup, open_sum, seal, seal_data,
                         seal_setup)
from .utils.trace import tracing_enabled

_TRACE = tracing_enabled()
# unchecked rounds the host may queue ahead of the GPU (see DeviceAggregator.throttle)
_MAX_INFLIGHT = 2


class AggregationError(RuntimeError):
    pass


_SIDE_STREAMS: dict = {}


def concurrent_stream(device, tries: int = 12, spin_us: int = 250, slot: str = "side",
                      beside: Sequence["torch.cuda.Stream"] = ()) -> "torch.cuda.Stream":
    """A stream whose kernels really run beside the current stream's (and beside
    those of the streams in `beside`); one per current stream and `slot`.

    HIP multiplexes a process's streams onto few hardware queues (4 by default),
    and two streams on one queue serialise -- which of them share a queue
    depends on how many streams the process (and RCCL) created before. The
    side stream carries latency-bound X25519 ladders that must overlap the
    main stream's bulk kernels, so candidates are probed: the main stream runs
    a bounded 250 us wait (a gate the host never posts), the candidate a no-op;
    a candidate that finishes while the wait is still running sits on another
    queue. Falls back to the last candidate (correct, only slower)."""
    dev = torch.device(device)
    main = torch.cuda.current_stream(dev)
    key = (dev.index, main.cuda_stream, slot)
    if key in _SIDE_STREAMS:
        return _SIDE_STREAMS[key]
    gate = torch.zeros(1, dtype=torch.int32, device=dev)
    cand = None
    with torch.cuda.device(dev):
        for _ in range(tries):
            cand = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(cand):
                # a stream's first launch attaches it to its hardware queue, which takes
                # longer than the spin below: measured cold, every candidate looked late
                G.gate_wait((gate, 0), timeout_us=1)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            torch.cuda.synchronize(dev)
            e0.record(main)
            G.gate_wait((gate, 1), timeout_us=spin_us)  # main: never posted, ends at the limit
            if beside:
                # a wait for the end of that spin queued on each of them: a stream's wait
                # holds up everything behind it in its hardware queue, other streams'
                # kernels included (seen in a kernel trace: key agreement submitted on
                # one stream stood behind the result path's wait for the main stream)
                spun = torch.cuda.Event()
                spun.record(main)
                for other in beside:
                    other.wait_event(spun)
            with torch.cuda.stream(cand):
                G.gate_wait((gate, 0), timeout_us=1)    # candidate: returns at once
                e1.record(cand)
            e2.record(main)
            torch.cuda.synchronize(dev)
            if e0.elapsed_time(e1) < 0.5 * e0.elapsed_time(e2):
                break
    _SIDE_STREAMS[key] = cand
    return cand


def _words(b: bytes) -> list[int]:
    return [int.from_bytes(b[4 * i:4 * i + 4], "little", signed=True) for i in range(len(b) // 4)]


@dataclass
class KeyTable:
    """X25519 keypairs: index 0..n-1 = clerks, index n = recipient.

    A process that plays only some of the parties holds only their secret
    keys: `sk_bytes[i]` is None (and row i of `sks` zero) for the others."""

    pks: torch.Tensor  # int32 [K][8]
    sks: torch.Tensor  # int32 [K][8]
    pk_bytes: list = field(default_factory=list)
    sk_bytes: list = field(default_factory=list)

    @classmethod
    def from_bytes(cls, pk: list, sk: list, device) -> "KeyTable":
        zero = bytes(32)
        pks = torch.tensor([_words(p) for p in pk], dtype=torch.int32, device=device)
        sks = torch.tensor([_words(s if s is not None else zero) for s in sk], dtype=torch.int32,
                           device=device)
        return cls(pks, sks, list(pk), list(sk))

    def holds(self, i: int) -> bool:
        return self.sk_bytes[i] is not None

    # launches of at least this many boxes use the keys' fixed-base tables (the
    # many-message form of the seal-side key agreement, keys.hip)
    TABLE_MIN_BOXES = 65536

    def tables(self, boxes: int | None = None):
        """Fixed-base tables of the public keys (int32 [K][KEY_TABLE_WORDS], built on
        the host once and kept): with them a sealed box's shared point costs 64 table
        additions instead of a 255-step ladder. None below `TABLE_MIN_BOXES` boxes, where
        the launch is latency-bound and the two-ladder kernel runs anyway."""
        if boxes is not None and boxes < self.TABLE_MIN_BOXES:
            return None
        if getattr(self, "_tables", None) is None:
            blob, _ok = native().crypto.x25519_comb_tables(list(self.pk_bytes))
            t = torch.frombuffer(bytearray(blob), dtype=torch.int32)
            self._tables = t.view(len(self.pk_bytes), G.KEY_TABLE_WORDS).to(self.pks.device)
        return self._tables

    @classmethod
    def generate(cls, count: int, device) -> "KeyTable":
        c = native().crypto
        pairs = [c.box_keypair() for _ in range(count)]
        pk = [p for p, _ in pairs]
        sk = [s for _, s in pairs]
        pks = torch.tensor([_words(p) for p in pk], dtype=torch.int32, device=device)
        sks = torch.tensor([_words(s) for s in sk], dtype=torch.int32, device=device)
        return cls(pks, sks, pk, sk)


class RoundResult:
    """What a round returns: `output` (int32 [D], canonical in [0, m); None on the
    ranks of a reduced round that do not reveal), `clerks_used`, `stage_ms`, and
    `err`, the round's device error word (int32 [1]; see describe_error) -- already
    read and raised on when the round ran with check=True; callers that time
    unchecked rounds OR these together and read the result once.

    An unchecked round may have run its recipient stage on a stream of its own
    (DeviceAggregator.run_round): `output` and `err` then belong to that stream
    until first read, and reading them makes the *current* stream wait for it.
    A loop that wants the next round's kernels to start meanwhile reads them one
    round late."""

    def __init__(self, output, clerks_used, stage_ms, err: Optional[torch.Tensor] = None):
        self._output, self._err = output, err
        self.clerks_used, self.stage_ms = clerks_used, stage_ms
        self._ready = None  # (event, device) while the recipient stage's stream owns the tensors

    def _join(self):
        if self._ready is not None:
            ev, dev = self._ready
            self._ready = None
            cur = torch.cuda.current_stream(dev)
            cur.wait_event(ev)
            for t in (self._output, self._err):
                if t is not None:
                    t.record_stream(cur)

    @property
    def output(self):
        self._join()
        return self._output

    @output.setter
    def output(self, value):
        self._output = value

    @property
    def err(self):
        self._join()
        return self._err

    @err.setter
    def err(self, value):
        self._err = value


class DeviceAggregator:
    """Runs complete aggregation rounds for one :class:`AggregationSpec`."""

    def __init__(self, spec: AggregationSpec, device=None, keys: KeyTable | None = None,
                 time_stages: bool = False, pss_backend: str = "auto", share_storage: str = "auto"):
        self.spec = spec
        self.device = torch.device(device or "cuda")
        self.n = spec.n_clerks
        self.m = spec.field_modulus
        self.keys = keys or KeyTable.generate(self.n + 1, self.device)
        self.vdtype = G.value_dtype(self.m)
        if isinstance(spec.sharing, PackedShamir) and self.m <= 256 and share_storage != "u16":
            self.vdtype = torch.uint8  # a field element per byte
        self.time_stages = time_stages
        # rounds run their result path on a stream of its own (_reveal_beside)
        self.overlap_reveal = True
        self._round = 0
        if isinstance(spec.sharing, PackedShamir):
            p = spec.sharing.native()
            p.validate()
            self._pss = p
            self._share_matrix = torch.tensor(p.share_matrix(), dtype=torch.int64).to(
                torch.int32).to(self.device)
            ps = spec.sharing
            big = ps.secret_count > 8 or ps.privacy_threshold_ > 16 or ps.share_count > 64
            if pss_backend not in ("auto", "mfma", "valu"):
                raise ValueError("pss_backend must be auto, mfma or valu")
            if pss_backend == "valu" and big:
                raise ValueError("the register (VALU) PSS kernel supports k<=8, t<=16, n<=64")
            # matrix cores (int8-limb MFMA GEMM) for the large parameter sets
            self._pss_mfma = pss_backend == "mfma" or (pss_backend == "auto" and big)
            if self._pss_mfma:
                self._Kp = G.padded_k(ps.secret_count + ps.privacy_threshold_)
                self._limbs = G.limb_count(self.m, self._Kp)
                self._M_limbs = G.limbs_of(
                    self._share_matrix.view(self.n, ps.secret_count + ps.privacy_threshold_),
                    self._Kp, self.m)
                self._M_frag = G.a_fragments(self._M_limbs) if self._Kp <= G.PANEL_MAX_K else None
        else:
            self._pss = None
            self._pss_mfma = False

    # ------------------------------------------------------------ helpers ----
    def _key_idx(self, values: Sequence[int]) -> torch.Tensor:
        return torch.tensor(list(values), dtype=torch.int32, device=self.device)

    def _mark(self, marks, name):
        # stage boundary: a roctx marker under SDA_TRACE=1 (rocprofv3 --marker-trace),
        # a timing event with time_stages
        if _TRACE:
            torch.cuda.nvtx.mark(f"sda:{name}")
        if self.time_stages:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append((name, ev))

    # ---------------------------------------------------------- the round ----
    def _share(self, secrets, rng_key, owner_base, err):
        """Mask + share (+ byte counts): shares [n][P][B], cnt, mask values/seeds."""
        spec, n, m = self.spec, self.n, self.m
        P, D = secrets.shape
        B = spec.batches
        dev = self.device
        shares = torch.empty(n, P, B, dtype=self.vdtype, device=dev)
        cnt = torch.empty(n * P * G.tiles(B), dtype=torch.int32, device=dev)
        mask_vals, mask_cnt = None, None
        full = isinstance(spec.masking, FullMask)
        if isinstance(spec.masking, ChaChaMask):
            # masking/chacha.rs:29-45: a fresh seed per participant, masked = secret +
            # its rand-0.3 stream. A pre-pass, so the shares come from the fast kernels;
            # what travels to the recipient is the seed.
            mask_vals = G.chacha_seeds(P, spec.masking.seed_words, rng_key, owner_base, dev)
            secrets = G.chacha_mask_apply(secrets, mask_vals, m, err)
        elif full:
            # the masks in the shares' storage type (u16 where m <= 65536: half the
            # bytes written here and read by the encoder), 32-bit ahead of the limb GEMM
            mask_vals = torch.empty(P, D, dtype=torch.int32 if self._pss_mfma else self.vdtype,
                                    device=dev)
            mask_cnt = torch.empty(P * G.tiles(D), dtype=torch.int32, device=dev)
        if self._pss_mfma:
            # masks (if any) first, then S = M . X on the matrix cores
            masked = secrets
            if full:
                masked = G.mask_secrets(secrets, m, rng_key, owner_base, mask_vals, mask_cnt)
            ps = spec.sharing
            X = G.pss_x_limbs(masked, ps.secret_count, ps.privacy_threshold_, m, rng_key, owner_base)
            cnt.zero_()  # the GEMM epilogue adds the boxes' varint bytes into it
            G.modgemm_i8(self._M_limbs, X, m, shares, ldc_z=B, ldc_m=P * B, ldc_n=1,
                         limit=n * P * B, cnt=cnt, a_frag=self._M_frag)
            return shares, cnt, mask_vals, mask_cnt
        mode = G.MASK_FULL if full else G.MASK_NONE
        if self._pss is None:
            G.share_additive(secrets, n, m, shares, cnt, mode, rng_key, owner_base,
                             mask_out=mask_vals if full else None, mask_cnt=mask_cnt)
        else:
            ps = spec.sharing
            G.share_pss(secrets, n, ps.secret_count, ps.privacy_threshold_, m,
                        self._share_matrix, shares, cnt, mode, rng_key, owner_base,
                        mask_out=mask_vals if full else None)
            mask_cnt = None  # PSS batches do not align with mask tiles: recounted
        return shares, cnt, mask_vals, mask_cnt

    def _gate_token(self):
        """A fresh (tensor, value) dispatch token for a side-stream setup kernel
        that a main-stream `gate_wait` orders ahead of the next big grid."""
        if getattr(self, "_gate", None) is None:
            self._gate = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._gate_val = 0
        self._gate_val = (self._gate_val + 1) & 0x7FFFFFFF or 1
        return self._gate, self._gate_val

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            # default priority, like every stream of the process: its kernels are
            # latency-bound X25519 ladders that raise their own wave priority
            self._side = concurrent_stream(self.device)
        return self._side

    def _tail_stream(self):
        if getattr(self, "_tail", None) is None:
            # beside the main stream and beside the side stream: on the side stream's
            # queue the next round's key agreement would wait for this round's result
            # path, and the main stream's first grid waits for that key agreement
            self._tail = concurrent_stream(self.device, slot="tail", beside=[self._side_stream()])
        return self._tail

    def _live(self, clerks):
        spec, n = self.spec, self.n
        live = list(range(n)) if clerks is None else sorted(set(int(c) for c in clerks))
        if self._pss is None and len(live) != n:
            raise AggregationError("additive sharing needs every clerk's result")
        if self._pss is not None and len(live) < spec.sharing.reconstruction_threshold():
            raise AggregationError("Not enough shares to reconstruct")
        return live

    def corrupt_next_round(self) -> None:
        """Fault injection: flip one ciphertext bit of the next round's first
        sealed box in transit (the clerk's MAC check must then fail the round)."""
        self._corrupt = True

    def _inject_corruption(self, arena: Arena) -> None:
        if getattr(self, "_corrupt", False):
            self._corrupt = False
            arena.ct[G.SEAL_OVERHEAD + 5] ^= 1

    def new_error_word(self) -> torch.Tensor:
        return torch.zeros(1, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------- planning ----
    def free_bytes(self) -> int:
        """Device memory a round can still claim: what the driver reports free plus
        what the caching allocator holds but has not handed out."""
        free, _ = torch.cuda.mem_get_info(self.device)
        held = torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        return int(free + max(0, held))

    def plan(self, participants: int, input_resident: bool = True, free_bytes: int | None = None):
        """The :class:`sda_amd.planner.RoundPlan` for `participants` vectors on this
        device now (cached per participant count)."""
        from .planner import plan_round

        if free_bytes is None:
            free_bytes = getattr(self, "memory_limit_bytes", None)  # a cap set by the caller
        cache = self.__dict__.setdefault("_plans", {})
        key = (participants, input_resident, free_bytes)
        if key not in cache:
            cache[key] = plan_round(
                self.spec, participants, self.free_bytes() if free_bytes is None else free_bytes,
                pss_backend="mfma" if self._pss_mfma else ("valu" if self._pss is not None else "auto"),
                share_storage="u16" if self.vdtype == torch.int16 else "auto",
                input_resident=input_resident)
        return cache[key]

    def run_round(self, secrets: torch.Tensor, clerks: Sequence[int] | None = None,
                  check: bool = True, reducer=None, owner_base: int = 0) -> RoundResult:
        """One full round for participant vectors `secrets` [P][D] (int32, on device).

        = :meth:`participate_and_clerk` (+ `reducer`) + :meth:`reveal`.

        `reducer(partials) -> reduced | None` (the multi-GPU ``owner`` layout,
        a non-private upper bound): called with the per-clerk column sums over
        this device's participants -- int64 [len(live) (+1 with a mask)][max(B,
        D)] -- before the recipient stage; it returns the sums over all
        devices on the root and None elsewhere (which then skips the recipient
        stage and returns ``output=None``). `owner_base` offsets the
        participants' RNG stream ids. The protocol-faithful multi-GPU round is
        :class:`sda_amd.parallel.DistributedAggregator`'s ``committee`` layout.
        """
        live = self._live(clerks)
        plan = self.plan(secrets.shape[0])
        if not plan.resident:
            # too large to be resident: the same round in participant waves (only the
            # clerks' running sums persist between them) instead of an out-of-memory error
            from .streaming import StreamingAggregator

            st = StreamingAggregator(self, wave=plan.wave)
            sr = st.run(secrets.shape[0], lambda w, first, count: secrets[first:first + count],
                        clerks=clerks, reducer=reducer, owner_base=owner_base, check=check)
            return RoundResult(sr.output, sr.clerks_used, sr.stage_ms, err=sr.err)
        err = self.new_error_word()
        marks: list = []
        self._mark(marks, "start")
        combined, mask_sum = self.participate_and_clerk(secrets, live, err, owner_base=owner_base,
                                                        marks=marks)
        main = torch.cuda.current_stream(self.device)
        if self.overlap_reveal and reducer is None and not self.time_stages:
            # checked rounds too: the same path (and the same stream's memory pool)
            # whether or not the caller reads the result at once
            result = self._reveal_beside(main, combined, mask_sum, live, err)
            if check:
                e = int(result.err.item())  # joins the tail stream, then the host
                if e:
                    raise AggregationError(f"device error word 0x{e:x} ({describe_error(e)})")
            return result
        if getattr(self, "_tail_ev", None) is not None:
            # an earlier round's recipient stage ran on the tail stream: whatever it
            # created there for later rounds (cached matrices) is ordered before this one
            main.wait_event(self._tail_ev)
        # the recipient's key agreement queues on the side stream BEHIND the
        # participants' and clerks' (needed last; ahead of them it delayed the
        # first encrypt by the length of an X25519 ladder)
        rk = self.prepare_reveal(live, err)
        if reducer is not None:
            combined, mask_sum = self.reduce_partials(combined, mask_sum, reducer, marks)
            if combined is None:
                return self._finish(err, marks, check, RoundResult(None, live, {}))
        out = self.reveal(combined, mask_sum, live, err, marks=marks, keys=rk)
        return self._finish(err, marks, check, RoundResult(out, live, {}))

    def _reveal_beside(self, main, combined, mask_sum, live, err) -> RoundResult:
        """The result path of a round -- clerks seal their sums, the recipient
        opens, reconstructs and unmasks -- on a third stream. It is a
        chain of ~15 dependent launches over a handful of boxes, 0.2 ms during
        which the card is nearly idle; on the main stream the next round's first
        grid waited for it. The result's tensors belong to that stream until
        first read (RoundResult)."""
        tail = self._tail_stream()
        # the recipient's key agreement is queued on the side stream first: should the
        # tail stream share its hardware queue after all, the wait below must not stand
        # in front of it
        rk = self.prepare_reveal(live, err)
        tail.wait_stream(main)
        for t in (combined, mask_sum, err, rk[0].ct, rk[0].pt_len, rk[1], rk[2]):
            if t is not None:  # tensors of the main and side streams used on the tail
                t.record_stream(tail)
        with torch.cuda.stream(tail):
            out = self.reveal(combined, mask_sum, live, err, keys=rk)
            result = self._finish(err, [], False, RoundResult(out, live, {}))
            ev = torch.cuda.Event()
            ev.record(tail)
        result._ready = (ev, self.device)
        self._tail_ev = ev
        return result

    def participate_and_clerk(self, secrets: torch.Tensor, live, err, owner_base: int = 0,
                              marks=None):
        """Participants mask + share + seal; clerks open + combine.

        Returns (combined [len(live)][B] int32 in [0, m), mask_sum [D] int32 or
        None): the clerks' sums over these participants and the recipient's
        sum of their masks. A fresh 256-bit round key is drawn per call, so
        ephemeral keys and share streams never repeat across calls (waves).

        Stream schedule: every X25519 / key-derivation kernel (participants'
        ephemeral keys, clerks' key agreement) runs on a side stream concurrently
        with the bandwidth-bound share/encode/MAC kernels of the main stream;
        the main stream waits on events only where it consumes derived keys.
        """
        marks = [] if marks is None else marks
        st = self._participate(secrets, live, err, owner_base)
        self._mark(marks, "participate")
        out = self._clerk(st, live, err)
        self._mark(marks, "clerk")
        return out

    def _participate(self, secrets, live, err, owner_base):
        """Mask + share + seal one batch of participants; returns the state the
        clerk half needs (arenas and derived keys)."""
        spec, n, m = self.spec, self.n, self.m
        if secrets.dim() != 2 or secrets.shape[1] != spec.dimension:
            raise ValueError("secrets must be [P][dimension]")
        if secrets.dtype != torch.int32 or secrets.device.type != "cuda":
            raise ValueError("secrets must be an int32 GPU tensor")
        secrets = secrets.contiguous()
        P, D = secrets.shape
        B = spec.batches
        dev = self.device
        rng_key = native().crypto.random_bytes(32)
        self._round += 1
        main = torch.cuda.current_stream(dev)
        side = self._side_stream()
        pks = self.keys.pks

        # ---- arenas (participants -> clerks, participants -> recipient)
        clerk_arena = Arena.empty(n * P, B, m, dev)
        mask_arena = None
        if isinstance(spec.masking, FullMask):
            mask_arena = Arena.empty(P, D, m, dev)
        elif isinstance(spec.masking, ChaChaMask):
            mask_arena = Arena.empty(P, spec.masking.seed_words, 0, dev)
        kidx_clerk = self._kidx_clerk(P)
        kidx_rcpt_p = self._kidx_recipient(P) if mask_arena is not None else None

        # ---- side stream: key agreement (data independent)
        gate = self._gate_token()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            # Poly1305 tables on the side stream too: the encrypt is ~3 ms away
            ks_clerk = seal_setup(clerk_arena, kidx_clerk, pks, rng_key, 0, err, gate=gate,
                                  pk_tables=self.keys.tables(n * P)).with_powers()
            ks_mask = (seal_setup(mask_arena, kidx_rcpt_p, pks, rng_key, n * P, err).with_powers()
                       if mask_arena is not None else None)
            ev_sealkeys = torch.cuda.Event()
            ev_sealkeys.record(side)

        def open_keys():
            with torch.cuda.stream(side):
                ko_clerk = self._open_keys(clerk_arena, kidx_clerk, live, P, err)
                ko_mask = (open_setup(mask_arena, kidx_rcpt_p, self.keys.sks, pks, err)
                           if mask_arena is not None else None)
                ev_openkeys = torch.cuda.Event()
                ev_openkeys.record(side)
            return ko_clerk, ko_mask, ev_openkeys

        # ---- participants: mask + share, then encrypt (waits for the seal keys)
        G.gate_wait(gate)  # the setup waves are resident before the share grid
        shares, cnt, mask_vals, mask_cnt = self._share(secrets, rng_key, owner_base, err)
        # the clerks' key agreement queues behind the share kernel, not beside it (beside
        # it, its ladder waves took register space from the share grid: measured slower)
        side.wait_stream(main)
        ko_clerk, ko_mask, ev_openkeys = open_keys()
        for t in [ks_clerk, ks_mask, ko_mask] + ko_clerk:
            if t is not None:
                t.record_stream(main)
        main.wait_event(ev_sealkeys)
        seal_data(clerk_arena, ks_clerk, shares.view(n * P, B), err, cnt)
        self._inject_corruption(clerk_arena)
        del shares
        if mask_arena is not None:
            seal_data(mask_arena, ks_mask, mask_vals, err, mask_cnt)
        return {"P": P, "kidx": kidx_clerk, "ev_openkeys": ev_openkeys, "mask_arena": mask_arena,
                "ko_mask": ko_mask, "inbox": clerk_arena, "ko_clerk": ko_clerk}

    def _clerk(self, st, live, err):
        """Open + combine an inbox (the local arena or the routed one)."""
        P = st["P"]
        main = torch.cuda.current_stream(self.device)
        main.wait_event(st["ev_openkeys"])
        inbox = st.pop("inbox")
        ko_clerk = st["ko_clerk"]
        combined = self._open_combine(inbox, ko_clerk, live, P, err)
        del inbox
        # recipient's share of the mask work is data-parallel too: open these
        # participants' mask boxes and sum them
        mask_sum = None
        mask_arena = st["mask_arena"]
        if mask_arena is not None:
            mask_sum = self._open_masks(mask_arena, st["ko_mask"], err)
        return combined, mask_sum

    def _open_combine(self, box: Arena, keys, live, P: int, err) -> torch.Tensor:
        """The clerks' open + combine (clerk.rs:79-86) of a clerk-major inbox of
        n x P boxes: [len(live)][B] int32 sums mod m, decode fused with the sum
        (:func:`open_sum`). `keys`: one KeySet for all n x P boxes, or a list
        with one per live clerk (``_open_keys``)."""
        n = self.n
        out = torch.empty(len(live), self.spec.batches, dtype=torch.int32, device=self.device)
        if isinstance(keys, list) and len(keys) == 1:
            keys = keys[0]
        if len(live) == n:
            open_sum(box, keys, err, rows=n, out=out)
        else:
            for i, c in enumerate(live):
                kc = keys[i] if isinstance(keys, list) else keys.slice(c * P, P)
                open_sum(box.slice(c * P, P), kc, err, rows=1, out=out[i])
        return out

    def _open_masks(self, mask_arena: Arena, keys, err) -> torch.Tensor:
        """Recipient: open the participants' mask boxes and sum the masks
        (full.rs:37-52) or re-expand and sum the ChaCha seeds (chacha.rs:56-77)."""
        D, m = self.spec.dimension, self.m
        mask_sum = torch.empty(D, dtype=torch.int32, device=self.device)
        if isinstance(self.spec.masking, FullMask):
            open_sum(mask_arena, keys, err, rows=1, out=mask_sum)
        else:
            seeds = open_data(mask_arena, keys, err, out_dtype=torch.int32)
            G.chacha_mask_sum(seeds, D, m, mask_sum, err)
        return mask_sum

    def reduce_partials(self, combined, mask_sum, reducer, marks=None):
        """Bucket the clerk rows (B wide) and the mask row (D wide) into one
        int64 buffer, reduce over devices, unpack on the root."""
        B, D, m = self.spec.batches, self.spec.dimension, self.m
        rows = combined.shape[0]
        nrow = rows + (1 if mask_sum is not None else 0)
        partials = torch.zeros(nrow, max(B, D), dtype=torch.int64, device=self.device)
        partials[:rows, :B] = combined
        if mask_sum is not None:
            partials[rows, :D] = mask_sum
        reduced = reducer(partials)
        if marks is not None:
            self._mark(marks, "reduce")
        if reduced is None:
            return None, None
        reduced = torch.remainder(reduced, m).to(torch.int32)
        combined = reduced[:rows, :B].contiguous()
        if mask_sum is not None:
            mask_sum = reduced[rows, :D].contiguous()
        return combined, mask_sum

    def prepare_reveal(self, live, err):
        """Key agreement for the clerks -> recipient boxes, on the side stream
        (latency-bound X25519 ladders for a handful of messages: kept off the
        critical path). Returns what :meth:`reveal` consumes."""
        n, m, dev = self.n, self.m, self.device
        pks, sks = self.keys.pks, self.keys.sks
        rng_key = native().crypto.random_bytes(32)
        main = torch.cuda.current_stream(dev)
        side = self._side_stream()
        # Everything is allocated on the side stream and nothing here waits for
        # the main stream: called after the round's participant/clerk work has
        # been queued, it must not serialise behind it. (`err` and the key
        # tensors are long-lived; `err` is only OR-ed into.)
        with torch.cuda.stream(side):
            res_arena = Arena.empty(len(live), self.spec.batches, m, dev)
            kidx = torch.full((len(live),), n, dtype=torch.int32, device=dev)
            ks = seal_setup(res_arena, kidx, pks, rng_key, 0, err).with_powers()
            ko = open_setup(res_arena, kidx, sks, pks, err)
            ev = torch.cuda.Event()
            ev.record(side)
        for t in (res_arena.ct, res_arena.pt_len, ks, ko):  # side-stream tensors used on main
            t.record_stream(main)
        return res_arena, ks, ko, ev

    def reveal(self, combined, mask_sum, live, err, marks=None, keys=None) -> torch.Tensor:
        """Clerks seal their sums for the recipient; the recipient opens them,
        reconstructs (sum / Lagrange over the live clerks) and unmasks."""
        spec, n, m = self.spec, self.n, self.m
        B, D, dev = spec.batches, spec.dimension, self.device
        if keys is None:  # not prepared ahead: order after this round's main work (err init)
            self._side_stream().wait_stream(torch.cuda.current_stream(dev))
            keys = self.prepare_reveal(live, err)
        res_arena, ks_res, ko_res, ev = keys
        torch.cuda.current_stream(dev).wait_event(ev)
        self.seal_results(res_arena, ks_res, combined, err)
        out = self.open_results(res_arena, ko_res, live, err, mask_sum)
        if marks is not None:
            self._mark(marks, "reveal")
        return out

    def seal_results(self, res_arena: Arena, ks_res: KeySet, combined: torch.Tensor, err) -> Arena:
        """Clerk side of the result path (clerk.rs:99-100): seal the combined
        shares -- one row per clerk -- for the recipient."""
        res_vals = combined if self.vdtype == torch.int32 else combined.to(self.vdtype)
        return seal_data(res_arena, ks_res, res_vals, err)

    def open_results(self, res_arena: Arena, ko_res: KeySet, live, err, mask_sum=None,
                     rows: Sequence[int] | None = None) -> torch.Tensor:
        """Recipient side (receive.rs:127-152): open the clerks' sealed results,
        reconstruct (sum / Lagrange over the clerks `live`) and unmask.

        `res_arena` row i holds clerk live[i]'s result, or -- with `rows` --
        row rows[i] does (results that never arrived leave their rows unused)."""
        spec, m = self.spec, self.m
        D, dev = spec.dimension, self.device
        masked = torch.empty(D, dtype=torch.int32, device=dev)
        if rows is not None and list(rows) == list(range(res_arena.M)):
            rows = None
        if self._pss is None:  # additive: the reconstruction is the sum of the n results
            if rows is not None or len(live) != self.n:
                raise AggregationError("additive sharing needs every clerk's result")
            open_sum(res_arena, ko_res, err, rows=1, out=masked)
        else:
            if len(live) < spec.sharing.reconstruction_threshold():
                raise AggregationError("Not enough shares to reconstruct")
            if rows is None:
                ys = open_data(res_arena, ko_res, err, out_dtype=torch.int32)
            else:
                ys = torch.cat([open_data(res_arena.slice(r, 1), ko_res.slice(r, 1), err,
                                          out_dtype=torch.int32) for r in rows])
            if self._pss_mfma:
                lag_limbs, kp = self._lagrange_limbs(live)
                G.modgemm_i8(lag_limbs, G.limbs_t(ys, kp, m), m, masked, ldc_z=0,
                             ldc_m=1, ldc_n=spec.sharing.secret_count, limit=D)
            else:
                lag = self._lagrange(live)
                G.pss_reconstruct(ys, lag, spec.sharing.secret_count, D, m, masked)
        out = masked
        if mask_sum is not None:
            out = torch.empty(D, dtype=torch.int32, device=dev)
            G.sub_mod(masked, mask_sum, m, out)
        return out

    def _kidx_clerk(self, P: int) -> torch.Tensor:
        cache = getattr(self, "_kidx_cache", None)
        if cache is None:
            cache = self._kidx_cache = {}
        if P not in cache:
            cache[P] = torch.arange(self.n, dtype=torch.int32,
                                    device=self.device).repeat_interleave(P)
        return cache[P]

    def _kidx_recipient(self, P: int) -> torch.Tensor:
        """P times the recipient's key index (the participants' mask boxes), cached."""
        cache = self.__dict__.setdefault("_kidx_rcpt_cache", {})
        if P not in cache:
            cache[P] = torch.full((P,), self.n, dtype=torch.int32, device=self.device)
        return cache[P]

    def _open_keys(self, arena, kidx, live, P, err):
        """Key agreement for the clerks' boxes: one launch over every slot, also with
        clerks dropped -- the ladders are latency-bound (a launch over 8000 boxes
        takes 2.5 ms, five launches over 1000 each 6 ms), and the unused key sets
        of the dropped clerks' slots cost nothing more."""
        return [open_setup(arena, kidx, self.keys.sks, self.keys.pks, err)]

    def throttle(self) -> None:
        """Mark the end of a round (or streamed wave) on the current stream and wait
        for the one before the previous: at most two in flight. The host queues a
        round in 1-2 ms, the GPU needs ~13: left alone the host runs dozens of rounds
        ahead, and every round in flight holds its own multi-GB arenas (a freed block
        that a second stream has touched is not reusable before the GPU has passed
        that use), so the allocator keeps mapping fresh memory instead of recycling."""
        inflight = getattr(self, "_inflight", None)
        if inflight is None:
            inflight = self._inflight = collections.deque()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        inflight.append(ev)
        while len(inflight) > _MAX_INFLIGHT:
            inflight.popleft().synchronize()

    def _finish(self, err, marks, check, result: RoundResult) -> RoundResult:
        result.err = err
        # the round's error word into the running OR of the stream it ends on
        acc = self.__dict__.setdefault("_err_acc", {})
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream not in acc:
            acc[cur.cuda_stream] = (torch.zeros_like(err), cur)
        acc[cur.cuda_stream][0].bitwise_or_(err)
        self.throttle()
        if check or self.time_stages:
            e = int(err.item())
            if e:
                raise AggregationError(f"device error word 0x{e:x} ({describe_error(e)})")
            for (a, ea), (b, eb) in zip(marks, marks[1:]):
                result.stage_ms[b] = ea.elapsed_time(eb)
        return result

    def take_errors(self) -> torch.Tensor:
        """The OR of the error words of every round since the last call (int32 [1], on
        the current stream; see describe_error), and a fresh start. A loop of
        unchecked rounds reads this once at its end instead of a word per round:
        reading a round's own word orders the reader behind that round's result
        path, which otherwise runs beside the next round's first kernels."""
        cur = torch.cuda.current_stream(self.device)
        total = self.new_error_word()
        for word, stream in self.__dict__.pop("_err_acc", {}).values():
            if stream != cur:
                cur.wait_stream(stream)
                word.record_stream(cur)
            total |= word
        return total

    def _lagrange_limbs(self, live):
        key = ("limbs",) + tuple(live)
        cache = getattr(self, "_lag_cache", None)
        if cache is None:
            cache = self._lag_cache = {}
        if key not in cache:
            kp = G.padded_k(len(live))
            lag = self._lagrange(live).view(self.spec.sharing.secret_count, len(live))
            cache[key] = (G.limbs_of(lag, kp, self.m), kp)
        return cache[key]

    def _lagrange(self, live):
        key = tuple(live)
        cache = getattr(self, "_lag_cache", None)
        if cache is None:
            cache = self._lag_cache = {}
        if key not in cache:
            cache[key] = torch.tensor(self._pss.lagrange_matrix(list(live)), dtype=torch.int64).to(
                torch.int32).to(self.device)
        return cache[key]


def describe_error(e: int) -> str:
    names = []
    if e & 1:
        names.append("bad public key")
    if e & 2:
        names.append("MAC verification failed")
    if e & 4:
        names.append("malformed varint stream")
    if e & 8:
        names.append("ChaCha mask stream: more than half of the draws rejected")
    if e & 16:
        names.append("value out of range")
    return ", ".join(names) or "none"


def reference_sum(secrets: torch.Tensor, modulus: int) -> torch.Tensor:
    """Plain PyTorch int64 reference: sum over participants mod m in [0, m)."""
    return torch.remainder(secrets.to(torch.int64).sum(0), modulus).to(torch.int32)
