"""HBM planner: does a round fit the card, and if not, in waves of how many.

An MI355X has 288 GB of HBM3E; a resident round keeps, per participant, the
clerk-major share tensor, one fixed-stride ciphertext slot per clerk, two key
sets (80-byte stream keys + 26 KB of Poly1305 tables per box, for sealing and
for opening) and -- with a mask -- the mask values and their box. The engine
queues at most two rounds ahead of the GPU, so what a wave holds until its boxes
are opened counts twice (what it only needs while sharing counts once).
Rounds that do not fit are *streamed*: participants go through the
participate + clerk phase in waves and only the clerks' running sums persist
(`sda_amd.streaming`). This module prices both from the aggregation spec alone
-- no allocation, no GPU -- so that

  * `DeviceAggregator.run_round` streams instead of running out of memory,
  * `StreamingAggregator` picks its wave when the caller gives none,
  * the benchmark configurations report the plan they ran under.

The byte model follows the allocations of `engine._participate` / `_clerk` and
`ops.sealed.open_sum` one by one (the reference holds whole vectors in RAM and
JSON and has no such notion: client/src/crypto/sharing/batched.rs:19-53).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from .models.schemes import AggregationSpec, ChaChaMask, FullMask, PackedShamir

# constants of the kernels (csrc/kernels/kernels.hpp); mirrored in ops/gpu.py, which
# needs torch -- the planner must not
TILE_VALUES = 4096
CHUNK_BYTES = 16384
SUB_PER_CHUNK = 16
SUM_TILE = 6144
MSGKEY_BYTES = 80
POW_WORDS = 6560
POW_SHORT_WORDS = 320   # boxes of at most SHORT_MAX_CHUNKS chunks: the one-pass MAC's table
SHORT_MAX_CHUNKS = 4
SEAL_OVERHEAD = 48

HBM_BYTES_MI355X = 288 * 10 ** 9
# share of the free memory a plan may claim (allocator rounding, RCCL buffers, the
# caller's own tensors) and rounds the host may have queued at once
HEADROOM = 0.80
IN_FLIGHT = 2


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def varint_max_len(modulus: int) -> int:
    if modulus == 0:
        return 5
    z, n = 2 * (modulus - 1), 1
    while z >= 128:
        z >>= 7
        n += 1
    return n


def slot_stride(L: int, modulus: int) -> int:
    return _round_up(SEAL_OVERHEAD + _round_up(L * varint_max_len(modulus), 16), 64)


def chunks_for(max_pt: int) -> int:
    return (max_pt + 32 + CHUNK_BYTES - 1) // CHUNK_BYTES


def _box_bytes(L: int, modulus: int, opened: bool) -> int:
    """One sealed box of L values: slot, stream key + Poly1305 tables, MAC partials
    and (when it is opened here) the terminator counts of the decode."""
    K = chunks_for(L * varint_max_len(modulus))
    short = K <= SHORT_MAX_CHUNKS
    tables = (POW_SHORT_WORDS if short else POW_WORDS) * 4 + (0 if short else K * 32)
    b = slot_stride(L, modulus) + MSGKEY_BYTES + tables + 4
    if opened:
        b += MSGKEY_BYTES + tables + K * SUB_PER_CHUNK * 4 + 8 + \
            ((L + SUM_TILE - 1) // SUM_TILE + 1) * 4
    return b


@dataclass(frozen=True)
class RoundPlan:
    participants: int
    resident: bool
    wave: int                      # participants per wave (== participants when resident)
    waves: int
    per_participant_bytes: int     # peak bytes one participant of a wave accounts for
    fixed_bytes: int               # accumulators, slabs, outputs: independent of the wave
    budget_bytes: int              # what the plan was allowed to claim
    planned_bytes: int             # fixed + in-flight waves at the chosen wave size
    note: str = ""

    def as_dict(self) -> dict:
        return {"resident": self.resident, "wave": self.wave, "waves": self.waves,
                "per_participant_bytes": self.per_participant_bytes,
                "fixed_bytes": self.fixed_bytes, "budget_bytes": self.budget_bytes,
                "planned_bytes": self.planned_bytes, "note": self.note}


def value_bytes(spec: AggregationSpec, share_storage: str = "auto") -> int:
    m = spec.field_modulus
    if isinstance(spec.sharing, PackedShamir) and m <= 256 and share_storage != "u16":
        return 1
    return 2 if m <= 65536 else 4


def uses_mfma(spec: AggregationSpec, pss_backend: str = "auto") -> bool:
    if not isinstance(spec.sharing, PackedShamir):
        return False
    ps = spec.sharing
    big = ps.secret_count > 8 or ps.privacy_threshold_ > 16 or ps.share_count > 64
    return pss_backend == "mfma" or (pss_backend == "auto" and big)


def participant_bytes(spec: AggregationSpec, pss_backend: str = "auto",
                      share_storage: str = "auto", clerks_here: Optional[int] = None):
    """(held, short) device bytes of one participant of a wave.

    `held` lives from the wave's key agreement until its boxes are opened -- the
    ciphertext slots and both key sets -- so with the host queuing `in_flight`
    waves ahead it is there that many times. `short` is produced and consumed
    inside the participant half (shares, byte counts, limb planes, mask values, the
    ChaCha pre-pass copy): the allocator hands those blocks to the next wave as
    soon as this one's seal kernels are queued, so they count once.
    `clerks_here`: clerks whose boxes this GPU opens (all of them on one GPU; a
    committee rank opens its piece, i.e. the same number of boxes)."""
    n, m, D, B = spec.n_clerks, spec.field_modulus, spec.dimension, spec.batches
    vb = value_bytes(spec, share_storage)
    opened = n if clerks_here is None else clerks_here
    held = opened * _box_bytes(B, m, True) + (n - opened) * _box_bytes(B, m, False)
    short = n * B * vb                                       # shares [n][P][B]
    short += n * ((B + TILE_VALUES - 1) // TILE_VALUES) * 4  # tile byte counts
    mfma = uses_mfma(spec, pss_backend)
    if mfma:
        ps = spec.sharing
        kp = _round_up(ps.secret_count + ps.privacy_threshold_, 64)
        # the GEMM's limb_scheme: three limbs (7-bit, or signed 8-bit up to 2^24 - 2^18), else four
        limbs = 3 if m < 2 ** 21 or (m < 2 ** 24 - 2 ** 18 and kp <= 4096) else 4
        short += limbs * B * kp                              # X limb planes
    if isinstance(spec.masking, FullMask):
        held += _box_bytes(D, m, True)
        short += D * (4 if mfma else vb) + ((D + TILE_VALUES - 1) // TILE_VALUES) * 4
        if mfma:
            short += D * 4                                   # masked copy ahead of the limb kernel
    elif isinstance(spec.masking, ChaChaMask):
        w = spec.masking.seed_words
        held += w * 4 + _box_bytes(w, 0, True)
        short += D * 4                                       # masked copy (the pre-pass)
        short += 4 * (2 + (2 * D + 4096 + 2047) // 2048)     # repair scratch
    return held, short


def per_participant_bytes(spec: AggregationSpec, pss_backend: str = "auto",
                          share_storage: str = "auto", clerks_here: Optional[int] = None,
                          in_flight: int = IN_FLIGHT) -> int:
    """Peak device bytes a participant of a wave accounts for with `in_flight`
    waves queued."""
    held, short = participant_bytes(spec, pss_backend, share_storage, clerks_here)
    return in_flight * held + short


def fixed_bytes(spec: AggregationSpec, streamed: bool) -> int:
    """What a round holds whatever the wave: decode-sum slabs (~10k blocks of one
    tile each), combined shares, the result boxes, the output; running int64 sums
    when streamed."""
    n, m, D, B = spec.n_clerks, spec.field_modulus, spec.dimension, spec.batches
    slabs = 10_000 * SUM_TILE * (8 if m > 2 ** 27 else 4) + n * B * 4   # 64-bit sums above 2^27
    b = slabs + n * B * 4 + n * _box_bytes(B, m, True) + 2 * D * 4
    if spec.masking.has_mask():
        b += 10_000 * SUM_TILE * 4 + D * 4 + D * 8   # mask slabs / sums / ChaCha fix-up words
    if streamed:
        b += n * B * 8 + (D * 8 if spec.masking.has_mask() else 0)
    return b


def plan_round(spec: AggregationSpec, participants: int, free_bytes: int = HBM_BYTES_MI355X,
               pss_backend: str = "auto", share_storage: str = "auto",
               in_flight: int = IN_FLIGHT, headroom: float = HEADROOM,
               input_resident: bool = True) -> RoundPlan:
    """Resident or streamed, and the wave size, for `participants` vectors on a GPU
    with `free_bytes` free. `input_resident`: the caller's [P][D] int32 input is
    already on the device (and already counted out of `free_bytes`); streamed
    callers that produce their waves on the fly pass False and the wave's own input
    is priced in."""
    if participants <= 0:
        raise ValueError("participants must be positive")
    per_p = per_participant_bytes(spec, pss_backend, share_storage, in_flight=in_flight)
    budget = int(free_bytes * headroom)
    fixed_res = fixed_bytes(spec, streamed=False)
    need_res = fixed_res + participants * per_p
    if need_res <= budget:
        return RoundPlan(participants, True, participants, 1, per_p, fixed_res, budget, need_res,
                         "the whole round is resident")
    per_wave_p = per_p + (0 if input_resident else spec.dimension * 4)
    fixed_str = fixed_bytes(spec, streamed=True)
    room = budget - fixed_str
    wave = room // per_wave_p if room > 0 else 0
    if wave < 1:
        raise MemoryError(
            f"one participant of this aggregation needs {per_wave_p + fixed_str} bytes "
            f"in flight, the budget is {budget}")
    wave = min(int(wave), participants)
    if wave >= 16:
        wave -= wave % 8   # whole multiples keep the kernels' grids even
    waves = (participants + wave - 1) // wave
    return RoundPlan(participants, False, wave, waves, per_wave_p, fixed_str, budget,
                     fixed_str + wave * per_wave_p,
                     f"streamed: {waves} waves of {wave} participants")
