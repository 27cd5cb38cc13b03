"""HBM planner (CPU): resident or streamed, and the wave, for the benchmark
configurations at the card's 288 GB and at 64 GB.

The reference materialises whole vectors in RAM and JSON
(client/src/crypto/sharing/batched.rs:19-53) and has no notion of a memory
budget; here a round that does not fit is cut into participant waves.
"""
import pytest

from sda_amd.models.configs import bench_config
from sda_amd.planner import (HBM_BYTES_MI355X, per_participant_bytes, plan_round, slot_stride,
                             varint_max_len)

GB = 10 ** 9


def _plan(number, free, participants=None):
    cfg = bench_config(number)
    spec = cfg.spec()
    return plan_round(spec, participants or cfg.participants, free, pss_backend=cfg.pss_backend,
                      input_resident=not cfg.streamed)


def test_shapes_match_the_arena_rules(native):
    assert varint_max_len(433) == 2 and varint_max_len(2 ** 31 - 1) == 5 and varint_max_len(0) == 5
    assert slot_stride(1_000_000, 433) == 2_000_064
    assert slot_stride(4, 433) == 64


# (config, free bytes) -> (resident, wave)
PINNED = {
    (2, 288): (True, 1000), (2, 64): (True, 1000),
    (3, 288): (True, 1000), (3, 64): (True, 1000),
    (5, 288): (True, 1000), (5, 64): (True, 1000),
    (7, 288): (True, 1000), (7, 64): (True, 1000),
    (9, 288): (True, 1000), (9, 64): (True, 1000),
    (10, 288): (True, 1000), (10, 64): (True, 1000),
}


@pytest.mark.parametrize("number,free_gb", sorted(PINNED))
def test_resident_configs(native, number, free_gb):
    plan = _plan(number, free_gb * GB)
    assert (plan.resident, plan.wave) == PINNED[(number, free_gb)], plan
    assert plan.planned_bytes <= plan.budget_bytes


def test_config4_streams_and_fills_the_card(native):
    """10k x 125M cannot be resident (13 TB of shares): waves sized to the memory."""
    big = _plan(4, HBM_BYTES_MI355X)
    small = _plan(4, 64 * GB)
    assert not big.resident and not small.resident
    assert big.wave == 88 and small.wave == 16, (big, small)  # pinned: 8-aligned
    assert big.waves == -(-10_000 // big.wave)
    # the plan uses what it may: one more wave-8 step would not fit
    step = 8 * big.per_participant_bytes
    assert big.budget_bytes - step < big.planned_bytes <= big.budget_bytes


def test_many_clerk_configs(native):
    c6 = _plan(6, HBM_BYTES_MI355X)     # 728 clerks: resident on 288 GB ...
    assert c6.resident and c6.planned_bytes > 80 * GB
    c6s = _plan(6, 64 * GB)             # ... in waves on 64 GB
    assert not c6s.resident and c6s.wave == 592
    c8 = _plan(8, HBM_BYTES_MI355X)     # 19,682 clerks x 16 participants
    assert c8.resident
    c8s = _plan(8, 32 * GB)
    assert not c8s.resident and c8s.wave == 8


def test_larger_rounds_stream_instead_of_failing(native):
    cfg = bench_config(2)
    p = plan_round(cfg.spec(), 50_000, HBM_BYTES_MI355X)
    assert not p.resident and p.wave * p.per_participant_bytes + p.fixed_bytes <= p.budget_bytes
    assert 10_000 <= p.wave < 50_000 and p.wave % 8 == 0
    with pytest.raises(MemoryError):
        plan_round(bench_config(4).spec(), 10, 2 * GB)


def test_masks_cost_what_they_allocate(native):
    plain = per_participant_bytes(bench_config(2).spec())
    full = per_participant_bytes(bench_config(9).spec())
    chacha = per_participant_bytes(bench_config(10).spec())
    assert 18_000_000 < plain < 19_000_000  # two slots + key sets in flight twice, shares once
    assert full - plain > 4_000_000      # u16 masks + their sealed box
    assert chacha - plain > 4_000_000    # the masked copy of the vector
