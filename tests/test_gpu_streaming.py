"""Participant-wave streaming and accumulator checkpoint/resume on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _waves(m, D, seed=5):
    def make(w, first, count):
        g = torch.Generator(device="cuda").manual_seed(seed + w)
        return torch.randint(0, m, (count, D), dtype=torch.int32, device="cuda", generator=g)
    return make


def _reference(make, total, wave, m):
    acc = None
    for w in range((total + wave - 1) // wave):
        x = make(w, w * wave, min(wave, total - w * wave)).to(torch.int64).sum(0)
        acc = x if acc is None else acc + x
    return torch.remainder(acc, m).to(torch.int32)


@pytest.mark.parametrize("name", ["additive_fullmask", "pss"])
def test_streamed_round_matches_reference(cuda, name):
    from sda_amd.engine import DeviceAggregator
    from sda_amd.models import PSS_4_8_3, Additive, AggregationSpec, FullMask
    from sda_amd.streaming import StreamingAggregator

    m, D, total, wave = 433, 3001, 37, 8
    spec = (AggregationSpec(D, m, Additive(3, m), FullMask(m)) if name != "pss"
            else AggregationSpec(D, m, PSS_4_8_3))
    make = _waves(m, D)
    res = StreamingAggregator(DeviceAggregator(spec), wave=wave).run(total, make)
    assert res.waves == 5
    assert torch.equal(res.output, _reference(make, total, wave, m))


def test_streamed_checkpoint_resume(cuda, tmp_path):
    from sda_amd.engine import AggregationError, DeviceAggregator
    from sda_amd.models import PSS_4_8_3, AggregationSpec
    from sda_amd.streaming import StreamingAggregator

    m, D, total, wave = 433, 2000, 40, 6
    spec = AggregationSpec(D, m, PSS_4_8_3)
    make = _waves(m, D, seed=11)
    ck = str(tmp_path / "acc.safetensors")
    eng = DeviceAggregator(spec)
    first = StreamingAggregator(eng, wave=wave, checkpoint=ck, checkpoint_every=2)
    part = first.run(total, make, stop_after=3)  # "crash" after 3 waves
    assert part.output is None
    # a fresh process would rebuild the engine; the clerk keys stay the same
    second = StreamingAggregator(DeviceAggregator(spec, keys=eng.keys), wave=wave, checkpoint=ck)
    res = second.run(total, make)
    assert res.resumed_from == 3 and res.waves == 7 - 3
    assert torch.equal(res.output, _reference(make, total, wave, m))
    # a checkpoint from another aggregation is refused
    other = StreamingAggregator(DeviceAggregator(spec, keys=eng.keys), wave=wave + 1, checkpoint=ck)
    with pytest.raises(AggregationError):
        other.run(total, make)


def test_run_round_streams_when_the_round_does_not_fit(cuda):
    """A round larger than the memory it may use runs in planner-sized waves
    instead of failing: same output, and the plan says so."""
    from sda_amd.engine import DeviceAggregator, reference_sum
    from sda_amd.models import Additive, AggregationSpec, FullMask

    m, D, P = 433, 50_000, 96
    spec = AggregationSpec(D, m, Additive(3, m), FullMask(m))
    agg = DeviceAggregator(spec)
    x = torch.randint(0, m, (P, D), dtype=torch.int32, device="cuda")
    assert agg.plan(P).resident
    ref = reference_sum(x, m)
    assert torch.equal(agg.run_round(x).output, ref)
    small = DeviceAggregator(spec, keys=agg.keys)
    small.memory_limit_bytes = 700 * 10 ** 6  # the slabs and sums alone are ~0.5 GB
    plan = small.plan(P)
    assert not plan.resident and 1 <= plan.wave < P, plan
    res = small.run_round(x)
    assert torch.equal(res.output, ref) and int(res.err.item()) == 0
    with pytest.raises(MemoryError):
        small.memory_limit_bytes = 10 ** 6
        small.plan(P + 1)


def test_planner_picks_the_wave_and_checkpoints_do_not_block(cuda, tmp_path):
    from sda_amd.engine import DeviceAggregator
    from sda_amd.models import PSS_4_8_3, AggregationSpec
    from sda_amd.streaming import StreamingAggregator

    m, D, total = 433, 30_000, 120
    spec = AggregationSpec(D, m, PSS_4_8_3)
    eng = DeviceAggregator(spec)
    eng.memory_limit_bytes = 350 * 10 ** 6  # the fixed part is ~250 MB: room for ~60 participants
    make = _waves(m, D, seed=3)
    st = StreamingAggregator(eng, checkpoint=str(tmp_path / "ck.safetensors"), checkpoint_every=1)
    res = st.run(total, make)
    assert res.plan is not None and res.wave == res.plan["wave"] and 1 <= res.wave < total
    assert res.waves == -(-total // res.wave)
    assert torch.equal(res.output, _reference(make, total, res.wave, m))
    # a checkpoint per wave was written by the background writer
    assert res.checkpoint["written"] == res.waves
    # resuming adopts the checkpoint's wave size even when the planner would pick another
    eng2 = DeviceAggregator(spec, keys=eng.keys)
    again = StreamingAggregator(eng2, checkpoint=str(tmp_path / "ck.safetensors")).run(total, make)
    assert again.resumed_from == res.waves and again.waves == 0
    assert torch.equal(again.output, res.output)


def test_a_checkpoint_is_never_written_from_a_failed_wave(cuda, tmp_path):
    from sda_amd.engine import AggregationError, DeviceAggregator
    from sda_amd.models import Additive, AggregationSpec
    from sda_amd.streaming import StreamingAggregator

    spec = AggregationSpec(5000, 433, Additive(3, 433))
    eng = DeviceAggregator(spec)
    eng.corrupt_next_round()  # the first wave's first box fails its MAC
    ck = tmp_path / "ck.safetensors"
    st = StreamingAggregator(eng, wave=4, checkpoint=str(ck), checkpoint_every=1)
    with pytest.raises(AggregationError, match="MAC"):
        st.run(12, _waves(433, 5000))
    assert not ck.exists()
