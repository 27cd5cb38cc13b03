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
