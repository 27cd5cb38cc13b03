"""Additive share kernel with 16-bit draws (k_share_additive16): exactness under
heavy rejection (m = 40000 rejects 39% of the halves, exercising the deferred
and the overflow replacement paths), byte counts, masks, and uniformity."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(m, n, P, D, mask):
    from sda_amd.ops import gpu as G

    g = torch.Generator(device="cuda").manual_seed(m + n)
    secrets = torch.randint(-m, m, (P, D), dtype=torch.int32, device="cuda", generator=g)
    shares = torch.empty(n, P, D, dtype=torch.int16, device="cuda")
    cnt = torch.empty(n * P * G.tiles(D), dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    mask_out = torch.empty(P, D, dtype=torch.int16, device="cuda") if mask else None
    mask_cnt = torch.empty(P * G.tiles(D), dtype=torch.int32, device="cuda") if mask else None
    G.share_additive(secrets, n, m, shares, cnt, G.MASK_FULL if mask else G.MASK_NONE,
                     bytes(range(32)), 0, mask_out=mask_out, mask_cnt=mask_cnt)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    sh = shares.to(torch.int64) & 0xFFFF
    assert int(sh.max()) < m
    total = torch.remainder(sh.sum(0), m)
    expect = torch.remainder(secrets.to(torch.int64) + ((mask_out.to(torch.int64) & 0xFFFF) if mask else 0), m)
    assert torch.equal(total, expect)
    # tile byte counts equal a recount of the stored values
    recount = torch.empty_like(cnt)
    G.count(shares.view(n * P, D), recount)
    assert torch.equal(cnt, recount)
    if mask:
        mv = mask_out.to(torch.int64) & 0xFFFF
        assert int(mv.max()) < m and int(mv.min()) >= 0
        mrecount = torch.empty_like(mask_cnt)
        G.count(mask_out, mrecount)
        assert torch.equal(mask_cnt, mrecount)
    return sh


# m^3 < 2^32 (m <= 1625) takes the three-draws-per-word kernel (1291: ~50% of the
# words rejected, so spare and retry-stream replacements run constantly)
@pytest.mark.parametrize("m", [433, 40000, 65521, 2, 3, 1000, 1291, 1625, 1626, 8192, 8193, 20000,
                               32768])
@pytest.mark.parametrize("n,mask", [(3, False), (2, True), (5, True), (8, False)])
def test_share16_exact(cuda, m, n, mask):
    _run(m, n, 3, 70001, mask)  # D not a multiple of the 16384-element block


@pytest.mark.parametrize("m", [40000, 1291, 433])
def test_share16_uniform_under_rejection(cuda, m):
    sh = _run(m, 3, 16, 200000, False)
    for r in range(2):  # both random rows (the third is secret - their sum)
        row = sh[r].reshape(-1)
        if m > 4096:  # 20 equal-width buckets (m = 40000: 2000 values each)
            counts, dof = torch.histc(row.float(), bins=20, min=0, max=m), 19
        else:  # every residue
            counts, dof = torch.bincount(row, minlength=m).double(), m - 1
        expected = row.numel() / counts.numel()
        chi2 = float(((counts - expected) ** 2 / expected).sum())
        assert chi2 < dof + 6 * (2 * dof) ** 0.5, (m, r, chi2)
