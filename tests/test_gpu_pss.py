"""Packed-Shamir share kernels (k_share_pss48 for the k = 3, n = 8 small-field
sets, k_share_pss otherwise): shares reconstruct to the secrets through the
host Lagrange matrix (every clerk and a dropout subset), tile byte counts
match a recount, and with zero secrets every clerk's shares are uniform."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _shares(cuda, ps, secrets, switch=1):
    from sda_amd._native import gpu
    from sda_amd.ops import gpu as G

    nat = ps.native()
    n, k, t, m = ps.share_count, ps.secret_count, ps.privacy_threshold_, ps.prime_modulus
    M = torch.tensor(nat.share_matrix(), dtype=torch.int64).to(torch.int32).to(cuda)
    P, D = secrets.shape
    B = -(-D // k)
    shares = torch.empty(n, P, B, dtype=torch.int16, device=cuda)
    cnt = torch.empty(n * P * G.tiles(B), dtype=torch.int32, device=cuda)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    gpu().set_pss48(switch)
    try:
        G.share_pss(secrets, n, k, t, m, M, shares, cnt, G.MASK_NONE, bytes(range(32)), 0, err=err)
        torch.cuda.synchronize()
    finally:
        gpu().set_pss48(1)
    assert int(err.item()) == 0
    recount = torch.empty_like(cnt)
    G.count(shares.view(n * P, B), recount)
    assert torch.equal(cnt, recount)
    return nat, shares.to(torch.int64) & 0xFFFF


def _reconstruct(nat, ys, live, k, m, D):
    lag = torch.tensor(nat.lagrange_matrix(list(live)), dtype=torch.int64).view(k, len(live))
    n, P, B = ys.shape
    rec = torch.remainder(lag @ ys[list(live)].cpu().reshape(len(live), P * B), m)  # int64 matmul on CPU
    return rec.view(k, P, B).permute(1, 2, 0).reshape(P, B * k)[:, :D]


@pytest.mark.parametrize("name", ["483", "5of8"])
@pytest.mark.parametrize("switch", [1, 0])  # small-field kernel / generic kernel
def test_pss_shares_reconstruct(cuda, name, switch):
    from sda_amd.models import PSS_4_8_3
    from sda_amd.models.schemes import pss_5_of_8

    ps = PSS_4_8_3 if name == "483" else pss_5_of_8()
    m, k = ps.prime_modulus, ps.secret_count
    P, D = 3, 3 * 9000 + 2  # batches past a count tile, zero-padded last batch
    g = torch.Generator(device="cuda").manual_seed(7)
    secrets = torch.randint(0, m, (P, D), dtype=torch.int32, device=cuda, generator=g)
    nat, ys = _shares(cuda, ps, secrets, switch)
    assert int(ys.max()) < m
    assert torch.equal(_reconstruct(nat, ys, range(ps.share_count), k, m, D), secrets.cpu().to(torch.int64))
    live = [c for c in range(ps.share_count) if c != 1][:ps.reconstruction_threshold()]  # clerk 1 dropped
    assert torch.equal(_reconstruct(nat, ys, live, k, m, D), secrets.cpu().to(torch.int64))


@pytest.mark.parametrize("name", ["483", "5of8"])
def test_pss_shares_uniform(cuda, name):
    from sda_amd.models import PSS_4_8_3
    from sda_amd.models.schemes import pss_5_of_8

    ps = PSS_4_8_3 if name == "483" else pss_5_of_8()
    m = ps.prime_modulus
    secrets = torch.zeros(8, 3 * 60000, dtype=torch.int32, device=cuda)
    _, ys = _shares(cuda, ps, secrets)
    for c in range(ps.share_count):
        counts = torch.bincount(ys[c].reshape(-1), minlength=m).double()
        expected = ys[c].numel() / m
        chi2 = float(((counts - expected) ** 2 / expected).sum())
        dof = m - 1
        assert chi2 < dof + 6 * (2 * dof) ** 0.5, (c, chi2)
