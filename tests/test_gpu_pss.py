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
        G.share_pss(secrets, n, k, t, m, M, shares, cnt, G.MASK_NONE, bytes(range(32)), 0)
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


# ---- parity with the tss 0.2 FFT construction on the device paths ---------------
def _fft_model_shares(ps, secrets_rows, seed):
    """Shares [n][rows] of the FFT construction (tests/helpers.py) for random inputs."""
    import random

    from helpers import tss_share

    rng = random.Random(seed)
    p = ps.prime_modulus
    cols = []
    for s in secrets_rows:
        r = [rng.randrange(p) for _ in range(ps.privacy_threshold_)]
        cols.append(tss_share(list(s), r, ps.privacy_threshold_, ps.share_count, ps.secret_count, p,
                              ps.omega_secrets, ps.omega_shares))
    return torch.tensor(cols, dtype=torch.int64).T.contiguous()  # [n][batches]


@pytest.mark.parametrize("name", ["483", "4_26_3"])
def test_fft_model_shares_reconstruct_on_device(cuda, name):
    """Shares made by the reference's FFT construction (client/src/crypto/sharing/
    packed_shamir.rs:40-43 -> tss share) reconstruct through the GPU Lagrange
    kernel (k_pss_reconstruct) and the int8-MFMA GEMM, from every clerk and
    from dropout subsets (packed_shamir.rs:73-77 -> tss reconstruct)."""
    import random

    from sda_amd.models import PSS_4_8_3, PSS_4_26_3
    from sda_amd.ops import gpu as G

    ps = PSS_4_8_3 if name == "483" else PSS_4_26_3
    nat, p, n, k = ps.native(), ps.prime_modulus, ps.share_count, ps.secret_count
    B = 257
    rng = random.Random(11)
    secrets = [[rng.randrange(p) for _ in range(k)] for _ in range(B)]
    ys_all = _fft_model_shares(ps, secrets, seed=3)
    D = B * k - 1  # truncated last batch
    want = torch.tensor(secrets, dtype=torch.int64).reshape(-1)[:D]
    need = ps.reconstruction_threshold()
    for live in (list(range(n)), sorted(rng.sample(range(n), need)),
                 sorted(rng.sample(range(n), need + 1))):
        ys = ys_all[live].to(torch.int32).cuda().contiguous()
        lag = torch.tensor(nat.lagrange_matrix(live), dtype=torch.int64).to(torch.int32).cuda()
        out = torch.empty(D, dtype=torch.int32, device="cuda")
        G.pss_reconstruct(ys, lag, k, D, p, out)
        assert torch.equal(out.cpu().to(torch.int64), want), live
        kp = G.padded_k(len(live))
        out2 = torch.full((D,), -1, dtype=torch.int32, device="cuda")
        G.modgemm_i8(G.limbs_of(lag.view(k, len(live)), kp, p), G.limbs_t(ys, kp, p), p,
                     out2, ldc_z=0, ldc_m=1, ldc_n=k, limit=D)
        assert torch.equal(out2.cpu().to(torch.int64), want), live


def test_device_shares_are_the_fft_construction(cuda):
    """The matrix the share kernels apply is the FFT construction: device
    shares of PSS_4_8_3 interpolate (big-integer Lagrange through {1} u
    {omega_shares^(i+1)}) to a polynomial of degree <= t + k that is 0 at 1 and
    holds the secrets at omega_secrets^(1..k)."""
    from sda_amd.models import PSS_4_8_3

    ps = PSS_4_8_3
    p, n, k, t = ps.prime_modulus, ps.share_count, ps.secret_count, ps.privacy_threshold_
    g = torch.Generator(device="cuda").manual_seed(21)
    secrets = torch.randint(0, p, (2, 3 * 40), dtype=torch.int32, device=cuda, generator=g)
    _, ys = _shares(cuda, ps, secrets)
    ys = ys.cpu()

    def interp_at(points, values, x):
        acc = 0
        for i, (xi, yi) in enumerate(zip(points, values)):
            num = den = 1
            for j, xj in enumerate(points):
                if j != i:
                    num, den = num * (x - xj) % p, den * (xi - xj) % p
            acc = (acc + yi * num * pow(den, p - 2, p)) % p
        return acc

    pts = [pow(ps.omega_shares, i + 1, p) for i in range(n)]
    for part in range(2):
        for b in range(0, 40, 7):
            vals = [int(ys[c, part, b]) for c in range(n)]
            # all n = 8 shares lie on one polynomial of degree <= t + k = 7 with f(1) = 0
            assert interp_at(pts, vals, 1) == 0
            for e in range(k):
                assert interp_at(pts, vals, pow(ps.omega_secrets, e + 1, p)) == int(secrets[part, b * k + e])


# ---- u8 share storage (primes below 256) ------------------------------------------
@pytest.mark.parametrize("backend", ["valu", "mfma"])
@pytest.mark.parametrize("storage", ["auto", "u16"])
def test_round_small_prime_u8_storage(cuda, backend, storage):
    """5-of-8 packed Shamir over p = 241 with three clerks dropped
    (protocol/src/crypto.rs:79-155 semantics: any t + k results reconstruct): a
    field element per byte of share storage, on the register kernel and on the
    int8-limb MFMA GEMM, against the plain sum -- and the same with u16 storage."""
    from sda_amd.engine import DeviceAggregator, reference_sum
    from sda_amd.models import AggregationSpec
    from sda_amd.models.configs import small_prime_5_of_8

    ps = small_prime_5_of_8()
    m = ps.prime_modulus
    spec = AggregationSpec(3 * 5000 + 1, m, ps)
    agg = DeviceAggregator(spec, cuda, pss_backend=backend, share_storage=storage)
    assert agg.vdtype == (torch.uint8 if storage == "auto" else torch.int16)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randint(0, m, (7, spec.dimension), dtype=torch.int32, device=cuda, generator=g)
    for clerks in (None, [0, 2, 3, 5, 7]):
        res = agg.run_round(x, clerks=clerks)
        assert torch.equal(res.output, reference_sum(x, m))
