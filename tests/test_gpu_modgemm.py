"""Packed Shamir on the matrix cores: int8-limb MFMA modular GEMM (modgemm.hip).

Numerics: the GEMM is compared with a plain PyTorch int64 matmul mod p; the
engine paths are checked end to end (large reference parameter sets, dropout,
and the MFMA backend forced on PSS_4_8_3 against the register kernel).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prime", [746497, 5038849, 433])
@pytest.mark.parametrize("M,N,K,Z", [(37, 45, 100, 2), (64, 64, 64, 1), (5, 300, 255, 3),
                                     (130, 17, 700, 1)])
def test_modgemm_matches_torch(cuda, prime, M, N, K, Z):
    from sda_amd.ops import gpu as G

    g = torch.Generator().manual_seed(M * N + K)
    A = torch.randint(0, prime, (M, K), generator=g, dtype=torch.int64)
    Bm = torch.randint(0, prime, (Z, N, K), generator=g, dtype=torch.int64)  # B stored transposed
    L = G.limb_count(prime)
    Kp = G.padded_k(K)
    Al = G.limbs_of(A.to(torch.int32).cuda(), Kp, L)
    Bl = torch.stack([G.limbs_of(Bm[z].to(torch.int32).cuda(), Kp, L) for z in range(Z)], 1)
    out = torch.zeros(Z * M * N, dtype=torch.int32, device="cuda")
    G.modgemm_i8(Al.contiguous(), Bl.contiguous(), prime, out, ldc_z=M * N, ldc_m=N, ldc_n=1,
                 limit=Z * M * N)
    # exact reference: split K to keep int64 products exact
    ref = torch.stack([(A @ Bm[z].T) % prime for z in range(Z)]) if prime < 2 ** 21 else \
        torch.stack([sum((A[:, i:i + 1] * Bm[z][:, i:i + 1].T) % prime for i in range(K)) % prime
                     for z in range(Z)])
    assert torch.equal(out.cpu().view(Z, M, N).to(torch.int64), ref)


def test_modgemm_transposed_truncated_store(cuda):
    from sda_amd.ops import gpu as G

    p, k, R, N = 746497, 100, 255, 40
    g = torch.Generator().manual_seed(3)
    Lm = torch.randint(0, p, (k, R), generator=g, dtype=torch.int64)
    Y = torch.randint(0, p, (R, N), generator=g, dtype=torch.int64)
    Kp = G.padded_k(R)
    D = k * N - 37  # truncation of the last batch
    out = torch.full((D,), -1, dtype=torch.int32, device="cuda")
    G.modgemm_i8(G.limbs_of(Lm.to(torch.int32).cuda(), Kp, 3),
                 G.limbs_t(Y.to(torch.int32).cuda(), Kp, 3), p, out, ldc_z=0, ldc_m=1, ldc_n=k,
                 limit=D)
    ref = ((Lm @ Y) % p).T.reshape(-1)[:D]
    assert torch.equal(out.cpu().to(torch.int64), ref)


def _round(spec, P, clerks=None, **kw):
    from sda_amd.engine import DeviceAggregator, reference_sum

    agg = DeviceAggregator(spec, **kw)
    x = torch.randint(0, spec.field_modulus, (P, spec.dimension), dtype=torch.int32, device="cuda")
    res = agg.run_round(x, clerks=clerks)
    assert torch.equal(res.output, reference_sum(x, spec.field_modulus))
    return agg


def test_round_pss_155_728_100_mfma(cuda):
    from sda_amd.models import PSS_155_728_100, AggregationSpec

    agg = _round(AggregationSpec(1500, PSS_155_728_100.prime_modulus, PSS_155_728_100), 3)
    assert agg._pss_mfma


def test_round_pss_155_728_100_dropout_fullmask(cuda):
    from sda_amd.models import PSS_155_728_100, AggregationSpec, FullMask

    p = PSS_155_728_100.prime_modulus
    live = [c for c in range(728) if c % 3 != 1]  # drop a third of the committee
    _round(AggregationSpec(777, p, PSS_155_728_100, FullMask(p)), 2, clerks=live)


def test_round_pss_155_19682_100_four_limbs(cuda):
    from sda_amd.models import PSS_155_19682_100, AggregationSpec

    spec = AggregationSpec(150, PSS_155_19682_100.prime_modulus, PSS_155_19682_100)
    # 19682 clerks; reconstruct from 300 of them (t + k = 255 needed)
    agg = _round(spec, 1, clerks=list(range(0, 600, 2)))
    assert agg._limbs == 4


def test_pss_4_8_3_mfma_backend_matches(cuda):
    from sda_amd.models import PSS_4_8_3, AggregationSpec, ChaChaMask

    _round(AggregationSpec(4001, 433, PSS_4_8_3), 5, pss_backend="mfma")
    _round(AggregationSpec(999, 433, PSS_4_8_3, ChaChaMask(433, 999)), 3, pss_backend="mfma",
           clerks=[0, 1, 2, 3, 5, 6, 7])
