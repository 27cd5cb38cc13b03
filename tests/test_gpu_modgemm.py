"""Packed Shamir on the matrix cores: int8-limb MFMA modular GEMM (modgemm.hip).

Numerics: the GEMM is compared with a plain PyTorch int64 matmul mod p; the
engine paths are checked end to end (large reference parameter sets, dropout,
and the MFMA backend forced on PSS_4_8_3 against the register kernel).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prime,fold24", [(746497, 1), (746497, 0), (5038849, 2), (2097169, 2),
                                          ((1 << 24) - (1 << 18) - 1, 2),
                                          (433, 1), (433, 0), (16777213, 2), (16777213, 1), (16777213, 0),
                                          ((1 << 27) - 39, 2), ((1 << 27) - 39, 0),
                                          ((1 << 28) - 57, 2)])
@pytest.mark.parametrize("M,N,K,Z,panel", [(37, 45, 100, 2, 0), (64, 64, 64, 1, 0), (5, 300, 255, 3, 0),
                                           (130, 17, 700, 1, 0), (37, 45, 100, 2, 1),
                                           (5, 300, 255, 3, 1), (333, 200, 190, 2, 1), (130, 301, 100, 2, 1),
                                           (64, 128, 64, 1, 1)])
def test_modgemm_matches_torch(cuda, prime, fold24, M, N, K, Z, panel):
    """Every limb scheme and epilogue: three signed base-256 limbs (2^21 <= p < 2^24 - 2^18,
    both ends of that range); 7-bit limbs with the 64-bit fold reduced through the
    double-precision unit (the default) and, with it switched off, the Horner chain of
    32-bit Barrett steps (p < 2^24) and the 64-bit Barrett fold (p >= 2^24); under the
    general kernel and,
    for K <= 256, the panel-resident one (one, two, three and six row blocks, ragged edges,
    rows of C that start off a 16-byte boundary)."""
    from sda_amd._native import gpu
    from sda_amd.ops import gpu as G

    g = torch.Generator().manual_seed(M * N + K)
    A = torch.randint(0, prime, (M, K), generator=g, dtype=torch.int64)
    Bm = torch.randint(0, prime, (Z, N, K), generator=g, dtype=torch.int64)  # B stored transposed
    Kp = G.padded_k(K)
    Al = G.limbs_of(A.to(torch.int32).cuda(), Kp, prime)
    Bl = torch.stack([G.limbs_of(Bm[z].to(torch.int32).cuda(), Kp, prime) for z in range(Z)], 1)
    out = torch.zeros(Z * M * N, dtype=torch.int32, device="cuda")
    gpu().set_gemm_fold_f64(fold24)
    gpu().set_gemm_panel(panel)
    try:
        G.modgemm_i8(Al.contiguous(), Bl.contiguous(), prime, out, ldc_z=M * N, ldc_m=N, ldc_n=1,
                     limit=Z * M * N)
    finally:
        gpu().set_gemm_fold_f64(2)
        gpu().set_gemm_panel(-1)
    # exact reference: split K to keep int64 products exact
    ref = torch.stack([(A @ Bm[z].T) % prime for z in range(Z)]) if prime < 2 ** 21 else \
        torch.stack([sum((A[:, i:i + 1] * Bm[z][:, i:i + 1].T) % prime for i in range(K)) % prime
                     for z in range(Z)])
    assert torch.equal(out.cpu().view(Z, M, N).to(torch.int64), ref)


@pytest.mark.parametrize("panel", [0, 1])
@pytest.mark.parametrize("p", [746497, 5038849, (1 << 27) - 39])  # limbs_t in every scheme
def test_modgemm_transposed_truncated_store(cuda, panel, p):
    from sda_amd._native import gpu
    from sda_amd.ops import gpu as G

    k, R, N = 100, 255, 40
    g = torch.Generator().manual_seed(3)
    Lm = torch.randint(0, p, (k, R), generator=g, dtype=torch.int64)
    Y = torch.randint(0, p, (R, N), generator=g, dtype=torch.int64)
    Kp = G.padded_k(R)
    D = k * N - 37  # truncation of the last batch
    out = torch.full((D,), -1, dtype=torch.int32, device="cuda")
    gpu().set_gemm_panel(panel)
    try:
        G.modgemm_i8(G.limbs_of(Lm.to(torch.int32).cuda(), Kp, p),
                     G.limbs_t(Y.to(torch.int32).cuda(), Kp, p), p, out, ldc_z=0, ldc_m=1, ldc_n=k,
                     limit=D)
    finally:
        gpu().set_gemm_panel(-1)
    ref = (sum((Lm[:, i:i + 1] * Y[i:i + 1, :]) % p for i in range(R)) % p).T.reshape(-1)[:D]
    assert torch.equal(out.cpu().to(torch.int64), ref)


@pytest.mark.parametrize("p", [433, 746497, 5038849, (1 << 27) - 39])
@pytest.mark.parametrize("R,N", [(255, 40), (300, 130), (64, 64), (5, 1), (1000, 257)])
def test_limbs_t_is_limbs_of_the_transpose(cuda, p, R, N):
    """The tiled transpose-to-limbs kernel against the elementwise limb split (every limb
    scheme; ragged row and column tiles)."""
    from sda_amd.ops import gpu as G

    g = torch.Generator().manual_seed(R * N)
    Y = torch.randint(0, p, (R, N), generator=g, dtype=torch.int64).to(torch.int32).cuda()
    Kp = G.padded_k(R)
    got = G.limbs_t(Y, Kp, p)
    ref = G.limbs_of(Y.T.contiguous(), Kp, p)
    assert torch.equal(got[:, 0], ref)


@pytest.mark.parametrize("prime,dtype", [(746497, torch.int32), (5038849, torch.int32),
                                         (433, torch.int16), (60013, torch.int16)])
@pytest.mark.parametrize("M,N,Z,panel", [(37, 45, 2, 0), (70, 4096 + 300, 3, 0), (9, 9000, 1, 0),
                                         (37, 45, 2, 1), (270, 4096 + 300, 3, -1), (9, 9000, 1, 1),
                                         (130, 4097 + 300, 2, 1)])  # odd N: unaligned wide stores
def test_modgemm_epilogue_counts_varint_bytes(cuda, prime, dtype, M, N, Z, panel):
    """The share layout (C[m][z][n]) with `cnt`: the epilogue's byte counts per
    (row, batch, 4096-column tile) equal the counting kernel's over the stored output
    (general kernel, panel-resident kernel, and the launcher's own choice)."""
    from sda_amd._native import gpu
    from sda_amd.ops import gpu as G

    K = 130
    g = torch.Generator().manual_seed(N + Z)
    A = torch.randint(0, prime, (M, K), generator=g, dtype=torch.int64)
    Bm = torch.randint(0, prime, (Z, N, K), generator=g, dtype=torch.int64)
    Bm[:, ::5] = 0  # short codes too: whole output columns of zeros
    Kp = G.padded_k(K)
    Al = G.limbs_of(A.to(torch.int32).cuda(), Kp, prime)
    Bl = torch.stack([G.limbs_of(Bm[z].to(torch.int32).cuda(), Kp, prime) for z in range(Z)], 1)
    out = torch.zeros(M, Z, N, dtype=dtype, device="cuda")
    T = G.tiles(N)
    cnt = torch.zeros(M * Z * T, dtype=torch.int32, device="cuda")
    gpu().set_gemm_panel(panel)
    try:
        G.modgemm_i8(Al.contiguous(), Bl.contiguous(), prime, out, ldc_z=N, ldc_m=Z * N, ldc_n=1,
                     limit=M * Z * N, cnt=cnt)
    finally:
        gpu().set_gemm_panel(-1)
    ref = torch.empty(M * Z, T, dtype=torch.int32, device="cuda")
    G.count(out.view(M * Z, N), ref)
    assert torch.equal(cnt.view(M * Z, T), ref)
    v = out.cpu().to(torch.int64) & (0xFFFF if dtype == torch.int16 else 0xFFFFFFFF)
    z2 = 2 * v
    lens = 1 + (z2 >= 1 << 7).long() + (z2 >= 1 << 14).long() + (z2 >= 1 << 21).long() + (z2 >= 1 << 28).long()
    assert int(lens.sum()) == int(cnt.sum())


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


def test_round_pss_155_19682_100_signed_limbs(cuda):
    from sda_amd.models import PSS_155_19682_100, AggregationSpec

    spec = AggregationSpec(150, PSS_155_19682_100.prime_modulus, PSS_155_19682_100)
    # 19682 clerks; reconstruct from 300 of them (t + k = 255 needed)
    agg = _round(spec, 1, clerks=list(range(0, 600, 2)))
    assert agg._limbs == 3  # p = 5,038,849: three signed base-256 limbs


def test_pss_4_8_3_mfma_backend_matches(cuda):
    from sda_amd.models import PSS_4_8_3, AggregationSpec, ChaChaMask

    _round(AggregationSpec(4001, 433, PSS_4_8_3), 5, pss_backend="mfma")
    _round(AggregationSpec(999, 433, PSS_4_8_3, ChaChaMask(433, 999)), 3, pss_backend="mfma",
           clerks=[0, 1, 2, 3, 5, 6, 7])
