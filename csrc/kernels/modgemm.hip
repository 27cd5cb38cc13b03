// Modular GEMM on the matrix cores: C = A . B mod p for field elements p < 2^28.
//
// Packed Shamir with the reference's large parameter sets (PSS_155_728_100:
// K = t + k = 255 inputs, n = 728 shares, p = 746497; PSS_155_19682_100) turns
// share generation into S = M . X (n x K times K x batches, per participant) and
// reconstruction into L_I . Y (k x |I| times |I| x batches) -- SURVEY K2/K10.
// Values are split into L = 3 (p < 2^21) or 4 (p < 2^28) 7-bit limbs (int8,
// non-negative), so every limb product fits the i8 MFMA and a K-sum of up to L
// limb products per degree stays below 2^31 (K * 127^2 * L < 2^31). The L^2
// limb products per K-step go into 2L - 1 accumulators by degree d = i + j;
// the epilogue folds sum_d (acc_d mod p) * (2^(7d) mod p) with Barrett steps.
//
// Layouts: A limbs [3][M][Kp] (row-major, k contiguous), B limbs
// [3][batch][N][Kp] (B stored transposed: each column contiguous in k); Kp is a
// multiple of 64 with zero padding. C element (m, n) of batch z is written to
// C[z*ldc_z + m*ldc_m + n*ldc_n] if that linear index < limit.
// Tile: 256 threads = 4 waves (2 x 2), each wave 32 x 32 = 2 x 2 MFMA
// 16x16x64 tiles; workgroup tile 64 x 64.
#include "device_crypto.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kLimbBits = 7;

// Fragment of a 16 x 64 int8 operand: lane l holds row (l & 15), k = 16*(l>>4) .. +15.
SDA_DEV v4i load_frag(const int8_t* base, int row, int rows, int64_t ld, int k0, int lane) {
  const int r = row + (lane & 15);
  if (r >= rows) return v4i{0, 0, 0, 0};
  return *reinterpret_cast<const v4i*>(base + (int64_t)r * ld + k0 + 16 * (lane >> 4));
}

template <typename VT, int kLimbs>
__global__ void __launch_bounds__(256)
    k_modgemm_i8(int M, int N, int Kp, ModParams mp, const int8_t* __restrict__ A,
                 const int8_t* __restrict__ B, int64_t b_batch, VT* __restrict__ C,
                 int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.y * 64 + (wave >> 1) * 32;
  const int n0 = blockIdx.x * 64 + (wave & 1) * 32;
  const int z = blockIdx.z;
  const int64_t a_plane = (int64_t)M * Kp;
  const int8_t* Bz = B + (int64_t)z * (int64_t)N * Kp;
  const int64_t b_plane = b_batch;  // bytes between limb planes of B
  v4i acc[2][2][2 * kLimbs - 1];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int d = 0; d < 2 * kLimbs - 1; ++d) acc[i][j][d] = v4i{0, 0, 0, 0};

  for (int k0 = 0; k0 < Kp; k0 += 64) {
    v4i fa[2][kLimbs], fb[2][kLimbs];
#pragma unroll
    for (int l = 0; l < kLimbs; ++l)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i][l] = load_frag(A + l * a_plane, m0 + 16 * i, M, Kp, k0, lane);
        fb[i][l] = load_frag(Bz + l * b_plane, n0 + 16 * i, N, Kp, k0, lane);
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int la = 0; la < kLimbs; ++la)
#pragma unroll
          for (int lb = 0; lb < kLimbs; ++lb)
            acc[i][j][la + lb] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i][la], fb[j][lb], acc[i][j][la + lb], 0, 0, 0);
  }
  // epilogue: C/D map col = lane & 15, row = 4*(lane >> 4) + r
  uint32_t w[2 * kLimbs - 1];
#pragma unroll
  for (int d = 0; d < 2 * kLimbs - 1; ++d) w[d] = (uint32_t)(((uint64_t)1 << (kLimbBits * d)) % mp.m);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 16 * i + 4 * (lane >> 4) + r;
        const int col = n0 + 16 * j + (lane & 15);
        if (row >= M || col >= N) continue;
        uint64_t s = 0;
#pragma unroll
        for (int d = 0; d < 2 * kLimbs - 1; ++d)
          s += (uint64_t)mod32((uint32_t)acc[i][j][d][r], mp) * w[d];  // < 7 * 2^56
        const int64_t idx = (int64_t)z * ldc_z + (int64_t)row * ldc_m + (int64_t)col * ldc_n;
        if (idx < limit) C[idx] = (VT)mod64(s, mp);
      }
}

template <int kLimbs>
SDA_DEV void put_limbs(int8_t* dst, int64_t plane, const uint32_t (&v)[16]) {
#pragma unroll
  for (int l = 0; l < kLimbs; ++l) {
    uint32_t q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) x |= ((v[4 * u + b] >> (kLimbBits * l)) & 0x7fu) << (8 * b);
      q[u] = x;
    }
    *reinterpret_cast<uint4*>(dst + l * plane) = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

// X limbs of packed-Shamir share generation: row b of participant p is
// [s_{b k} .. s_{b k + k-1} | r_1 .. r_t | 0 ...] (length Kp). One thread per 16
// positions; position j's randomness is word j % 16 of ChaCha block
// (b * Kp/16 + j/16) of the participant's share stream (exact uniform with the
// retry stream for rejected words), so every draw is a pure function of
// (round key, participant, batch, position).
template <int kLimbs>
__global__ void __launch_bounds__(256)
    k_pss_x_limbs(int P, int D, int B, int k, int t, int Kp, ModParams mp,
                  const int32_t* __restrict__ secrets, RngKeyArg rng, uint64_t owner_base,
                  int8_t* __restrict__ X) {
  const int groups = Kp / 16;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (gid >= (int64_t)B * groups) return;
  const int b = (int)(gid / groups), g = (int)(gid % groups);
  RngKey rk;
#pragma unroll
  for (int i = 0; i < 8; ++i) rk.k[i] = rng.k[i];
  const uint64_t owner = owner_base + (uint64_t)p;
  const int j0 = 16 * g;
  uint32_t v[16];
  const bool rnd = j0 + 16 > k && j0 < k + t;
  uint32_t w[16];
  if (rnd) rng_block(w, rk, stream_id(kPurposeShares, owner), (uint64_t)b * groups + g);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = j0 + i;
    uint32_t x = 0;
    if (j < k) {
      const int64_t e = (int64_t)b * k + j;
      x = e < D ? canon_i32(secrets[(int64_t)p * D + e], mp) : 0u;
    } else if (j < k + t) {
      x = (uint64_t)w[i] < mp.zone32
              ? mod32(w[i], mp)
              : uniform_fixup(rk, kPurposeSharesRetry, owner, (uint64_t)b * Kp + j, mp.m,
                              (uint32_t)mp.zone32);
    }
    v[i] = x;
  }
  const int64_t plane = (int64_t)P * B * Kp;
  put_limbs<kLimbs>(X + ((int64_t)p * B + b) * Kp + j0, plane, v);
}

// Limbs of a [R][N] u32 matrix, transposed to [3][N][Kp] (Kp >= R, zero padded):
// the B operand of reconstruction (rows = surviving clerks, columns = batches).
template <int kLimbs>
__global__ void __launch_bounds__(256)
    k_limbs_t(int R, int N, int Kp, const uint32_t* __restrict__ Y, int8_t* __restrict__ out) {
  const int groups = Kp / 16;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)N * groups) return;
  const int col = (int)(gid / groups), g = (int)(gid % groups);
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = 16 * g + i;
    v[i] = r < R ? Y[(int64_t)r * N + col] : 0u;
  }
  put_limbs<kLimbs>(out + (int64_t)col * Kp + 16 * g, (int64_t)N * Kp, v);
}

}  // namespace

void launch_modgemm_i8(int M, int N, int Kp, int batches, int limbs, uint32_t p, const int8_t* A,
                       const int8_t* B, int64_t b_plane, int value_bytes, void* C, int64_t ldc_z,
                       int64_t ldc_m, int64_t ldc_n, int64_t limit, hipStream_t s) {
  if (M <= 0 || N <= 0 || batches <= 0) return;
  ModParams mp = make_mod_params(p);
  dim3 grid((N + 63) / 64, (M + 63) / 64, batches);
#define SDA_GEMM(VT, L)                                                                      \
  hipLaunchKernelGGL((k_modgemm_i8<VT, L>), grid, dim3(256), 0, s, M, N, Kp, mp, A, B, b_plane, \
                     (VT*)C, ldc_z, ldc_m, ldc_n, limit)
  if (value_bytes == 2) {
    if (limbs == 3) SDA_GEMM(uint16_t, 3); else SDA_GEMM(uint16_t, 4);
  } else {
    if (limbs == 3) SDA_GEMM(uint32_t, 3); else SDA_GEMM(uint32_t, 4);
  }
#undef SDA_GEMM
}

void launch_pss_x_limbs(int P, int D, int B, int k, int t, int Kp, int limbs, uint32_t p,
                        const int32_t* secrets, RngKeyArg rng, uint64_t owner_base, int8_t* X,
                        hipStream_t s) {
  if (P <= 0 || B <= 0) return;
  const int64_t threads = (int64_t)B * (Kp / 16);
  dim3 grid((unsigned)((threads + 255) / 256), P);
  if (limbs == 3)
    hipLaunchKernelGGL(k_pss_x_limbs<3>, grid, dim3(256), 0, s, P, D, B, k, t, Kp,
                       make_mod_params(p), secrets, rng, owner_base, X);
  else
    hipLaunchKernelGGL(k_pss_x_limbs<4>, grid, dim3(256), 0, s, P, D, B, k, t, Kp,
                       make_mod_params(p), secrets, rng, owner_base, X);
}

void launch_limbs_t(int R, int N, int Kp, int limbs, const uint32_t* Y, int8_t* out,
                    hipStream_t s) {
  if (R <= 0 || N <= 0) return;
  const int64_t threads = (int64_t)N * (Kp / 16);
  dim3 grid((unsigned)((threads + 255) / 256));
  if (limbs == 3)
    hipLaunchKernelGGL(k_limbs_t<3>, grid, dim3(256), 0, s, R, N, Kp, Y, out);
  else
    hipLaunchKernelGGL(k_limbs_t<4>, grid, dim3(256), 0, s, R, N, Kp, Y, out);
}

}  // namespace sdagpu
