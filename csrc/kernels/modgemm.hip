// Modular GEMM on the matrix cores: C = A . B mod p for field elements p < 2^28.
//
// Packed Shamir with the reference's large parameter sets (PSS_155_728_100:
// K = t + k = 255 inputs, n = 728 shares, p = 746497; PSS_155_19682_100) turns
// share generation into S = M . X (n x K times K x batches, per participant) and
// reconstruction into L_I . Y (k x |I| times |I| x batches).
// Values are split into int8 limbs (limb_scheme): L = 3 (p < 2^21) or 4 (p < 2^28)
// non-negative 7-bit digits, or -- 2^21 <= p < 2^24 - 2^18, K <= 4096 -- three signed
// base-256 digits of the balanced residue (|x| <= p / 2): the i8 MFMA multiplies signed
// bytes, and nine products per K-step and five degree sums instead of sixteen and seven
// is what the 19,682-clerk field (p = 5,038,849) saves by it. Every limb product fits
// the MFMA and a K-sum of up to L limb products per degree stays inside 32 bits
// (K * 127^2 * L, K * 128^2 * L < 2^31). The L^2 limb products per K-step go into
// 2L - 1 accumulators by degree d = i + j; the epilogue folds sum_d acc_d 2^(b d) mod p
// (b = 7 or 8; kFold below).
//
// Layouts: A limbs [L][M][Kp] (row-major, k contiguous), B limbs
// [L][batch][N][Kp] (B stored transposed: each column contiguous in k); Kp is a
// multiple of 64 with zero padding. C element (m, n) of batch z is written to
// C[z*ldc_z + m*ldc_m + n*ldc_n] if that linear index < limit.
//
// Tiling: a workgroup of 4 waves (2 x 2) owns a 64 (M) x 128 (N) tile of C, a
// wave 32 x 64 = 2 x 4 MFMA 16x16x64 tiles with 2L - 1 accumulators each. Every
// K-step's A (64 x 64 B per limb) and B (128 x 64 B per limb) tiles are staged
// through LDS -- each byte is fetched from L2/HBM once per workgroup instead of
// once per wave -- in two buffers: the next step's tiles are loaded into
// registers before the current step's MFMAs and written to the other buffer
// after them, one barrier per step. Rows are 64 B; a row's four 16-byte chunks
// are stored XOR-swizzled (chunk ^ {0,2,3,1}[(row >> 2) & 3]) so that the 16
// lanes ds_read_b128 services together (which mix two chunk indices and three
// row ranges) hit 16 different 16-byte slots of the 256-byte bank row.
// K = t + k is short in share generation (255 -> 4 steps), so the epilogue matters as
// much as the MFMAs, and restaging B for every row block more than either: those
// shapes go to the panel-resident kernel further down (k_modgemm_panel); this one
// serves long K (reconstruction over many clerks) and matrices of a few row blocks.
// What was tried on it and measured neutral: reductions on the 24-bit multipliers
// (every 32-bit integer multiply is full rate on this chip) and operand reuse through
// the L2 (the block id remap below).
//
// Share generation also needs every sealed box's varint length per 4096-value
// tile before the encoder can place its bytes (kernels.hpp, launch_count). With
// `cnt` the epilogue adds them up itself -- the lengths of a lane's outputs per
// row, summed over the 16 lanes of a row group on the VALU (DPP), one atomic add
// per (row, wave) -- instead of a second pass over the stored shares.
#include <algorithm>
#include <type_traits>

#include "block_utils.hpp"
#include "device_crypto.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kLimbBits = 7;
constexpr int kBM = 64, kBN = 128, kBK = 64;

SDA_DEV int swz(int row, int chunk) {  // position of a row's 16-byte chunk inside its 64 bytes
  return chunk ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);  // {0, 2, 3, 1}
}

// kFold: how the epilogue folds the degree sums acc_d (< 2^31) into sum_d acc_d 2^(7d)
// mod p. 1: in 64-bit integers -- one multiply-add per degree -- reduced through the
// double-precision unit (modf64): all five degrees at once with three limbs (the
// caller checks sum < 2^53), degrees 3..6 first and then the rest with four. 0: a
// Horner chain of 32-bit Barrett steps (p < 2^24: s < p and acc_d < 2^31 keep
// s * 2^7 + acc_d below 2^32). 2: 64-bit multiply-adds by 2^(7d) mod p and one 64-bit
// Barrett reduction (any p < 2^28). 0 and 2 are the integer-only references. 3: signed
// base-256 limbs (three of them): sum_d acc_d w_d in doubles with w_d = 2^(8 d) for
// d < 4 and 2^32 mod p for d = 4, plus a multiple of p that makes the sum positive --
// one reduction: every term is below K 2^40 in size and K <= 4096.
//
// Epilogue of a wave's 32 x 16 kJT outputs held as degree sums in `acc` (rows from
// m_blk + 32 wm, columns from n_blk + 16 kJT wn, C/D map of the 16x16 MFMA): fold,
// store, and -- with `cnt` -- the byte counts.
template <typename VT, int kLimbs, int kFold, int kJT, bool kVec, int kBlockN>
__device__ __forceinline__ void gemm_epilogue(const v4i (&acc)[2][kJT][2 * kLimbs - 1], int m_blk, int n_blk,
                                              int z, int wm, int wn, int lane, int M, int N, int batches,
                                              const ModParams& mp, const ModF64& mf, VT* __restrict__ C,
                                              int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit,
                                              uint32_t* __restrict__ cnt, int cnt_tiles) {
  constexpr int kDeg = 2 * kLimbs - 1;
  // C/D map of the MFMA: tile column lane & 15, tile row 4*(lane >> 4) + r. Which matrix
  // column a tile column stands for is the caller's choice of B rows: tile j's column c
  // is column 16 j + c of the wave's 16 kJT, or -- kVec -- column kJT c + j: a lane's
  // kJT outputs of one row are then neighbours in memory and leave in one store.
  // Output indices are built from per-lane bases by additions (the general z/m/n strides
  // would cost three 64-bit multiplies per element otherwise).
  uint32_t w[kDeg];
  if constexpr (kFold == 2) {
#pragma unroll
    for (int d = 0; d < kDeg; ++d) w[d] = (uint32_t)(((uint64_t)1 << (kLimbBits * d)) % mp.m);
  }
  const int row0 = m_blk + wm * 32 + 4 * (lane >> 4);
  const int col0 = n_blk + wn * (16 * kJT) + (kVec ? kJT : 1) * (lane & 15);
  constexpr int kColStep = kVec ? 1 : 16;  // matrix columns between tiles j and j + 1
  const int64_t base = (int64_t)z * ldc_z + (int64_t)row0 * ldc_m + (int64_t)col0 * ldc_n;
  const int64_t step_j = kColStep * ldc_n, step_i = 16 * ldc_m;
  uint32_t bytes[2][2] = {{0, 0}, {0, 0}};  // varint bytes of rows (i, r): two 16-bit sums per word
  auto fold = [&](int i, int j, int r) -> uint32_t {
    if constexpr (kFold == 3) {
      static_assert(kFold != 3 || kLimbs == 3, "signed limbs come in threes");
      double s = mf.off + (double)acc[i][j][0][r];
      s = __builtin_fma((double)acc[i][j][1][r], 256.0, s);
      s = __builtin_fma((double)acc[i][j][2][r], 65536.0, s);
      s = __builtin_fma((double)acc[i][j][3][r], 16777216.0, s);
      s = __builtin_fma((double)acc[i][j][4][r], mf.w4, s);
      return modf64d(s, mf);
    } else if constexpr (kFold == 1) {
      // neighbouring degrees pair up in 32 bits (acc_d 2^7 + acc_(d-1) < 2^32: the
      // caller's bound on K), the pairs meet as doubles: exact integers below 2^53
      auto pair = [&](int d) -> double {  // acc_(d+1) 2^7 + acc_d, or acc_d alone at the top
        uint32_t v = (uint32_t)acc[i][j][d][r];
        if (d + 1 < kDeg) v += (uint32_t)acc[i][j][d + 1][r] << kLimbBits;
        return (double)v;
      };
      if constexpr (kLimbs == 3) {
        const double s = __builtin_fma(pair(4), 268435456.0, __builtin_fma(pair(2), 16384.0, pair(0)));
        return modf64d(s, mf);
      } else {
        // degrees 4..6 first (below 2^46), reduced; then with the low four (below 2^53)
        const double hi = __builtin_fma(pair(6), 16384.0, pair(4));
        const double rh = (double)modf64d(hi, mf);
        const double s = __builtin_fma(rh, 268435456.0, __builtin_fma(pair(2), 16384.0, pair(0)));
        return modf64d(s, mf);
      }
    } else if constexpr (kFold == 0) {
      // acc_d < 2^31, s < p < 2^24: s * 2^7 + acc_d < 2^32
      uint32_t s = mod32((uint32_t)acc[i][j][kDeg - 1][r], mp);
#pragma unroll
      for (int d = kDeg - 2; d >= 0; --d) s = mod32((s << kLimbBits) + (uint32_t)acc[i][j][d][r], mp);
      return s;
    } else {
      uint64_t s = 0;
#pragma unroll
      for (int d = 0; d < kDeg; ++d)
        s += (uint64_t)mod32((uint32_t)acc[i][j][d][r], mp) * w[d];  // < 7 * 2^56
      return mod64(s, mp);
    }
  };
  // zigzag code z = 2 * out of b bits (b of 2 * out + 1: the same, and 1 for 0):
  // ceil(b / 7) bytes = ((b + 6) * 37) >> 8 for b + 6 <= 35, b = 32 - clz
  auto varint_len = [](uint32_t out) -> uint32_t {
    return (1406u - 37u * (uint32_t)__builtin_clz((out << 1) | 1u)) >> 8;
  };
  // A block whose whole tile is inside the matrix and below `limit` (nine in ten of the
  // share GEMMs' blocks) stores without any per-element test: the tests are a compare
  // or two and a branch per element otherwise.
  const bool inside = m_blk + kBM <= M && n_blk + kBlockN <= N && limit < 0 && (!kVec || ldc_n == 1);  // uniform
  if (inside) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t idx = base + i * step_i + r * ldc_m;
        VT o[kJT];
#pragma unroll
        for (int j = 0; j < kJT; ++j) {
          const uint32_t out = fold(i, j, r);
          o[j] = (VT)out;
          bytes[i][r >> 1] += varint_len(out) << (16 * (r & 1));
        }
        if constexpr (kVec) {
          __builtin_memcpy(C + idx, o, sizeof(o));  // one store of kJT neighbours (C is only VT-aligned)
        } else {
#pragma unroll
          for (int j = 0; j < kJT; ++j) C[idx + j * step_j] = o[j];
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 16 * i + r;
        if (row >= M) continue;
        int64_t idx = base + i * step_i + r * ldc_m;
#pragma unroll
        for (int j = 0; j < kJT; ++j, idx += step_j) {
          if (col0 + kColStep * j >= N) continue;
          if (limit >= 0 && idx >= limit) continue;  // limit < 0: every in-range element is stored
          const uint32_t out = fold(i, j, r);
          C[idx] = (VT)out;
          bytes[i][r >> 1] += varint_len(out) << (16 * (r & 1));
        }
      }
  }
  if (cnt == nullptr) return;  // uniform
  // the block's columns lie inside one count tile (kTileValues is a multiple of kBlockN)
  static_assert(kTileValues % kBlockN == 0, "a block's columns must not straddle a count tile");
  const int tile = n_blk / kTileValues;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // a row's columns of this wave: kJT per lane, over the 16 lanes of the row group
      const uint32_t sum = row16_incl_scan(bytes[i][h]);
      if ((lane & 15) != 15) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int row = row0 + 16 * i + 2 * h + q;
        const uint32_t v = (sum >> (16 * q)) & 0xffffu;
        if (row < M && v != 0)
          atomicAdd(&cnt[((int64_t)row * batches + z) * cnt_tiles + tile], v);
      }
    }
}

// Block id -> tile. K is short, so the kernel lives on operand reuse between blocks: a
// column panel of B (128 columns of one batch) is read by every row block, a row block
// of A by every panel. Consecutive block ids go round the 8 XCDs, each with its own
// L2: ids congruent mod 8 share one. Each such class walks super-tiles of gm row
// blocks x gp panels (row blocks fastest), sized so that a super-tile's operands stay
// in the 4 MB L2: every operand tile is then fetched from HBM / the Infinity Cache once
// per super-tile instead of once per block (728 clerks: the 7.7 GB of B limbs went
// through 12 times). Ragged edges are blocks that exit at once.
struct GemmGrid {
  int gx, gy, panels;  // column blocks per batch, row blocks, gx * batches
  int gm, gp, tiles_m;
};
constexpr int kXcds = 8;

template <typename VT, int kLimbs, int kFold>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
    k_modgemm_i8(int M, int N, int Kp, int batches, GemmGrid gg, ModParams mp, ModF64 mf,
                 const int8_t* __restrict__ A, const int8_t* __restrict__ B, int64_t b_batch,
                 VT* __restrict__ C, int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit,
                 uint32_t* __restrict__ cnt, int cnt_tiles) {
  constexpr int kRows = kBM + kBN;                       // staged rows per limb
  constexpr int kStage = kLimbs * kRows * kBK;           // bytes per buffer
  constexpr int kDeg = 2 * kLimbs - 1;
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * kStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int m_blk, n_blk, z;
  {
    const int cls = blockIdx.x % kXcds, seq = blockIdx.x / kXcds;
    const int per = gg.gm * gg.gp;
    const int tile = seq / per, i = seq % per;
    const int mb = (tile % gg.tiles_m) * gg.gm + i % gg.gm;
    const int panel = ((tile / gg.tiles_m) * gg.gp + i / gg.gm) * kXcds + cls;
    if (mb >= gg.gy || panel >= gg.panels) return;  // block-uniform
    m_blk = mb * kBM;
    n_blk = (panel % gg.gx) * kBN;
    z = panel / gg.gx;
  }
  const int64_t a_plane = (int64_t)M * Kp;
  const int8_t* Bz = B + (int64_t)z * (int64_t)N * Kp;

  // this thread's staging pieces: chunk (tid & 3) of A row tid >> 2 and of B rows
  // tid >> 2 and 64 + (tid >> 2), for every limb plane: 3 row pointers, 3 LDS offsets
  static_assert(kBM == 64 && kBN == 128, "staging map assumes a 64 + 128 row stage");
  const int chunk = tid & 3, srow = tid >> 2;
  const int8_t* src[3];
  int dst[3];
  int64_t plane[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const bool isA = u == 0;
    const int row = isA ? srow : srow + 64 * (u - 1);
    const int grow = (isA ? m_blk : n_blk) + row;
    const bool ok = grow < (isA ? M : N);
    src[u] = !ok ? nullptr : (isA ? A : Bz) + (int64_t)grow * Kp + 16 * chunk;
    plane[u] = isA ? a_plane : b_batch;
    dst[u] = ((isA ? 0 : kBM) + row) * kBK + 16 * swz(row, chunk);
  }
  v4i acc[2][4][kDeg];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int d = 0; d < kDeg; ++d) acc[i][j][d] = v4i{0, 0, 0, 0};

  v4i stage[kLimbs][3];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int l = 0; l < kLimbs; ++l)
#pragma unroll
      for (int u = 0; u < 3; ++u)
        stage[l][u] = src[u] ? *reinterpret_cast<const v4i*>(src[u] + l * plane[u] + k0) : v4i{0, 0, 0, 0};
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int l = 0; l < kLimbs; ++l)
#pragma unroll
      for (int u = 0; u < 3; ++u)
        *reinterpret_cast<v4i*>(lds + buf * kStage + l * kRows * kBK + dst[u]) = stage[l][u];
  };
  // fragment addresses: lane l reads row (l & 15) of a 16-row tile, chunk l >> 4
  const int fr = lane & 15, fg = lane >> 4;
  const int a_off = (wm * 32 + fr) * kBK + 16 * swz(fr, fg);
  const int b_off = (kBM + wn * 64 + fr) * kBK + 16 * swz(fr, fg);

  fetch(0);
  commit(0);
  __syncthreads();
  const int nk = Kp / kBK;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) fetch((ks + 1) * kBK);
    const int8_t* base = lds + cur * kStage;
    v4i fa[2][kLimbs];
#pragma unroll
    for (int l = 0; l < kLimbs; ++l)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i][l] = *reinterpret_cast<const v4i*>(base + l * kRows * kBK + a_off + 16 * i * kBK);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v4i fb[kLimbs];
#pragma unroll
      for (int l = 0; l < kLimbs; ++l)
        fb[l] = *reinterpret_cast<const v4i*>(base + l * kRows * kBK + b_off + 16 * j * kBK);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int la = 0; la < kLimbs; ++la)
#pragma unroll
          for (int lb = 0; lb < kLimbs; ++lb)
            acc[i][j][la + lb] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i][la], fb[lb], acc[i][j][la + lb], 0, 0, 0);
    }
    if (ks + 1 < nk) commit(cur ^ 1);
    __syncthreads();
  }
  gemm_epilogue<VT, kLimbs, kFold, 4, false, kBN>(acc, m_blk, n_blk, z, wm, wn, lane, M, N, batches, mp, mf, C, ldc_z,
                                             ldc_m, ldc_n, limit, cnt, cnt_tiles);
}

// The same product for short K (Kp <= 256: share generation, K = t + k), one workgroup
// per column panel of B. The general kernel above restages its B panel for every row
// block, and its waves meet at a barrier every K-step, so the MFMAs of a tile and the
// epilogue of the tile before it rarely overlap: measured, a tile took 15.8k cycles of
// a SIMD for 4.6k cycles of MFMAs and about as many of other instructions. Here the
// panel's limbs (128 columns x Kp x L bytes, 96 / 128 KB) are loaded into LDS once and
// the workgroup walks down all row blocks of A against them. A is small and shared by
// every panel (it stays in each XCD's L2), so each wave loads its own A fragments
// straight from global memory, one step ahead of the MFMAs that use them, from a copy of
// A in fragment order (launch_a_fragments: [row block][K-step][limb][16-row tile][lane]
// [16 bytes], lane (r, g) = bytes [16 g, 16 g + 16) of row r): one load instruction is
// 1 KB of consecutive bytes. (From the row-major limbs the same instruction touched 16
// half cache lines; the A traffic alone then held the kernel at 11.6 ms of 19.) After
// the panel is in LDS nothing is written to it and no wave waits for another.
// The panel's rows are stored so that MFMA tile j's column c is column kJT c + j of the
// wave's columns: a lane's kJT outputs of a row are neighbours in C and leave in one
// 16-byte store (the plain order gives 4-byte stores, 64 B runs per instruction; the
// stores cost 5.5 of the 19 ms).
// Eight waves: with three limbs two teams of 2 x 2 waves (32 x 64 outputs per wave, 160
// accumulator registers) take alternate row blocks; with four limbs one team of 2 x 4
// (32 x 32 per wave, 112 registers).
// Where the time goes (728 clerks x 1000 participants, 17.3 ms; the general kernel
// 26 ms): 8.9 ms of MFMAs per SIMD and ~950 other VALU instructions per wave and tile.
// The matrix pipe does run under another wave's VALU work (scripts/ubench_mfma_valu.hip)
// but a single wave issues one VALU instruction every ~6 cycles, not 4, and every MFMA
// issue costs the other wave ~6 more: by that micro-benchmark's rates this structure
// ends at ~14 ms. Tried on top and measured neutral: holding the second four waves back
// half a tile, alternating MFMA and epilogue slots between the two waves of a SIMD
// under workgroup barriers, raised wave priority in the epilogue, 64-column panels.
// The fused byte counts cost 1 ms of it (their atomics), filling C alone takes 4.9 ms.
constexpr int kPanelMaxK = 256;

template <typename VT, int kLimbs, int kFold, int kPN, int kJT, int kTeams>
__global__ void __launch_bounds__(kPN / (16 * kJT) * 128 * kTeams)
    __attribute__((amdgpu_waves_per_eu(2, 2)))
    k_modgemm_panel(int M, int N, int Kp, int batches, int gx, int gy, ModParams mp, ModF64 mf,
                    const int8_t* __restrict__ Afrag, const int8_t* __restrict__ B, int64_t b_batch,
                    VT* __restrict__ C, int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit,
                    uint32_t* __restrict__ cnt, int cnt_tiles) {
  // kPN panel columns, kJT 16-column tiles per wave: kPN / (16 kJT) waves across the
  // panel, two down the row block, kTeams such teams on alternate row blocks
  static_assert(kPN % (16 * kJT) == 0, "panel width");
  constexpr int kDeg = 2 * kLimbs - 1;
  constexpr int kWavesN = kPN / (16 * kJT);
  constexpr int kThreads = kWavesN * 128 * kTeams;
  constexpr int kSteps = kPanelMaxK / kBK;
  constexpr int kPlane = kPN * kBK;         // one (limb, K-step) slab of the panel
  __shared__ __attribute__((aligned(16))) int8_t Bs[kLimbs * kSteps * kPlane];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % kWavesN, wm = (wave / kWavesN) & 1, team = wave / (2 * kWavesN);
  const int n_blk = ((int)blockIdx.x % gx) * kPN, z = (int)blockIdx.x / gx;
  const int nk = Kp / kBK;
  {
    // the panel: rows = columns of C, 16-byte pieces; 16 consecutive threads take one
    // row's Kp bytes. All loads are issued before the first LDS write.
    const int8_t* Bz = B + (int64_t)z * (int64_t)N * Kp;
    const int cpr = Kp / 16, pieces = kLimbs * kPN * cpr;
    constexpr int kMine = (kLimbs * kPN * (kPanelMaxK / 16) + kThreads - 1) / kThreads;
    v4i t[kMine];
    int dst[kMine];
#pragma unroll
    for (int u = 0; u < kMine; ++u) {
      const int id = u * kThreads + tid;
      const int c = id % cpr, rl = id / cpr, row = rl % kPN, l = rl / kPN;
      // LDS row `row` = tile (row / 16) % kJT, tile column row % 16 of wave row / (16 kJT)
      constexpr int kW = 16 * kJT;
      const int grow = n_blk + (row / kW) * kW + kJT * (row & 15) + ((row >> 4) % kJT);
      const bool ok = id < pieces;
      dst[u] = ok ? ((l * kSteps + (c >> 2)) * kPN + row) * kBK + 16 * swz(row, c & 3) : -1;
      t[u] = ok && grow < N ? *reinterpret_cast<const v4i*>(Bz + l * b_batch + (int64_t)grow * Kp + 16 * c)
                            : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kMine; ++u)
      if (dst[u] >= 0) *reinterpret_cast<v4i*>(Bs + dst[u]) = t[u];
  }
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  const int b_off = (wn * (16 * kJT) + fr) * kBK + 16 * swz(fr, fg);
  // this wave's two 16-row tiles of (row block mb, step ks), limb l: 1 KB each
  const int8_t* af = Afrag + ((int64_t)(2 * wm) * 64 + lane) * 16;
  auto load_a = [&](v4i (&f)[2][kLimbs], int mb, int ks) {
    const int8_t* p = af + (int64_t)(mb * nk + ks) * (kLimbs * 4096);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int l = 0; l < kLimbs; ++l) f[i][l] = *reinterpret_cast<const v4i*>(p + (l * 4 + i) * 1024);
  };
  // The next step's fragments are requested before this step's MFMAs and taken over
  // after them -- a K-step of MFMAs (1,152 cycles) covers the L2 latency. The loads are
  // unconditional (past the last row block they fetch row block `mb` again) and the
  // hand-over sits before the epilogue: with a branch around the loads, or the
  // epilogue's stores between request and use, the compiler's wait-count bookkeeping
  // turns conservative and every step waits for the loads it has just issued.
  v4i fa[2][kLimbs], fnext[2][kLimbs];
  auto take = [&] {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int l = 0; l < kLimbs; ++l) fa[i][l] = fnext[i][l];
  };
  load_a(fnext, min(team, gy - 1), 0);
  take();
  for (int mb = team; mb < gy; mb += kTeams) {
    v4i acc[2][kJT][kDeg];
    // the first K-step starts every degree from a zero C operand: no clearing pass
    auto step = [&](int ks, auto first) {
      constexpr bool kFirst = decltype(first)::value;
      const bool more = ks + 1 < nk;
      const int nmb = more || mb + kTeams >= gy ? mb : mb + kTeams;
      load_a(fnext, nmb, more ? ks + 1 : 0);
      __builtin_amdgcn_sched_barrier(0);  // or the scheduler sinks the loads below the MFMAs
      const int8_t* base = Bs + ks * kPlane + b_off;
#pragma unroll
      for (int j = 0; j < kJT; ++j) {
        v4i fb[kLimbs];
#pragma unroll
        for (int l = 0; l < kLimbs; ++l)
          fb[l] = *reinterpret_cast<const v4i*>(base + l * kSteps * kPlane + 16 * j * kBK);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int la = 0; la < kLimbs; ++la)
#pragma unroll
            for (int lb = 0; lb < kLimbs; ++lb) {
              // (la, lb) with la == 0 or lb == kLimbs - 1 is its degree's first product
              const bool fresh = kFirst && (la == 0 || lb == kLimbs - 1);
              acc[i][j][la + lb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                  fa[i][la], fb[lb], fresh ? v4i{0, 0, 0, 0} : acc[i][j][la + lb], 0, 0, 0);
            }
      }
      __builtin_amdgcn_sched_barrier(0);
      take();
      __builtin_amdgcn_sched_barrier(0);
    };
    step(0, std::true_type{});
    for (int ks = 1; ks < nk; ++ks) step(ks, std::false_type{});
    gemm_epilogue<VT, kLimbs, kFold, kJT, true, kPN>(acc, mb * kBM, n_blk, z, wm, wn, lane, M, N, batches, mp, mf,
                                                     C, ldc_z, ldc_m, ldc_n, limit, cnt, cnt_tiles);
  }
}

// Sixteen canonical values -> their limbs, 16 bytes per limb plane. kBits == 7: the
// non-negative base-128 digits. kBits == 8 (three limbs): the signed base-256 digits of
// the balanced residue x - (x > p / 2 ? p : 0): d0 = low byte as int8, then the same of
// (x - d0) >> 8, and what is left (|.| <= 128 by limb_scheme's bound on p).
template <int kLimbs, int kBits>
SDA_DEV void put_limbs(int8_t* dst, int64_t plane, const uint32_t (&v)[16], uint32_t p) {
  uint32_t q[kLimbs][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint32_t x[kLimbs];
#pragma unroll
    for (int l = 0; l < kLimbs; ++l) x[l] = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if constexpr (kBits == 7) {
#pragma unroll
        for (int l = 0; l < kLimbs; ++l) x[l] |= ((v[4 * u + b] >> (kLimbBits * l)) & 0x7fu) << (8 * b);
      } else {
        static_assert(kBits == 7 || kLimbs == 3, "signed limbs come in threes");
        int32_t t = (int32_t)v[4 * u + b];
        if ((uint32_t)t > (p >> 1)) t -= (int32_t)p;
        const int32_t d0 = (int32_t)(int8_t)(t & 0xff);
        t = (t - d0) >> 8;
        const int32_t d1 = (int32_t)(int8_t)(t & 0xff);
        t = (t - d1) >> 8;
        x[0] |= ((uint32_t)d0 & 0xffu) << (8 * b);
        x[1] |= ((uint32_t)d1 & 0xffu) << (8 * b);
        x[2] |= ((uint32_t)t & 0xffu) << (8 * b);
      }
    }
#pragma unroll
    for (int l = 0; l < kLimbs; ++l) q[l][u] = x[l];
  }
#pragma unroll
  for (int l = 0; l < kLimbs; ++l)
    *reinterpret_cast<uint4*>(dst + l * plane) = make_uint4(q[l][0], q[l][1], q[l][2], q[l][3]);
}

// X limbs of packed-Shamir share generation: row b of participant p is
// [s_{b k} .. s_{b k + k-1} | r_1 .. r_t | 0 ...] (length Kp). One thread per 16
// positions; position j's randomness is word j % 16 of ChaCha block
// (b * Kp/16 + j/16) of the participant's share stream (exact uniform with the
// retry stream for rejected words), so every draw is a pure function of
// (round key, participant, batch, position).
template <int kLimbs, int kBits>
__global__ void __launch_bounds__(256)
    k_pss_x_limbs(int P, int D, int B, int k, int t, int Kp, ModParams mp,
                  const int32_t* __restrict__ secrets, RngKeyArg rng, uint64_t owner_base,
                  int8_t* __restrict__ X) {
  const int groups = Kp / 16;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (gid >= (int64_t)B * groups) return;
  // Groups [g_lo, g_hi) hold random positions and cost a ChaCha block each, the others
  // a few loads. Threads are numbered with the random groups of all rows first, so a
  // wave is all generator work or none (row-major, 10 of a row's 16 groups draw with
  // k = 100, t = 155: three lanes in eight sat idle through every ChaCha block).
  const int g_lo = k / 16, g_hi = min(groups, (k + t + 15) / 16);
  const int R = g_hi - g_lo, S = groups - R;
  int b, g;
  if (gid < (int64_t)B * R) {
    b = (int)(gid / R);
    g = g_lo + (int)(gid % R);
  } else {
    const int64_t rest = gid - (int64_t)B * R;
    b = (int)(rest / S);
    const int i = (int)(rest % S);
    g = i < g_lo ? i : i - g_lo + g_hi;
  }
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
  put_limbs<kLimbs, kBits>(X + ((int64_t)p * B + b) * Kp + j0, plane, v, mp.m);
}

// Limbs of a [R][N] u32 matrix, transposed to [L][N][Kp] (Kp >= R, zero padded): the B
// operand of reconstruction (rows = surviving clerks, columns = batches). A workgroup
// turns a 64 x 64 tile through LDS: rows of Y are read 256 bytes at a time, and the four
// threads of a column write 64 consecutive bytes of its limb rows. (One thread per 16
// rows of a column straight from global memory read 4 bytes per 40 KB stride: 1.3 ms
// for the 19,682-clerk committee's 0.8 GB, now the time of the traffic.)
template <int kLimbs, int kBits>
__global__ void __launch_bounds__(256)
    k_limbs_t(int R, int N, int Kp, uint32_t p, const uint32_t* __restrict__ Y, int8_t* __restrict__ out) {
  __shared__ uint32_t tile[64][65];
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + 4 * i + (tid >> 6), c = c0 + (tid & 63);
    tile[4 * i + (tid >> 6)][tid & 63] = r < R && c < N ? Y[(int64_t)r * N + c] : 0u;
  }
  __syncthreads();
  const int g = tid & 3, col = tid >> 2;
  if (c0 + col >= N) return;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = tile[16 * g + i][col];
  put_limbs<kLimbs, kBits>(out + (int64_t)(c0 + col) * Kp + r0 + 16 * g, (int64_t)N * Kp, v, p);
}

// A limbs [L][M][Kp] in the order the panel kernel's waves load them: [row block]
// [K-step][limb][16-row tile (4)][lane (64)][16 bytes], lane (r, g) holding bytes
// [16 g, 16 g + 16) of the step of row r of the tile; rows past M are zero.
__global__ void __launch_bounds__(256)
    k_a_fragments(int M, int Kp, int limbs, const int8_t* __restrict__ A, int8_t* __restrict__ out) {
  const int nk = Kp / kBK, gy = (M + kBM - 1) / kBM;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)gy * nk * limbs * 256) return;
  const int lane = (int)(id & 63), t = (int)((id >> 6) & 3);
  const int64_t rest = id >> 8;
  const int l = (int)(rest % limbs), ks = (int)((rest / limbs) % nk), mb = (int)(rest / limbs / nk);
  const int row = mb * kBM + 16 * t + (lane & 15), col = ks * kBK + 16 * (lane >> 4);
  v4i v = {0, 0, 0, 0};
  if (row < M) v = *reinterpret_cast<const v4i*>(A + ((int64_t)l * M + row) * Kp + col);
  *reinterpret_cast<v4i*>(out + id * 16) = v;
}

}  // namespace

int64_t a_fragments_bytes(int M, int Kp, int limbs) {
  return (int64_t)((M + kBM - 1) / kBM) * kBM * Kp * limbs;
}
void launch_a_fragments(int M, int Kp, int limbs, const int8_t* A, int8_t* out, hipStream_t s) {
  if (M <= 0) return;
  const int64_t pieces = a_fragments_bytes(M, Kp, limbs) / 16;
  hipLaunchKernelGGL(k_a_fragments, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, s, M, Kp, limbs, A, out);
}

static int g_gemm_fold_f64 = 2;  // 0 never, 1 three-limb fields only, 2 every field below 2^24 (default)
void set_gemm_fold_f64(int mode) { g_gemm_fold_f64 = mode; }
static int g_gemm_panel = -1;  // -1: the panel kernel where it pays, 0 never, 1 wherever Kp allows
void set_gemm_panel(int mode) { g_gemm_panel = mode; }

void launch_modgemm_i8(int M, int N, int Kp, int batches, int limbs, uint32_t p, const int8_t* A,
                       const int8_t* a_frag, const int8_t* B, int64_t b_plane, int value_bytes, void* C,
                       int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit, uint32_t* cnt,
                       hipStream_t s) {
  if (M <= 0 || N <= 0 || batches <= 0) return;
  ModParams mp = make_mod_params(p);
  ModF64 mf = make_modf64(p);
  const LimbScheme sch = limb_scheme(p, Kp);
  if (sch.limbs != limbs) return;  // the operands were not made for this field (callers check)
  // no truncation: the per-element bound check goes away (the kernel takes limit < 0)
  if ((int64_t)(batches - 1) * ldc_z + (int64_t)(M - 1) * ldc_m + (int64_t)(N - 1) * ldc_n < limit &&
      ldc_z >= 0 && ldc_m >= 0 && ldc_n >= 0)
    limit = -1;
  // three limbs fold all five degrees in one 64-bit sum: acc_d <= Kp 127^2 min(d + 1, 5 - d)
  // and the 32-bit pairs: (acc_(d+1) << 7) + acc_d with at most `limbs` products per degree
  const bool fits53 = (limbs == 4 || (uint64_t)Kp * 127 * 127 * ((1ull << 28) + (2ull << 21) + (3ull << 14) +
                                                                (2ull << 7) + 1) < (1ull << 53)) &&
                      (uint64_t)Kp * 127 * 127 * limbs * 129 < (1ull << 32);
  // measured on the share GEMMs of the two large reference fields, against the Horner
  // chain: three limbs 28.9 -> 27.8 ms, four limbs 21.0 -> 20.4 ms (four limbs: the
  // second stage's r 2^28 + ... stays below 2^53 only for p < 2^24)
  const bool f64 = p >= 16 && ((g_gemm_fold_f64 == 2 && p < (1u << 24)) || (g_gemm_fold_f64 == 1 && limbs == 3));
  int fold = f64 && fits53 ? 1 : (p >= (1u << 24) ? 2 : 0);
  if (sch.bits == 8) {
    fold = 3;
    mf = make_modf64_signed(p, Kp);
  }
  const int cnt_tiles = (N + kTileValues - 1) / kTileValues;
  const int gy = (M + kBM - 1) / kBM;
  // short K and enough row blocks to pay for loading the panel
  if (a_frag != nullptr && Kp <= kPanelMaxK && (int64_t)((N + 127) / 128) * batches <= 0x7fffffff &&
      (g_gemm_panel > 0 || (g_gemm_panel < 0 && gy >= 4))) {
    // 128-column panels, eight waves, one workgroup a CU. (64-column panels with two
    // workgroups a CU, so that one loads its panel while the other computes, measured
    // the same with 32 x 64 wave tiles and 30 % slower with 32 x 32 ones, which load
    // every A fragment twice as often.)
    constexpr int pn = 128;
    const int gx = (N + pn - 1) / pn;
    dim3 grid((unsigned)(gx * batches));
#define SDA_PANEL_K(VT, L, F, PN, JT, T)                                                                       \
  hipLaunchKernelGGL((k_modgemm_panel<VT, L, F, PN, JT, T>), grid, dim3(PN / (16 * JT) * 128 * T), 0, s, M, N, Kp, \
                     batches, gx, gy, mp, mf, a_frag, B, b_plane, (VT*)C, ldc_z, ldc_m, ldc_n, limit, cnt,     \
                     cnt_tiles)
#define SDA_PANEL3(VT, F) SDA_PANEL_K(VT, 3, F, 128, 4, 2)
#define SDA_PANEL4(VT, F) SDA_PANEL_K(VT, 4, F, 128, 2, 1)
#define SDA_PANEL_VT(VT)                                                    \
  do {                                                                      \
    if (limbs == 3) {                                                       \
      if (fold == 3) SDA_PANEL3(VT, 3);                                     \
      else if (fold == 1) SDA_PANEL3(VT, 1);                                \
      else SDA_PANEL3(VT, 0);                                               \
    } else if (fold == 2) {                                                 \
      SDA_PANEL4(VT, 2);                                                    \
    } else if (fold == 1) {                                                 \
      SDA_PANEL4(VT, 1);                                                    \
    } else {                                                                \
      SDA_PANEL4(VT, 0);                                                    \
    }                                                                       \
  } while (0)
    if (value_bytes == 1) SDA_PANEL_VT(uint8_t);
    else if (value_bytes == 2) SDA_PANEL_VT(uint16_t);
    else SDA_PANEL_VT(uint32_t);
#undef SDA_PANEL_VT
#undef SDA_PANEL3
#undef SDA_PANEL4
#undef SDA_PANEL_K
    return;
  }
  GemmGrid gg;
  gg.gx = (N + kBN - 1) / kBN;
  gg.gy = (M + kBM - 1) / kBM;
  gg.panels = gg.gx * batches;
  {
    // super-tile: all row blocks if they are few, else 8; panels to fill ~2 MB of L2
    const int64_t a_tile = (int64_t)kBM * Kp * limbs, b_panel = (int64_t)kBN * Kp * limbs;
    gg.gm = gg.gy <= 16 ? gg.gy : 8;
    const int64_t room = (2 << 20) - gg.gm * a_tile;
    gg.gp = (int)std::max<int64_t>(1, std::min<int64_t>(8, room / b_panel));
    gg.tiles_m = (gg.gy + gg.gm - 1) / gg.gm;
  }
  const int panels_x = (gg.panels + kXcds - 1) / kXcds;          // panels per id class
  const int tiles_p = (panels_x + gg.gp - 1) / gg.gp;
  const int64_t blocks = (int64_t)kXcds * gg.tiles_m * tiles_p * gg.gm * gg.gp;
  if (blocks > 0x7fffffff) return;  // cannot happen below 2^31 output tiles
  dim3 grid((unsigned)blocks);
#define SDA_GEMM(VT, L, F)                                                                        \
  hipLaunchKernelGGL((k_modgemm_i8<VT, L, F>), grid, dim3(256), 0, s, M, N, Kp, batches, gg, mp, mf, A, B, b_plane, \
                     (VT*)C, ldc_z, ldc_m, ldc_n, limit, cnt, cnt_tiles)
#define SDA_GEMM_VT(VT)                                                     \
  do {                                                                      \
    if (limbs == 3) {                                                       \
      if (fold == 3) SDA_GEMM(VT, 3, 3);                                    \
      else if (fold == 1) SDA_GEMM(VT, 3, 1);                               \
      else SDA_GEMM(VT, 3, 0);                                              \
    } else if (fold == 2) {                                                 \
      SDA_GEMM(VT, 4, 2);                                                   \
    } else if (fold == 1) {                                                 \
      SDA_GEMM(VT, 4, 1);                                                   \
    } else {                                                                \
      SDA_GEMM(VT, 4, 0);                                                   \
    }                                                                       \
  } while (0)
  if (value_bytes == 1) SDA_GEMM_VT(uint8_t);
  else if (value_bytes == 2) SDA_GEMM_VT(uint16_t);
  else SDA_GEMM_VT(uint32_t);
#undef SDA_GEMM_VT
#undef SDA_GEMM
}

void launch_pss_x_limbs(int P, int D, int B, int k, int t, int Kp, uint32_t p, const int32_t* secrets,
                        RngKeyArg rng, uint64_t owner_base, int8_t* X, hipStream_t s) {
  if (P <= 0 || B <= 0) return;
  const int64_t threads = (int64_t)B * (Kp / 16);
  dim3 grid((unsigned)((threads + 255) / 256), P);
  const LimbScheme sch = limb_scheme(p, Kp);
  auto kern = sch.bits == 8 ? k_pss_x_limbs<3, 8> : sch.limbs == 3 ? k_pss_x_limbs<3, 7> : k_pss_x_limbs<4, 7>;
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, P, D, B, k, t, Kp, make_mod_params(p), secrets, rng,
                     owner_base, X);
}

void launch_limbs_t(int R, int N, int Kp, uint32_t p, const uint32_t* Y, int8_t* out, hipStream_t s) {
  if (R <= 0 || N <= 0) return;
  dim3 grid((unsigned)(Kp / 64), (unsigned)((N + 63) / 64));
  const LimbScheme sch = limb_scheme(p, Kp);
  auto kern = sch.bits == 8 ? k_limbs_t<3, 8> : sch.limbs == 3 ? k_limbs_t<3, 7> : k_limbs_t<4, 7>;
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, R, N, Kp, p, Y, out);
}

}  // namespace sdagpu
