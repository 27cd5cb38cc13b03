// Participant-side kernels: masking + secret sharing + varint byte counting.
//
// Reference semantics:
//  * additive sharing  client/src/crypto/sharing/additive.rs:32-51 (n-1 uniform
//    shares, last = secret - sum), batched per clerk (batched.rs:19-52)
//  * packed Shamir     client/src/crypto/sharing/packed_shamir.rs:40-43 -> tss
//    share(); here as the equivalent n x (k+t) matrix product
//  * masks             masking/full.rs:22-34 (uniform mask), masking/chacha.rs:22-53
//    (rand-0.3 ChaChaRng expansion of a per-participant seed)
//
// Randomness: counter-mode ChaCha20 keyed per round from OS entropy, one stream
// per (purpose, participant); every draw is exact-uniform (rejection with a
// deterministic retry stream), so outputs are a pure function of (key, indices).
// The share kernel writes shares clerk-major ([n][P][B]) so each clerk's block
// is contiguous -- the "transpose" of the snapshot step (server/src/stores.rs:86-101)
// is free.
#include "block_utils.hpp"
#include "device_crypto.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

SDA_DEV RngKey to_key(const RngKeyArg& a) {
  RngKey k;
#pragma unroll
  for (int i = 0; i < 8; ++i) k.k[i] = a.k[i];
  return k;
}

// zigzag-varint length of a canonical (non-negative, < 2^32) value
SDA_DEV uint32_t vlen(uint32_t v) {
  uint64_t z = (uint64_t)v << 1;
  return 1u + (z >= (1ull << 7)) + (z >= (1ull << 14)) + (z >= (1ull << 21)) + (z >= (1ull << 28));
}

template <typename VT>
SDA_DEV void store16(VT* dst, const uint32_t (&v)[16], int valid, bool vec_ok) {
  if (vec_ok && valid == 16) {
    if constexpr (sizeof(VT) == 2) {
      uint4 a, b;
      a.x = v[0] | (v[1] << 16); a.y = v[2] | (v[3] << 16);
      a.z = v[4] | (v[5] << 16); a.w = v[6] | (v[7] << 16);
      b.x = v[8] | (v[9] << 16); b.y = v[10] | (v[11] << 16);
      b.z = v[12] | (v[13] << 16); b.w = v[14] | (v[15] << 16);
      reinterpret_cast<uint4*>(dst)[0] = a;
      reinterpret_cast<uint4*>(dst)[1] = b;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        reinterpret_cast<uint4*>(dst)[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < valid) dst[i] = (VT)v[i];
  }
}

SDA_DEV void load16_secrets(uint32_t (&x)[16], const int32_t* src, int valid, bool vec_ok,
                            const ModParams& mp) {
  int32_t s[16];
  if (vec_ok && valid == 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int4 a = reinterpret_cast<const int4*>(src)[q];
      s[4 * q] = a.x; s[4 * q + 1] = a.y; s[4 * q + 2] = a.z; s[4 * q + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = i < valid ? src[i] : 0;
  }
  // all 16 already canonical (the usual case): their OR is below m exactly then
  // (a value is at most the OR; a negative one sets bit 31)
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) any |= (uint32_t)s[i];
  if (any < mp.m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = (uint32_t)s[i];
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = canon_i32(s[i], mp);
  }
}

SDA_DEV uint32_t draw(uint32_t w, const RngKey& rk, uint64_t retry_purpose, uint64_t owner,
                      uint64_t idx, const ModParams& mp) {
  if ((uint64_t)w < mp.zone32) return mod32(w, mp);
  return uniform_fixup(rk, retry_purpose, owner, idx, mp.m, (uint32_t)mp.zone32);
}

// ------------------------------------------------------------- additive ----
// 16 exact-uniform draws in [0, m) from one ChaCha block: the common path is a
// Barrett reduction per word; rejected words (probability < m / 2^32 each) are
// re-drawn from a private retry stream in a rarely taken, lane-divergent branch.
SDA_DEV void draw16(uint32_t (&w)[16], const RngKey& rk, uint64_t purpose, uint64_t retry,
                    uint64_t owner, uint64_t block, uint64_t idx0, uint64_t idx_stride,
                    const ModParams& mp) {
  rng_block(w, rk, stream_id(purpose, owner), block);
  uint32_t rej = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    rej |= ((uint64_t)w[i] >= mp.zone32 ? 1u : 0u) << i;
    w[i] = mod32(w[i], mp);
  }
  if (rej) {
    for (int i = 0; i < 16; ++i)
      if ((rej >> i) & 1)
        w[i] = uniform_fixup(rk, retry, owner, idx0 + (uint64_t)i * idx_stride, mp.m,
                             (uint32_t)mp.zone32);
  }
}

// Per-clerk tile byte counts: wave partial sums in LDS, one barrier at the end.
constexpr int kMaxCountSlots = 256;

template <typename VT, int MASK>
__global__ void __launch_bounds__(kBlock)
    k_share_additive(int P, int D, int n, ModParams mp, const int32_t* __restrict__ secrets,
                     RngKeyArg rng, uint64_t owner_base, VT* __restrict__ shares,
                     uint32_t* __restrict__ cnt, VT* __restrict__ mask_out,
                     uint32_t* __restrict__ mask_cnt) {
  __shared__ uint32_t partial[kMaxCountSlots + 1][kWaves];
  const int t = blockIdx.x, p = blockIdx.y, T = gridDim.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int e0 = t * kTileValues + tid * 16;
  const int valid = max(0, min(16, D - e0));
  const uint64_t owner = owner_base + (uint64_t)p;
  const uint64_t gidx = (uint64_t)e0 / 16;  // 16-element group index = ChaCha block id
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;
  const bool vec_ok = (D % 16) == 0;

  // `last` starts as the (masked) secret and becomes secret - sum(random shares)
  uint32_t last[16];
  load16_secrets(last, secrets + (size_t)p * D + e0, valid, vec_ok, mp);

  if constexpr (MASK == kMaskFull) {
    uint32_t w[16];
    draw16(w, rk, kPurposeMaskFull, kPurposeMaskRetry, owner, gidx, (uint64_t)e0, 1, mp);
    uint32_t bytes = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      last[i] = add_mod(last[i], w[i], m);
      bytes += i < valid ? vlen(w[i]) : 0u;
    }
    store16<VT>(mask_out + (size_t)p * D + e0, w, valid, vec_ok);
    bytes = wave_sum(bytes);
    if (lane == 0) partial[kMaxCountSlots][wave] = bytes;
  }

  const int w_draws = n - 1;
  for (int c = 0; c < w_draws; ++c) {
    uint32_t w[16];
    draw16(w, rk, kPurposeShares, kPurposeSharesRetry, owner, gidx * (uint64_t)w_draws + c,
           (uint64_t)e0 * (uint64_t)w_draws + c, (uint64_t)w_draws, mp);
    uint32_t bytes = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      last[i] = sub_mod(last[i], w[i], m);
      bytes += i < valid ? vlen(w[i]) : 0u;
    }
    store16<VT>(shares + ((size_t)c * P + p) * D + e0, w, valid, vec_ok);
    bytes = wave_sum(bytes);
    if (lane == 0) partial[c][wave] = bytes;
  }
  {
    uint32_t bytes = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) bytes += i < valid ? vlen(last[i]) : 0u;
    store16<VT>(shares + ((size_t)(n - 1) * P + p) * D + e0, last, valid, vec_ok);
    bytes = wave_sum(bytes);
    if (lane == 0) partial[n - 1][wave] = bytes;
  }
  __syncthreads();
  for (int c = tid; c < n; c += kBlock) {
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += partial[c][w];
    cnt[((size_t)c * P + p) * T + t] = s;
  }
  if constexpr (MASK == kMaskFull) {
    if (tid == 0) {
      uint32_t s = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) s += partial[kMaxCountSlots][w];
      mask_cnt[(size_t)p * T + t] = s;
    }
  }
}

// ------------------------------------------------ additive, 16-bit draws ----
// For m < 2^16 one ChaCha block yields 32 draws (its 16-bit halves) instead of
// 16, halving the keystream work of the largest participant kernel. Each lane
// covers 64 elements (4 count tiles of 4096 per block: lane l, group g ->
// elements blk*16384 + g*4096 + l*16 .. +15); every row pair of draws costs one
// block per group. A rejected half (probability (2^16 mod m) / 2^16: 0.23% for
// m = 433) is replaced on the spot by the next accepted half of the lane's
// private retry block, generated once per lane and kept in registers; a lane
// that exhausts its 32 spares falls back to the per-element retry stream. Every
// share stays an exact, independent uniform draw. (A deferred variant that
// patched stores after the fact needed an out-of-line call whose ABI cost more
// registers than the halved keystream saved.)
constexpr int kG16 = 4;        // groups of 16 elements per lane
constexpr int kMaxRows16 = 64; // rows (n - 1 draws + mask) handled by this kernel

SDA_DEV uint32_t half16(const uint32_t (&w)[16], int k) { return (w[k >> 1] >> (16 * (k & 1))) & 0xffffu; }

template <int MASK>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_share_additive16(int P, int D, int n, ModParams mp, uint32_t zone16,
                       const int32_t* __restrict__ secrets, RngKeyArg rng, uint64_t owner_base,
                       uint16_t* __restrict__ shares, uint32_t* __restrict__ cnt,
                       uint16_t* __restrict__ mask_out, uint32_t* __restrict__ mask_cnt) {
  // partial[row][group][wave] byte counts; the final share at index kMaxRows16
  __shared__ uint32_t partial[kMaxRows16 + 1][kG16][kWaves];
  const int blk = blockIdx.x, p = blockIdx.y;
  const int T = (D + kTileValues - 1) / kTileValues;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t owner = owner_base + (uint64_t)p;
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;
  const bool vec_ok = (D % 16) == 0;
  constexpr int kMaskRows = MASK == kMaskFull ? 1 : 0;
  const int rows = kMaskRows + (n - 1);
  const int64_t Gtot = ((int64_t)D + 15) / 16;
  const uint64_t lane_id = (uint64_t)blk * kBlock + tid;

  uint32_t rw[16];  // this lane's spare halves
  rng_block(rw, rk, stream_id(kPurposeRetry16, owner), lane_id);
  uint32_t rused = 0;
  uint16_t* lastrow = shares + ((size_t)(n - 1) * P + p) * D;

#pragma unroll 1
  for (int g = 0; g < kG16; ++g) {
    const int e0 = blk * (kG16 * kTileValues) + g * kTileValues + tid * 16;
    const int valid = max(0, min(16, D - e0));
    uint32_t last[16];
    load16_secrets(last, secrets + (size_t)p * D + e0, valid, vec_ok, mp);
    for (int q = 0; 2 * q < rows; ++q) {
      uint32_t w[16];
      rng_block(w, rk, stream_id(kPurposeShares16, owner), (uint64_t)q * Gtot + e0 / 16);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = 2 * q + h;
        if (row >= rows) break;
        const bool is_mask = row < kMaskRows;
        uint32_t v[16];
        uint32_t rej = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t x = half16(w, 16 * h + i);
          v[i] = mod32(x, mp);
          rej |= (uint32_t)(x >= zone16) << i;
        }
        if (rej) {  // rare per lane (~4% of rows at m = 433)
          for (uint32_t bits = rej; bits; bits &= bits - 1) {
            const int i = __builtin_ctz(bits);
            uint32_t x = 0xffffffffu;
            while (rused < 32 && x >= zone16) {
              uint32_t word = 0;
#pragma unroll
              for (int k = 0; k < 16; ++k) word = (k == (int)(rused >> 1)) ? rw[k] : word;
              x = (word >> (16 * (rused & 1))) & 0xffffu;
              ++rused;
            }
            const uint32_t r = x < zone16
                ? mod32(x, mp)
                : uniform_fixup(rk, kPurposeSharesRetry, owner, ((uint64_t)row << 40) | (uint64_t)(e0 + i), m,
                                (uint32_t)mp.zone32);
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = k == i ? r : v[k];
          }
        }
        uint32_t bytes = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          last[i] = is_mask ? add_mod(last[i], v[i], m) : sub_mod(last[i], v[i], m);
          bytes += i < valid ? vlen(v[i]) : 0u;
        }
        if (is_mask) {
          store16<uint16_t>(mask_out + (size_t)p * D + e0, v, valid, vec_ok);
        } else {
          store16<uint16_t>(shares + ((size_t)(row - kMaskRows) * P + p) * D + e0, v, valid,
                            vec_ok);
        }
        bytes = wave_sum(bytes);
        if (lane == 0) partial[row][g][wave] = bytes;
      }
    }
    // the final share of this group
    uint32_t bytes = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) bytes += i < valid ? vlen(last[i]) : 0u;
    store16<uint16_t>(lastrow + e0, last, valid, vec_ok);
    bytes = wave_sum(bytes);
    if (lane == 0) partial[kMaxRows16][g][wave] = bytes;
  }
  __syncthreads();
  // tile byte counts: (rows + final) x 4 groups, each group one count tile
  for (int x = tid; x < (rows + 1) * kG16; x += kBlock) {
    const int r = x / kG16, g = x % kG16;
    const int prow = r < rows ? r : kMaxRows16;
    const int t = blk * kG16 + g;
    if (t >= T) continue;
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += partial[prow][g][w];
    if (r < kMaskRows) mask_cnt[(size_t)p * T + t] = s;
    else if (r < rows) cnt[((size_t)(r - kMaskRows) * P + p) * T + t] = s;
    else cnt[((size_t)(n - 1) * P + p) * T + t] = s;
  }
}

// ------------------------------------- additive, 16-bit draws, packed pairs ----
// The same exact-uniform 16-bit draws as k_share_additive16, with every
// per-value step after the ChaCha core done on packed u16 pairs (m <= 32768, so
// a pair's modular sum / difference never leaves 16 bits):
//   add/sub mod m   v_pk_add/sub_u16 + v_pk_min_u16 (3 ops per 2 values)
//   byte counts     zigzag length 1 + (v >= 64) (+ (v >= 8192)): one add + mask
//                   + v_bcnt per pair
//   rejection       a v_pk_max_u16 sweep over the block's 16 words; only a wave
//                   holding a rejected half walks the replacement path
// and 8 count tiles per lane so the lane's spare-draw block (one ChaCha block)
// is amortised over 256 draws. The per-value path of k_share_additive16 spent
// as many VALU instructions as its ChaCha cores (the round is VALU-bound).
constexpr int kGP = 8;  // count tiles (groups of 16 elements) per lane

SDA_DEV uint32_t pk_add_mod(uint32_t a, uint32_t b, u16x2 mm) {
  const u16x2 t = __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(t, t - mm));
}
SDA_DEV uint32_t pk_sub_mod(uint32_t a, uint32_t b, u16x2 mm) {
  const u16x2 t = __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(t, t + mm));
}
// x mod m for a 16-bit x (q = floor(x * mu32 / 2^32) is floor(x/m) or one less)
SDA_DEV uint32_t mod16(uint32_t x, const ModParams& mp) {
  const uint32_t q = __umulhi(x, mp.mu32);
  const uint32_t r = x - __umul24(q, mp.m);
  return min(r, r - mp.m);
}
// zigzag-varint bytes of the two canonical values of a pair (< 2^15)
template <bool kShort>
SDA_DEV uint32_t pk_vlen(uint32_t p) {
  uint32_t n = 2u + __builtin_popcount((p + 0x7fc07fc0u) & 0x80008000u);  // v >= 64
  if constexpr (!kShort) n += __builtin_popcount((p + 0x60006000u) & 0x80008000u);  // v >= 8192
  return n;
}

// byte count of the first `valid` of 16 values held as 8 pairs
template <bool kShort>
SDA_DEV uint32_t pairs_bytes(const uint32_t (&vp)[8], int valid) {
  uint32_t bytes = 0;
  if (valid == 16) {
#pragma unroll
    for (int k = 0; k < 8; ++k) bytes += pk_vlen<kShort>(vp[k]);
  } else {
    for (int i = 0; i < valid; ++i) bytes += vlen((vp[i >> 1] >> (16 * (i & 1))) & 0xffffu);
  }
  return bytes;
}
SDA_DEV void store_pairs(uint16_t* dst, const uint32_t (&vp)[8], int valid, bool vec_ok) {
  if (vec_ok && valid == 16) {
    reinterpret_cast<uint4*>(dst)[0] = make_uint4(vp[0], vp[1], vp[2], vp[3]);
    reinterpret_cast<uint4*>(dst)[1] = make_uint4(vp[4], vp[5], vp[6], vp[7]);
  } else {
    for (int i = 0; i < valid; ++i) dst[i] = (uint16_t)(vp[i >> 1] >> (16 * (i & 1)));
  }
}

template <int MASK, bool kShort>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_share_additive16p(int P, int D, int n, ModParams mp, uint32_t zone16,
                        const int32_t* __restrict__ secrets, RngKeyArg rng, uint64_t owner_base,
                        uint16_t* __restrict__ shares, uint32_t* __restrict__ cnt,
                        uint16_t* __restrict__ mask_out, uint32_t* __restrict__ mask_cnt) {
  __shared__ uint32_t partial[kMaxRows16 + 1][kGP][kWaves];
  const int blk = blockIdx.x, p = blockIdx.y;
  const int T = (D + kTileValues - 1) / kTileValues;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t owner = owner_base + (uint64_t)p;
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;
  const u16x2 mm = {(uint16_t)m, (uint16_t)m};
  const bool vec_ok = (D % 16) == 0;
  constexpr int kMaskRows = MASK == kMaskFull ? 1 : 0;
  const int rows = kMaskRows + (n - 1);
  const int64_t Gtot = ((int64_t)D + 15) / 16;
  const uint64_t lane_id = (uint64_t)blk * kBlock + tid;

  uint32_t rw[16];  // this lane's spare halves
  rng_block(rw, rk, stream_id(kPurposeRetry16, owner), lane_id);
  uint32_t rused = 0;
  uint16_t* lastrow = shares + ((size_t)(n - 1) * P + p) * D;

#pragma unroll 1
  for (int g = 0; g < kGP; ++g) {
    const int e0 = blk * (kGP * kTileValues) + g * kTileValues + tid * 16;
    const int valid = max(0, min(16, D - e0));
    uint32_t lastp[8];  // the (masked) secret, becoming secret - sum(random shares)
    {
      uint32_t s[16];
      load16_secrets(s, secrets + (size_t)p * D + e0, valid, vec_ok, mp);
#pragma unroll
      for (int k = 0; k < 8; ++k) lastp[k] = s[2 * k] | (s[2 * k + 1] << 16);
    }
    for (int q = 0; 2 * q < rows; ++q) {
      uint32_t w[16];
      rng_block(w, rk, stream_id(kPurposeShares16, owner), (uint64_t)q * Gtot + e0 / 16);
      // rejected halves (>= zone16, probability (2^16 mod m) / 2^16 each) are
      // replaced by the lane's next accepted spare; the wave-uniform test keeps
      // the walk out of waves that have none
      u16x2 hmax = __builtin_bit_cast(u16x2, w[0]);
#pragma unroll
      for (int k = 1; k < 16; ++k) hmax = __builtin_elementwise_max(hmax, __builtin_bit_cast(u16x2, w[k]));
      const bool any_rej = hmax.x >= zone16 || hmax.y >= zone16;
      if (__builtin_amdgcn_ballot_w64(any_rej) != 0 && any_rej) {
        uint32_t rej = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
          rej |= (((w[k] & 0xffffu) >= zone16 ? 1u : 0u) | ((w[k] >> 16) >= zone16 ? 2u : 0u)) << (2 * k);
        while (rej) {
          const int b = __builtin_ctz(rej);
          rej &= rej - 1;
          uint32_t x = 0xffffffffu;
          while (rused < 32 && x >= zone16) {
            uint32_t word = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) word = (k == (int)(rused >> 1)) ? rw[k] : word;
            x = (word >> (16 * (rused & 1))) & 0xffffu;
            ++rused;
          }
          if (x >= zone16) {  // spares exhausted: an exact draw from the per-element retry stream
            const int row = 2 * q + (b >> 4);
            x = uniform_fixup(rk, kPurposeSharesRetry, owner,
                              ((uint64_t)row << 40) | (uint64_t)(e0 + ((b >> 1) & 7) * 2 + (b & 1)), m,
                              (uint32_t)mp.zone32);
          }
          const uint32_t sh = 16u * (uint32_t)(b & 1);
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (k == (b >> 1)) w[k] = (w[k] & ~(0xffffu << sh)) | (x << sh);
        }
      }
      uint32_t bytes2 = 0;  // this pair of rows' byte counts in the two halves
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = 2 * q + h;
        if (row >= rows) break;
        const bool is_mask = row < kMaskRows;
        uint32_t vp[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          vp[k] = mod16(w[8 * h + k] & 0xffffu, mp) | (mod16(w[8 * h + k] >> 16, mp) << 16);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          lastp[k] = is_mask ? pk_add_mod(lastp[k], vp[k], mm) : pk_sub_mod(lastp[k], vp[k], mm);
        bytes2 |= pairs_bytes<kShort>(vp, valid) << (16 * h);
        if (is_mask) {
          uint32_t v[16];
#pragma unroll
          for (int k = 0; k < 8; ++k) { v[2 * k] = vp[k] & 0xffffu; v[2 * k + 1] = vp[k] >> 16; }
          store16<uint16_t>(mask_out + (size_t)p * D + e0, v, valid, vec_ok);
        } else {
          store_pairs(shares + ((size_t)(row - kMaskRows) * P + p) * D + e0, vp, valid, vec_ok);
        }
      }
      bytes2 = wave_sum(bytes2);  // both rows at once (each < 2^16)
      if (lane == 0) {
        partial[2 * q][g][wave] = bytes2 & 0xffffu;
        if (2 * q + 1 < rows) partial[2 * q + 1][g][wave] = bytes2 >> 16;
      }
    }
    store_pairs(lastrow + e0, lastp, valid, vec_ok);
    const uint32_t bytes = wave_sum(pairs_bytes<kShort>(lastp, valid));
    if (lane == 0) partial[kMaxRows16][g][wave] = bytes;
  }
  __syncthreads();
  for (int x = tid; x < (rows + 1) * kGP; x += kBlock) {
    const int r = x / kGP, g = x % kGP;
    const int prow = r < rows ? r : kMaxRows16;
    const int t = blk * kGP + g;
    if (t >= T) continue;
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += partial[prow][g][w];
    if (r < kMaskRows) mask_cnt[(size_t)p * T + t] = s;
    else if (r < rows) cnt[((size_t)(r - kMaskRows) * P + p) * T + t] = s;
    else cnt[((size_t)(n - 1) * P + p) * T + t] = s;
  }
}

// ---------------------------------- additive, three draws per 32-bit word ----
// For m^3 < 2^32 (m <= 1625) one ChaCha word x yields three draws by Lemire's
// multiply-shift: d0 = hi(x m), x1 = lo(x m), d1 = hi(x1 m), x2 = lo(x1 m),
// d2 = hi(x2 m). Then d0 m^2 + d1 m + d2 = floor(x m^3 / 2^32) and lo(x m^3) is
// the remainder, so rejecting x when lo(x m^3) < 2^32 mod m^3 leaves that floor
// exactly uniform on [0, m^3): three independent exact-uniform draws per word,
// 48 per ChaCha block (16-bit halves give 32) -- a third fewer ChaCha cores,
// which are most of the kernel's VALU work, and 7 VALU ops per 3 draws instead
// of a Barrett step per draw. A rejected word (1.7% at m = 433) is replaced by
// the lane's next acceptable spare word (one private ChaCha block, screened
// once), then by the per-word retry stream.
// Layout: lane l of block b covers, per "triple" tt, elements l*16 .. +15 of
// the three count tiles 3 (b kT3 + tt) + c; word i of a row's block gives
// element i of each: digit c -> tile c.
// triples per lane: 6 (18 count tiles per block: the lane's spare block is 1/6 of a
// ChaCha block per triple) for big launches, 3 where that would leave too few blocks

// An acceptable word (x m3 >= t3) from the per-word retry stream of `idx`.
SDA_DEV uint32_t retry_word3(const RngKey& rk, uint64_t owner, uint64_t idx, uint32_t m3,
                             uint32_t t3) {
  for (uint64_t blk = 0;; ++blk) {
    uint32_t w[16];
    rng_block(w, rk, stream_id(kPurposeSharesRetry, owner), (idx << 8) | blk);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (w[i] * m3 >= t3) return w[i];
  }
}

template <int MASK, int kT3>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
    k_share_additive48(int P, int D, int n, ModParams mp, uint32_t m3, uint32_t t3,
                       const int32_t* __restrict__ secrets, RngKeyArg rng, uint64_t owner_base,
                       uint16_t* __restrict__ shares, uint32_t* __restrict__ cnt,
                       uint16_t* __restrict__ mask_out, uint32_t* __restrict__ mask_cnt) {
  __shared__ uint32_t partial[kMaxRows16 + 1][3 * kT3][kWaves];
  const int blk = blockIdx.x, p = blockIdx.y;
  const int T = (D + kTileValues - 1) / kTileValues;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t owner = owner_base + (uint64_t)p;
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;
  const u16x2 mm = {(uint16_t)m, (uint16_t)m};
  const bool vec_ok = (D % 16) == 0;
  constexpr int kMaskRows = MASK == kMaskFull ? 1 : 0;
  const int rows = kMaskRows + (n - 1);
  const uint64_t slots = (uint64_t)gridDim.x * kT3 * kBlock;  // (triple, lane) slots per row

  // this lane's spare words (in LDS: dynamically indexed, and no registers
  // held across the kernel); racc = the acceptable ones not used yet
  __shared__ uint32_t spare[16][kBlock];
  uint32_t racc = 0;
  {
    uint32_t rw[16];
    rng_block(rw, rk, stream_id(kPurposeRetry48, owner), (uint64_t)blk * kBlock + tid);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      spare[k][tid] = rw[k];
      racc |= (rw[k] * m3 >= t3 ? 1u : 0u) << k;
    }
  }
  uint16_t* lastrow = shares + ((size_t)(n - 1) * P + p) * D;

#pragma unroll 1
  for (int tt = 0; tt < kT3; ++tt) {
    int e0[3], valid[3];
    uint32_t lastp[3][8];  // (masked) secrets becoming secret - sum(random shares), as pairs
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      e0[c] = blk * (3 * kT3 * kTileValues) + (3 * tt + c) * kTileValues + tid * 16;
      valid[c] = max(0, min(16, D - e0[c]));
      uint32_t s[16];
      load16_secrets(s, secrets + (size_t)p * D + e0[c], valid[c], vec_ok, mp);
#pragma unroll
      for (int k = 0; k < 8; ++k) lastp[c][k] = s[2 * k] | (s[2 * k + 1] << 16);
    }
    const uint64_t slot = ((uint64_t)blk * kT3 + tt) * kBlock + tid;
    for (int r = 0; r < rows; ++r) {
      uint32_t w[16];
      rng_block(w, rk, stream_id(kPurposeShares48, owner), (uint64_t)r * slots + slot);
      uint32_t rej = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) rej |= (w[k] * m3 < t3 ? 1u : 0u) << k;
      if (__builtin_amdgcn_ballot_w64(rej != 0) != 0 && rej != 0) {
        while (rej) {
          const int b = __builtin_ctz(rej);
          rej &= rej - 1;
          uint32_t x;
          if (racc) {
            x = spare[__builtin_ctz(racc)][tid];
            racc &= racc - 1;
          } else {  // spares used up: exact draw from this word's retry stream
            x = retry_word3(rk, owner, ((uint64_t)r << 40) | (slot * 16 + (uint64_t)b), m3, t3);
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) w[k] = k == b ? x : w[k];
        }
      }
      // digit c of every word (hi(x m), then x <- lo(x m)), as u16 pairs -> tile c
      const bool is_mask = r < kMaskRows;
      uint32_t bytes[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        uint32_t vp[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) vp[k] = __umulhi(w[2 * k], m) | (__umulhi(w[2 * k + 1], m) << 16);
        if (c < 2) {
#pragma unroll
          for (int k = 0; k < 16; ++k) w[k] *= m;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
          lastp[c][k] = is_mask ? pk_add_mod(lastp[c][k], vp[k], mm) : pk_sub_mod(lastp[c][k], vp[k], mm);
        bytes[c] = pairs_bytes<true>(vp, valid[c]);
        if (is_mask) {
          uint32_t v[16];
#pragma unroll
          for (int k = 0; k < 8; ++k) { v[2 * k] = vp[k] & 0xffffu; v[2 * k + 1] = vp[k] >> 16; }
          store16<uint16_t>(mask_out + (size_t)p * D + e0[c], v, valid[c], vec_ok);
        } else {
          store_pairs(shares + ((size_t)(r - kMaskRows) * P + p) * D + e0[c], vp, valid[c], vec_ok);
        }
      }
      const uint32_t b01 = wave_sum(bytes[0] | (bytes[1] << 16));  // each < 2^16
      const uint32_t b2 = wave_sum(bytes[2]);
      if (lane == 0) {
        partial[r][3 * tt][wave] = b01 & 0xffffu;
        partial[r][3 * tt + 1][wave] = b01 >> 16;
        partial[r][3 * tt + 2][wave] = b2;
      }
    }
    // the final shares of this triple
    uint32_t lb[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      store_pairs(lastrow + e0[c], lastp[c], valid[c], vec_ok);
      lb[c] = pairs_bytes<true>(lastp[c], valid[c]);
    }
    const uint32_t l01 = wave_sum(lb[0] | (lb[1] << 16));
    const uint32_t l2 = wave_sum(lb[2]);
    if (lane == 0) {
      partial[kMaxRows16][3 * tt][wave] = l01 & 0xffffu;
      partial[kMaxRows16][3 * tt + 1][wave] = l01 >> 16;
      partial[kMaxRows16][3 * tt + 2][wave] = l2;
    }
  }
  __syncthreads();
  for (int x = tid; x < (rows + 1) * 3 * kT3; x += kBlock) {
    const int r = x / (3 * kT3), g = x % (3 * kT3);
    const int prow = r < rows ? r : kMaxRows16;
    const int t = blk * 3 * kT3 + g;
    if (t >= T) continue;
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += partial[prow][g][w];
    if (r < kMaskRows) mask_cnt[(size_t)p * T + t] = s;
    else if (r < rows) cnt[((size_t)(r - kMaskRows) * P + p) * T + t] = s;
    else cnt[((size_t)(n - 1) * P + p) * T + t] = s;
  }
}

// --------------------------------------------------------- packed Shamir ----
constexpr int kPssMaxK = 8;
constexpr int kPssMaxT = 16;
constexpr int kPssMaxN = 64;

template <typename VT, int MASK>
__global__ void __launch_bounds__(kBlock)
    k_share_pss(int P, int D, int n, int k, int t, ModParams mp, int small_acc,
                const int32_t* __restrict__ secrets, const uint32_t* __restrict__ mat,
                RngKeyArg rng, uint64_t owner_base, VT* __restrict__ shares,
                uint32_t* __restrict__ cnt, VT* __restrict__ mask_out,
                uint32_t* __restrict__ mask_cnt) {
  __shared__ uint32_t sM[kPssMaxN * (kPssMaxK + kPssMaxT)];
  __shared__ uint32_t scratch[kWaves];
  const int K = k + t;
  for (int i = threadIdx.x; i < n * K; i += kBlock) sM[i] = mat[i];
  __syncthreads();
  const int tile = blockIdx.x, p = blockIdx.y, T = gridDim.x;
  const int tid = threadIdx.x;
  const int B = (D + k - 1) / k;
  const uint64_t owner = owner_base + (uint64_t)p;
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;

  uint32_t mask_bytes = 0;

  // per-clerk byte counters live in LDS-free registers only for small n; use
  // one pass per clerk group of 8 to bound registers.
  for (int cg = 0; cg < n; cg += 8) {
    uint32_t bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 16; ++i) {
      const int b = tile * kTileValues + tid + kBlock * i;
      if (b >= B) break;
      uint32_t v[kPssMaxK + kPssMaxT];
      // secrets (+mask) of this batch
#pragma unroll
      for (int j = 0; j < kPssMaxK; ++j) {
        if (j < k) {
          const int e = b * k + j;
          uint32_t x = e < D ? canon_i32(secrets[(size_t)p * D + e], mp) : 0u;
          if (e < D) {
            if constexpr (MASK == kMaskFull) {
              uint32_t w[16];
              rng_block(w, rk, stream_id(kPurposeMaskFull, owner), (uint64_t)e / 16);
              uint32_t mk = draw(w[e % 16], rk, kPurposeMaskRetry, owner, (uint64_t)e, mp);
              x = add_mod(x, mk, m);
              if (cg == 0) {
                mask_out[(size_t)p * D + e] = (VT)mk;
                mask_bytes += vlen(mk);
              }
            }
          }
          v[j] = x;
        } else {
          v[j] = 0;
        }
      }
      // t uniform draws: one ChaCha block per batch
      {
        uint32_t w[16];
        rng_block(w, rk, stream_id(kPurposeShares, owner), (uint64_t)b);
#pragma unroll
        for (int d = 0; d < kPssMaxT; ++d)
          v[kPssMaxK + d] = d < t ? draw(w[d], rk, kPurposeSharesRetry, owner,
                                         (uint64_t)b * 16 + d, mp)
                                  : 0u;
      }
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) {
        const int c = cg + cc;
        if (c >= n) break;
        const uint32_t* row = sM + c * K;
        uint32_t y;
        if (small_acc) {
          uint64_t acc = 0;
#pragma unroll
          for (int j = 0; j < kPssMaxK; ++j)
            if (j < k) acc += (uint64_t)row[j] * v[j];
#pragma unroll
          for (int d = 0; d < kPssMaxT; ++d)
            if (d < t) acc += (uint64_t)row[k + d] * v[kPssMaxK + d];
          y = mod64(acc, mp);
        } else {
          uint32_t acc = 0;
#pragma unroll
          for (int j = 0; j < kPssMaxK; ++j)
            if (j < k) acc = add_mod(acc, mod64((uint64_t)row[j] * v[j], mp), m);
#pragma unroll
          for (int d = 0; d < kPssMaxT; ++d)
            if (d < t) acc = add_mod(acc, mod64((uint64_t)row[k + d] * v[kPssMaxK + d], mp), m);
          y = acc;
        }
        shares[((size_t)c * P + p) * B + b] = (VT)y;
        bytes[cc] += vlen(y);
      }
    }
    for (int cc = 0; cc < 8; ++cc) {
      const int c = cg + cc;
      if (c >= n) break;
      uint32_t tot = block_sum(bytes[cc], scratch);
      if (tid == 0) cnt[((size_t)c * P + p) * T + tile] = tot;
    }
  }
  if constexpr (MASK == kMaskFull) {
    // mask message tiles are over D elements with kTileValues per tile; the
    // engine recounts them with k_count (PSS batches do not align with them).
    (void)mask_bytes;
    (void)mask_cnt;
  }
}

// ------------------------------------- packed Shamir, small fields (VALU) ----
// The reference parameter sets with n = 8 clerks and k = 3 secrets per batch
// (PSS_4_8_3 and the 5-of-8 set, t = 4 / 2) over p = 433: shares = M [s; r] per
// batch with u32 accumulation (K (p-1)^2 < 2^32: 24-bit multiply-adds) and one
// Barrett step per share. The t field elements of randomness of 32 / t batches
// come from one ChaCha block as Lemire triples (11 of its 16 words; rejected
// words are replaced by its other 5, then by the per-word retry stream) --
// where k_share_pss spends a whole block on every batch. Thread i of block b
// handles 16 batches of count tile b in runs of 4 / sizeof(share) adjacent ones
// (consecutive lanes store consecutive 32-bit words of shares). M is read through
// scalar loads (its addresses are uniform) and multiplied from SGPRs.
struct __attribute__((packed, aligned(1))) Word32 {
  uint32_t v;
};
struct __attribute__((packed, aligned(4))) Words2 {
  uint2 v;
};
constexpr int kPssKS = 3;  // secrets per batch
constexpr int kPssNC = 8;  // clerks

template <int T, typename VT, bool kMod24>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(T == 4 ? 3 : 2)))
    k_share_pss48(int P, int D, ModParams mp, Mod24 m24, uint32_t m3, uint32_t t3,
                  const int32_t* __restrict__ secrets, const uint32_t* __restrict__ mat,
                  RngKeyArg rng, uint64_t owner_base, VT* __restrict__ shares,
                  uint32_t* __restrict__ cnt) {
  constexpr int K = kPssKS + T;
  constexpr int kPerBlock = 32 / T;      // batches per ChaCha block
  constexpr int kAdj = 4 / sizeof(VT);   // adjacent batches per thread: one 32-bit store per clerk
  constexpr int kRounds = 16 / kPerBlock;
  __shared__ uint32_t partial[kPssNC][kWaves];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tile = blockIdx.x, p = blockIdx.y, Tt = gridDim.x;
  const int B = (D + kPssKS - 1) / kPssKS;
  const uint64_t owner = owner_base + (uint64_t)p;
  const RngKey rk = to_key(rng);
  const uint32_t m = mp.m;
  uint32_t extra[kPssNC];  // per clerk: shares of two varint bytes (v >= 64)
#pragma unroll
  for (int c = 0; c < kPssNC; ++c) extra[c] = 0;
  uint32_t nvalid = 0;

#pragma unroll 1
  for (int rd = 0; rd < kRounds; ++rd) {
    // this round's batches. A thread takes runs of kAdj adjacent batches (4 bytes of
    // shares per clerk), so that a run's shares leave in one 32-bit store and its
    // secrets arrive as consecutive words -- requested here, ahead of the ChaCha
    // block, which covers their latency.
    int32_t raw[kPerBlock * kPssKS];
#pragma unroll
    for (int q = 0; q < kPerBlock / kAdj; ++q) {
      const int b0 = tile * kTileValues + kAdj * (tid + kBlock * (rd * (kPerBlock / kAdj) + q));
      const int32_t* src = reinterpret_cast<const int32_t*>(
          reinterpret_cast<const char*>(secrets + (size_t)p * D) + (uint32_t)b0 * (uint32_t)(kPssKS * 4));
      int32_t* dst = raw + q * kAdj * kPssKS;
      if ((b0 + kAdj) * kPssKS <= D) {  // the run's secrets are all there: consecutive words
        const Words2* v = reinterpret_cast<const Words2*>(src);
#pragma unroll
        for (int i = 0; i < kAdj * kPssKS / 2; ++i) {
          const uint2 d = v[i].v;
          dst[2 * i] = (int32_t)d.x;
          dst[2 * i + 1] = (int32_t)d.y;
        }
      } else {
#pragma unroll
        for (int i = 0; i < kAdj * kPssKS; ++i) dst[i] = b0 * kPssKS + i < D ? src[i] : 0;
      }
    }
    uint32_t w[16];
    const uint64_t ctr = ((uint64_t)tile * kBlock + tid) * kRounds + rd;
    rng_block(w, rk, stream_id(kPurposeSharesPss48, owner), ctr);
    uint32_t rej = 0, spare = 0;
#pragma unroll
    for (int i = 0; i < 11; ++i) rej |= (w[i] * m3 < t3 ? 1u : 0u) << i;
#pragma unroll
    for (int i = 11; i < 16; ++i) spare |= (w[i] * m3 >= t3 ? 1u : 0u) << i;
    if (__builtin_amdgcn_ballot_w64(rej != 0) != 0 && rej != 0) {
      while (rej) {
        const int bi = __builtin_ctz(rej);
        rej &= rej - 1;
        uint32_t x;
        if (spare) {
          const int si = __builtin_ctz(spare);
          spare &= spare - 1;
          x = 0;
#pragma unroll
          for (int i = 11; i < 16; ++i) x = i == si ? w[i] : x;
        } else {
          x = retry_word3(rk, owner, (ctr << 4) | (uint64_t)bi, m3, t3);
        }
#pragma unroll
        for (int i = 0; i < 11; ++i) w[i] = i == bi ? x : w[i];
      }
    }
    uint32_t dg[33];
#pragma unroll
    for (int i = 0; i < 11; ++i) {
      const uint32_t x0 = w[i], x1 = x0 * m;
      dg[3 * i] = __umulhi(x0, m);
      dg[3 * i + 1] = __umulhi(x1, m);
      dg[3 * i + 2] = __umulhi(x1 * m, m);
    }
    // secrets (canonical) of this round's batches
    uint32_t s[kPerBlock][kPssKS];
    bool ok[kPerBlock];
    // batch indices as unsigned 32-bit offsets from the clerk's (uniform) row pointer:
    // one address register per run instead of a 64-bit pair per (clerk, run)
    uint32_t bidx[kPerBlock];
#pragma unroll
    for (int g = 0; g < kPerBlock; ++g) {
      const int q = g / kAdj, a = g % kAdj;
      bidx[g] = (uint32_t)(tile * kTileValues + kAdj * (tid + kBlock * (rd * (kPerBlock / kAdj) + q)) + a);
      ok[g] = bidx[g] < (uint32_t)B;
#pragma unroll
      for (int j = 0; j < kPssKS; ++j) s[g][j] = canon_i32(raw[g * kPssKS + j], mp);
      nvalid += ok[g] ? 1u : 0u;
    }
#pragma unroll
    for (int c = 0; c < kPssNC; ++c) {
      // the clerk's row of M: uniform addresses, i.e. scalar loads into SGPRs (a VGPR
      // copy of all 8 rows next to the 64 accumulators left 2 waves per SIMD)
      uint32_t row[K];
#pragma unroll
      for (int j = 0; j < K; ++j) row[j] = mat[c * K + j];
      VT* out = shares + ((size_t)c * P + p) * B;
#pragma unroll
      for (int q = 0; q < kPerBlock / kAdj; ++q) {
        uint32_t y[kAdj];
#pragma unroll
        for (int a = 0; a < kAdj; ++a) {
          const int g = q * kAdj + a;
          uint32_t acc = 0;
#pragma unroll
          for (int j = 0; j < kPssKS; ++j) acc += __umul24(row[j], s[g][j]);
#pragma unroll
          for (int d = 0; d < T; ++d) acc += __umul24(row[kPssKS + d], dg[g * T + d]);
          y[a] = kMod24 ? mod24(acc, m24) : mod32(acc, mp);
          extra[c] += (ok[g] && y[a] >= 64u) ? 1u : 0u;
        }
        if (ok[q * kAdj + kAdj - 1]) {  // the whole run lies inside the row
          uint32_t word = 0;
#pragma unroll
          for (int a = 0; a < kAdj; ++a) word |= y[a] << (8 * sizeof(VT) * a);
          // (row starts are only VT-aligned)
          reinterpret_cast<Word32*>(reinterpret_cast<char*>(out) + bidx[q * kAdj] * (uint32_t)sizeof(VT))->v = word;
        } else {
#pragma unroll
          for (int a = 0; a < kAdj; ++a)
            if (ok[q * kAdj + a]) out[bidx[q * kAdj + a]] = (VT)y[a];
        }
      }
    }
  }
  // per-clerk tile byte counts: one byte per share, two for v >= 64 (p <= 8192)
#pragma unroll
  for (int c = 0; c < kPssNC; ++c) {
    const uint32_t v = wave_sum(nvalid + extra[c]);
    if (lane == 0) partial[c][wave] = v;
  }
  __syncthreads();
  if (tid < kPssNC) {
    uint32_t v = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) v += partial[tid][w];
    cnt[((size_t)tid * P + p) * Tt + tile] = v;
  }
}

// ----------------------------------------------------------------- count ---
template <typename VT>
__global__ void __launch_bounds__(kBlock) k_count(int L, const VT* __restrict__ vals,
                                                  uint32_t* __restrict__ cnt) {
  __shared__ uint32_t scratch[kWaves];
  const int t = blockIdx.x, j = blockIdx.y, T = gridDim.x;
  const int e0 = t * kTileValues + threadIdx.x * 16;
  const VT* src = vals + (size_t)j * L;
  uint32_t bytes = 0;
  if (e0 + 16 <= L) {
    // 16-byte loads from an address that is only value-aligned (rows start at j * L)
    struct __attribute__((packed, aligned(1))) Q { uint32_t w[4]; };
    constexpr int kQ = (int)sizeof(VT) * 16 / 16;
    const Q* q = reinterpret_cast<const Q*>(src + e0);
#pragma unroll
    for (int i = 0; i < kQ; ++i) {
      const Q d = q[i];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (sizeof(VT) == 4) {
          bytes += vlen(d.w[u]);
        } else if constexpr (sizeof(VT) == 2) {
          bytes += vlen(d.w[u] & 0xffffu) + vlen(d.w[u] >> 16);
        } else {
          bytes += vlen(d.w[u] & 0xffu) + vlen((d.w[u] >> 8) & 0xffu) + vlen((d.w[u] >> 16) & 0xffu) +
                   vlen(d.w[u] >> 24);
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (e0 + i < L) bytes += vlen((uint32_t)src[e0 + i]);
  }
  uint32_t tot = block_sum(bytes, scratch);
  if (threadIdx.x == 0) cnt[(size_t)j * T + t] = tot;
}

}  // namespace

static int g_share16 = 1;
void set_share16(int mode) { g_share16 = mode; }
static int g_pss48 = 1;
void set_pss48(int mode) { g_pss48 = mode; }

void launch_share_additive(int P, int D, int n, uint32_t m, int value_bytes, const int32_t* secrets,
                           int mask_mode, RngKeyArg rng, uint64_t owner_base, void* shares,
                           uint32_t* cnt, void* mask_out, uint32_t* mask_cnt, hipStream_t s) {
  if (P <= 0 || D <= 0) return;
  if (n < 1 || n > kMaxCountSlots) return;  // rejected by the binding (n == 1: masking only)
  if (mask_mode != kMaskNone && mask_mode != kMaskFull) return;  // ChaCha masks: launch_chacha_mask_apply
  ModParams mp = make_mod_params(m);
  // 16-bit draws: u16 shares, no ChaCha mask, room for the rows in LDS
  const bool rows_ok = (n - 1) + (mask_mode == kMaskFull ? 1 : 0) <= kMaxRows16;
  const uint64_t m3 = (uint64_t)m * m * m;
  if (g_share16 == 1 && value_bytes == 2 && m3 < (1ull << 32) && rows_ok) {
    const uint32_t t3 = (uint32_t)((1ull << 32) % m3);  // reject x with lo(x m^3) < t3
    // six triples per block amortise the lanes' spare ChaCha block better (2.50 -> 2.43 ms
    // at 1000 x 1M); small launches (participant waves) keep three for twice the blocks
    const int64_t blocks6 = (int64_t)P * ((D + 18 * kTileValues - 1) / (18 * kTileValues));
    const int t3n = blocks6 >= 8192 ? 6 : 3;
    dim3 grid((D + 3 * t3n * kTileValues - 1) / (3 * t3n * kTileValues), P);
    auto kern = mask_mode == kMaskFull
                    ? (t3n == 6 ? k_share_additive48<kMaskFull, 6> : k_share_additive48<kMaskFull, 3>)
                    : (t3n == 6 ? k_share_additive48<kMaskNone, 6> : k_share_additive48<kMaskNone, 3>);
    hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, s, P, D, n, mp, (uint32_t)m3, t3, secrets, rng,
                       owner_base, (uint16_t*)shares, cnt, (uint16_t*)mask_out, mask_cnt);
    return;
  }
  if (g_share16 && value_bytes == 2 && m <= 32768u && rows_ok) {
    const uint32_t zone16 = 65536u - (65536u % m);
    dim3 grid((D + kGP * kTileValues - 1) / (kGP * kTileValues), P);
#define SDA_P16(MK, SH)                                                                      \
  hipLaunchKernelGGL((k_share_additive16p<MK, SH>), grid, dim3(kBlock), 0, s, P, D, n, mp, zone16, \
                     secrets, rng, owner_base, (uint16_t*)shares, cnt, (uint16_t*)mask_out, mask_cnt)
    if (mask_mode == kMaskFull) {
      if (m <= 8192u) SDA_P16(kMaskFull, true); else SDA_P16(kMaskFull, false);
    } else {
      if (m <= 8192u) SDA_P16(kMaskNone, true); else SDA_P16(kMaskNone, false);
    }
#undef SDA_P16
    return;
  }
  if (g_share16 && value_bytes == 2 && m < 65536u && rows_ok) {
    const uint32_t zone16 = 65536u - (65536u % m);
    dim3 grid16((D + kG16 * kTileValues - 1) / (kG16 * kTileValues), P);
    if (mask_mode == kMaskFull)
      hipLaunchKernelGGL(k_share_additive16<kMaskFull>, grid16, dim3(kBlock), 0, s, P, D, n, mp,
                         zone16, secrets, rng, owner_base, (uint16_t*)shares, cnt,
                         (uint16_t*)mask_out, mask_cnt);
    else
      hipLaunchKernelGGL(k_share_additive16<kMaskNone>, grid16, dim3(kBlock), 0, s, P, D, n, mp,
                         zone16, secrets, rng, owner_base, (uint16_t*)shares, cnt,
                         (uint16_t*)mask_out, mask_cnt);
    return;
  }
  dim3 grid((D + kTileValues - 1) / kTileValues, P);
#define SDA_ADD_LAUNCH(VT, MK)                                                                \
  hipLaunchKernelGGL((k_share_additive<VT, MK>), grid, dim3(kBlock), 0, s, P, D, n, mp,        \
                     secrets, rng, owner_base, (VT*)shares, cnt, (VT*)mask_out, mask_cnt)
  if (value_bytes == 2) {
    if (mask_mode == kMaskFull) SDA_ADD_LAUNCH(uint16_t, kMaskFull);
    else SDA_ADD_LAUNCH(uint16_t, kMaskNone);
  } else {
    if (mask_mode == kMaskFull) SDA_ADD_LAUNCH(uint32_t, kMaskFull);
    else SDA_ADD_LAUNCH(uint32_t, kMaskNone);
  }
#undef SDA_ADD_LAUNCH
}

void launch_share_pss(int P, int D, int n, int k, int t, uint32_t p, int value_bytes,
                      const int32_t* secrets, const uint32_t* share_matrix, int mask_mode,
                      RngKeyArg rng, uint64_t owner_base, void* shares, uint32_t* cnt,
                      void* mask_out, uint32_t* mask_cnt, hipStream_t s) {
  if (P <= 0 || D <= 0) return;
  if (mask_mode != kMaskNone && mask_mode != kMaskFull) return;  // ChaCha masks: launch_chacha_mask_apply
  ModParams mp = make_mod_params(p);
  const int B = (D + k - 1) / k;
  // accumulate in u64 without intermediate reduction when K*(p-1)^2 < 2^64
  const double bound = (double)(k + t) * (double)(p - 1) * (double)(p - 1);
  const int small_acc = bound < 1.8e19 ? 1 : 0;
  dim3 grid((B + kTileValues - 1) / kTileValues, P);
  const uint64_t p3 = (uint64_t)p * p * p;
  if (g_pss48 && value_bytes <= 2 && mask_mode == kMaskNone && k == kPssKS && n == kPssNC &&
      (t == 2 || t == 4) && p <= 8192u && p3 < (1ull << 32)) {
    const uint32_t t3 = (uint32_t)((1ull << 32) % p3);
    // a share is a sum of k + t products of canonical values
    const Mod24 m24 = make_mod24(p, (uint64_t)(k + t) * (p - 1) * (p - 1));
#define SDA_PSS48(TT, VT)                                                                     \
  do {                                                                                        \
    if (m24.c)                                                                                \
      hipLaunchKernelGGL((k_share_pss48<TT, VT, true>), grid, dim3(kBlock), 0, s, P, D, mp, m24, \
                         (uint32_t)p3, t3, secrets, share_matrix, rng, owner_base, (VT*)shares,  \
                         cnt);                                                                \
    else                                                                                      \
      hipLaunchKernelGGL((k_share_pss48<TT, VT, false>), grid, dim3(kBlock), 0, s, P, D, mp, m24, \
                         (uint32_t)p3, t3, secrets, share_matrix, rng, owner_base, (VT*)shares,  \
                         cnt);                                                                \
  } while (0)
    if (value_bytes == 1) {  // p <= 256: a share per byte
      if (t == 4) SDA_PSS48(4, uint8_t); else SDA_PSS48(2, uint8_t);
    } else {
      if (t == 4) SDA_PSS48(4, uint16_t); else SDA_PSS48(2, uint16_t);
    }
#undef SDA_PSS48
    return;
  }
#define SDA_PSS_LAUNCH(VT, MK)                                                             \
  hipLaunchKernelGGL((k_share_pss<VT, MK>), grid, dim3(kBlock), 0, s, P, D, n, k, t, mp,       \
                     small_acc, secrets, share_matrix, rng, owner_base, (VT*)shares, cnt,      \
                     (VT*)mask_out, mask_cnt)
  if (value_bytes == 1) {
    if (mask_mode == kMaskFull) SDA_PSS_LAUNCH(uint8_t, kMaskFull);
    else SDA_PSS_LAUNCH(uint8_t, kMaskNone);
  } else if (value_bytes == 2) {
    if (mask_mode == kMaskFull) SDA_PSS_LAUNCH(uint16_t, kMaskFull);
    else SDA_PSS_LAUNCH(uint16_t, kMaskNone);
  } else {
    if (mask_mode == kMaskFull) SDA_PSS_LAUNCH(uint32_t, kMaskFull);
    else SDA_PSS_LAUNCH(uint32_t, kMaskNone);
  }
#undef SDA_PSS_LAUNCH
}

void launch_count(int M, int L, int value_bytes, const void* vals, uint32_t* cnt, hipStream_t s) {
  if (M <= 0 || L <= 0) return;
  dim3 grid((L + kTileValues - 1) / kTileValues, M);
  if (value_bytes == 1)
    hipLaunchKernelGGL(k_count<uint8_t>, grid, dim3(kBlock), 0, s, L, (const uint8_t*)vals, cnt);
  else if (value_bytes == 2)
    hipLaunchKernelGGL(k_count<uint16_t>, grid, dim3(kBlock), 0, s, L, (const uint16_t*)vals, cnt);
  else
    hipLaunchKernelGGL(k_count<uint32_t>, grid, dim3(kBlock), 0, s, L, (const uint32_t*)vals, cnt);
}

}  // namespace sdagpu
