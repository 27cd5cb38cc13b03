// ChaCha masks: rand-0.3 `ChaChaRng` seed expansion on the device, bit for bit.
//
// Reference: client/src/crypto/masking/chacha.rs:29-39 (participant: seed from
// the OS, `gen_range(0, m)` per element, masked = secret + mask), :56-77
// (recipient: re-expand every participant's seed and sum the masks). rand 0.3's
// `gen_range` for i64 draws u64 values (two ChaCha words, high word first) and
// *rejects* a draw at or above zone = u64::MAX - u64::MAX % m: element e of a
// stream is its (e + 1)-th accepted draw, so one rejection shifts every later
// element of that participant by one draw.
//
// A rejection has probability m / 2^64 per draw (1e-10 at m = 2^31): the fast
// kernels therefore take draw e for element e -- a lane expands one ChaCha block
// = 8 draws with no dependence on any other lane -- and only *record* which
// participants saw a rejected draw. The repair kernels, launched right behind
// them and gated on that record (they exit at once when it is empty, without a
// host round trip), redo the affected participants exactly: rejections are
// counted per 2048-draw chunk, scanned, and every accepted draw is re-indexed to
// its true element. Nothing limits how many draws are rejected, up to half of
// them (a stream is scanned over 2 D + 4096 draws).
#include <hip/hip_runtime.h>

#include "block_utils.hpp"
#include "device_crypto.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {

namespace {

constexpr int kDrawsPerLane = 8;                      // one ChaCha block: 16 words = 8 u64 draws
constexpr int kChunkDraws = kBlock * kDrawsPerLane;   // 2048

// scratch layout (u32 words): [0] any-rejection flag, [1] number of affected
// participants A, [2, 2 + P) per-participant "saw a rejection" marks, [2 + P, 2 + 2P)
// the affected participants in increasing order, then A * C (at most P * C)
// rejection counts / bases (C chunks of the scanned range), one row per affected one
constexpr int kScratchHead = 2;
// The repair grids have this many rows; row y serves affected participants y,
// y + kRepairRows, ...: with nothing to repair (the usual case) a repair launch is
// C * kRepairRows blocks that return at once, not C * P.
constexpr int kRepairRows = 8;

// rand-0.3 ChaChaRng block `ctr` (128-bit counter, here < 2^64) for a seed.
SDA_DEV void chacharng_block(uint32_t (&w)[16], const uint32_t (&key)[8], uint64_t ctr) {
  uint32_t in[16] = {kSigma0, kSigma1, kSigma2, kSigma3, key[0], key[1], key[2], key[3],
                     key[4],  key[5],  key[6],  key[7],  (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
  chacha_block<20>(w, in);
}

// `p` is wave-uniform at every call site: the key lives in SGPRs.
__device__ __forceinline__ void load_seed_key(uint32_t (&key)[8], const uint32_t* seeds, int p,
                                              int seed_words) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    key[i] = __builtin_amdgcn_readfirstlane(i < seed_words ? seeds[(size_t)p * seed_words + i] : 0u);
}

// The 8 draws of block `blk`: values mod m, and the mask of rejected ones.
__device__ __forceinline__ uint32_t draws8(uint32_t (&val)[8], const uint32_t (&key)[8], uint64_t blk,
                                           const ModParams& mp) {
  uint32_t w[16];
  chacharng_block(w, key, blk);
  uint32_t rej = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t v = ((uint64_t)w[2 * i] << 32) | w[2 * i + 1];  // next_u64: high word first
    rej |= (v >= mp.zone64 ? 1u : 0u) << i;
    val[i] = mod64(v, mp);
  }
  return rej;
}

__global__ void k_chacha_seeds(int P, int seed_words, RngKeyArg rng, uint64_t owner_base,
                               uint32_t* seeds) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  RngKey rk;
#pragma unroll
  for (int i = 0; i < 8; ++i) rk.k[i] = rng.k[i];
  uint32_t w[16];
  rng_block(w, rk, stream_id(kPurposeChaChaSeed, owner_base + p), 0);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < seed_words) seeds[(size_t)p * seed_words + i] = w[i];
}

__device__ __forceinline__ void note_rejection(uint32_t* scratch, int p) {
  scratch[0] = 1u;                 // plain stores of the same value: racing lanes agree
  scratch[kScratchHead + p] = 1u;
}

// ---- participants: masked = secret + mask, draw e for element e ------------------------
__global__ void __launch_bounds__(kBlock)
    k_cc_mask_apply(int D, ModParams mp, int seed_words, const uint32_t* __restrict__ seeds,
                    const int32_t* __restrict__ secrets, int32_t* __restrict__ masked,
                    uint32_t* __restrict__ scratch) {
  const int p = blockIdx.y;
  const int e0 = (blockIdx.x * kBlock + threadIdx.x) * kDrawsPerLane;
  if (e0 >= D) return;
  uint32_t key[8], mk[8];
  load_seed_key(key, seeds, p, seed_words);
  uint32_t rej = draws8(mk, key, (uint64_t)e0 / 8, mp);
  const int valid = min(kDrawsPerLane, D - e0);
  if (valid < 8) rej &= (1u << valid) - 1u;  // draws past D only matter once something shifted
  if (rej) note_rejection(scratch, p);
  const int32_t* src = secrets + (size_t)p * D + e0;
  int32_t* dst = masked + (size_t)p * D + e0;
  if (valid == 8 && (D % 4) == 0) {
    int4 a = reinterpret_cast<const int4*>(src)[0], b = reinterpret_cast<const int4*>(src)[1];
    const int32_t s[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    int32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (int32_t)add_mod(canon_i32(s[i], mp), mk[i], mp.m);
    reinterpret_cast<int4*>(dst)[0] = make_int4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<int4*>(dst)[1] = make_int4(o[4], o[5], o[6], o[7]);
  } else {
    for (int i = 0; i < valid; ++i) dst[i] = (int32_t)add_mod(canon_i32(src[i], mp), mk[i], mp.m);
  }
}

// ---- recipient: part[g][e] = sum over group g's participants of mask_p[e] --------------
// Blocks tile (elements, participant groups): a lane walks its group's participants
// with their keys in SGPRs and keeps 8 running sums; the groups' slabs are added by
// launch_colsum. `Pg` participants per group.
__global__ void __launch_bounds__(kBlock)
    k_cc_mask_sum(int P, int Pg, int D, ModParams mp, int seed_words,
                  const uint32_t* __restrict__ seeds, uint32_t* __restrict__ part,
                  uint32_t* __restrict__ scratch) {
  const int g = blockIdx.y;
  const int e0 = (blockIdx.x * kBlock + threadIdx.x) * kDrawsPerLane;
  if (e0 >= D) return;
  const int valid = min(kDrawsPerLane, D - e0);
  const uint32_t tail_mask = valid < 8 ? (1u << valid) - 1u : 0xffu;
  uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int p1 = min(P, (g + 1) * Pg);
  for (int p = g * Pg; p < p1; ++p) {
    uint32_t key[8], mk[8];
    load_seed_key(key, seeds, p, seed_words);
    const uint32_t rej = draws8(mk, key, (uint64_t)e0 / 8, mp) & tail_mask;
    if (rej) note_rejection(scratch, p);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = add_mod(acc[i], mk[i], mp.m);
  }
  uint32_t* o = part + (size_t)g * D + e0;
  if (valid == 8 && (D % 4) == 0) {
    reinterpret_cast<uint4*>(o)[0] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    reinterpret_cast<uint4*>(o)[1] = make_uint4(acc[4], acc[5], acc[6], acc[7]);
  } else {
    for (int i = 0; i < valid; ++i) o[i] = acc[i];
  }
}

// ---- repair, gated on scratch[0] -----------------------------------------------------------
// (0) the affected participants, compacted in increasing order (one block)
__global__ void __launch_bounds__(kBlock) k_cc_compact(int P, uint32_t* __restrict__ scratch) {
  __shared__ uint32_t red[kWaves];
  if (scratch[0] == 0u) return;
  uint32_t base = 0;
  for (int p0 = 0; p0 < P; p0 += kBlock) {
    const int p = p0 + threadIdx.x;
    const uint32_t hit = p < P && scratch[kScratchHead + p] != 0u ? 1u : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(hit, red, &total);
    if (hit) scratch[kScratchHead + P + base + ex] = (uint32_t)p;
    base += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) scratch[1] = base;
}

// (1) rejections per chunk of the affected participants' streams
__global__ void __launch_bounds__(kBlock)
    k_cc_rej_count(int C, ModParams mp, int seed_words, const uint32_t* __restrict__ seeds,
                   uint32_t* __restrict__ scratch, int P) {
  __shared__ uint32_t red[kWaves];
  if (scratch[0] == 0u) return;
  const int c = blockIdx.x;
  const int A = (int)scratch[1];
  for (int a = blockIdx.y; a < A; a += kRepairRows) {
    const int p = (int)scratch[kScratchHead + P + a];
    uint32_t key[8], mk[8];
    load_seed_key(key, seeds, p, seed_words);
    const uint32_t rej = draws8(mk, key, (uint64_t)c * kBlock + threadIdx.x, mp);
    const uint32_t tot = block_sum((uint32_t)__popc(rej), red);
    if (threadIdx.x == 0) scratch[kScratchHead + 2 * (size_t)P + (size_t)a * C + c] = tot;
    __syncthreads();
  }
}

// (2) per affected participant: counts -> exclusive bases; a stream that does not
// hold D accepted draws within the scanned range is reported
__global__ void __launch_bounds__(kBlock)
    k_cc_rej_scan(int C, int D, uint32_t* __restrict__ scratch, int P, uint32_t* err) {
  __shared__ uint32_t red[kWaves];
  if (scratch[0] == 0u) return;
  const int A = (int)scratch[1];
  for (int a = blockIdx.x; a < A; a += kRepairRows) {
    uint32_t* cnt = scratch + kScratchHead + 2 * (size_t)P + (size_t)a * C;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < C; c0 += kBlock) {
      const int c = c0 + threadIdx.x;
      const uint32_t v = c < C ? cnt[c] : 0u;
      uint32_t total;
      const uint32_t ex = block_excl_scan(v, red, &total);
      if (c < C) cnt[c] = carry + ex;
      carry += total;
      __syncthreads();
    }
    if (threadIdx.x == 0 && (uint64_t)C * kChunkDraws - carry < (uint64_t)D)
      atomicOr(err, kErrChaChaReject);
  }
}

// (3) every accepted draw of an affected stream goes to its true element.
//   kSum = false: masked[p][e] = secret[p][e] + draw           (participants)
//   kSum = true : fix[e] += draw, and fix[d] += m - draw_d for every position d < D,
//                 which takes back what the fast kernel added there   (recipient)
// Draws before a stream's first rejection sit where the fast kernel put them and
// are skipped.
template <bool kSum>
__global__ void __launch_bounds__(kBlock)
    k_cc_fix(int C, int D, ModParams mp, int seed_words, const uint32_t* __restrict__ seeds,
             const uint32_t* __restrict__ scratch, int P, const int32_t* __restrict__ secrets,
             int32_t* __restrict__ masked, unsigned long long* __restrict__ fix) {
  __shared__ uint32_t red[kWaves];
  if (scratch[0] == 0u) return;
  const int c = blockIdx.x;
  const int A = (int)scratch[1];
  for (int a = blockIdx.y; a < A; a += kRepairRows) {
    const int p = (int)scratch[kScratchHead + P + a];
    uint32_t key[8], mk[8];
    load_seed_key(key, seeds, p, seed_words);
    const uint64_t blk = (uint64_t)c * kBlock + threadIdx.x;
    const uint32_t rej = draws8(mk, key, blk, mp);
    uint32_t total;
    uint32_t before = block_excl_scan((uint32_t)__popc(rej), red, &total) +
                      scratch[kScratchHead + 2 * (size_t)P + (size_t)a * C + c];
    const uint64_t d0 = blk * kDrawsPerLane;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t d = d0 + i;
      const bool rejected = (rej >> i) & 1u;
      if (kSum && d < (uint64_t)D && (before != 0u || rejected))
        atomicAdd(&fix[d], (unsigned long long)(mp.m - mk[i]));
      if (rejected) {
        ++before;
        continue;
      }
      if (before == 0u) continue;  // unshifted: already right
      const uint64_t e = d - before;
      if (e >= (uint64_t)D) continue;
      if constexpr (kSum) {
        atomicAdd(&fix[e], (unsigned long long)mk[i]);
      } else {
        masked[(size_t)p * D + e] =
            (int32_t)add_mod(canon_i32(secrets[(size_t)p * D + e], mp), mk[i], mp.m);
      }
    }
    __syncthreads();
  }
}

// (4) recipient: out[e] = (out[e] + fix[e]) mod m
__global__ void __launch_bounds__(kBlock)
    k_cc_finish(int D, ModParams mp, const uint32_t* __restrict__ scratch,
                const unsigned long long* __restrict__ fix, uint32_t* __restrict__ out) {
  if (scratch[0] == 0u) return;
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e < D) out[e] = add_mod(out[e], mod64(fix[e], mp), mp.m);
}

__global__ void k_cc_clear(uint32_t* scratch, int words) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < words) scratch[i] = 0u;
}
__global__ void k_cc_clear64(unsigned long long* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0ull;
}

uint64_t g_zone_cap = ~0ull;

ModParams cc_params(uint32_t m) {
  ModParams mp = make_mod_params(m);
  if (g_zone_cap != ~0ull && m != 0) {
    const uint64_t z = g_zone_cap - g_zone_cap % m;
    if (z < mp.zone64) mp.zone64 = z;
  }
  return mp;
}

int scan_chunks(int D) {  // chunks covering 2 D + 4096 draws
  return (int)((2ull * (uint64_t)D + 4096 + kChunkDraws - 1) / kChunkDraws);
}

}  // namespace

void set_chacha_zone_cap(uint64_t cap) { g_zone_cap = cap; }

size_t chacha_scratch_words(int P, int D) {
  return (size_t)kScratchHead + 2 * (size_t)P + (size_t)P * scan_chunks(D);
}

int chacha_sum_groups(int P, int D) {
  // ~8k blocks when the elements alone do not fill the chip; at least 16
  // participants per group so the slabs stay a small fraction of the work
  const int tiles = (D + kChunkDraws - 1) / kChunkDraws;
  int groups = (8192 + tiles - 1) / tiles;
  groups = groups < 1 ? 1 : groups;
  const int by_p = (P + 15) / 16;
  if (groups > by_p) groups = by_p;
  return groups < 1 ? 1 : groups;
}

void launch_chacha_seeds(int P, int seed_words, RngKeyArg rng, uint64_t owner_base, uint32_t* seeds,
                         hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_chacha_seeds, dim3((P + 63) / 64), dim3(64), 0, s, P, seed_words, rng,
                     owner_base, seeds);
}

void launch_chacha_mask_apply(int P, int D, uint32_t m, int seed_words, const uint32_t* seeds,
                              const int32_t* secrets, int32_t* masked, uint32_t* scratch,
                              uint32_t* err, hipStream_t s) {
  if (P <= 0 || D <= 0) return;
  const ModParams mp = cc_params(m);
  const int C = scan_chunks(D);
  const int head = kScratchHead + P;  // flag, count and the marks
  hipLaunchKernelGGL(k_cc_clear, dim3((head + 255) / 256), dim3(256), 0, s, scratch, head);
  dim3 grid((D + kChunkDraws - 1) / kChunkDraws, P);
  hipLaunchKernelGGL(k_cc_mask_apply, grid, dim3(kBlock), 0, s, D, mp, seed_words, seeds, secrets,
                     masked, scratch);
  // repair (exits at once unless a draw was rejected)
  hipLaunchKernelGGL(k_cc_compact, dim3(1), dim3(kBlock), 0, s, P, scratch);
  hipLaunchKernelGGL(k_cc_rej_count, dim3(C, kRepairRows), dim3(kBlock), 0, s, C, mp, seed_words,
                     seeds, scratch, P);
  hipLaunchKernelGGL(k_cc_rej_scan, dim3(kRepairRows), dim3(kBlock), 0, s, C, D, scratch, P, err);
  hipLaunchKernelGGL(k_cc_fix<false>, dim3(C, kRepairRows), dim3(kBlock), 0, s, C, D, mp, seed_words,
                     seeds, scratch, P, secrets, masked, (unsigned long long*)nullptr);
}

void launch_chacha_mask_sum(int P, int D, uint32_t m, int seed_words, const uint32_t* seeds,
                            uint32_t* out, uint32_t* part, int groups, uint32_t* scratch,
                            uint64_t* fix, uint32_t* err, hipStream_t s) {
  if (D <= 0) return;
  const ModParams mp = cc_params(m);
  if (P <= 0) {
    hipLaunchKernelGGL(k_cc_clear, dim3((D + 255) / 256), dim3(256), 0, s, out, D);
    return;
  }
  const int C = scan_chunks(D);
  const int head = kScratchHead + P;
  const int Pg = (P + groups - 1) / groups;
  const int G = (P + Pg - 1) / Pg;  // groups actually used (<= groups)
  hipLaunchKernelGGL(k_cc_clear, dim3((head + 255) / 256), dim3(256), 0, s, scratch, head);
  dim3 grid((D + kChunkDraws - 1) / kChunkDraws, G);
  hipLaunchKernelGGL(k_cc_mask_sum, grid, dim3(kBlock), 0, s, P, Pg, D, mp, seed_words, seeds, part,
                     scratch);
  launch_colsum(1, G, D, m, 4, part, out, s);
  // repair (exits at once unless a draw was rejected)
  hipLaunchKernelGGL(k_cc_clear64, dim3((D + 255) / 256), dim3(256), 0, s, (unsigned long long*)fix, D);
  hipLaunchKernelGGL(k_cc_compact, dim3(1), dim3(kBlock), 0, s, P, scratch);
  hipLaunchKernelGGL(k_cc_rej_count, dim3(C, kRepairRows), dim3(kBlock), 0, s, C, mp, seed_words,
                     seeds, scratch, P);
  hipLaunchKernelGGL(k_cc_rej_scan, dim3(kRepairRows), dim3(kBlock), 0, s, C, D, scratch, P, err);
  hipLaunchKernelGGL(k_cc_fix<true>, dim3(C, kRepairRows), dim3(kBlock), 0, s, C, D, mp, seed_words,
                     seeds, scratch, P, (const int32_t*)nullptr, (int32_t*)nullptr,
                     (unsigned long long*)fix);
  hipLaunchKernelGGL(k_cc_finish, dim3((D + kBlock - 1) / kBlock), dim3(kBlock), 0, s, D, mp, scratch,
                     (const unsigned long long*)fix, out);
}

}  // namespace sdagpu
