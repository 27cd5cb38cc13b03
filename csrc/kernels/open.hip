// Clerk / recipient kernels after decryption: parallel varint decode, the
// per-clerk modular combine, packed-Shamir (Lagrange) reconstruction, unmask.
//
// Reference: sodium.rs:83-89 (decode until exhausted), sharing/combiner.rs:15-29
// (element-wise sum mod m), sharing/batched.rs:68-99 + tss reconstruct
// (reconstruct per batch, truncate to the dimension), masking/full.rs:54-67.
//
// Parallel decode: every byte with MSB = 0 terminates a varint, so a chunk's
// terminator count gives element ranks by an exclusive scan across chunks
// (launch_segscan over the per-chunk counts from k_mac_chunks<1>); inside a chunk
// the lanes rank their terminators with a block scan and each lane decodes the
// varints ending in its 64 bytes, reading at most 9 bytes back (a 16-byte LDS
// prefix of the previous chunk covers varints straddling the boundary).
#include "block_utils.hpp"
#include "device_crypto.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

// Canonical field value of a decoded zigzag varint (general path handles
// negative / oversized values from foreign encoders such as the reference's
// Rust-`%` shares, which can be negative: additive.rs:47).
SDA_DEV uint32_t canon_varint(uint64_t z, const ModParams& mp, bool& bad) {
  if (!(z & 1)) {
    const uint64_t mag = z >> 1;
    if (mp.m == 0) {
      bad |= mag > 0xffffffffULL;
      return (uint32_t)mag;
    }
    return mag < mp.m ? (uint32_t)mag : mod64(mag, mp);
  }
  if (mp.m == 0) {
    bad = true;
    return 0;
  }
  const uint32_t r = mod64((z >> 1) + 1, mp);  // value = -(z>>1) - 1
  return r == 0 ? 0u : mp.m - r;
}

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

// Two candidate values from a word holding two (previous byte, byte) pairs in
// its 16-bit halves: z = prev-is-continuation ? byte<<7 | prev&0x7f : byte,
// then zigzag-decode and reduce a value in (-m, m) into [0, m). Halves whose
// byte is not a terminator produce garbage the caller discards.
SDA_DEV uint32_t pair_values(uint32_t P, u16x2 mpair) {
  const uint32_t z2 = ((P >> 1) & 0x7f807f80u) | (P & 0x007f007fu);
  const uint32_t z1 = (P >> 8) & 0x00ff00ffu;
  const uint32_t sel = ((P >> 7) & 0x00010001u) * 0xffffu;
  const uint32_t z = (sel & z2) | (~sel & z1);
  const uint32_t neg = z & 0x00010001u;
  const uint32_t u = ((z >> 1) & 0x7fff7fffu) + neg;  // |value|, no carry across halves
  const uint32_t nsel = neg * 0xffffu;
  const uint32_t mu = __builtin_bit_cast(uint32_t, mpair - __builtin_bit_cast(u16x2, u));
  return (nsel & mu) | (~nsel & u);
}

// One block per (chunk, message). Each lane owns 64 plaintext bytes held in
// registers; terminator positions are a 64-bit mask (popcount -> block scan ->
// ranks); the bytes preceding a lane come from its neighbour by a shuffle (lane
// 0 of a wave loads them); decoded values are staged in LDS so the global store
// of the chunk's contiguous element range is coalesced. Varints of 3+ bytes
// (large moduli, ChaCha seeds) walk back through global memory.
template <typename VT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_decode(int L, ModParams mp, const uint8_t* __restrict__ pt, uint64_t stride,
             const uint32_t* __restrict__ pt_len, const uint32_t* __restrict__ elem_start,
             VT* __restrict__ vals, uint32_t* err) {
  __shared__ VT outb[kChunkBytes + 128];  // + a dummy dword per wave lane
  __shared__ uint32_t scratch[kWaves];
  const int k = blockIdx.x, j = blockIdx.y, K = gridDim.x;
  const int tid = threadIdx.x;
  const uint32_t N = pt_len[j];
  const int64_t kC = (int64_t)k * kChunkBytes;
  const int64_t start = kC >= 32 ? kC - 32 : 0;
  const int64_t end = min((int64_t)N, kC + kChunkBytes - 32);
  if (start >= end) return;
  const uint8_t* gmsg = pt + (size_t)j * stride + 48;
  const int64_t p0 = kC - 32 + 64 * tid;  // message position of this lane's first byte
  uint32_t w[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t pos = p0 + 16 * q;
    uint4 d = make_uint4(0, 0, 0, 0);
    if (pos >= 0 && pos < end) d = *reinterpret_cast<const uint4*>(gmsg + pos);
    w[4 * q] = d.x; w[4 * q + 1] = d.y; w[4 * q + 2] = d.z; w[4 * q + 3] = d.w;
  }
  // the 4 bytes before this lane's range, for lane 0 of each wave (the other
  // lanes take them from their neighbour below)
  uint32_t wave_prev = 0;
  if ((tid & 63) == 0 && p0 - 4 >= 0 && p0 - 4 < end) wave_prev = *reinterpret_cast<const uint32_t*>(gmsg + p0 - 4);
  // valid bytes [lo, hi) of this lane
  const int lo = (int)max((int64_t)0, start - p0);
  const int hi = (int)min((int64_t)64, end - p0);
  uint64_t vmask = 0;
  if (hi > lo) {
    const uint64_t upto = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
    vmask = upto & ~((1ull << lo) - 1);
  }
  uint64_t tmask = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t t = ~w[i] & 0x80808080u;
    const uint64_t bits = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
    tmask |= bits << (4 * i);
  }
  const uint64_t traw = tmask;
  tmask &= vmask;
  uint32_t total;
  uint32_t local = block_excl_scan((uint32_t)__popcll(tmask), scratch, &total);  // syncs
  bool bad = false;
  // The two bytes preceding this lane's range (previous lane's last word; lane 0
  // of each wave reads them from the LDS image, which holds the chunk prefix).
  uint32_t prev_word = __shfl_up(w[15], 1, 64);
  if ((tid & 63) == 0) prev_word = wave_prev;
  // Fast path (u16 values, modulus < 2^16, no varint longer than two bytes,
  // canonical range): SWAR over 16-bit halves -- one 32-bit op yields the
  // candidate values of two byte positions. Odd positions pair with the byte
  // before them inside the same half of the word; even positions use the word
  // realigned by one byte (v_alignbyte). Every position then stores its
  // candidate, non-terminators into a per-lane dummy slot. A lane that meets a
  // longer varint or an out-of-range value re-runs the generic path below.
  const uint32_t local0 = local;
  const uint32_t dummy = kChunkBytes + 2 * (tid & 63);  // own dword per lane of a wave
  const uint32_t tmask_lo = (uint32_t)tmask, tmask_hi = (uint32_t)(tmask >> 32);
  bool redo = true;
  if constexpr (sizeof(VT) == 2) {
    if (mp.m != 0 && mp.m < 65536u) {
      const uint64_t craw = ~traw;  // continuation bytes
      const uint32_t cm1 = prev_word >> 31, cm2 = (prev_word >> 23) & 1u;
      const bool longv = (craw & (craw << 1)) != 0 || (cm1 & ((uint32_t)craw & 1u)) || (cm1 & cm2);
      const u16x2 mpair = {(uint16_t)mp.m, (uint16_t)mp.m};
      u16x2 vmax = {0, 0};
      uint32_t wp = prev_word;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t W = w[i];
        const uint32_t Pe = __builtin_amdgcn_alignbyte(W, wp, 3);  // [wp.B3 W.B0 | W.B1 W.B2]
        const uint32_t ve = pair_values(Pe, mpair), vo = pair_values(W, mpair);
        const uint32_t t4 = ((i < 8 ? tmask_lo : tmask_hi) >> (4 * (i & 7))) & 15u;
        const uint32_t te = ((t4 & 1u) * 0xffffu) | (((t4 >> 2) & 1u) * 0xffff0000u);
        const uint32_t to = (((t4 >> 1) & 1u) * 0xffffu) | (((t4 >> 3) & 1u) * 0xffff0000u);
        vmax = __builtin_elementwise_max(vmax, __builtin_bit_cast(u16x2, ve & te));
        vmax = __builtin_elementwise_max(vmax, __builtin_bit_cast(u16x2, vo & to));
        uint32_t t;
        t = t4 & 1u;        outb[t ? local : dummy] = (VT)ve;         local += t;
        t = (t4 >> 1) & 1u; outb[t ? local : dummy] = (VT)vo;         local += t;
        t = (t4 >> 2) & 1u; outb[t ? local : dummy] = (VT)(ve >> 16); local += t;
        t = (t4 >> 3) & 1u; outb[t ? local : dummy] = (VT)(vo >> 16); local += t;
        wp = W;
      }
      redo = longv || vmax.x >= mp.m || vmax.y >= mp.m;
    }
  }
  if (redo) {
    // Generic path, all in registers (the LDS image is only touched by the
    // rare long-varint walk: lanes 64 B apart would all hit the same two LDS
    // banks). A terminator at b closes a 1-, 2- or 3-byte varint depending on
    // the continuation bits of bytes b-1, b-2; four bytes and more
    // (|value| >= 2^20) take the LDS walk.
    // opaque copies: stop the compiler from sharing (and keeping live across
    // the fast path) the per-byte terms it would otherwise CSE between paths
    uint32_t tlo = tmask_lo, thi = tmask_hi;
    local = local0;
    asm volatile("" : "+v"(tlo), "+v"(thi), "+v"(local));
    uint32_t long_mask_lo = 0, long_mask_hi = 0;  // terminators needing the slow path
    uint32_t b3 = (prev_word >> 8) & 0xffu, b2 = (prev_word >> 16) & 0xffu, b1 = prev_word >> 24;
    // Branch-free: every byte stores a value, non-terminators into a per-lane
    // dummy slot, so the unrolled loop compiles to straight-line VALU + ds_write.
    // Conditions are kept as integer 0/1 / all-ones masks (bools become SGPR
    // lane masks that the compiler then spills across the unrolled loop).
    uint32_t neg_raw = 0;
  #pragma unroll
    for (int b = 0; b < 64; ++b) {
      const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
      const uint32_t term = ((b < 32 ? tlo : thi) >> (b & 31)) & 1u;
      const uint32_t c1 = b1 >> 7, c2 = b2 >> 7, c3 = b3 >> 7;
      const uint32_t m1 = 0u - c1, m2 = 0u - c2;
      const uint32_t z2 = (b1 & 0x7f) | (byte << 7);
      const uint32_t z3 = (b2 & 0x7f) | ((b1 & 0x7f) << 7) | (byte << 14);
      const uint32_t z = (byte & ~m1) | (z2 & m1 & ~m2) | (z3 & m1 & m2);  // < 2^21
      const uint32_t lng = term & c1 & c2 & c3;
      if (b < 32) long_mask_lo |= lng << b; else long_mask_hi |= lng << (b - 32);
      const uint32_t neg = z & 1u;
      const uint32_t u = (z >> 1) + neg;  // |value| (value = -u when neg)
      const uint32_t r = mod32(u, mp);    // m == 0: raw
      const uint32_t nr = r == 0 ? 0u : mp.m - r;
      const uint32_t v = r ^ ((r ^ nr) & (0u - neg));
      neg_raw |= term & neg & (lng ^ 1u);
      const uint32_t addr = dummy ^ ((dummy ^ local) & (0u - term));
      outb[addr] = (VT)v;
      local += term;
      b3 = b2;
      b2 = b1;
      b1 = byte;
    }
    if (mp.m == 0) bad |= neg_raw != 0;  // a raw (modulus-free) stream holds no negatives
    // rare slow path: rewrite the values of >= 3-byte varints
    uint64_t lm = ((uint64_t)long_mask_hi << 32) | long_mask_lo;
    if (lm) {
      uint32_t rank0 = local - (uint32_t)__popcll(tmask);
      while (lm) {
        const int b = __builtin_ctzll(lm);
        lm &= lm - 1;
        const uint32_t r = rank0 + (uint32_t)__popcll(tmask & ((1ull << b) - 1));
        const int64_t q = p0 + b;
        int64_t s0 = q;
        int n = 0;
        while (n < 10 && s0 > 0 && (gmsg[s0 - 1] & 0x80)) { --s0; ++n; }
        bad |= n >= 10;
        uint64_t z = 0;
        for (int64_t u = s0; u <= q; ++u) {
          const uint32_t sh = 7u * (uint32_t)(u - s0);
          if (sh < 64) z |= (uint64_t)(gmsg[u] & 0x7f) << sh;
        }
        outb[r] = (VT)canon_varint(z, mp, bad);
      }
    }
  }
  // a message must end on a terminator
  if (hi > lo && p0 + hi == (int64_t)N && (gmsg[N - 1] & 0x80)) bad = true;
  __syncthreads();
  const uint32_t base = elem_start[(size_t)j * K + k];
  VT* out = vals + (size_t)j * L;
  for (uint32_t i = tid; i < total; i += kBlock) {
    if (base + i < (uint32_t)L) out[base + i] = outb[i];
    else bad = true;
  }
  if (bad) atomicOr(err, kErrMalformed);
}

template <typename VT, typename ACC>
__global__ void __launch_bounds__(kBlock)
    k_colsum(int R, int L, ModParams mp, const VT* __restrict__ vals, uint32_t* __restrict__ out) {
  const int g = blockIdx.y;
  const int l0 = (blockIdx.x * kBlock + threadIdx.x) * 8;
  if (l0 >= L) return;
  const VT* src = vals + (size_t)g * R * L;
  ACC acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool vec = (L % 8) == 0;
  if (vec) {
    for (int r = 0; r < R; ++r) {
      const VT* row = src + (size_t)r * L + l0;
      if constexpr (sizeof(VT) == 2) {
        uint4 q = *reinterpret_cast<const uint4*>(row);
        acc[0] += q.x & 0xffff; acc[1] += q.x >> 16; acc[2] += q.y & 0xffff; acc[3] += q.y >> 16;
        acc[4] += q.z & 0xffff; acc[5] += q.z >> 16; acc[6] += q.w & 0xffff; acc[7] += q.w >> 16;
      } else {
        uint4 a = reinterpret_cast<const uint4*>(row)[0];
        uint4 b = reinterpret_cast<const uint4*>(row)[1];
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
    }
  } else {
    for (int r = 0; r < R; ++r) {
      const VT* row = src + (size_t)r * L;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (l0 + i < L) acc[i] += row[l0 + i];
    }
  }
  uint32_t* o = out + (size_t)g * L;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (l0 + i < L) o[l0 + i] = mod64((uint64_t)acc[i], mp);
}

__global__ void __launch_bounds__(kBlock)
    k_pss_reconstruct(int B, int k, int nI, int D, ModParams mp, const uint32_t* __restrict__ lag,
                      const uint32_t* __restrict__ ys, uint32_t* __restrict__ out) {
  extern __shared__ uint32_t sL[];
  for (int i = threadIdx.x; i < k * nI; i += kBlock) sL[i] = lag[i];
  __syncthreads();
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  for (int s = 0; s < k; ++s) {
    const int e = b * k + s;
    if (e >= D) break;
    uint32_t acc = 0;
    for (int i = 0; i < nI; ++i)
      acc = add_mod(acc, mod64((uint64_t)sL[s * nI + i] * ys[(size_t)i * B + b], mp), mp.m);
    out[e] = acc;
  }
}

__global__ void k_sub_mod(int D, uint32_t m, const uint32_t* __restrict__ a,
                          const uint32_t* __restrict__ b, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D) out[i] = sub_mod(a[i], b[i], m);
}

}  // namespace

void launch_decode(int M, int K, int L, uint32_t m, int value_bytes, const uint8_t* pt,
                   uint64_t stride, const uint32_t* pt_len, const uint32_t* elem_start,
                   void* vals, uint32_t* err, hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  ModParams mp = make_mod_params(m);
  dim3 grid(K, M);
  if (value_bytes == 2)
    hipLaunchKernelGGL(k_decode<uint16_t>, grid, dim3(kBlock), 0, s, L, mp, pt, stride, pt_len,
                       elem_start, (uint16_t*)vals, err);
  else
    hipLaunchKernelGGL(k_decode<uint32_t>, grid, dim3(kBlock), 0, s, L, mp, pt, stride, pt_len,
                       elem_start, (uint32_t*)vals, err);
}

void launch_colsum(int G, int R, int L, uint32_t m, int value_bytes, const void* vals,
                   uint32_t* out, hipStream_t s) {
  if (G <= 0 || L <= 0) return;
  ModParams mp = make_mod_params(m);
  const int threads = (L + 7) / 8;
  dim3 grid((threads + kBlock - 1) / kBlock, G);
  if (value_bytes == 2 && (uint64_t)R * 65535ull < 0xffffffffull)
    hipLaunchKernelGGL((k_colsum<uint16_t, uint32_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint16_t*)vals, out);
  else if (value_bytes == 2)
    hipLaunchKernelGGL((k_colsum<uint16_t, uint64_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint16_t*)vals, out);
  else
    hipLaunchKernelGGL((k_colsum<uint32_t, uint64_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint32_t*)vals, out);
}

void launch_pss_reconstruct(int B, int k, int nI, int D, uint32_t p, const uint32_t* lag,
                            const uint32_t* ys, uint32_t* out, hipStream_t s) {
  if (B <= 0) return;
  ModParams mp = make_mod_params(p);
  hipLaunchKernelGGL(k_pss_reconstruct, dim3((B + kBlock - 1) / kBlock), dim3(kBlock),
                     (size_t)k * nI * sizeof(uint32_t), s, B, k, nI, D, mp, lag, ys, out);
}

void launch_sub_mod(int D, uint32_t m, const uint32_t* a, const uint32_t* b, uint32_t* out,
                    hipStream_t s) {
  if (D <= 0) return;
  hipLaunchKernelGGL(k_sub_mod, dim3((D + 255) / 256), dim3(256), 0, s, D, m, a, b, out);
}

}  // namespace sdagpu
