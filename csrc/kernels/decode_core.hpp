// Lane-level zigzag-varint decoding shared by the clerk / recipient kernels.
//
// Every byte with MSB = 0 terminates a varint (reference sodium.rs:83-89 decodes
// until the stream is exhausted), so a lane holding 64 plaintext bytes in
// registers can decode every varint that *ends* in them once it knows the rank
// of its first terminator (a block scan of terminator popcounts) and the bytes
// just before its range. The values go to a `Sink`:
//
//   put(local, v, term)   every byte position; `term` = 1 where a value ends
//                         (the sink routes term = 0 to a dummy slot, so the
//                         unrolled loop stays branch-free)
//   put_rank(rank, v)     a varint whose code does not fit 32 bits (six bytes and more,
//                         or a fifth byte above 15) recovered by the slow walk
//   kAdditive             the sink accumulates (an aborted fast pass is undone
//                         by re-adding its values negated); additive sinks also
//   put_masked(local, v)  take every position's value pre-masked (0 where no
//                         value ends) -- the canonical fast pass
#pragma once

#include "device_crypto.hpp"
#include "modarith.hpp"

namespace sdagpu {

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

// 64-bit mask of the terminator bytes (MSB clear) among 16 little-endian words.
SDA_DEV uint64_t term_mask64(const uint32_t (&w)[16]) {
  uint64_t tmask = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t t = ~w[i] & 0x80808080u;
    const uint64_t bits = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
    tmask |= bits << (4 * i);
  }
  return tmask;
}

// A lane's 64 message bytes [p0, p0 + 64) as 16-byte loads; pieces starting
// outside [0, end) read as zero (terminators, masked out by the caller's range).
SDA_DEV void load_lane_bytes(uint32_t (&w)[16], const uint8_t* __restrict__ gmsg, int64_t p0,
                             int64_t end) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t pos = p0 + 16 * q;
    uint4 d = make_uint4(0, 0, 0, 0);
    if (pos >= 0 && pos < end) d = *reinterpret_cast<const uint4*>(gmsg + pos);
    w[4 * q] = d.x; w[4 * q + 1] = d.y; w[4 * q + 2] = d.z; w[4 * q + 3] = d.w;
  }
}

SDA_DEV uint64_t byte_range_mask(int lo, int hi) {
  if (hi <= lo) return 0;
  const uint64_t upto = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
  return upto & ~((1ull << lo) - 1);
}

// SWAR fast pass (canonical u16 values, no varint longer than two bytes): one
// 32-bit op yields the candidate values of two byte positions. Odd positions
// pair with the byte before them inside the same half of the word; even
// positions use the word realigned by one byte (v_alignbyte). `negate` = ~0
// re-emits every value negated (undoes an additive pass). Returns the largest
// terminated candidate per half (>= m means the pass is invalid).
template <typename Sink>
SDA_DEV u16x2 decode_fast16(const uint32_t (&w)[16], uint32_t prev_word, uint64_t tmask,
                            uint32_t local, uint32_t m, Sink& sink, uint32_t negate) {
  const u16x2 mpair = {(uint16_t)m, (uint16_t)m};
  u16x2 vmax = {0, 0};
  const uint32_t tmask_lo = (uint32_t)tmask, tmask_hi = (uint32_t)(tmask >> 32);
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
    t = t4 & 1u;        sink.put(local, ((ve & 0xffffu) ^ negate) - negate, t); local += t;
    t = (t4 >> 1) & 1u; sink.put(local, ((vo & 0xffffu) ^ negate) - negate, t); local += t;
    t = (t4 >> 2) & 1u; sink.put(local, ((ve >> 16) ^ negate) - negate, t);     local += t;
    t = (t4 >> 3) & 1u; sink.put(local, ((vo >> 16) ^ negate) - negate, t);     local += t;
    wp = W;
  }
  return vmax;
}

// Zigzag codes of two (previous byte, byte) pairs held in the 16-bit halves of
// P: prev-is-continuation ? byte<<7 | prev&0x7f : byte (each < 2^15).
SDA_DEV uint32_t pair_z(uint32_t P) {
  const uint32_t z2 = ((P >> 1) & 0x7f807f80u) | (P & 0x007f007fu);
  const uint32_t z1 = (P >> 8) & 0x00ff00ffu;
  const uint32_t sel = ((P >> 7) & 0x00010001u) * 0xffffu;
  return (sel & z2) | (~sel & z1);
}

// Canonical fast pass for additive sinks: every terminated varint must be one
// or two bytes long (checked by the caller) and encode an even zigzag code
// below 2m (a canonical value < m). Per 4-byte word: two SWAR pair codes, the
// terminated halves kept by a mask, then each position adds its (masked) value
// at its rank -- non-terminators add 0 to the next rank's slot. `negate` = ~0
// re-adds every value negated (undo). Returns false if a terminated code is
// odd (a negative value) or >= 2m.
template <typename Sink>
SDA_DEV bool decode_canon(const uint32_t (&w)[16], uint32_t prev_word, uint64_t tmask,
                          uint32_t local, uint32_t m, Sink& sink, uint32_t negate) {
  uint32_t odd = 0;
  u16x2 zmax = {0, 0};
  const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
  uint32_t wp = prev_word;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t W = w[i];
    const uint32_t t4 = ((i < 8 ? tlo : thi) >> (4 * (i & 7))) & 15u;
    // halves of the even-position pairs (bytes 0, 2) and odd ones (1, 3)
    const uint32_t te = ((t4 & 1u) | ((t4 & 4u) << 14)) * 0xffffu;
    const uint32_t to = (((t4 >> 1) & 1u) | ((t4 & 8u) << 13)) * 0xffffu;
    const uint32_t ze = pair_z(__builtin_amdgcn_alignbyte(W, wp, 3)) & te;
    const uint32_t zo = pair_z(W) & to;
    odd |= ze | zo;
    zmax = __builtin_elementwise_max(zmax, __builtin_bit_cast(u16x2, ze));
    zmax = __builtin_elementwise_max(zmax, __builtin_bit_cast(u16x2, zo));
    sink.put_masked(local, (((ze >> 1) & 0x7fffu) ^ negate) - negate);
    local += t4 & 1u;
    sink.put_masked(local, (((zo >> 1) & 0x7fffu) ^ negate) - negate);
    local += (t4 >> 1) & 1u;
    sink.put_masked(local, ((ze >> 17) ^ negate) - negate);
    local += (t4 >> 2) & 1u;
    sink.put_masked(local, ((zo >> 17) ^ negate) - negate);
    local += t4 >> 3;
    wp = W;
  }
  const uint32_t m2 = 2u * m;
  return (odd & 0x00010001u) == 0 && zmax.x < m2 && zmax.y < m2;
}

// Decodes the varints terminated in one lane's 64 bytes.
//   w                       the lane's bytes (message order)
//   prev_word2, prev_word   the 8 bytes before them (bytes -8..-5 and -4..-1)
//   tmask, traw             valid terminators / raw terminator bits of all 64 bytes
//   local                   block-local rank of the lane's first valid terminator
//   gmsg, p0                the message in global memory and the lane's first position
//                           (codes beyond 32 bits walk back through it)
// Returns true if the stream is malformed.
template <bool kFast16, typename Sink>
SDA_DEV bool decode_lane(const uint32_t (&w)[16], uint32_t prev_word2, uint32_t prev_word, uint64_t tmask,
                         uint64_t traw, uint32_t local, const ModParams& mp,
                         const uint8_t* __restrict__ gmsg, int64_t p0, Sink& sink) {
  bool bad = false;
  const uint32_t local0 = local;
  bool redo = true;
  if constexpr (kFast16 && Sink::kAdditive) {
    // canonical values of at most two varint bytes (m <= 8192): decode_canon
    if (mp.m != 0 && mp.m <= 8192u) {
      const uint64_t craw = ~traw;  // continuation bytes
      const uint32_t cm1 = prev_word >> 31, cm2 = (prev_word >> 23) & 1u;
      const bool longv = (craw & (craw << 1)) != 0 || (cm1 & ((uint32_t)craw & 1u)) || (cm1 & cm2);
      if (!longv) {
        redo = !decode_canon(w, prev_word, tmask, local, mp.m, sink, 0u);
        // take the pass back out (opaque copies: see below); the wave-uniform
        // test keeps this rare branch out of line
        if (__builtin_amdgcn_ballot_w64(redo) != 0 && redo) {
          uint32_t w2[16], pw = prev_word, lc = local;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            w2[i] = w[i];
            asm volatile("" : "+v"(w2[i]));
          }
          asm volatile("" : "+v"(pw), "+v"(lc));
          (void)decode_canon(w2, pw, tmask, lc, mp.m, sink, ~0u);
        }
      }
    }
  } else if constexpr (kFast16) {
    if (mp.m != 0 && mp.m < 65536u) {
      const uint64_t craw = ~traw;  // continuation bytes
      const uint32_t cm1 = prev_word >> 31, cm2 = (prev_word >> 23) & 1u;
      const bool longv = (craw & (craw << 1)) != 0 || (cm1 & ((uint32_t)craw & 1u)) || (cm1 & cm2);
      const u16x2 vmax = decode_fast16(w, prev_word, tmask, local, mp.m, sink, 0u);
      redo = longv || vmax.x >= mp.m || vmax.y >= mp.m;
      // an additive sink already holds the invalid pass: take it back out
      // (recomputed from opaque copies: sharing the first pass's values with
      // this rarely taken branch would keep all of them live)
      if constexpr (Sink::kAdditive) {
        if (redo) {
          uint32_t w2[16], pw = prev_word, lc = local;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            w2[i] = w[i];
            asm volatile("" : "+v"(w2[i]));
          }
          asm volatile("" : "+v"(pw), "+v"(lc));
          (void)decode_fast16(w2, pw, tmask, lc, mp.m, sink, ~0u);
        }
      }
    }
  }
  if (redo) {
    // Generic path, all in registers: one pass over the bytes carrying the code of the
    // continuation run so far (`run`, its length as a shift `sh`). A terminator closes
    // the code run | byte << sh; codes of up to five bytes that fit 32 bits (every
    // canonical value of a modulus up to 2^31) end here, anything longer or larger is
    // flagged (`ovf`) and left to the walk below. The state before the lane's first byte
    // comes from the eight bytes before it; eight continuation bytes there mean a run
    // that began out of sight: flagged too.
    // opaque copies: stop the compiler from sharing (and keeping live across
    // the fast path) the per-byte terms it would otherwise CSE between paths
    uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
    local = local0;
    asm volatile("" : "+v"(tlo), "+v"(thi), "+v"(local));
    uint32_t long_mask_lo = 0, long_mask_hi = 0;  // terminators needing the slow path
    // Conditions are kept as integer 0/1 / all-ones masks (bools become SGPR
    // lane masks that the compiler then spills across the unrolled loop).
    uint32_t run = 0, sh = 0, ovf = 0;
    uint32_t z = 0;
    auto step = [&](uint32_t byte) {  // z = the code ending at `byte`; then the state after it
      const uint32_t cm = (uint32_t)((int32_t)(byte << 24) >> 31);  // all ones: continuation byte
      const uint64_t s64 = (uint64_t)(byte & 0x7fu) << sh;           // sh <= 35
      z = run | (uint32_t)s64;
      ovf |= (uint32_t)(s64 >> 32);
      const uint32_t flagged = ovf;
      uint32_t nsh = (sh + 7u) & cm;
      nsh = nsh < 35u ? nsh : 35u;
      run = z & cm;
      ovf = (ovf & cm) | (nsh >> 5);  // five continuation bytes in a row: six bytes or more
      sh = nsh;
      return flagged;
    };
    {
      uint32_t allc = 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t byte = ((i < 4 ? prev_word2 : prev_word) >> (8 * (i & 3))) & 0xffu;
        (void)step(byte);
        allc &= byte >> 7;
      }
      ovf |= allc;
    }
    uint32_t neg_raw = 0;
#pragma unroll
    for (int b = 0; b < 64; ++b) {
      const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
      const uint32_t term = ((b < 32 ? tlo : thi) >> (b & 31)) & 1u;
      const uint32_t lng = term & (step(byte) != 0u ? 1u : 0u);
      if (b < 32) long_mask_lo |= lng << b; else long_mask_hi |= lng << (b - 32);
      const uint32_t neg = z & 1u;
      const uint32_t u = (z >> 1) + neg;  // |value| (value = -u when neg), at most 2^31
      const uint32_t r = mod32(u, mp);    // m == 0: raw
      const uint32_t nr = r == 0 ? 0u : mp.m - r;
      const uint32_t v = r ^ ((r ^ nr) & (0u - neg));
      neg_raw |= term & neg & (lng ^ 1u);
      sink.put(local, v, term & (lng ^ 1u));  // flagged codes: written by the walk
      local += term;
    }
    if (mp.m == 0) bad |= neg_raw != 0;  // a raw (modulus-free) stream holds no negatives
    // rare slow path: codes that do not fit 32 bits
    uint64_t lm = ((uint64_t)long_mask_hi << 32) | long_mask_lo;
    while (lm) {
      const int b = __builtin_ctzll(lm);
      lm &= lm - 1;
      const uint32_t r = local0 + (uint32_t)__builtin_popcountll(tmask & ((1ull << b) - 1));
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
      sink.put_rank(r, canon_varint(z, mp, bad));
    }
  }
  return bad;
}

}  // namespace sdagpu
