// Device-side (gfx950) cryptographic building blocks.
//
// Everything here runs on 32-bit VALU lanes of a 64-wide wavefront:
//  * Salsa20 / HSalsa20 / ChaCha20 cores (ARX; rotates lower to v_alignbit_b32)
//  * BLAKE2b single-block compression (sealed-box nonce, libsodium
//    crypto_box_seal_nonce)
//  * Poly1305 in 5 x 26-bit limbs (32x32->64 products -> v_mad_u64_u32)
//  * GF(2^255-19) in 8 x 32-bit limbs for the X25519 Montgomery ladder
//
// Bit-exactness against the host oracle (csrc/src/crypto_*.cc) is covered by
// tests/test_gpu_kernels.py.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#define SDA_DEV __host__ __device__ __forceinline__

namespace sdagpu {

// two u16 lanes of a 32-bit register (v_pk_*_u16)
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

SDA_DEV uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
SDA_DEV uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u,
                   kSigma3 = 0x6b206574u;

// ---------------------------------------------------------------- Salsa20 ---
template <int kDoubleRounds = 10>
SDA_DEV void salsa20_rounds(uint32_t (&x)[16]) {
#pragma unroll
  for (int i = 0; i < kDoubleRounds; ++i) {
    x[4] ^= rotl32(x[0] + x[12], 7);   x[8] ^= rotl32(x[4] + x[0], 9);
    x[12] ^= rotl32(x[8] + x[4], 13);  x[0] ^= rotl32(x[12] + x[8], 18);
    x[9] ^= rotl32(x[5] + x[1], 7);    x[13] ^= rotl32(x[9] + x[5], 9);
    x[1] ^= rotl32(x[13] + x[9], 13);  x[5] ^= rotl32(x[1] + x[13], 18);
    x[14] ^= rotl32(x[10] + x[6], 7);  x[2] ^= rotl32(x[14] + x[10], 9);
    x[6] ^= rotl32(x[2] + x[14], 13);  x[10] ^= rotl32(x[6] + x[2], 18);
    x[3] ^= rotl32(x[15] + x[11], 7);  x[7] ^= rotl32(x[3] + x[15], 9);
    x[11] ^= rotl32(x[7] + x[3], 13);  x[15] ^= rotl32(x[11] + x[7], 18);
    x[1] ^= rotl32(x[0] + x[3], 7);    x[2] ^= rotl32(x[1] + x[0], 9);
    x[3] ^= rotl32(x[2] + x[1], 13);   x[0] ^= rotl32(x[3] + x[2], 18);
    x[6] ^= rotl32(x[5] + x[4], 7);    x[7] ^= rotl32(x[6] + x[5], 9);
    x[4] ^= rotl32(x[7] + x[6], 13);   x[5] ^= rotl32(x[4] + x[7], 18);
    x[11] ^= rotl32(x[10] + x[9], 7);  x[8] ^= rotl32(x[11] + x[10], 9);
    x[9] ^= rotl32(x[8] + x[11], 13);  x[10] ^= rotl32(x[9] + x[8], 18);
    x[12] ^= rotl32(x[15] + x[14], 7); x[13] ^= rotl32(x[12] + x[15], 9);
    x[14] ^= rotl32(x[13] + x[12], 13); x[15] ^= rotl32(x[14] + x[13], 18);
  }
}

// 64-byte Salsa20/20 block as 16 little-endian words.
SDA_DEV void salsa20_block(uint32_t (&out)[16], const uint32_t (&k)[8], uint32_t n0, uint32_t n1,
                           uint64_t ctr) {
  uint32_t j[16] = {kSigma0, k[0], k[1], k[2], k[3], kSigma1, n0, n1,
                    (uint32_t)ctr, (uint32_t)(ctr >> 32), kSigma2, k[4], k[5], k[6], k[7], kSigma3};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = j[i];
  salsa20_rounds(x);
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + j[i];
}

// The part of a block's first double round that does not depend on the block counter
// (its high word is zero: a message is far below 2^38 bytes): 60 of the 96 steps'
// operations. Every lane of a wave works on one message, so these values are
// wave-uniform: on the device the rotations are written for the scalar unit (which
// has no rotate: two shifts and an or), so that the whole prefix runs there, beside
// the vector work, instead of once per wave on the vector unit.
template <int N>
SDA_DEV uint32_t rotl32_uniform(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t hi, lo;
  asm("s_lshl_b32 %0, %2, %3\n\ts_lshr_b32 %1, %2, %4"
      : "=&s"(hi), "=&s"(lo)
      : "s"(x), "n"(N), "n"(32 - N)
      : "scc");
  return hi | lo;
#else
  return rotl32(x, N);
#endif
}
struct SalsaPrefix {
  uint32_t x1, x2, x3, x9, x10, x13, x14, x15;  // after the column round
  uint32_t x4c;                                 // x4 after the column round
  uint32_t t8a;                                 // rotl(x4c + x0, 9): x8 after the column round = counter ^ t8a
  uint32_t x4, x5, x6, x7;                      // after the row round (row 1 never sees the counter)
  uint32_t x11;                                 // after its row step
  uint32_t t8, t12;                             // what the row round xors into x8 and x12
};
SDA_DEV SalsaPrefix salsa20_prefix(const uint32_t (&k)[8], uint32_t n0, uint32_t n1) {
  uint32_t x1 = k[0], x2 = k[1], x3 = k[2], x4 = k[3], x5 = kSigma1, x6 = n0, x7 = n1, x9 = 0,
           x10 = kSigma2, x11 = k[4], x13 = k[6], x14 = k[7], x15 = kSigma3;
  SalsaPrefix p;
  x4 ^= rotl32_uniform<7>(kSigma0 + k[5]);
  p.x4c = x4;
  p.t8a = rotl32_uniform<9>(x4 + kSigma0);
  x9 ^= rotl32_uniform<7>(x5 + x1);    x13 ^= rotl32_uniform<9>(x9 + x5);
  x1 ^= rotl32_uniform<13>(x13 + x9);  x5 ^= rotl32_uniform<18>(x1 + x13);
  x14 ^= rotl32_uniform<7>(x10 + x6);  x2 ^= rotl32_uniform<9>(x14 + x10);
  x6 ^= rotl32_uniform<13>(x2 + x14);  x10 ^= rotl32_uniform<18>(x6 + x2);
  x3 ^= rotl32_uniform<7>(x15 + x11);  x7 ^= rotl32_uniform<9>(x3 + x15);
  x11 ^= rotl32_uniform<13>(x7 + x3);  x15 ^= rotl32_uniform<18>(x11 + x7);
  p.x1 = x1; p.x2 = x2; p.x3 = x3; p.x9 = x9; p.x10 = x10; p.x13 = x13; p.x14 = x14; p.x15 = x15;
  x6 ^= rotl32_uniform<7>(x5 + x4);    x7 ^= rotl32_uniform<9>(x6 + x5);
  x4 ^= rotl32_uniform<13>(x7 + x6);   x5 ^= rotl32_uniform<18>(x4 + x7);
  p.x4 = x4; p.x5 = x5; p.x6 = x6; p.x7 = x7;
  x11 ^= rotl32_uniform<7>(x10 + x9);
  p.x11 = x11;
  p.t8 = rotl32_uniform<9>(x11 + x10);
  p.t12 = rotl32_uniform<7>(x15 + x14);
  return p;
}
// salsa20_block for a counter below 2^32, given the message's prefix.
SDA_DEV void salsa20_block(uint32_t (&out)[16], const SalsaPrefix& p, const uint32_t (&k)[8],
                           uint32_t n0, uint32_t n1, uint32_t ctr) {
  uint32_t x[16];
  x[8] = ctr ^ p.t8a;  // column 0: what is left of it
  x[12] = k[5] ^ rotl32(x[8] + p.x4c, 13);
  x[0] = kSigma0 ^ rotl32(x[12] + x[8], 18);
  x[1] = p.x1 ^ rotl32(x[0] + p.x3, 7);  // row 0
  x[2] = p.x2 ^ rotl32(x[1] + x[0], 9);
  x[3] = p.x3 ^ rotl32(x[2] + x[1], 13);
  x[0] ^= rotl32(x[3] + x[2], 18);
  x[4] = p.x4; x[5] = p.x5; x[6] = p.x6; x[7] = p.x7;  // row 1
  x[11] = p.x11;  // row 2
  x[8] ^= p.t8;
  x[9] = p.x9 ^ rotl32(x[8] + x[11], 13);
  x[10] = p.x10 ^ rotl32(x[9] + x[8], 18);
  x[12] ^= p.t12;  // row 3
  x[13] = p.x13 ^ rotl32(x[12] + p.x15, 9);
  x[14] = p.x14 ^ rotl32(x[13] + x[12], 13);
  x[15] = p.x15 ^ rotl32(x[14] + x[13], 18);
  salsa20_rounds<9>(x);
  const uint32_t j[16] = {kSigma0, k[0], k[1], k[2], k[3], kSigma1, n0, n1,
                          ctr, 0u, kSigma2, k[4], k[5], k[6], k[7], kSigma3};
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + j[i];
}

SDA_DEV void hsalsa20(uint32_t (&out)[8], const uint32_t (&k)[8], const uint32_t (&in)[4]) {
  uint32_t x[16] = {kSigma0, k[0], k[1], k[2], k[3], kSigma1, in[0], in[1],
                    in[2],   in[3], kSigma2, k[4], k[5], k[6], k[7], kSigma3};
  salsa20_rounds(x);
  out[0] = x[0]; out[1] = x[5]; out[2] = x[10]; out[3] = x[15];
  out[4] = x[6]; out[5] = x[7]; out[6] = x[8]; out[7] = x[9];
}

// ---------------------------------------------------------------- ChaCha20 --
#define SDA_CHACHA_QR(a, b, c, d)            \
  a += b; d ^= a; d = rotl32(d, 16);         \
  c += d; b ^= c; b = rotl32(b, 12);         \
  a += b; d ^= a; d = rotl32(d, 8);          \
  c += d; b ^= c; b = rotl32(b, 7);

template <int ROUNDS = 20>
SDA_DEV void chacha_block(uint32_t (&out)[16], const uint32_t (&in)[16]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = in[i];
#pragma unroll
  for (int i = 0; i < ROUNDS; i += 2) {
    SDA_CHACHA_QR(x[0], x[4], x[8], x[12]);
    SDA_CHACHA_QR(x[1], x[5], x[9], x[13]);
    SDA_CHACHA_QR(x[2], x[6], x[10], x[14]);
    SDA_CHACHA_QR(x[3], x[7], x[11], x[15]);
    SDA_CHACHA_QR(x[0], x[5], x[10], x[15]);
    SDA_CHACHA_QR(x[1], x[6], x[11], x[12]);
    SDA_CHACHA_QR(x[2], x[7], x[8], x[13]);
    SDA_CHACHA_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

// Counter-mode device CSPRNG: ChaCha20(key, counter = block, nonce = stream id).
// State words 12..13 = 64-bit block counter, 14..15 = 64-bit stream id.
struct RngKey {
  uint32_t k[8];
};
SDA_DEV void rng_block(uint32_t (&out)[16], const RngKey& key, uint64_t stream, uint64_t block) {
  uint32_t in[16] = {kSigma0, kSigma1, kSigma2, kSigma3, key.k[0], key.k[1], key.k[2], key.k[3],
                     key.k[4], key.k[5], key.k[6], key.k[7], (uint32_t)block,
                     (uint32_t)(block >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  chacha_block<20>(out, in);
}

// Stream ids: purpose in the top byte, then the owner index.
enum RngPurpose : uint64_t {
  kPurposeShares = 1,
  kPurposeSharesRetry = 2,
  kPurposeMaskFull = 3,
  kPurposeMaskRetry = 4,
  kPurposeChaChaSeed = 5,
  kPurposeEphemeral = 6,
  kPurposeShares16 = 7,   // 16-bit share draws (two rows per ChaCha block)
  kPurposeRetry16 = 8,    // lane-private replacements for rejected 16-bit draws
  kPurposeShares48 = 9,   // three draws per 32-bit word (m^3 < 2^32)
  kPurposeRetry48 = 10,   // lane-private spare words for those
  kPurposeSharesPss48 = 11,  // packed-Shamir randomness, three draws per word
};
SDA_DEV uint64_t stream_id(uint64_t purpose, uint64_t owner) { return (purpose << 56) | owner; }

// Exact uniform draw in [0, m) for one (stream, draw index): the primary word is
// word `idx` of the stream; a rejected word falls back to a private retry stream
// keyed by (owner, idx) so the result stays a pure function of (stream, idx).
SDA_DEV uint32_t uniform_fixup(const RngKey& key, uint64_t retry_purpose, uint64_t owner,
                               uint64_t idx, uint32_t m, uint32_t zone) {
  // retry stream: owner in the stream id, (idx) as block counter high bits
  for (uint64_t blk = 0;; ++blk) {
    uint32_t w[16];
    rng_block(w, key, stream_id(retry_purpose, owner), (idx << 8) | blk);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (w[i] < zone) return w[i] % m;
  }
}

// ---------------------------------------------------------------- BLAKE2b ---
// BLAKE2b-192 of a 64-byte message given as 16 LE words (libsodium seal nonce).
SDA_DEV void blake2b_192_64(uint32_t (&out)[6], const uint32_t (&msg)[16]) {
  const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                          0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                          0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  const uint8_t S[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = (uint64_t)msg[2 * i] | ((uint64_t)msg[2 * i + 1] << 32);
#pragma unroll
  for (int i = 8; i < 16; ++i) m[i] = 0;
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = IV[i];
  h[0] ^= 0x01010000ULL ^ 24ULL;
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV[i]; }
  v[12] ^= 64ULL;  // t0 = 64 bytes
  v[14] = ~v[14];  // last block
#define SDA_B2G(a, b, c, d, x, y)                    \
  v[a] = v[a] + v[b] + (x); v[d] = rotr64(v[d] ^ v[a], 32); \
  v[c] = v[c] + v[d];       v[b] = rotr64(v[b] ^ v[c], 24); \
  v[a] = v[a] + v[b] + (y); v[d] = rotr64(v[d] ^ v[a], 16); \
  v[c] = v[c] + v[d];       v[b] = rotr64(v[b] ^ v[c], 63);
#pragma unroll
  for (int r = 0; r < 12; ++r) {
    SDA_B2G(0, 4, 8, 12, m[S[r][0]], m[S[r][1]]);
    SDA_B2G(1, 5, 9, 13, m[S[r][2]], m[S[r][3]]);
    SDA_B2G(2, 6, 10, 14, m[S[r][4]], m[S[r][5]]);
    SDA_B2G(3, 7, 11, 15, m[S[r][6]], m[S[r][7]]);
    SDA_B2G(0, 5, 10, 15, m[S[r][8]], m[S[r][9]]);
    SDA_B2G(1, 6, 11, 12, m[S[r][10]], m[S[r][11]]);
    SDA_B2G(2, 7, 8, 13, m[S[r][12]], m[S[r][13]]);
    SDA_B2G(3, 4, 9, 14, m[S[r][14]], m[S[r][15]]);
  }
#undef SDA_B2G
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    uint64_t hv = h[i] ^ v[i] ^ v[i + 8];
    out[2 * i] = (uint32_t)hv;
    out[2 * i + 1] = (uint32_t)(hv >> 32);
  }
}

// --------------------------------------------------------------- Poly1305 ---
struct P130 {
  uint32_t v[5];
};
constexpr uint32_t kM26 = 0x3ffffff;

SDA_DEV P130 p130_zero() { return P130{{0, 0, 0, 0, 0}}; }

// Clamped r from the 16 key bytes (4 LE words).
SDA_DEV P130 p130_r_from_key(const uint32_t (&k)[4]) {
  P130 r;
  r.v[0] = k[0] & 0x3ffffff;
  r.v[1] = ((k[0] >> 26) | (k[1] << 6)) & 0x3ffff03;
  r.v[2] = ((k[1] >> 20) | (k[2] << 12)) & 0x3ffc0ff;
  r.v[3] = ((k[2] >> 14) | (k[3] << 18)) & 0x3f03fff;
  r.v[4] = (k[3] >> 8) & 0x00fffff;
  return r;
}
// 16-byte block (4 LE words) with the 2^128 (or pad) bit
SDA_DEV P130 p130_block(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t hibit) {
  P130 c;
  c.v[0] = w0 & kM26;
  c.v[1] = ((w0 >> 26) | (w1 << 6)) & kM26;
  c.v[2] = ((w1 >> 20) | (w2 << 12)) & kM26;
  c.v[3] = ((w2 >> 14) | (w3 << 18)) & kM26;
  c.v[4] = (w3 >> 8) | hibit;
  return c;
}
SDA_DEV P130 p130_add(const P130& a, const P130& b) {
  P130 r;
#pragma unroll
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}
// General product mod 2^130-5, operand limbs < 2^27; result limbs < 2^26 (limb1 < 2^27).
SDA_DEV P130 p130_mul(const P130& h, const P130& r) {
  const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
  uint64_t d0 = (uint64_t)h.v[0] * r.v[0] + (uint64_t)h.v[1] * s4 + (uint64_t)h.v[2] * s3 +
                (uint64_t)h.v[3] * s2 + (uint64_t)h.v[4] * s1;
  uint64_t d1 = (uint64_t)h.v[0] * r.v[1] + (uint64_t)h.v[1] * r.v[0] + (uint64_t)h.v[2] * s4 +
                (uint64_t)h.v[3] * s3 + (uint64_t)h.v[4] * s2;
  uint64_t d2 = (uint64_t)h.v[0] * r.v[2] + (uint64_t)h.v[1] * r.v[1] + (uint64_t)h.v[2] * r.v[0] +
                (uint64_t)h.v[3] * s4 + (uint64_t)h.v[4] * s3;
  uint64_t d3 = (uint64_t)h.v[0] * r.v[3] + (uint64_t)h.v[1] * r.v[2] + (uint64_t)h.v[2] * r.v[1] +
                (uint64_t)h.v[3] * r.v[0] + (uint64_t)h.v[4] * s4;
  uint64_t d4 = (uint64_t)h.v[0] * r.v[4] + (uint64_t)h.v[1] * r.v[3] + (uint64_t)h.v[2] * r.v[2] +
                (uint64_t)h.v[3] * r.v[1] + (uint64_t)h.v[4] * r.v[0];
  P130 o;
  uint64_t c;
  c = d0 >> 26; o.v[0] = (uint32_t)d0 & kM26; d1 += c;
  c = d1 >> 26; o.v[1] = (uint32_t)d1 & kM26; d2 += c;
  c = d2 >> 26; o.v[2] = (uint32_t)d2 & kM26; d3 += c;
  c = d3 >> 26; o.v[3] = (uint32_t)d3 & kM26; d4 += c;
  c = d4 >> 26; o.v[4] = (uint32_t)d4 & kM26;
  uint64_t t = (uint64_t)o.v[0] + c * 5;
  o.v[0] = (uint32_t)t & kM26;
  o.v[1] += (uint32_t)(t >> 26);
  return o;
}
// Normalise limbs (< 2^26 each) after additions.
SDA_DEV P130 p130_carry(P130 h) {
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= kM26; h.v[1] += c;
  c = h.v[1] >> 26; h.v[1] &= kM26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= kM26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= kM26; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= kM26; h.v[0] += c * 5;
  c = h.v[0] >> 26; h.v[0] &= kM26; h.v[1] += c;
  return h;
}
SDA_DEV P130 p130_pow(P130 r, uint32_t e) {
  P130 acc = P130{{1, 0, 0, 0, 0}};
  while (e) {
    if (e & 1) acc = p130_mul(acc, r);
    r = p130_mul(r, r);
    e >>= 1;
  }
  return acc;
}
// Fully reduced representative of h (limbs < 2^26, value < p).
SDA_DEV P130 p130_freeze(const P130& x) {
  uint32_t h0 = x.v[0], h1 = x.v[1], h2 = x.v[2], h3 = x.v[3], h4 = x.v[4], c;
  c = h0 >> 26; h0 &= kM26; h1 += c;
  c = h1 >> 26; h1 &= kM26; h2 += c;
  c = h2 >> 26; h2 &= kM26; h3 += c;
  c = h3 >> 26; h3 &= kM26; h4 += c;
  c = h4 >> 26; h4 &= kM26; h0 += c * 5;
  c = h0 >> 26; h0 &= kM26; h1 += c;
  c = h1 >> 26; h1 &= kM26; h2 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= kM26;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= kM26;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= kM26;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= kM26;
  uint32_t g4 = h4 + c - (1u << 26);
  const uint32_t keep = (g4 >> 31) - 1;  // all ones iff h >= p
  return P130{{(h0 & ~keep) | (g0 & keep), (h1 & ~keep) | (g1 & keep), (h2 & ~keep) | (g2 & keep),
               (h3 & ~keep) | (g3 & keep), (h4 & ~keep) | (g4 & keep)}};
}
// 2^x mod p for x < 156 (2^130 = 5).
SDA_DEV P130 p130_bit(int x) {
  P130 r = p130_zero();
  if (x < 130) r.v[x / 26] = 1u << (x % 26);
  else r.v[0] = 5u << (x - 130);
  return r;
}
// 7-bit digit d (bits 7d .. 7d+6) of a frozen value, d < 19.
SDA_DEV uint32_t p130_digit7(const P130& w, int d) {
  const int bit = 7 * d, li = bit / 26, sh = bit % 26;
  uint64_t x = w.v[li];
  if (li < 4) x |= (uint64_t)w.v[li + 1] << 26;
  return (uint32_t)(x >> sh) & 0x7fu;
}

// ---- Poly1305 on the matrix cores (k_mac_chunks, tables from k_poly_powers) ----
// A 1 KiB segment of 64 full blocks c_j (j = 0..63, bytes u_pos, pos = 16 j + a)
// contributes h = sum_j c_j r^(64 - j) = sum_pos u_pos W(pos) + 2^128 sum_e r^e
// with the key-dependent weights W(pos) = 2^(8a) r^(64 - j) mod p. Splitting W
// into 19 digits D_d of 7 bits turns the sum into 19 integer dot products over
// the segment's bytes -- an int8 GEMM: the i8 MFMA takes the bytes recentred
// to u - 128 (signed) and the digits (0..127); per digit the dot product
// C_d lies in (-2^24, 2^24). With x_d = C_d + 2^24 >= 0:
//   h = sum_d x_d 2^(7d) + K_seg,
//   K_seg = 2^128 sum_{e=1..64} r^e + 128 sum_pos W(pos) - 2^24 sum_d 2^(7d)  (mod p).
SDA_DEV P130 poly_weight(const P130& rpow, int a) {
  return p130_freeze(p130_mul(rpow, p130_bit(8 * a)));
}
// K_seg from sum_e r^e and sum_pos W(pos) (both carried, limbs < 2^27).
SDA_DEV P130 poly_kseg(const P130& sum_r, const P130& sum_w) {
  const P130 t1 = p130_mul(sum_r, p130_bit(128));
  const P130 t2 = p130_mul(sum_w, P130{{128u, 0, 0, 0, 0}});
  P130 b = p130_zero();
#pragma unroll
  for (int d = 0; d < 19; ++d) b = p130_add(b, p130_bit(24 + 7 * d));  // distinct bits: no carries
  P130 k;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint32_t four_p = 4u * (i == 0 ? kM26 - 4u : kM26);
    k.v[i] = t1.v[i] + t2.v[i] + four_p - b.v[i];
  }
  return p130_carry(k);
}
// Segment value from its 19 digit dot products C_d (summed over K-slices).
SDA_DEV P130 poly_seg_value(const int32_t (&c)[19], const P130& kseg) {
  uint32_t l[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int d = 0; d < 19; ++d) {
    const uint32_t x = (uint32_t)(c[d] + (1 << 24));  // < 2^25
    const int bit = 7 * d, li = bit / 26, sh = bit % 26;
    const uint64_t v = (uint64_t)x << sh;
    l[li] += (uint32_t)v & kM26;
    l[li + 1] += (uint32_t)(v >> 26);
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    l[i + 1] += l[i] >> 26;
    l[i] &= kM26;
  }
  const P130 h = p130_carry(P130{{l[0] + 5u * l[5], l[1], l[2], l[3], l[4]}});
  return p130_carry(p130_add(h, kseg));
}

// ---- interleaved rows (k_encode_encrypt's MAC; tables: kernels.hpp) ----
// Row i of the chunk whose first keystream byte is kC takes the blocks jb = i + 16 t.
// A tile holding the keystream bytes [ks0, ks1) owns the pad bit of the blocks whose
// first byte (kC + 16 jb) lies in that range: for row i those with t in [T0, T1).
SDA_DEV void poly_row_owned(int64_t ks0, int64_t ks1, int64_t kC, int i, int& T0, int& T1) {
  const int64_t d0 = ks0 - kC, d1 = ks1 - kC;
  const int J0 = d0 <= 0 ? 0 : (int)(((d0 + 15) >> 4) < 1024 ? ((d0 + 15) >> 4) : 1024);
  const int J1 = d1 <= 0 ? 0 : (int)(((d1 + 15) >> 4) < 1024 ? ((d1 + 15) >> 4) : 1024);
  T0 = J0 > i ? (J0 - i + 15) >> 4 : 0;
  T1 = J1 > i ? (J1 - i + 15) >> 4 : 0;
}
// Row constant: koff + Q[T1] - Q[T0] (all carried, limbs < 2^26 + small).
SDA_DEV P130 poly_row_const(const uint32_t* koff, const uint32_t* q0, const uint32_t* q1) {
  P130 k;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const uint32_t four_p = 4u * (u == 0 ? kM26 - 4u : kM26);
    k.v[u] = koff[u] + q1[u] + four_p - q0[u];
  }
  return p130_carry(k);
}

// Final tag = (h mod p + s) mod 2^128, as 4 LE words.
SDA_DEV void p130_finish(uint32_t (&tag)[4], P130 h, const uint32_t (&s)[4]) {
  uint32_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4], c;
  c = h0 >> 26; h0 &= kM26; h1 += c;
  c = h1 >> 26; h1 &= kM26; h2 += c;
  c = h2 >> 26; h2 &= kM26; h3 += c;
  c = h3 >> 26; h3 &= kM26; h4 += c;
  c = h4 >> 26; h4 &= kM26; h0 += c * 5;
  c = h0 >> 26; h0 &= kM26; h1 += c;
  c = h1 >> 26; h1 &= kM26; h2 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= kM26;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= kM26;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= kM26;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= kM26;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;
  g0 &= mask; g1 &= mask; g2 &= mask; g3 &= mask; g4 &= mask;
  mask = ~mask;
  h0 = (h0 & mask) | g0; h1 = (h1 & mask) | g1; h2 = (h2 & mask) | g2;
  h3 = (h3 & mask) | g3; h4 = (h4 & mask) | g4;
  uint32_t w0 = h0 | (h1 << 26);
  uint32_t w1 = (h1 >> 6) | (h2 << 20);
  uint32_t w2 = (h2 >> 12) | (h3 << 14);
  uint32_t w3 = (h3 >> 18) | (h4 << 8);
  uint64_t f;
  f = (uint64_t)w0 + s[0]; tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + s[1] + (f >> 32); tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + s[2] + (f >> 32); tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + s[3] + (f >> 32); tag[3] = (uint32_t)f;
}

// -------------------------------------------------------- GF(2^255 - 19) ----
// ---- radix 2^25.5 representation (10 limbs, 26/25 bits alternating) -------
// Products accumulate into 10 independent 64-bit column sums (no carry chain
// inside the product), which gives the single-wave X25519 ladders the ILP the
// serial radix-2^32 schoolbook lacks. Limb i sits at bit ceil(25.5 i); a product
// of two odd limbs is doubled, and columns >= 10 wrap with a factor 19.
struct Fe10 {
  uint32_t v[10];
};
SDA_DEV Fe10 fe10_set(uint32_t x) { return Fe10{{x, 0, 0, 0, 0, 0, 0, 0, 0, 0}}; }

SDA_DEV Fe10 fe10_carry64(uint64_t (&h)[10]) {
  uint64_t c;
  c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffff;
  c = h[1] >> 25; h[2] += c; h[1] &= 0x1ffffff;
  c = h[2] >> 26; h[3] += c; h[2] &= 0x3ffffff;
  c = h[3] >> 25; h[4] += c; h[3] &= 0x1ffffff;
  c = h[4] >> 26; h[5] += c; h[4] &= 0x3ffffff;
  c = h[5] >> 25; h[6] += c; h[5] &= 0x1ffffff;
  c = h[6] >> 26; h[7] += c; h[6] &= 0x3ffffff;
  c = h[7] >> 25; h[8] += c; h[7] &= 0x1ffffff;
  c = h[8] >> 26; h[9] += c; h[8] &= 0x3ffffff;
  c = h[9] >> 25; h[0] += c * 19; h[9] &= 0x1ffffff;
  c = h[0] >> 26; h[1] += c; h[0] &= 0x3ffffff;
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)h[i];
  return r;
}
SDA_DEV Fe10 fe10_carry(const Fe10& a) {
  uint64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = a.v[i];
  return fe10_carry64(h);
}
SDA_DEV Fe10 fe10_add(const Fe10& a, const Fe10& b) {
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
  return fe10_carry(r);
}
// a - b + 2p, then carried (inputs carried: limbs <= 2^26 + small)
SDA_DEV Fe10 fe10_sub(const Fe10& a, const Fe10& b) {
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t two_p = (i == 0) ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu);
    r.v[i] = a.v[i] + two_p - b.v[i];
  }
  return fe10_carry(r);
}
// The same without the carry pass, for results that go straight into a product:
// with carried inputs (even limbs <= 2^26, odd <= 2^25, plus a few units) a sum has
// limbs <= 2^27 / 2^26 and a difference <= 3 * 2^26 / 3 * 2^25; fe10_mul / fe10_sq of
// two such operands keep 19 f < 2^32 and every column sum below 1120 * 2^52 < 2^63.
SDA_DEV Fe10 fe10_add_nc(const Fe10& a, const Fe10& b) {
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}
SDA_DEV Fe10 fe10_sub_nc(const Fe10& a, const Fe10& b) {
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t two_p = (i == 0) ? 0x7ffffdau : ((i & 1) ? 0x3fffffeu : 0x7fffffeu);
    r.v[i] = a.v[i] + two_p - b.v[i];
  }
  return r;
}
SDA_DEV Fe10 fe10_mul(const Fe10& f, const Fe10& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const uint32_t fi = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      if (i + j < 10) h[i + j] += (uint64_t)fi * g.v[j];
      else h[i + j - 10] += (uint64_t)fi * g19[j];
    }
  }
  return fe10_carry64(h);
}
SDA_DEV Fe10 fe10_sq(const Fe10& f) {
  uint32_t f19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    f19[i] = 19u * f.v[i];
    f2[i] = 2u * f.v[i];
  }
  uint64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      // symmetric pair counted twice (i != j); odd*odd doubles once more
      const bool odd2 = (i & 1) && (j & 1);
      uint32_t a = (i == j) ? (odd2 ? f2[i] : f.v[i]) : (odd2 ? 2u * f2[i] : f2[i]);
      if (i + j < 10) h[i + j] += (uint64_t)a * f.v[j];
      else h[i + j - 10] += (uint64_t)a * f19[j];
    }
  }
  return fe10_carry64(h);
}
SDA_DEV Fe10 fe10_mul121665(const Fe10& f) {
  uint64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = (uint64_t)f.v[i] * 121665u;
  return fe10_carry64(h);
}
SDA_DEV void fe10_cswap(Fe10& a, Fe10& b, uint32_t swap) {
  const uint32_t mask = 0u - swap;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t t = mask & (a.v[i] ^ b.v[i]);
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}
SDA_DEV Fe10 fe10_sqn(Fe10 a, int n) {
  for (int i = 0; i < n; ++i) a = fe10_sq(a);
  return a;
}
SDA_DEV Fe10 fe10_invert(const Fe10& z) {
  Fe10 z2 = fe10_sq(z);
  Fe10 z9 = fe10_mul(fe10_sqn(z2, 2), z);
  Fe10 z11 = fe10_mul(z9, z2);
  Fe10 z_5_0 = fe10_mul(fe10_sq(z11), z9);
  Fe10 z_10_0 = fe10_mul(fe10_sqn(z_5_0, 5), z_5_0);
  Fe10 z_20_0 = fe10_mul(fe10_sqn(z_10_0, 10), z_10_0);
  Fe10 z_40_0 = fe10_mul(fe10_sqn(z_20_0, 20), z_20_0);
  Fe10 z_50_0 = fe10_mul(fe10_sqn(z_40_0, 10), z_10_0);
  Fe10 z_100_0 = fe10_mul(fe10_sqn(z_50_0, 50), z_50_0);
  Fe10 z_200_0 = fe10_mul(fe10_sqn(z_100_0, 100), z_100_0);
  Fe10 z_250_0 = fe10_mul(fe10_sqn(z_200_0, 50), z_50_0);
  return fe10_mul(fe10_sqn(z_250_0, 5), z11);
}
SDA_DEV Fe10 fe10_from_words(const uint32_t (&w)[8]) {
  // bit offsets 0,26,51,77,102,128,153,179,204,230
  const int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  Fe10 r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int p = pos[i], wi = p >> 5, sh = p & 31;
    const int width = (i & 1) ? 25 : 26;
    uint64_t x = w[wi];
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << 32;
    r.v[i] = (uint32_t)(x >> sh) & ((1u << width) - 1);
  }
  r.v[9] &= 0x1ffffff;  // bit 255 ignored (limb 9 covers bits 230..254)
  return r;
}
SDA_DEV void fe10_to_words(uint32_t (&w)[8], const Fe10& a) {
  // fully reduce: carry, then subtract p if h >= p
  uint64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = a.v[i];
  Fe10 t = fe10_carry64(h);
  t = fe10_carry(t);
  // q = 1 iff t >= p: propagate (t + 19) carries to bit 255
  uint32_t q = (19u * 1u + t.v[0]) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (t.v[i] + q) >> ((i & 1) ? 25 : 26);
  uint64_t hh[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) hh[i] = t.v[i];
  hh[0] += 19u * q;
  uint64_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int width = (i & 1) ? 25 : 26;
    c = hh[i] >> width;
    hh[i + 1] += c;
    hh[i] &= (1u << width) - 1;
  }
  hh[9] &= 0x1ffffff;
  const int pos[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int p = pos[i], wi = p >> 5, sh = p & 31;
    const uint64_t x = hh[i] << sh;
    w[wi] |= (uint32_t)x;
    if (wi + 1 < 8) w[wi + 1] |= (uint32_t)(x >> 32);
  }
}

// RFC 7748 ladder: X25519(scalar, u) = x2 / z2 (0 when z2 = 0). Words are little-endian.
SDA_DEV void x25519_xz(Fe10& x2_out, Fe10& z2_out, const uint32_t (&scalar)[8], const uint32_t (&u)[8]) {
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = scalar[i];
  k[0] &= 0xfffffff8u;
  k[7] &= 0x7fffffffu;
  k[7] |= 0x40000000u;
  const Fe10 x1 = fe10_from_words(u);
  Fe10 x2 = fe10_set(1), z2 = fe10_set(0), x3 = x1, z3 = fe10_set(1);
  uint32_t swap = 0;
  for (int t = 254; t >= 0; --t) {
    const uint32_t kt = (k[t >> 5] >> (t & 31)) & 1;
    swap ^= kt;
    fe10_cswap(x2, x3, swap);
    fe10_cswap(z2, z3, swap);
    swap = kt;
    // every sum / difference feeds a product directly: no carry passes (fe10_add_nc)
    const Fe10 A = fe10_add_nc(x2, z2), B = fe10_sub_nc(x2, z2);
    const Fe10 C = fe10_add_nc(x3, z3), D = fe10_sub_nc(x3, z3);
    const Fe10 AA = fe10_sq(A), BB = fe10_sq(B);
    const Fe10 DA = fe10_mul(D, A), CB = fe10_mul(C, B);
    const Fe10 E = fe10_sub_nc(AA, BB);
    x3 = fe10_sq(fe10_add_nc(DA, CB));
    z3 = fe10_mul(x1, fe10_sq(fe10_sub_nc(DA, CB)));
    x2 = fe10_mul(AA, BB);
    z2 = fe10_mul(E, fe10_add_nc(AA, fe10_mul121665(E)));
  }
  fe10_cswap(x2, x3, swap);
  fe10_cswap(z2, z3, swap);
  x2_out = x2;
  z2_out = z2;
}
SDA_DEV void x25519(uint32_t (&out)[8], const uint32_t (&scalar)[8], const uint32_t (&u)[8]) {
  Fe10 x2, z2;
  x25519_xz(x2, z2, scalar, u);
  fe10_to_words(out, fe10_mul(x2, fe10_invert(z2)));
}

// ---- fixed-base: X25519(scalar, 9) from a table of edwards25519 multiples ----
// A sealed box's ephemeral public key is esk . 9, always the same point: with the
// table of (j + 1) 256^i B (i < 32, j < 8; scripts/gen_ed25519_base.py) the scalar's
// 64 signed radix-16 digits cost 64 mixed additions and 4 doublings -- about 500 field
// multiplications against the ladder's 2,500 -- and the Montgomery u-coordinate is
// (Z + Y) / (Z - Y) (the route of libsodium's crypto_scalarmult_base). Lanes index the
// table by their own secret digits: there is no cache-timing observer on the device
// worth the constant-time scan of eight entries per addition.
constexpr int kEdEntryWords = 32;  // y+x, y-x, 2dxy: 3 x 10 limbs, padded
struct GeP3 {
  Fe10 X, Y, Z, T;
};
struct GeP1 {  // "completed" point: (X : Z) x (Y : T)
  Fe10 X, Y, Z, T;
};
SDA_DEV GeP3 ge_p1_to_p3(const GeP1& r) {
  return GeP3{fe10_mul(r.X, r.T), fe10_mul(r.Y, r.Z), fe10_mul(r.Z, r.T), fe10_mul(r.X, r.Y)};
}
// p + (sign ? -q : q) for the table entry q = (y+x, y-x, 2dxy) at `e`
SDA_DEV GeP1 ge_madd(const GeP3& p, const uint32_t* e, bool neg) {
  Fe10 ypx, ymx, xy2d;
  const uint4* e4 = reinterpret_cast<const uint4*>(e);
  uint32_t w[kEdEntryWords];
#pragma unroll
  for (int i = 0; i < kEdEntryWords / 4; ++i) {
    const uint4 q = e4[i];
    w[4 * i] = q.x; w[4 * i + 1] = q.y; w[4 * i + 2] = q.z; w[4 * i + 3] = q.w;
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    ypx.v[i] = neg ? w[10 + i] : w[i];
    ymx.v[i] = neg ? w[i] : w[10 + i];
    xy2d.v[i] = w[20 + i];
  }
  if (neg) xy2d = fe10_sub_nc(fe10_set(0), xy2d);  // 2p - x: a product operand
  GeP1 r;
  const Fe10 a = fe10_mul(fe10_add_nc(p.Y, p.X), ypx);
  const Fe10 b = fe10_mul(fe10_sub_nc(p.Y, p.X), ymx);
  const Fe10 c = fe10_mul(xy2d, p.T);
  const Fe10 d = fe10_add(p.Z, p.Z);
  r.X = fe10_sub_nc(a, b);
  r.Y = fe10_add_nc(a, b);
  r.Z = fe10_add(d, c);
  r.T = fe10_sub(d, c);
  return r;
}
// 2 (X : Y : Z) as a completed point
SDA_DEV GeP1 ge_dbl(const Fe10& X, const Fe10& Y, const Fe10& Z) {
  const Fe10 xx = fe10_sq(X), yy = fe10_sq(Y);
  const Fe10 zz = fe10_sq(Z);
  const Fe10 b = fe10_add(zz, zz);
  const Fe10 a = fe10_sq(fe10_add_nc(X, Y));
  GeP1 r;
  r.Y = fe10_add(yy, xx);
  r.Z = fe10_sub(yy, xx);
  r.X = fe10_sub(a, r.Y);
  r.T = fe10_sub(b, r.Z);
  return r;
}
// X25519(scalar, 9) = num / den
SDA_DEV void x25519_base_nd(Fe10& num_out, Fe10& den_out, const uint32_t (&scalar)[8], const uint32_t* table) {
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = scalar[i];
  k[0] &= 0xfffffff8u;
  k[7] &= 0x7fffffffu;
  k[7] |= 0x40000000u;
  // signed radix-16 digits, -8 <= e_i < 8 (the top one <= 8): nibble + carry, eight
  // per word, kept packed as biased bytes (digit + 8)
  uint32_t dig[16];  // four digits per word
  {
    uint32_t carry = 0;
#pragma unroll
    for (int wi = 0; wi < 8; ++wi) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        uint32_t v = ((k[wi] >> (4 * n)) & 15u) + carry;
        carry = (v + 8u) >> 4;
        if (wi == 7 && n == 7) carry = 0;  // the last digit keeps its carry (<= 8)
        v = v - (carry << 4) + 8u;         // biased: 0 .. 16
        if (n < 4) lo |= v << (8 * n); else hi |= v << (8 * (n - 4));
      }
      dig[2 * wi] = lo;
      dig[2 * wi + 1] = hi;
    }
  }
  auto digit = [&](int i) -> int {  // i < 64
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) w = (i >> 2) == q ? dig[q] : w;
    return (int)((w >> (8 * (i & 3))) & 0xffu) - 8;
  };
  GeP3 h{fe10_set(0), fe10_set(1), fe10_set(1), fe10_set(0)};
  auto step = [&](int i) {
    const int e = digit(i);
    if (e == 0) return;  // + identity
    const int mag = e < 0 ? -e : e;
    h = ge_p1_to_p3(ge_madd(h, table + ((size_t)(i >> 1) * 8 + (mag - 1)) * kEdEntryWords, e < 0));
  };
#pragma unroll 1
  for (int i = 1; i < 64; i += 2) step(i);
  // h <- 16 h
  GeP1 r = ge_dbl(h.X, h.Y, h.Z);
#pragma unroll 1
  for (int q = 0; q < 3; ++q) {
    const Fe10 x = fe10_mul(r.X, r.T), y = fe10_mul(r.Y, r.Z), z = fe10_mul(r.Z, r.T);
    r = ge_dbl(x, y, z);
  }
  h = ge_p1_to_p3(r);
#pragma unroll 1
  for (int i = 0; i < 64; i += 2) step(i);
  num_out = fe10_add(h.Z, h.Y);
  den_out = fe10_sub(h.Z, h.Y);
}
SDA_DEV void x25519_base(uint32_t (&out)[8], const uint32_t (&scalar)[8], const uint32_t* table) {
  Fe10 num, den;
  x25519_base_nd(num, den, scalar, table);
  fe10_to_words(out, fe10_mul(num, fe10_invert(den)));
}
// The same with the recipient's key as a fixed base too: a public key that seals many
// boxes (a clerk's, once per participant) gets its own table (host: x25519_comb_table),
// and the shared point is 64 table additions like the public key. One loop for both
// tables, one inversion for both results.
SDA_DEV void x25519_seal_pair_tables(uint32_t (&epk)[8], uint32_t (&shared)[8], const uint32_t (&esk)[8],
                                     const uint32_t* base_table, const uint32_t* key_table) {
  Fe10 num0 = fe10_set(0), den0 = num0, num1 = num0, den1 = num0;
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    Fe10 n, d;
    x25519_base_nd(n, d, esk, h ? key_table : base_table);
    if (h == 0) { num0 = n; den0 = d; } else { num1 = n; den1 = d; }
  }
  const Fe10 inv = fe10_invert(fe10_mul(den0, den1));
  fe10_to_words(epk, fe10_mul(num0, fe10_mul(inv, den1)));
  fe10_to_words(shared, fe10_mul(num1, fe10_mul(inv, den0)));
}
// Both halves of a sealed box's key agreement, epk = esk . 9 and shared = esk . pk,
// with one field inversion for the two (1 / (z2 den), then times the other
// denominator). A zero z2 (a low-order pk: the shared point is rejected anyway) makes
// both outputs zero.
SDA_DEV void x25519_seal_pair(uint32_t (&epk)[8], uint32_t (&shared)[8], const uint32_t (&esk)[8],
                              const uint32_t (&pk)[8], const uint32_t* table) {
  Fe10 num, den, x2, z2;
  x25519_base_nd(num, den, esk, table);
  x25519_xz(x2, z2, esk, pk);
  const Fe10 inv = fe10_invert(fe10_mul(z2, den));
  fe10_to_words(epk, fe10_mul(num, fe10_mul(inv, z2)));
  fe10_to_words(shared, fe10_mul(x2, fe10_mul(inv, den)));
}

// ------------------------------------------------------------------ varint --
// zigzag(LEB128) length of a canonical value v in [0, 2^31): z = 2v.
SDA_DEV uint32_t varint_len_canon(uint32_t v) {
  uint32_t z = v << 1;
  return 1u + (z >= (1u << 7)) + (z >= (1u << 14)) + (z >= (1u << 21)) + (z >= (1u << 28));
}

}  // namespace sdagpu
