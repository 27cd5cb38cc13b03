// Salsa20 / HSalsa20 / XSalsa20, ChaCha20 and the rand-0.3 `ChaChaRng`, plus
// Poly1305 — host reference implementations.
//
// XSalsa20-Poly1305 is the libsodium secretbox used under crypto_box_seal
// (reference client/src/crypto/encryption/sodium.rs:43,78). ChaChaRng reproduces
// `rand::ChaChaRng::from_seed` + `gen_range(0, m)` used by the ChaCha mask
// (client/src/crypto/masking/chacha.rs:29-39,67-72).
#include <atomic>
#include <cstring>

#include "sda/crypto.hpp"

namespace sda {
namespace crypto {
namespace {

inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
inline uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline void st32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

const uint32_t kSigma[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};

// 20-round Salsa20 permutation on x (no feed-forward).
void salsa20_rounds(uint32_t x[16]) {
  for (int i = 0; i < 10; ++i) {
    // column round
    x[4] ^= rotl32(x[0] + x[12], 7);   x[8] ^= rotl32(x[4] + x[0], 9);
    x[12] ^= rotl32(x[8] + x[4], 13);  x[0] ^= rotl32(x[12] + x[8], 18);
    x[9] ^= rotl32(x[5] + x[1], 7);    x[13] ^= rotl32(x[9] + x[5], 9);
    x[1] ^= rotl32(x[13] + x[9], 13);  x[5] ^= rotl32(x[1] + x[13], 18);
    x[14] ^= rotl32(x[10] + x[6], 7);  x[2] ^= rotl32(x[14] + x[10], 9);
    x[6] ^= rotl32(x[2] + x[14], 13);  x[10] ^= rotl32(x[6] + x[2], 18);
    x[3] ^= rotl32(x[15] + x[11], 7);  x[7] ^= rotl32(x[3] + x[15], 9);
    x[11] ^= rotl32(x[7] + x[3], 13);  x[15] ^= rotl32(x[11] + x[7], 18);
    // row round
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

void salsa20_setup(uint32_t x[16], const uint8_t key[32], const uint8_t in16[16]) {
  x[0] = kSigma[0];
  x[1] = ld32(key + 0); x[2] = ld32(key + 4); x[3] = ld32(key + 8); x[4] = ld32(key + 12);
  x[5] = kSigma[1];
  x[6] = ld32(in16 + 0); x[7] = ld32(in16 + 4); x[8] = ld32(in16 + 8); x[9] = ld32(in16 + 12);
  x[10] = kSigma[2];
  x[11] = ld32(key + 16); x[12] = ld32(key + 20); x[13] = ld32(key + 24); x[14] = ld32(key + 28);
  x[15] = kSigma[3];
}

void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  a += b; d ^= a; d = rotl32(d, 16);
  c += d; b ^= c; b = rotl32(b, 12);
  a += b; d ^= a; d = rotl32(d, 8);
  c += d; b ^= c; b = rotl32(b, 7);
}

}  // namespace

void salsa20_block(uint8_t out[64], const uint8_t key[32], const uint8_t nonce[8],
                   uint64_t counter) {
  uint8_t in16[16];
  std::memcpy(in16, nonce, 8);
  for (int i = 0; i < 8; ++i) in16[8 + i] = (uint8_t)(counter >> (8 * i));
  uint32_t x[16], j[16];
  salsa20_setup(j, key, in16);
  std::memcpy(x, j, sizeof(x));
  salsa20_rounds(x);
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + j[i]);
}

void hsalsa20(uint8_t out[32], const uint8_t key[32], const uint8_t in16[16]) {
  uint32_t x[16];
  salsa20_setup(x, key, in16);
  salsa20_rounds(x);
  st32(out + 0, x[0]); st32(out + 4, x[5]); st32(out + 8, x[10]); st32(out + 12, x[15]);
  st32(out + 16, x[6]); st32(out + 20, x[7]); st32(out + 24, x[8]); st32(out + 28, x[9]);
}

void xsalsa20_xor(uint8_t* out, const uint8_t* in, size_t n, const uint8_t nonce[24],
                  const uint8_t key[32], uint64_t ofs) {
  uint8_t subkey[32];
  hsalsa20(subkey, key, nonce);
  uint8_t block[64];
  size_t done = 0;
  while (done < n) {
    uint64_t pos = ofs + done;
    uint64_t ctr = pos / 64;
    size_t within = (size_t)(pos % 64);
    salsa20_block(block, subkey, nonce + 16, ctr);
    size_t take = std::min(n - done, (size_t)64 - within);
    for (size_t i = 0; i < take; ++i) out[done + i] = in[done + i] ^ block[within + i];
    done += take;
  }
  secure_zero(subkey, sizeof(subkey));
  secure_zero(block, sizeof(block));
}

void chacha20_block_words(uint32_t out[16], const uint32_t in[16], int rounds) {
  uint32_t x[16];
  std::memcpy(x, in, sizeof(x));
  for (int i = 0; i < rounds; i += 2) {
    chacha_qr(x[0], x[4], x[8], x[12]);
    chacha_qr(x[1], x[5], x[9], x[13]);
    chacha_qr(x[2], x[6], x[10], x[14]);
    chacha_qr(x[3], x[7], x[11], x[15]);
    chacha_qr(x[0], x[5], x[10], x[15]);
    chacha_qr(x[1], x[6], x[11], x[12]);
    chacha_qr(x[2], x[7], x[8], x[13]);
    chacha_qr(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

// ---- rand 0.3 ChaChaRng ----------------------------------------------------
ChaChaRng::ChaChaRng(const uint32_t* seed, size_t nwords) {
  for (int i = 0; i < 4; ++i) state_[i] = kSigma[i];
  for (int i = 0; i < 8; ++i) state_[4 + i] = (size_t)i < nwords ? seed[i] : 0u;
  for (int i = 12; i < 16; ++i) state_[i] = 0;
  index_ = 16;
}
void ChaChaRng::refill() {
  chacha20_block_words(buf_, state_, 20);
  index_ = 0;
  for (int i = 12; i < 16; ++i) {
    if (++state_[i] != 0) break;
  }
}
uint32_t ChaChaRng::next_u32() {
  if (index_ == 16) refill();
  return buf_[index_++];
}
uint64_t ChaChaRng::next_u64() {
  uint64_t hi = next_u32();
  uint64_t lo = next_u32();
  return (hi << 32) | lo;
}
namespace {
std::atomic<uint64_t> g_zone_cap{UINT64_MAX};
}
void set_chacha_zone_cap(uint64_t cap) { g_zone_cap.store(cap); }

int64_t ChaChaRng::gen_range(int64_t low, int64_t high) {
  if (!(low < high)) throw SdaError("gen_range: empty range");
  uint64_t range = (uint64_t)high - (uint64_t)low;
  uint64_t zone = UINT64_MAX - UINT64_MAX % range;
  const uint64_t cap = g_zone_cap.load(std::memory_order_relaxed);
  if (cap != UINT64_MAX && cap - cap % range < zone) zone = cap - cap % range;  // test hook
  for (;;) {
    uint64_t v = next_u64();
    if (v < zone) return (int64_t)((uint64_t)low + v % range);
  }
}

// ---- Poly1305 (26-bit limbs, the same radix the GPU kernels use) -----------
void poly1305(uint8_t tag[16], const uint8_t* m, size_t n, const uint8_t key[32]) {
  const uint32_t r0 = ld32(key + 0) & 0x3ffffff;
  const uint32_t r1 = (ld32(key + 3) >> 2) & 0x3ffff03;
  const uint32_t r2 = (ld32(key + 6) >> 4) & 0x3ffc0ff;
  const uint32_t r3 = (ld32(key + 9) >> 6) & 0x3f03fff;
  const uint32_t r4 = (ld32(key + 12) >> 8) & 0x00fffff;
  const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
  uint8_t last[16];
  while (n > 0) {
    const uint8_t* blk = m;
    uint32_t hibit = 1u << 24;
    size_t take = 16;
    if (n < 16) {
      std::memset(last, 0, 16);
      std::memcpy(last, m, n);
      last[n] = 1;
      blk = last;
      hibit = 0;
      take = n;
    }
    h0 += ld32(blk + 0) & 0x3ffffff;
    h1 += (ld32(blk + 3) >> 2) & 0x3ffffff;
    h2 += (ld32(blk + 6) >> 4) & 0x3ffffff;
    h3 += (ld32(blk + 9) >> 6) & 0x3ffffff;
    h4 += (ld32(blk + 12) >> 8) | hibit;
    uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff; d1 += c;
    c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff; d2 += c;
    c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff; d3 += c;
    c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff; d4 += c;
    c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff; h0 += c * 5;
    c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
    m += take;
    n -= take;
  }
  uint32_t c;
  c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
  c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
  c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
  c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
  c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;  // all-ones when h >= p
  g0 &= mask; g1 &= mask; g2 &= mask; g3 &= mask; g4 &= mask;
  mask = ~mask;
  h0 = (h0 & mask) | g0; h1 = (h1 & mask) | g1; h2 = (h2 & mask) | g2;
  h3 = (h3 & mask) | g3; h4 = (h4 & mask) | g4;
  h0 = (h0 | (h1 << 26));
  h1 = ((h1 >> 6) | (h2 << 20));
  h2 = ((h2 >> 12) | (h3 << 14));
  h3 = ((h3 >> 18) | (h4 << 8));
  uint64_t f;
  f = (uint64_t)h0 + ld32(key + 16); h0 = (uint32_t)f;
  f = (uint64_t)h1 + ld32(key + 20) + (f >> 32); h1 = (uint32_t)f;
  f = (uint64_t)h2 + ld32(key + 24) + (f >> 32); h2 = (uint32_t)f;
  f = (uint64_t)h3 + ld32(key + 28) + (f >> 32); h3 = (uint32_t)f;
  st32(tag + 0, h0); st32(tag + 4, h1); st32(tag + 8, h2); st32(tag + 12, h3);
}

bool verify16(const uint8_t a[16], const uint8_t b[16]) {
  uint8_t d = 0;
  for (int i = 0; i < 16; ++i) d |= a[i] ^ b[i];
  return d == 0;
}

}  // namespace crypto
}  // namespace sda
