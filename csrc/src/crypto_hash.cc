// SHA-512 (FIPS 180-4) and BLAKE2b (RFC 7693), host implementations.
//
// Used by Ed25519 (client/src/crypto/signing/mod.rs:72-132 in the reference) and
// by the sealed-box nonce BLAKE2b-192(epk || pk) (sodium.rs:43,78 -> libsodium
// crypto_box_seal). The SHA-512 round constants and the shared SHA-512/BLAKE2b IV
// are *derived* at start-up (fractional parts of cube / square roots of primes)
// with an exact integer root, so no constant table is typed in by hand.
#include <cstring>

#include "sda/crypto.hpp"

namespace sda {
namespace crypto {
namespace {

// ---- tiny fixed-width bignum for exact integer roots ---------------------
struct Big {
  uint32_t w[14] = {0};  // 448 bits
};
Big big_mul(const Big& a, const Big& b) {
  Big r;
  uint64_t acc[28] = {0};
  for (int i = 0; i < 14; ++i)
    for (int j = 0; i + j < 14 && j < 14; ++j) {
      uint64_t p = (uint64_t)a.w[i] * b.w[j];
      acc[i + j] += p & 0xffffffffu;
      acc[i + j + 1] += p >> 32;
    }
  uint64_t c = 0;
  for (int i = 0; i < 14; ++i) {
    uint64_t t = acc[i] + c;
    r.w[i] = (uint32_t)t;
    c = t >> 32;
  }
  return r;
}
int big_cmp(const Big& a, const Big& b) {
  for (int i = 13; i >= 0; --i) {
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  }
  return 0;
}
// floor(root_k(p * 2^(64k))) mod 2^64 : the first 64 fractional bits of p^(1/k)
uint64_t frac_root_bits(uint32_t p, int k) {
  Big target;
  int shift = 64 * k;  // p << shift
  target.w[shift / 32] = p;
  // x < 2^(64 + 9) since p < 512
  Big lo, hi;
  hi.w[2] = 1u << 10;  // 2^74
  // binary search for the largest x with x^k <= target
  for (int it = 0; it < 80; ++it) {
    // mid = (lo + hi) / 2
    Big mid;
    uint64_t c = 0;
    for (int i = 0; i < 14; ++i) {
      uint64_t t = (uint64_t)lo.w[i] + hi.w[i] + c;
      mid.w[i] = (uint32_t)t;
      c = t >> 32;
    }
    for (int i = 0; i < 14; ++i) {
      uint32_t next = (i + 1 < 14) ? mid.w[i + 1] : (uint32_t)c;
      mid.w[i] = (mid.w[i] >> 1) | (next << 31);
    }
    Big pw = mid;
    for (int e = 1; e < k; ++e) pw = big_mul(pw, mid);
    if (big_cmp(pw, target) <= 0) lo = mid; else hi = mid;
  }
  return ((uint64_t)lo.w[1] << 32) | lo.w[0];
}

struct Constants {
  uint64_t K[80];
  uint64_t IV[8];
  Constants() {
    uint32_t primes[80];
    int n = 0;
    for (uint32_t c = 2; n < 80; ++c) {
      bool prime = true;
      for (uint32_t d = 2; d * d <= c; ++d)
        if (c % d == 0) { prime = false; break; }
      if (prime) primes[n++] = c;
    }
    for (int i = 0; i < 80; ++i) K[i] = frac_root_bits(primes[i], 3);
    for (int i = 0; i < 8; ++i) IV[i] = frac_root_bits(primes[i], 2);
  }
};
const Constants& C() {
  static Constants c;
  return c;
}

inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint64_t load64_be(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
inline void store64_be(uint8_t* p, uint64_t v) {
  for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; }
}
inline uint64_t load64_le(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

void sha512_compress(uint64_t h[8], const uint8_t block[128]) {
  const uint64_t* K = C().K;
  uint64_t w[80];
  for (int i = 0; i < 16; ++i) w[i] = load64_be(block + 8 * i);
  for (int i = 16; i < 80; ++i) {
    uint64_t s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    uint64_t s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 80; ++i) {
    uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K[i] + w[i];
    uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    uint64_t maj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + maj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// ---- BLAKE2b ---------------------------------------------------------------
const uint8_t kSigma[12][16] = {
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
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
};

void blake2b_compress(uint64_t h[8], const uint8_t block[128], uint64_t t0, uint64_t t1,
                      bool last) {
  const uint64_t* IV = C().IV;
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; ++i) m[i] = load64_le(block + 8 * i);
  for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV[i]; }
  v[12] ^= t0;
  v[13] ^= t1;
  if (last) v[14] = ~v[14];
  auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
    v[a] = v[a] + v[b] + x; v[d] = rotr64(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];     v[b] = rotr64(v[b] ^ v[c], 24);
    v[a] = v[a] + v[b] + y; v[d] = rotr64(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];     v[b] = rotr64(v[b] ^ v[c], 63);
  };
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = kSigma[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

}  // namespace

Sha512::Sha512() { std::memcpy(h, C().IV, sizeof(h)); }
void Sha512::update(const uint8_t* p, size_t n) {
  total += n;
  while (n > 0) {
    size_t take = std::min(n, (size_t)128 - fill);
    std::memcpy(buf + fill, p, take);
    fill += take; p += take; n -= take;
    if (fill == 128) { sha512_compress(h, buf); fill = 0; }
  }
}
void Sha512::final(uint8_t out[64]) {
  uint64_t bits = total * 8;
  uint8_t pad = 0x80;
  update(&pad, 1);
  uint8_t zero = 0;
  while (fill != 112) update(&zero, 1);
  uint8_t len[16] = {0};
  store64_be(len + 8, bits);
  update(len, 16);
  for (int i = 0; i < 8; ++i) store64_be(out + 8 * i, h[i]);
}

void sha512(const uint8_t* in, size_t n, uint8_t out[64]) {
  Sha512 s;
  s.update(in, n);
  s.final(out);
}

void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen, const uint8_t* key,
             size_t keylen) {
  if (outlen == 0 || outlen > 64 || keylen > 64) throw SdaError("blake2b: bad parameters");
  uint64_t h[8];
  std::memcpy(h, C().IV, sizeof(h));
  h[0] ^= 0x01010000ULL ^ ((uint64_t)keylen << 8) ^ (uint64_t)outlen;
  uint8_t block[128];
  uint64_t t = 0;
  size_t fill = 0;
  auto absorb = [&](const uint8_t* p, size_t n) {
    while (n > 0) {
      if (fill == 128) {  // compress only when more data follows
        t += 128;
        blake2b_compress(h, block, t, 0, false);
        fill = 0;
      }
      size_t take = std::min(n, (size_t)128 - fill);
      std::memcpy(block + fill, p, take);
      fill += take; p += take; n -= take;
    }
  };
  if (keylen > 0) {
    uint8_t kb[128] = {0};
    std::memcpy(kb, key, keylen);
    absorb(kb, 128);
  }
  absorb(in, inlen);
  t += fill;
  std::memset(block + fill, 0, 128 - fill);
  blake2b_compress(h, block, t, 0, true);
  uint8_t full[64];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) full[8 * i + j] = (uint8_t)(h[i] >> (8 * j));
  std::memcpy(out, full, outlen);
}

// Exposed for self-tests: derived constants must match the published tables.
uint64_t sha512_round_constant(int i) { return C().K[i]; }
uint64_t sha512_iv(int i) { return C().IV[i]; }

}  // namespace crypto
}  // namespace sda
