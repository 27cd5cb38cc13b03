// Curve25519 host arithmetic: X25519 (RFC 7748) and Ed25519 (RFC 8032) with
// libsodium's key conventions (64-byte secret key = seed || pk).
//
// Reference usage: encryption keypairs `box_::gen_keypair`
// (client/src/crypto/encryption/sodium.rs:95-109) and signing
// `sign::gen_keypair / sign_detached / verify_detached`
// (client/src/crypto/signing/mod.rs:28-132). Curve constants (d, sqrt(-1), the
// base point) are computed at start-up from their definitions.
#include <cstring>
#include <vector>

#include "sda/crypto.hpp"

namespace sda {
namespace crypto {
namespace {

typedef unsigned __int128 u128;
constexpr uint64_t M51 = (1ULL << 51) - 1;

struct fe {
  uint64_t v[5];
};

inline uint64_t load64(const uint8_t* p) {
  uint64_t r = 0;
  for (int i = 7; i >= 0; --i) r = (r << 8) | p[i];
  return r;
}

fe fe_zero() { return fe{{0, 0, 0, 0, 0}}; }
fe fe_one() { return fe{{1, 0, 0, 0, 0}}; }
fe fe_small(uint64_t x) { return fe{{x, 0, 0, 0, 0}}; }

fe fe_frombytes(const uint8_t s[32]) {
  fe h;
  h.v[0] = load64(s) & M51;
  h.v[1] = (load64(s + 6) >> 3) & M51;
  h.v[2] = (load64(s + 12) >> 6) & M51;
  h.v[3] = (load64(s + 19) >> 1) & M51;
  h.v[4] = (load64(s + 24) >> 12) & M51;
  return h;
}

fe fe_carry(fe a) {
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= M51; a.v[0] += 19 * c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  return a;
}

void fe_tobytes(uint8_t s[32], fe h) {
  h = fe_carry(h);
  h = fe_carry(h);
  uint64_t q = (h.v[0] + 19) >> 51;
  q = (h.v[1] + q) >> 51;
  q = (h.v[2] + q) >> 51;
  q = (h.v[3] + q) >> 51;
  q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c;
  c = h.v[0] >> 51; h.v[0] &= M51; h.v[1] += c;
  c = h.v[1] >> 51; h.v[1] &= M51; h.v[2] += c;
  c = h.v[2] >> 51; h.v[2] &= M51; h.v[3] += c;
  c = h.v[3] >> 51; h.v[3] &= M51; h.v[4] += c;
  h.v[4] &= M51;
  uint64_t w0 = h.v[0] | (h.v[1] << 51);
  uint64_t w1 = (h.v[1] >> 13) | (h.v[2] << 38);
  uint64_t w2 = (h.v[2] >> 26) | (h.v[3] << 25);
  uint64_t w3 = (h.v[3] >> 39) | (h.v[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

fe fe_add(const fe& a, const fe& b) {
  fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
  return fe_carry(r);
}
fe fe_sub(const fe& a, const fe& b) {
  // a + 4p - b ; limbs of b are < 2^52 after carry
  fe r;
  r.v[0] = a.v[0] + 0x1FFFFFFFFFFFB4ULL - b.v[0];
  r.v[1] = a.v[1] + 0x1FFFFFFFFFFFFCULL - b.v[1];
  r.v[2] = a.v[2] + 0x1FFFFFFFFFFFFCULL - b.v[2];
  r.v[3] = a.v[3] + 0x1FFFFFFFFFFFFCULL - b.v[3];
  r.v[4] = a.v[4] + 0x1FFFFFFFFFFFFCULL - b.v[4];
  return fe_carry(r);
}
fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

fe fe_mul(const fe& a, const fe& b) {
  const uint64_t b1_19 = b.v[1] * 19, b2_19 = b.v[2] * 19, b3_19 = b.v[3] * 19,
                 b4_19 = b.v[4] * 19;
  u128 r0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4_19 + (u128)a.v[2] * b3_19 +
            (u128)a.v[3] * b2_19 + (u128)a.v[4] * b1_19;
  u128 r1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4_19 +
            (u128)a.v[3] * b3_19 + (u128)a.v[4] * b2_19;
  u128 r2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] +
            (u128)a.v[3] * b4_19 + (u128)a.v[4] * b3_19;
  u128 r3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] +
            (u128)a.v[3] * b.v[0] + (u128)a.v[4] * b4_19;
  u128 r4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] +
            (u128)a.v[3] * b.v[1] + (u128)a.v[4] * b.v[0];
  fe r;
  uint64_t c;
  r.v[0] = (uint64_t)r0 & M51; c = (uint64_t)(r0 >> 51);
  r1 += c; r.v[1] = (uint64_t)r1 & M51; c = (uint64_t)(r1 >> 51);
  r2 += c; r.v[2] = (uint64_t)r2 & M51; c = (uint64_t)(r2 >> 51);
  r3 += c; r.v[3] = (uint64_t)r3 & M51; c = (uint64_t)(r3 >> 51);
  r4 += c; r.v[4] = (uint64_t)r4 & M51; c = (uint64_t)(r4 >> 51);
  r.v[0] += c * 19;
  c = r.v[0] >> 51; r.v[0] &= M51; r.v[1] += c;
  return r;
}
fe fe_sq(const fe& a) { return fe_mul(a, a); }

// a^e for a little-endian 32-byte exponent
fe fe_pow(const fe& a, const uint8_t e[32]) {
  fe r = fe_one();
  for (int i = 255; i >= 0; --i) {
    r = fe_sq(r);
    if ((e[i >> 3] >> (i & 7)) & 1) r = fe_mul(r, a);
  }
  return r;
}
fe fe_invert(const fe& a) {
  uint8_t e[32];
  std::memset(e, 0xff, 32);
  e[0] = 0xeb;  // p - 2 = 2^255 - 21
  e[31] = 0x7f;
  return fe_pow(a, e);
}
fe fe_pow22523(const fe& a) {
  uint8_t e[32];
  std::memset(e, 0xff, 32);
  e[0] = 0xfd;  // 2^252 - 3
  e[31] = 0x0f;
  return fe_pow(a, e);
}
bool fe_iszero(const fe& a) {
  uint8_t s[32];
  fe_tobytes(s, a);
  uint8_t d = 0;
  for (int i = 0; i < 32; ++i) d |= s[i];
  return d == 0;
}
bool fe_isneg(const fe& a) {
  uint8_t s[32];
  fe_tobytes(s, a);
  return s[0] & 1;
}
bool fe_eq(const fe& a, const fe& b) { return fe_iszero(fe_sub(a, b)); }
void fe_cswap(fe& a, fe& b, uint64_t swap) {
  uint64_t mask = 0 - swap;
  for (int i = 0; i < 5; ++i) {
    uint64_t t = mask & (a.v[i] ^ b.v[i]);
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}
fe fe_cmov(const fe& a, const fe& b, uint64_t take_b) {
  uint64_t mask = 0 - take_b;
  fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] ^ (mask & (a.v[i] ^ b.v[i]));
  return r;
}

// ---- Edwards25519 ------------------------------------------------------------
struct ge {
  fe X, Y, Z, T;
};

struct CurveConsts {
  fe d, d2, sqrtm1;
  ge B;
  CurveConsts();
};
const CurveConsts& K();

ge ge_identity() { return ge{fe_zero(), fe_one(), fe_one(), fe_zero()}; }

ge ge_add(const ge& p, const ge& q) {
  const CurveConsts& k = K();
  fe A = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  fe Bv = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  fe C = fe_mul(fe_mul(p.T, k.d2), q.T);
  fe D = fe_mul(fe_add(p.Z, p.Z), q.Z);
  fe E = fe_sub(Bv, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(Bv, A);
  return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
ge ge_dbl(const ge& p) {
  fe A = fe_sq(p.X), Bv = fe_sq(p.Y);
  fe C = fe_sq(p.Z);
  C = fe_add(C, C);
  fe D = fe_neg(A);
  fe E = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), A), Bv);
  fe G = fe_add(D, Bv);
  fe F = fe_sub(G, C);
  fe H = fe_sub(D, Bv);
  return ge{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
ge ge_neg(const ge& p) { return ge{fe_neg(p.X), p.Y, p.Z, fe_neg(p.T)}; }
ge ge_cmov(const ge& a, const ge& b, uint64_t take_b) {
  return ge{fe_cmov(a.X, b.X, take_b), fe_cmov(a.Y, b.Y, take_b), fe_cmov(a.Z, b.Z, take_b),
            fe_cmov(a.T, b.T, take_b)};
}
// Scalar multiplication (double-and-always-add with conditional select).
ge ge_scalarmult(const ge& p, const uint8_t s[32]) {
  ge r = ge_identity();
  for (int i = 255; i >= 0; --i) {
    r = ge_dbl(r);
    ge t = ge_add(r, p);
    r = ge_cmov(r, t, (s[i >> 3] >> (i & 7)) & 1);
  }
  return r;
}
void ge_tobytes(uint8_t s[32], const ge& p) {
  fe zi = fe_invert(p.Z);
  fe x = fe_mul(p.X, zi), y = fe_mul(p.Y, zi);
  fe_tobytes(s, y);
  s[31] ^= (uint8_t)(fe_isneg(x) << 7);
}
bool fe_is_canonical(const uint8_t s[32]) {
  // y < p with the sign bit ignored
  uint8_t t[32];
  std::memcpy(t, s, 32);
  t[31] &= 0x7f;
  fe y = fe_frombytes(t);
  uint8_t back[32];
  fe_tobytes(back, y);
  return std::memcmp(back, t, 32) == 0;
}
bool ge_frombytes(ge& out, const uint8_t s[32]) {
  const CurveConsts& k = K();
  if (!fe_is_canonical(s)) return false;
  fe y = fe_frombytes(s);
  fe y2 = fe_sq(y);
  fe u = fe_sub(y2, fe_one());
  fe v = fe_add(fe_mul(y2, k.d), fe_one());
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe x = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  fe vx2 = fe_mul(v, fe_sq(x));
  if (!fe_eq(vx2, u)) {
    if (fe_eq(vx2, fe_neg(u))) x = fe_mul(x, k.sqrtm1);
    else return false;
  }
  int sign = s[31] >> 7;
  if (fe_iszero(x) && sign) return false;
  if ((int)fe_isneg(x) != sign) x = fe_neg(x);
  out = ge{x, y, fe_one(), fe_mul(x, y)};
  return true;
}
bool ge_is_identity(const ge& p) { return fe_iszero(p.X) && fe_eq(p.Y, p.Z); }
bool ge_has_small_order(const ge& p) {
  ge q = ge_dbl(ge_dbl(ge_dbl(p)));
  return ge_is_identity(q);
}

CurveConsts::CurveConsts() {
  // d = -121665 / 121666
  d = fe_mul(fe_neg(fe_small(121665)), fe_invert(fe_small(121666)));
  d2 = fe_add(d, d);
  // sqrt(-1) = 2^((p-1)/4)
  uint8_t e[32];
  std::memset(e, 0xff, 32);
  e[0] = 0xfb;  // (p-1)/4 = 2^253 - 5
  e[31] = 0x1f;
  sqrtm1 = fe_pow(fe_small(2), e);
  // B: y = 4/5, x even
  fe y = fe_mul(fe_small(4), fe_invert(fe_small(5)));
  uint8_t enc[32];
  fe_tobytes(enc, y);
  ge b;
  // decompression needs d/sqrtm1 already set (done above), so do it inline
  fe y2 = fe_sq(y);
  fe u = fe_sub(y2, fe_one());
  fe v = fe_add(fe_mul(y2, d), fe_one());
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe x = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  if (!fe_eq(fe_mul(v, fe_sq(x)), u)) x = fe_mul(x, sqrtm1);
  if (fe_isneg(x)) x = fe_neg(x);
  b = ge{x, y, fe_one(), fe_mul(x, y)};
  B = b;
}
const CurveConsts& K() {
  static CurveConsts k;
  return k;
}

// ---- scalars mod L -----------------------------------------------------------
// L = 2^252 + 27742317777372353535851937790883648493
const uint64_t kL[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};

bool sc_ge_L(const uint64_t r[4]) {
  for (int i = 3; i >= 0; --i) {
    if (r[i] != kL[i]) return r[i] > kL[i];
  }
  return true;
}
void sc_sub_L(uint64_t r[4]) {
  u128 borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 t = (u128)r[i] - kL[i] - borrow;
    r[i] = (uint64_t)t;
    borrow = (t >> 64) ? 1 : 0;
  }
}
// Reduce a little-endian number of `nbytes` bytes modulo L (bit-serial).
void sc_reduce_bytes(uint8_t out[32], const uint8_t* in, size_t nbytes) {
  uint64_t r[4] = {0, 0, 0, 0};
  for (int bit = (int)(nbytes * 8) - 1; bit >= 0; --bit) {
    // r = 2r + b ; r < L < 2^253 so 2r+1 < 2^254 fits
    r[3] = (r[3] << 1) | (r[2] >> 63);
    r[2] = (r[2] << 1) | (r[1] >> 63);
    r[1] = (r[1] << 1) | (r[0] >> 63);
    r[0] = (r[0] << 1) | ((in[bit >> 3] >> (bit & 7)) & 1);
    if (sc_ge_L(r)) sc_sub_L(r);
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(r[i] >> (8 * j));
}
// out = (a*b + c) mod L
void sc_muladd(uint8_t out[32], const uint8_t a[32], const uint8_t b[32], const uint8_t c[32]) {
  uint64_t A[4], Bv[4], Cv[4];
  for (int i = 0; i < 4; ++i) { A[i] = load64(a + 8 * i); Bv[i] = load64(b + 8 * i); Cv[i] = load64(c + 8 * i); }
  uint64_t prod[9] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 carry = 0;
    for (int j = 0; j < 4; ++j) {
      u128 t = (u128)A[i] * Bv[j] + prod[i + j] + carry;
      prod[i + j] = (uint64_t)t;
      carry = t >> 64;
    }
    prod[i + 4] += (uint64_t)carry;
  }
  u128 carry = 0;
  for (int i = 0; i < 9; ++i) {
    u128 t = (u128)prod[i] + (i < 4 ? Cv[i] : 0) + carry;
    prod[i] = (uint64_t)t;
    carry = t >> 64;
  }
  uint8_t bytes[72];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 8; ++j) bytes[8 * i + j] = (uint8_t)(prod[i] >> (8 * j));
  sc_reduce_bytes(out, bytes, 72);
}
bool sc_is_canonical(const uint8_t s[32]) {
  uint64_t r[4];
  for (int i = 0; i < 4; ++i) r[i] = load64(s + 8 * i);
  return !sc_ge_L(r);
}

}  // namespace

// ---- X25519 ------------------------------------------------------------------
bool x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]) {
  uint8_t k[32];
  std::memcpy(k, scalar, 32);
  k[0] &= 248;
  k[31] &= 127;
  k[31] |= 64;
  uint8_t u[32];
  std::memcpy(u, point, 32);
  u[31] &= 127;
  fe x1 = fe_frombytes(u);
  fe x2 = fe_one(), z2 = fe_zero(), x3 = x1, z3 = fe_one();
  uint64_t swap = 0;
  const fe a24 = fe_small(121665);
  for (int t = 254; t >= 0; --t) {
    uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
    swap ^= kt;
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    swap = kt;
    fe A = fe_add(x2, z2), AA = fe_sq(A);
    fe Bv = fe_sub(x2, z2), BB = fe_sq(Bv);
    fe E = fe_sub(AA, BB);
    fe C = fe_add(x3, z3), D = fe_sub(x3, z3);
    fe DA = fe_mul(D, A), CB = fe_mul(C, Bv);
    x3 = fe_sq(fe_add(DA, CB));
    z3 = fe_mul(x1, fe_sq(fe_sub(DA, CB)));
    x2 = fe_mul(AA, BB);
    z2 = fe_mul(E, fe_add(AA, fe_mul(a24, E)));
  }
  fe_cswap(x2, x3, swap);
  fe_cswap(z2, z3, swap);
  fe_tobytes(out, fe_mul(x2, fe_invert(z2)));
  secure_zero(k, sizeof(k));
  uint8_t d = 0;
  for (int i = 0; i < 32; ++i) d |= out[i];
  return d != 0;
}

void x25519_base(uint8_t out[32], const uint8_t scalar[32]) {
  uint8_t nine[32] = {9};
  x25519(out, scalar, nine);
}

// ---- fixed-base tables for X25519 with a long-lived public key -------------------
// Entry (i, j), i < 32, j < 8, is (j + 1) 256^i P as (y + x, y - x, 2 d x y), 10 limbs of
// 26 / 25 bits each (limb k at bit ceil(25.5 k)), padded to 32 words; word 30 of every
// entry is 1 (a table of zeros marks a key without one). P is the edwards25519 point
// with u = (1 + y) / (1 - y) = the key and even x (either x gives the same X25519
// results). A key on the twist has no such point: false, and callers keep the ladder.
namespace {
void fe_to_limbs10(uint32_t out[10], const fe& v) {
  uint8_t b[32];
  fe_tobytes(b, v);
  int bit = 0;
  for (int k = 0; k < 10; ++k) {
    const int w = (k & 1) ? 25 : 26;
    uint64_t x = 0;
    for (int q = 0; q < 5; ++q) {
      const int idx = (bit >> 3) + q;
      if (idx < 32) x |= (uint64_t)b[idx] << (8 * q);
    }
    out[k] = (uint32_t)((x >> (bit & 7)) & ((1ULL << w) - 1));
    bit += w;
  }
}
}  // namespace

bool x25519_comb_table(uint32_t* out, const uint8_t pk[32]) {
  constexpr int kEntries = 32 * 8, kWords = 32;
  std::memset(out, 0, sizeof(uint32_t) * kEntries * kWords);
  uint8_t ub[32];
  std::memcpy(ub, pk, 32);
  ub[31] &= 127;
  const fe u = fe_frombytes(ub);
  const fe den = fe_add(u, fe_one());
  if (fe_iszero(den)) return false;
  const fe y0 = fe_mul(fe_sub(u, fe_one()), fe_invert(den));
  uint8_t enc[32];
  fe_tobytes(enc, y0);  // sign bit clear: the even x
  ge P;
  if (!ge_frombytes(P, enc)) return false;
  std::vector<ge> rows(kEntries);
  ge base = P;
  for (int i = 0; i < 32; ++i) {
    ge pt = base;
    for (int j = 0; j < 8; ++j) {
      rows[8 * i + j] = pt;
      pt = ge_add(pt, base);
    }
    for (int q = 0; q < 8; ++q) base = ge_dbl(base);
  }
  // one inversion for all 256 denominators
  std::vector<fe> pref(kEntries);
  fe acc = fe_one();
  for (int e = 0; e < kEntries; ++e) {
    pref[e] = acc;
    acc = fe_mul(acc, rows[e].Z);
  }
  fe inv = fe_invert(acc);
  const fe d2 = K().d2;
  for (int e = kEntries - 1; e >= 0; --e) {
    const fe zi = fe_mul(inv, pref[e]);
    inv = fe_mul(inv, rows[e].Z);
    const fe x = fe_mul(rows[e].X, zi), y = fe_mul(rows[e].Y, zi);
    uint32_t* w = out + (size_t)e * kWords;
    fe_to_limbs10(w, fe_add(y, x));
    fe_to_limbs10(w + 10, fe_sub(y, x));
    fe_to_limbs10(w + 20, fe_mul(fe_mul(x, y), d2));
    w[30] = 1;
  }
  return true;
}

// ---- Ed25519 -----------------------------------------------------------------
void ed25519_keypair_from_seed(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]) {
  uint8_t h[64];
  sha512(seed, 32, h);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  ge A = ge_scalarmult(K().B, h);
  ge_tobytes(pk, A);
  std::memcpy(sk, seed, 32);
  std::memcpy(sk + 32, pk, 32);
  secure_zero(h, sizeof(h));
}

void ed25519_keypair(uint8_t pk[32], uint8_t sk[64]) {
  uint8_t seed[32];
  os_random(seed, 32);
  ed25519_keypair_from_seed(pk, sk, seed);
  secure_zero(seed, sizeof(seed));
}

void ed25519_sign(uint8_t sig[64], const uint8_t* msg, size_t n, const uint8_t sk[64]) {
  uint8_t h[64];
  sha512(sk, 32, h);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  uint8_t rh[64], r[32];
  Sha512 s1;
  s1.update(h + 32, 32);
  s1.update(msg, n);
  s1.final(rh);
  sc_reduce_bytes(r, rh, 64);
  ge R = ge_scalarmult(K().B, r);
  ge_tobytes(sig, R);
  uint8_t kh[64], k[32];
  Sha512 s2;
  s2.update(sig, 32);
  s2.update(sk + 32, 32);
  s2.update(msg, n);
  s2.final(kh);
  sc_reduce_bytes(k, kh, 64);
  sc_muladd(sig + 32, k, h, r);
  secure_zero(h, sizeof(h));
  secure_zero(r, sizeof(r));
}

bool ed25519_verify(const uint8_t sig[64], const uint8_t* msg, size_t n, const uint8_t pk[32]) {
  if (!sc_is_canonical(sig + 32)) return false;
  ge A, R;
  if (!ge_frombytes(A, pk)) return false;
  if (!ge_frombytes(R, sig)) return false;
  if (ge_has_small_order(A) || ge_has_small_order(R)) return false;
  uint8_t kh[64], k[32];
  Sha512 s;
  s.update(sig, 32);
  s.update(pk, 32);
  s.update(msg, n);
  s.final(kh);
  sc_reduce_bytes(k, kh, 64);
  ge sB = ge_scalarmult(K().B, sig + 32);
  ge kA = ge_scalarmult(A, k);
  ge Rp = ge_add(sB, ge_neg(kA));
  uint8_t enc[32];
  ge_tobytes(enc, Rp);
  return std::memcmp(enc, sig, 32) == 0;
}

}  // namespace crypto
}  // namespace sda
