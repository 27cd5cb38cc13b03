// Modular arithmetic helpers for canonical field values (modulus < 2^31).
//
// The reference keeps everything in i64 with Rust's truncated `%`
// (client/src/crypto/sharing/additive.rs:37-48); on the GPU we keep canonical
// representatives in [0, m) in 32-bit lanes and use Barrett reductions instead
// of the multi-instruction integer divide.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_crypto.hpp"

namespace sdagpu {

struct ModParams {
  uint32_t m;       // modulus (0 = "no modulus": raw u32 values)
  uint32_t mu32;    // floor((2^32 - 1) / m)
  uint64_t mu64;    // floor((2^64 - 1) / m)
  uint64_t zone32;  // accept a u32 draw w iff w < zone32   (2^32 - 2^32 % m)
  uint64_t zone64;  // rand-0.3 u64 zone: u64::MAX - u64::MAX % m
};

inline ModParams make_mod_params(uint32_t m) {
  ModParams p{};
  p.m = m;
  if (m == 0) return p;
  p.mu32 = (uint32_t)(0xffffffffu / m);
  p.mu64 = 0xffffffffffffffffULL / m;
  p.zone32 = 0x100000000ULL - (0x100000000ULL % m);
  p.zone64 = 0xffffffffffffffffULL - (0xffffffffffffffffULL % m);
  return p;
}

// High halves of the products: the device instructions, or plain C for the host runs
// of the device algorithms (host_emul.cpp).
SDA_DEV uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}
SDA_DEV uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
SDA_DEV uint32_t mod32(uint32_t w, const ModParams& P) {
  uint32_t q = mulhi32(w, P.mu32);
  uint32_t r = w - q * P.m;
  return r >= P.m ? r - P.m : r;
}
// Exact reduction of small sums on the full-rate 24-bit multipliers (mod32's 32-bit
// multiplies run at a quarter of the rate): for w <= wmax,
//   q = ((w << k) * c) >> 32 = floor(w / m),  c = ceil(2^(32 - k) / m),
// whenever c < 2^24, (wmax << k) < 2^24 and wmax * m < 2^(32 - k) (then the excess
// of c over 2^(32-k)/m, below 1, moves w c / 2^(32-k) by less than 1/m).
struct Mod24 {
  uint32_t k, c, m;  // c == 0: no valid (k, c) for this modulus and bound
};
inline Mod24 make_mod24(uint32_t m, uint64_t wmax) {
  for (uint32_t k = 0; k <= 8; ++k) {
    const uint64_t pw = 1ull << (32 - k);
    const uint64_t c = (pw + m - 1) / m;
    if (c < (1u << 24) && (wmax << k) < (1u << 24) && wmax * m < pw) return Mod24{k, (uint32_t)c, m};
  }
  return Mod24{0, 0, m};
}
SDA_DEV uint32_t mod24(uint32_t w, const Mod24& P) {
  const uint32_t q = (uint32_t)(((uint64_t)((w << P.k) & 0xffffffu) * (uint64_t)(P.c & 0xffffffu)) >> 32);
  return w - (q & 0xffffffu) * (P.m & 0xffffffu);  // q, m < 2^24: a 24-bit multiply-subtract
}
// Exact reduction of an integer 0 <= v < 2^53 through the double-precision unit (full
// rate on this chip, like the 32-bit integer multiplies), for m >= 16. `inv` is 1/m
// scaled down by 2^-50: with the three roundings on the way (1/m, the scaling, the
// product; 2^-53 each) v * inv lies in (v/m (1 - 11 2^-53), v/m), so q = trunc(v * inv)
// is floor(v / m) or one less (v/m 11 2^-53 < 1), never more; v - q m, exact in one
// fused multiply-add, is in [0, 2m) and one conditional subtraction finishes. Seven
// instructions, whatever v's size -- a 64-bit Barrett step (mod64) takes about thirty.
struct ModF64 {
  double m, inv;
  double off, w4;  // the signed-limb fold of the modular GEMM: a multiple of m above its sums, 2^32 mod m
};
inline ModF64 make_modf64(uint32_t m) {
  return ModF64{(double)m, m ? (1.0 / (double)m) * (1.0 - 0x1p-50) : 0.0, 0.0, 0.0};
}
// The same for the modular GEMM's signed-limb fold (three signed base-256 limbs, K-sums
// of up to Kp products): |sum_d acc_d w_d| <= Kp 128^2 (w4 + 2 2^24 + 3 2^16 + 2 2^8 + 1)
// with w4 = 2^32 mod m; `off`, the next multiple of m, lifts the sum to [0, 2^53) for
// Kp <= 4096 and m < 2^24.
inline ModF64 make_modf64_signed(uint32_t m, int Kp) {
  ModF64 P = make_modf64(m);
  const uint64_t w4 = (1ull << 32) % m;
  const uint64_t bound = (uint64_t)Kp * 16384 * (w4 + (2ull << 24) + (3ull << 16) + (2ull << 8) + 1);
  P.off = (double)((bound + m - 1) / m * m);
  P.w4 = (double)w4;
  return P;
}
// v given as a double (an exact integer below 2^53)
SDA_DEV uint32_t modf64d(double vd, const ModF64& P) {
  const double q = __builtin_trunc(vd * P.inv);
  const uint32_t r = (uint32_t)__builtin_fma(-q, P.m, vd);  // in [0, 2m)
  const uint32_t t = r - (uint32_t)P.m;                     // wraps above r when r < m
  return t < r ? t : r;
}
SDA_DEV uint32_t modf64(uint64_t v, const ModF64& P) { return modf64d((double)(int64_t)v, P); }
SDA_DEV uint32_t mod64(uint64_t v, const ModParams& P) {
  uint64_t q = mulhi64(v, P.mu64);
  uint64_t r = v - q * (uint64_t)P.m;  // q >= floor(v/m) - 2
  r = r >= P.m ? r - P.m : r;
  r = r >= P.m ? r - P.m : r;
  return (uint32_t)r;
}
SDA_DEV uint32_t add_mod(uint32_t a, uint32_t b, uint32_t m) {
  uint32_t s = a + b;  // a, b < m < 2^31: no overflow
  return s >= m ? s - m : s;
}
SDA_DEV uint32_t sub_mod(uint32_t a, uint32_t b, uint32_t m) {
  return a >= b ? a - b : a + m - b;
}
// Zigzag-LEB128 codes of a pair of u16 values, both below 2^13 (codes of one or
// two bytes; zigzag of a non-negative v is z = 2 v), computed on both halves of
// the dword at once: half h of `codes` = byte 0 (low 7 bits of z, bit 7 = "a second
// byte follows") | byte 1 (z >> 7) << 8, and bit 16 h of `two` = the value needs
// two bytes (v >= 64). No step carries from the low half into the high one.
SDA_DEV void varint_pair16(uint32_t p, uint32_t& codes, uint32_t& two) {
  two = ((p + 0x7fc07fc0u) >> 15) & 0x00010001u;
  const uint32_t z2 = p << 1;
  codes = (z2 & 0x007f007fu) | ((z2 << 1) & 0x7f007f00u) | (two << 7);
}
// Canonical representative of a signed 32-bit input.
SDA_DEV uint32_t canon_i32(int32_t s, const ModParams& P) {
  if (s >= 0 && (uint32_t)s < P.m) return (uint32_t)s;
  if (s >= 0) return mod32((uint32_t)s, P);
  uint32_t r = mod32((uint32_t)(-(int64_t)s), P);  // |s| mod m
  return r == 0 ? 0 : P.m - r;
}

}  // namespace sdagpu
