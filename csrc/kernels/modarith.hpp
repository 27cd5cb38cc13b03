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

SDA_DEV uint32_t mod32(uint32_t w, const ModParams& P) {
  uint32_t q = __umulhi(w, P.mu32);
  uint32_t r = w - q * P.m;
  return r >= P.m ? r - P.m : r;
}
SDA_DEV uint32_t mod64(uint64_t v, const ModParams& P) {
  uint64_t q = __umul64hi(v, P.mu64);
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
// Canonical representative of a signed 32-bit input.
SDA_DEV uint32_t canon_i32(int32_t s, const ModParams& P) {
  if (s >= 0 && (uint32_t)s < P.m) return (uint32_t)s;
  if (s >= 0) return mod32((uint32_t)s, P);
  uint32_t r = mod32((uint32_t)(-(int64_t)s), P);  // |s| mod m
  return r == 0 ? 0 : P.m - r;
}

}  // namespace sdagpu
