// Prime-field helpers and the packed Shamir construction (host side).
//
// The reference delegates packed sharing to the external crate
// threshold-secret-sharing 0.2 (client/src/crypto/sharing/packed_shamir.rs:4-87):
// values [0, s_1..s_k, r_1..r_t] at w_s^0..w_s^(t+k) -> inverse radix-2 FFT ->
// zero-pad -> radix-3 FFT with w_n -> drop point 0; reconstruction by Newton
// interpolation through {1} U {w_n^(i+1)} evaluated at w_s^1..w_s^k
// (threshold-secret-sharing 0.2, used at client/src/crypto/sharing/packed_shamir.rs). Both maps are linear, so we express them as matrices:
//   shares  = M . [s; r]        M: n x (k+t)
//   secrets = L_I . shares_I    L_I: k x |I|   (any |I| >= t+k: clerk dropout)
// computed with Lagrange bases, which also covers parameter sets whose point
// counts are not FFT sizes (e.g. "5-of-8").
#pragma once

#include <cstdint>
#include <vector>

#include "sda/common.hpp"

namespace sda {

uint64_t mod_pow(uint64_t b, uint64_t e, uint64_t p);
uint64_t mod_inv(uint64_t a, uint64_t p);  // p prime
// Rust's truncated remainder (sign of the dividend), as used by the reference.
inline int64_t rust_rem(int64_t a, int64_t m) { return a % m; }
inline uint64_t canon(int64_t a, int64_t m) {
  int64_t r = a % m;
  return (uint64_t)(r < 0 ? r + m : r);
}

struct PackedShamirParams {
  int secret_count = 0;       // k
  int share_count = 0;        // n
  int privacy_threshold = 0;  // t
  int64_t prime = 0;          // p
  int64_t omega_secrets = 0;  // w_s
  int64_t omega_shares = 0;   // w_n

  int reconstruct_limit() const { return privacy_threshold + secret_count; }
  // Throws SdaError(Invalid) when points collide or the field is too large for
  // the 32-bit GPU representation.
  void validate() const;
  // n x (k+t), row-major
  std::vector<uint32_t> share_matrix() const;
  // k x |I|, row-major; `indices` are 0-based clerk indices
  std::vector<uint32_t> lagrange_matrix(const std::vector<int>& indices) const;
  // CPU share / reconstruct through the matrices (randomness supplied)
  std::vector<int64_t> share(const std::vector<int64_t>& secrets,
                             const std::vector<int64_t>& randomness) const;
  std::vector<int64_t> reconstruct(const std::vector<int>& indices,
                                   const std::vector<int64_t>& shares) const;
};

// The well-known parameter sets of threshold-secret-sharing 0.2.
PackedShamirParams pss_4_8_3();
PackedShamirParams pss_4_26_3();
PackedShamirParams pss_155_728_100();
PackedShamirParams pss_155_19682_100();

// Multiplicative order of w modulo p (small orders only; returns 0 if > limit).
uint64_t mult_order(uint64_t w, uint64_t p, uint64_t limit = 1u << 22);

}  // namespace sda
