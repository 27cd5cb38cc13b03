// Host (CPU) cryptographic primitives, written from the public specifications.
//
// These are the wire-compatible building blocks of the reference's libsodium
// usage (client/src/crypto/encryption/sodium.rs:36-117,
// client/src/crypto/signing/mod.rs:28-132, client/src/crypto/masking/chacha.rs):
//   * X25519 (RFC 7748), Ed25519 (RFC 8032, libsodium 64-byte secret keys)
//   * Salsa20 / HSalsa20 / XSalsa20, Poly1305 (RFC 8439 MAC), BLAKE2b (RFC 7693)
//   * crypto_box_seal / crypto_box_seal_open (libsodium sealed boxes)
//   * ChaCha20 and a rand-0.3 compatible `ChaChaRng` for the ChaCha mask scheme
//
// They double as the bit-exact oracle for the HIP kernels in csrc/kernels.
#pragma once

#include <array>
#include <cstdint>
#include <string>

#include "sda/common.hpp"

namespace sda {
namespace crypto {

// ---- OS entropy ------------------------------------------------------------
void os_random(uint8_t* out, size_t n);
uint32_t os_random_u32();
uint64_t os_random_u64();
// Uniform in [0, m) from OS entropy (exact rejection sampling).
int64_t os_random_range(int64_t m);

// ---- hashes ----------------------------------------------------------------
void sha512(const uint8_t* in, size_t n, uint8_t out[64]);
struct Sha512 {
  uint64_t h[8];
  uint8_t buf[128];
  uint64_t total = 0;
  size_t fill = 0;
  Sha512();
  void update(const uint8_t* p, size_t n);
  void final(uint8_t out[64]);
};

// BLAKE2b with variable output length (1..64) and optional key (0..64 bytes).
void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen,
             const uint8_t* key = nullptr, size_t keylen = 0);

// ---- Salsa20 family --------------------------------------------------------
// Salsa20/20 core: out = 64-byte block for (key, nonce8, counter)
void salsa20_block(uint8_t out[64], const uint8_t key[32], const uint8_t nonce[8],
                   uint64_t counter);
// HSalsa20: 32-byte subkey from a 32-byte key and 16-byte input.
void hsalsa20(uint8_t out[32], const uint8_t key[32], const uint8_t in16[16]);
// XOR `n` bytes with the XSalsa20 keystream starting at byte offset `ofs`.
void xsalsa20_xor(uint8_t* out, const uint8_t* in, size_t n, const uint8_t nonce[24],
                  const uint8_t key[32], uint64_t ofs = 0);

// ---- ChaCha20 --------------------------------------------------------------
// Raw ChaCha20 block with the state words given directly (16 x u32 input).
void chacha20_block_words(uint32_t out[16], const uint32_t in[16], int rounds = 20);

// rand 0.3 `ChaChaRng` (client/src/crypto/masking/chacha.rs:29-39): key = seed words (zero-filled to 8),
// 128-bit counter in state words 12..15 starting at 0, 20 rounds.
class ChaChaRng {
 public:
  explicit ChaChaRng(const uint32_t* seed, size_t nwords);
  uint32_t next_u32();
  uint64_t next_u64();  // high word first (rand 0.3 default next_u64)
  // rand 0.3 gen_range(low, high) for i64: rejection zone on u64
  int64_t gen_range(int64_t low, int64_t high);

 private:
  void refill();
  uint32_t state_[16];
  uint32_t buf_[16];
  int index_;
};

// Test hook: cap the acceptance zone of ChaChaRng::gen_range (draws at or above
// cap - cap % range are rejected), so that rejections -- at most 1e-10 per draw for
// 31-bit moduli -- can be made frequent; the device kernels have the same hook
// (kernels.hpp). UINT64_MAX = no cap. Process-wide.
void set_chacha_zone_cap(uint64_t cap);

// ---- Poly1305 --------------------------------------------------------------
void poly1305(uint8_t tag[16], const uint8_t* msg, size_t n, const uint8_t key[32]);
bool verify16(const uint8_t a[16], const uint8_t b[16]);

// ---- Curve25519 ------------------------------------------------------------
// Returns false when the result is all-zero (libsodium crypto_scalarmult -1).
bool x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t point[32]);
void x25519_base(uint8_t out[32], const uint8_t scalar[32]);
// Fixed-base table of a long-lived X25519 public key for the GPU key agreement
// (csrc/kernels/device_crypto.hpp, x25519_base_nd): 32 x 8 entries of 32 words. False
// (and a table of zeros) for a key on the twist, which has no edwards25519 point.
constexpr size_t kX25519CombTableWords = 32 * 8 * 32;
bool x25519_comb_table(uint32_t* out, const uint8_t pk[32]);

// ---- Ed25519 (libsodium conventions: sk = seed || pk) ----------------------
void ed25519_keypair_from_seed(uint8_t pk[32], uint8_t sk[64], const uint8_t seed[32]);
void ed25519_keypair(uint8_t pk[32], uint8_t sk[64]);
void ed25519_sign(uint8_t sig[64], const uint8_t* msg, size_t n, const uint8_t sk[64]);
bool ed25519_verify(const uint8_t sig[64], const uint8_t* msg, size_t n, const uint8_t pk[32]);

// ---- crypto_box / sealed boxes (libsodium) ---------------------------------
constexpr size_t kBoxPublicKeyBytes = 32;
constexpr size_t kBoxSecretKeyBytes = 32;
constexpr size_t kBoxMacBytes = 16;
constexpr size_t kSealBytes = 48;  // epk || mac

void box_keypair(uint8_t pk[32], uint8_t sk[32]);
// crypto_box_beforenm: k = HSalsa20(X25519(sk, pk), 0). Returns false on an
// all-zero shared secret.
bool box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32]);
// crypto_secretbox_easy with precomputed key: out = mac || ct (n + 16 bytes).
void secretbox_easy(uint8_t* out, const uint8_t* m, size_t n, const uint8_t nonce[24],
                    const uint8_t k[32]);
bool secretbox_open_easy(uint8_t* out, const uint8_t* c, size_t n, const uint8_t nonce[24],
                         const uint8_t k[32]);
// nonce = BLAKE2b-192(epk || pk)
void seal_nonce(uint8_t nonce[24], const uint8_t epk[32], const uint8_t pk[32]);
// crypto_box_seal: out = epk || mac || ct (n + 48 bytes). `esk` optional fixed
// ephemeral secret (tests / deterministic GPU-vs-CPU checks); null = random.
Bytes box_seal(const uint8_t* m, size_t n, const uint8_t pk[32], const uint8_t* esk = nullptr);
// Returns false on authentication failure.
bool box_seal_open(Bytes& out, const uint8_t* c, size_t n, const uint8_t pk[32],
                   const uint8_t sk[32]);

}  // namespace crypto
}  // namespace sda
