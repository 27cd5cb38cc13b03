// libsodium-compatible crypto_box / crypto_box_seal and OS entropy.
//
// Sealed box layout (reference: client/src/crypto/encryption/sodium.rs:43,78 ->
// sodiumoxide::crypto::sealedbox): epk(32) || mac(16) || ct, with
// nonce = BLAKE2b-192(epk || pk), k = HSalsa20(X25519(esk, pk), 0^16), and the
// XSalsa20-Poly1305 secretbox convention (Poly1305 key = keystream bytes 0..31,
// message XORed from keystream offset 32).
#include <sys/random.h>

#include <cerrno>
#include <cstring>

#include "sda/crypto.hpp"

namespace sda {

Bytes from_hex(const std::string& s) {
  auto nib = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    throw SdaError("invalid hex digit");
  };
  if (s.size() % 2) throw SdaError("odd hex length");
  Bytes out(s.size() / 2);
  for (size_t i = 0; i < out.size(); ++i) out[i] = (uint8_t)(nib(s[2 * i]) << 4 | nib(s[2 * i + 1]));
  return out;
}

void secure_zero(void* p, size_t n) {
  volatile uint8_t* v = static_cast<volatile uint8_t*>(p);
  while (n--) *v++ = 0;
}

namespace crypto {

void os_random(uint8_t* out, size_t n) {
  size_t done = 0;
  while (done < n) {
    ssize_t r = getrandom(out + done, n - done, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw SdaError("getrandom failed");
    }
    done += (size_t)r;
  }
}
uint32_t os_random_u32() {
  uint32_t v;
  os_random(reinterpret_cast<uint8_t*>(&v), sizeof(v));
  return v;
}
uint64_t os_random_u64() {
  uint64_t v;
  os_random(reinterpret_cast<uint8_t*>(&v), sizeof(v));
  return v;
}
int64_t os_random_range(int64_t m) {
  if (m <= 0) throw SdaError("os_random_range: modulus must be positive");
  uint64_t range = (uint64_t)m;
  uint64_t zone = UINT64_MAX - UINT64_MAX % range;
  for (;;) {
    uint64_t v = os_random_u64();
    if (v < zone) return (int64_t)(v % range);
  }
}

void box_keypair(uint8_t pk[32], uint8_t sk[32]) {
  os_random(sk, 32);
  x25519_base(pk, sk);
}

bool box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32]) {
  uint8_t s[32];
  bool ok = x25519(s, sk, pk);
  const uint8_t zero16[16] = {0};
  hsalsa20(k, s, zero16);
  secure_zero(s, sizeof(s));
  return ok;
}

void secretbox_easy(uint8_t* out, const uint8_t* m, size_t n, const uint8_t nonce[24],
                    const uint8_t k[32]) {
  uint8_t subkey[32];
  hsalsa20(subkey, k, nonce);
  uint8_t block0[64];
  salsa20_block(block0, subkey, nonce + 16, 0);
  // ciphertext = m XOR keystream[32..]
  xsalsa20_xor(out + 16, m, n, nonce, k, 32);
  poly1305(out, out + 16, n, block0);
  secure_zero(subkey, sizeof(subkey));
  secure_zero(block0, sizeof(block0));
}

bool secretbox_open_easy(uint8_t* out, const uint8_t* c, size_t n, const uint8_t nonce[24],
                         const uint8_t k[32]) {
  if (n < 16) return false;
  uint8_t subkey[32];
  hsalsa20(subkey, k, nonce);
  uint8_t block0[64];
  salsa20_block(block0, subkey, nonce + 16, 0);
  uint8_t tag[16];
  poly1305(tag, c + 16, n - 16, block0);
  secure_zero(subkey, sizeof(subkey));
  secure_zero(block0, sizeof(block0));
  if (!verify16(tag, c)) return false;
  xsalsa20_xor(out, c + 16, n - 16, nonce, k, 32);
  return true;
}

void seal_nonce(uint8_t nonce[24], const uint8_t epk[32], const uint8_t pk[32]) {
  uint8_t in[64];
  std::memcpy(in, epk, 32);
  std::memcpy(in + 32, pk, 32);
  blake2b(nonce, 24, in, 64);
}

Bytes box_seal(const uint8_t* m, size_t n, const uint8_t pk[32], const uint8_t* esk_in) {
  uint8_t epk[32], esk[32];
  if (esk_in) {
    std::memcpy(esk, esk_in, 32);
    x25519_base(epk, esk);
  } else {
    box_keypair(epk, esk);
  }
  uint8_t nonce[24], k[32];
  seal_nonce(nonce, epk, pk);
  if (!box_beforenm(k, pk, esk)) throw SdaError("box_seal: invalid public key");
  Bytes out(n + kSealBytes);
  std::memcpy(out.data(), epk, 32);
  secretbox_easy(out.data() + 32, m, n, nonce, k);
  secure_zero(esk, sizeof(esk));
  secure_zero(k, sizeof(k));
  return out;
}

bool box_seal_open(Bytes& out, const uint8_t* c, size_t n, const uint8_t pk[32],
                   const uint8_t sk[32]) {
  if (n < kSealBytes) return false;
  uint8_t nonce[24], k[32];
  seal_nonce(nonce, c, pk);
  if (!box_beforenm(k, c, sk)) return false;
  out.assign(n - kSealBytes, 0);
  bool ok = secretbox_open_easy(out.data(), c + 32, n - 32, nonce, k);
  secure_zero(k, sizeof(k));
  if (!ok) out.clear();
  return ok;
}

}  // namespace crypto
}  // namespace sda
