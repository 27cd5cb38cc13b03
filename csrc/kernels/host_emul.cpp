// Host emulation of the device sealed-box algorithms (debug / CI self-test).
//
// Runs the __host__ __device__ primitives of device_crypto.hpp and a lane-by-lane
// emulation of k_mac_chunks / k_mac_final / k_encode_encrypt against the host
// oracle (csrc/src/crypto_*.cc), so algorithm bugs are found without a GPU.
// Build: make emul ; run: build/hip/host_emul
#include <cstdio>
#include <cstring>
#include <vector>

#include "decode_core.hpp"
#include "device_crypto.hpp"
#include "encode_units.hpp"
#include "kernels.hpp"
#include "modarith.hpp"
#include "sda/crypto.hpp"

using namespace sdagpu;
namespace hc = sda::crypto;

static int failures = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);                  \
      std::printf("\n");                         \
      ++failures;                                \
    }                                            \
  } while (0)

static void words(uint32_t* w, const uint8_t* b, int n) {
  for (int i = 0; i < n; ++i) w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}
static void bytes(uint8_t* b, const uint32_t* w, int n) {
  for (int i = 0; i < n; ++i) for (int k = 0; k < 4; ++k) b[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
}

// emulate derive_msg_key from keys.hip
static MsgKey derive(const uint32_t (&shared)[8], const uint32_t (&epk)[8], const uint32_t (&pk)[8]) {
  const uint32_t zero4[4] = {0, 0, 0, 0};
  uint32_t k[8];
  hsalsa20(k, shared, zero4);
  uint32_t msg[16];
  for (int i = 0; i < 8; ++i) { msg[i] = epk[i]; msg[8 + i] = pk[i]; }
  uint32_t nonce[6];
  blake2b_192_64(nonce, msg);
  const uint32_t n4[4] = {nonce[0], nonce[1], nonce[2], nonce[3]};
  uint32_t sub[8];
  hsalsa20(sub, k, n4);
  uint32_t b0[16];
  salsa20_block(b0, sub, nonce[4], nonce[5], 0);
  MsgKey out{};
  for (int i = 0; i < 8; ++i) out.subkey[i] = sub[i];
  out.nonce[0] = nonce[4];
  out.nonce[1] = nonce[5];
  for (int i = 0; i < 4; ++i) { out.poly_r[i] = b0[i]; out.poly_s[i] = b0[4 + i]; }
  return out;
}

static P130 load_block(const uint8_t* lds, int64_t i, int64_t kC, uint32_t N) {
  const int64_t off = 32 + 16 * i - kC;
  uint32_t w[4];
  std::memcpy(w, lds + off, 16);
  uint32_t hibit = 1u << 24;
  const int64_t rem = (int64_t)N - 16 * i;
  if (rem < 16) {
    for (int b = 0; b < 16; ++b) {
      const int wi = b >> 2, sh = (b & 3) * 8;
      uint32_t byte = (w[wi] >> sh) & 0xff;
      uint32_t nb = b < rem ? byte : (b == rem ? 1u : 0u);
      w[wi] = (w[wi] & ~(0xffu << sh)) | (nb << sh);
    }
    hibit = 0;
  }
  return p130_block(w[0], w[1], w[2], w[3], hibit);
}

// emulate k_mac_chunks<0> + k_mac_final over the ciphertext `ct` (N bytes)
static void emul_mac(uint32_t (&tag)[4], const MsgKey& key, const uint8_t* ctbytes, uint32_t N) {
  const int C = kChunkBytes;
  const int K = (int)(((int64_t)N + 32 + C - 1) / C);
  std::vector<P130> parts(K);
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  for (int k = 0; k < K; ++k) {
    std::vector<uint8_t> buf(C, 0xAA);
    const int64_t kC = (int64_t)k * C;
    const int64_t start = kC >= 32 ? kC - 32 : 0;
    const int64_t end = std::min((int64_t)N, kC + C - 32);
    if (start >= end) { parts[k] = p130_zero(); continue; }
    for (int64_t pos = start; pos < end; ++pos) buf[pos - (kC - 32)] = ctbytes[pos];
    const int64_t fb = start / 16, eb = (end + 15) / 16;
    std::vector<P130> h(256);
    for (int tid = 0; tid < 256; ++tid) {
      P130 hh = p130_zero();
      for (int q = 0; q < 4; ++q) {
        const int64_t i = eb - 4 * (int64_t)(256 - tid) + q;
        P130 c = p130_zero();
        if (i >= fb) c = load_block(buf.data(), i, kC, N);
        hh = p130_mul(p130_add(hh, c), r);
      }
      h[tid] = hh;
    }
    P130 R = p130_mul(r, r);
    R = p130_mul(R, R);
    for (int l = 0; l < 8; ++l) {
      const int s = 1 << l;
      std::vector<P130> tree = h;
      for (int tid = 0; tid < 256; ++tid)
        if ((tid & (2 * s - 1)) == 2 * s - 1) h[tid] = p130_carry(p130_add(p130_mul(tree[tid - s], R), h[tid]));
      R = p130_mul(R, R);
    }
    parts[k] = h[255];
  }
  const P130 rC = p130_pow(r, C / 16);
  P130 H = p130_zero();
  int64_t prev = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t e = (k < K - 1) ? ((int64_t)(k + 1) * C - 32) / 16 : ((int64_t)N + 15) / 16;
    if (k == 0) H = parts[k];
    else {
      const int64_t d = e - prev;
      const P130 Rd = (d == C / 16) ? rC : p130_pow(r, (uint32_t)d);
      H = p130_carry(p130_add(p130_mul(H, Rd), parts[k]));
    }
    prev = e;
  }
  const uint32_t s4[4] = {key.poly_s[0], key.poly_s[1], key.poly_s[2], key.poly_s[3]};
  p130_finish(tag, H, s4);
}

static P130 carry64(uint64_t (&d)[5]) {
  uint64_t c;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  c = d[1] >> 26; d[1] &= kM26; d[2] += c;
  c = d[2] >> 26; d[2] &= kM26; d[3] += c;
  c = d[3] >> 26; d[3] &= kM26; d[4] += c;
  c = d[4] >> 26; d[4] &= kM26; d[0] += c * 5;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  return P130{{(uint32_t)d[0], (uint32_t)d[1], (uint32_t)d[2], (uint32_t)d[3], (uint32_t)d[4]}};
}

// the tables of k_poly_powers (layout: kernels.hpp)
static std::vector<uint32_t> emul_tables(const P130& r) {
  std::vector<uint32_t> pw(kPowWords, 0);
  P130 r4 = p130_mul(r, r);
  r4 = p130_mul(r4, r4);
  for (int t = 0; t < 256; ++t) {
    const P130 f = p130_carry(p130_pow(r4, (uint32_t)(255 - t)));
    for (int u = 0; u < 5; ++u) pw[t * 5 + u] = f.v[u];
  }
  P130 r16 = p130_mul(r4, r4);
  r16 = p130_mul(r16, r16);
  std::vector<P130> rp(64);
  for (int t = 0; t < 64; ++t) rp[t] = p130_carry(p130_pow(r16, (uint32_t)(63 - t)));
  int8_t* tab = reinterpret_cast<int8_t*>(pw.data() + kPowTabOff);
  uint64_t sw[5] = {0, 0, 0, 0, 0};
  for (int pos = 0; pos < kSegBytes; ++pos) {
    const P130 w = poly_weight(rp[pos / 16], pos % 16);
    for (int u = 0; u < 5; ++u) sw[u] += w.v[u];
    for (int d = 0; d < kPolyDigits; ++d) tab[d * kSegBytes + pos] = (int8_t)p130_digit7(w, d);
  }
  const P130 koff = poly_kseg(p130_zero(), carry64(sw));
  for (int u = 0; u < 5; ++u) pw[kPowKsegOff + u] = koff.v[u];
  for (int i = 0; i < 16; ++i) {
    const P130 f = p130_carry(p130_pow(r, (uint32_t)(16 - i)));
    for (int u = 0; u < 5; ++u) pw[kPowRowOff + i * 5 + u] = f.v[u];
  }
  for (int T = 0; T <= 64; ++T) {
    uint64_t d[5] = {0, 0, 0, 0, 0};
    for (int q = 0; q < T; ++q)
      for (int u = 0; u < 5; ++u) d[u] += rp[q].v[u];
    const P130 q128 = p130_carry(p130_mul(carry64(d), p130_bit(128)));
    for (int u = 0; u < 5; ++u) pw[kPowQOff + T * 5 + u] = q128.v[u];
  }
  return pw;
}

// emulate k_poly_powers tables + k_mac_horner (first / last chunk) + the matrix-core
// k_mac_chunks<0> (middle chunks as 16 interleaved rows; the MFMA is an explicit
// integer dot product) + k_mac_final
static void emul_mac_mfma(uint32_t (&tag)[4], const MsgKey& key, const uint8_t* ctbytes, uint32_t N) {
  const int C = kChunkBytes;
  const int K = (int)(((int64_t)N + 32 + C - 1) / C);
  const int last = (int)(((int64_t)N + 31) / C);
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  const std::vector<uint32_t> pw = emul_tables(r);
  const int8_t* tab = reinterpret_cast<const int8_t*>(pw.data() + kPowTabOff);
  std::vector<P130> parts(K);
  for (int k = 0; k < K; ++k) {
    std::vector<uint8_t> buf(C, 0xAA);
    const int64_t kC = (int64_t)k * C;
    const int64_t start = kC >= 32 ? kC - 32 : 0;
    const int64_t end = std::min((int64_t)N, kC + C - 32);
    if (start >= end) { parts[k] = p130_zero(); continue; }
    for (int64_t pos = start; pos < end; ++pos) buf[pos - (kC - 32)] = ctbytes[pos];
    const int64_t fb = start / 16, eb = (end + 15) / 16;
    uint64_t d[5] = {0, 0, 0, 0, 0};
    if (k != 0 && k != last) {  // middle: 16 "MFMA" rows
      for (int i = 0; i < 16; ++i) {
        int32_t c[kPolyDigits];
        for (int dd = 0; dd < kPolyDigits; ++dd) {
          int32_t acc = 0;
          for (int t = 0; t < 64; ++t)
            for (int b = 0; b < 16; ++b)
              acc += (int32_t)(int8_t)(buf[16 * (i + 16 * t) + b] ^ 0x80) * tab[dd * kSegBytes + 16 * t + b];
          c[dd] = acc;
        }
        P130 kseg;
        for (int u = 0; u < 5; ++u) kseg.v[u] = pw[kPowKsegOff + u] + pw[kPowQOff + 64 * 5 + u];
        const uint32_t* rf = pw.data() + kPowRowOff + i * 5;
        const P130 h = p130_mul(poly_seg_value(c, p130_carry(kseg)), P130{{rf[0], rf[1], rf[2], rf[3], rf[4]}});
        for (int u = 0; u < 5; ++u) d[u] += h.v[u];
      }
    } else {  // k_mac_horner: lane t sums the 4 blocks ending 4 (255 - t) blocks before eb
      for (int tid = 0; tid < 256; ++tid) {
        P130 hh = p130_zero();
        for (int q = 0; q < 4; ++q) {
          const int64_t i = eb - 4 * (int64_t)(256 - tid) + q;
          P130 cb = p130_zero();
          if (i >= fb) cb = load_block(buf.data(), i, kC, N);
          hh = p130_mul(p130_add(hh, cb), r);
        }
        const uint32_t* pf = pw.data() + tid * 5;
        hh = p130_mul(hh, P130{{pf[0], pf[1], pf[2], pf[3], pf[4]}});
        for (int u = 0; u < 5; ++u) d[u] += hh.v[u];
      }
    }
    parts[k] = carry64(d);
  }
  const P130 rC = p130_pow(r, C / 16);
  P130 H = p130_zero();
  int64_t prev = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t e = (k < K - 1) ? ((int64_t)(k + 1) * C - 32) / 16 : ((int64_t)N + 15) / 16;
    if (k == 0) H = parts[k];
    else {
      const int64_t dd = e - prev;
      const P130 Rd = (dd == C / 16) ? rC : p130_pow(r, (uint32_t)dd);
      H = p130_carry(p130_add(p130_mul(H, Rd), parts[k]));
    }
    prev = e;
  }
  const uint32_t s4[4] = {key.poly_s[0], key.poly_s[1], key.poly_s[2], key.poly_s[3]};
  p130_finish(tag, H, s4);
}

// emulate the seal-side MAC that k_encode_encrypt computes per tile (interleaved
// rows cut by the tile borders), k_mac_horner for the first
// and last chunk (by the definition of a chunk partial) and k_mac_final. `cuts` are
// the tile borders (message byte offsets, ascending, first 0, last N).
static void emul_mac_fused(uint32_t (&tag)[4], const MsgKey& key, const uint8_t* ctbytes, uint32_t N,
                           const std::vector<uint32_t>& cuts) {
  const int C = kChunkBytes;
  const int K = (int)(((int64_t)N + 32 + C - 1) / C);
  const int last = (int)(((int64_t)N + 31) / C);
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  const std::vector<uint32_t> pw = emul_tables(r);
  const int8_t* tab = reinterpret_cast<const int8_t*>(pw.data() + kPowTabOff);
  // ---- tiles
  std::vector<uint32_t> partials((size_t)K * 8, 0);
  for (size_t ti = 0; ti + 1 < cuts.size(); ++ti) {
    const uint32_t a = cuts[ti], tile_bytes = cuts[ti + 1] - cuts[ti];
    if (tile_bytes == 0) continue;
    const uint32_t b0 = (32u + a) >> 6, base = 32u + a - 64u * b0;
    std::vector<uint8_t> lds(base + tile_bytes + 128, 0xEE);  // garbage outside the tile ...
    std::memcpy(lds.data() + base, ctbytes + a, tile_bytes);
    const uint32_t v1 = base + tile_bytes;
    for (uint32_t x = base & ~15u; x < base; ++x) lds[x] = 0;  // ... but the edge blocks are cleared
    for (uint32_t x = v1; x < ((v1 + 15u) & ~15u); ++x) lds[x] = 0;
    const int32_t v0a = (int32_t)(base & ~15u), v1a = (int32_t)((v1 + 15u) & ~15u);
    const uint32_t ks0 = 32u + a, ks1 = ks0 + tile_bytes;
    const int kf = (int)(ks0 / C), kl = (int)((ks1 - 1u) / C);
    CHECK(kl - kf < 4, "tile spans too many chunks");
    for (int k = kf; k <= kl; ++k) {
      if (k == 0 || k >= last) continue;
      const int32_t xc = (int32_t)((uint32_t)k * C - 64u * b0);
      uint64_t dsum[5] = {0, 0, 0, 0, 0};
      for (int i = 0; i < 16; ++i) {
        int32_t c[kPolyDigits];
        for (int d = 0; d < kPolyDigits; ++d) c[d] = 0;
        for (int t = 0; t < 64; ++t) {
          const int32_t x = xc + 16 * i + 256 * t;
          uint8_t piece[16] = {0};
          if (x >= v0a && x < v1a) std::memcpy(piece, lds.data() + x, 16);
          for (int b = 0; b < 16; ++b) {
            const int8_t av = (int8_t)(piece[b] ^ 0x80);
            for (int d = 0; d < kPolyDigits; ++d) c[d] += (int32_t)av * tab[d * kSegBytes + 16 * t + b];
          }
        }
        int T0, T1;
        poly_row_owned((int64_t)ks0, (int64_t)ks1, (int64_t)k * C, i, T0, T1);
        const P130 krow = poly_row_const(pw.data() + kPowKsegOff, pw.data() + kPowQOff + T0 * 5,
                                         pw.data() + kPowQOff + T1 * 5);
        const uint32_t* rf = pw.data() + kPowRowOff + i * 5;
        const P130 h = p130_mul(poly_seg_value(c, krow), P130{{rf[0], rf[1], rf[2], rf[3], rf[4]}});
        for (int u = 0; u < 5; ++u) dsum[u] += h.v[u];
      }
      const P130 part = carry64(dsum);
      for (int u = 0; u < 5; ++u) partials[(size_t)k * 8 + u] += part.v[u];
    }
  }
  // ---- first and last chunk by definition: sum_i c_i r^(eb - i)
  for (int k : {0, last}) {
    if (k == last && last == 0 && k != 0) continue;
    const int64_t kC = (int64_t)k * C;
    const int64_t start = kC >= 32 ? kC - 32 : 0;
    const int64_t end = std::min((int64_t)N, kC + C - 32);
    P130 h = p130_zero();
    if (start < end) {
      std::vector<uint8_t> buf(C + 16, 0);
      for (int64_t pos = start; pos < end; ++pos) buf[pos - (kC - 32)] = ctbytes[pos];
      const int64_t fb = start / 16, eb = (end + 15) / 16;
      for (int64_t i = fb; i < eb; ++i) h = p130_mul(p130_carry(p130_add(h, load_block(buf.data(), i, kC, N))), r);
    }
    for (int u = 0; u < 5; ++u) partials[(size_t)k * 8 + u] = h.v[u];
    if (last == 0) break;
  }
  // ---- k_mac_final
  const P130 rC = p130_pow(r, C / 16);
  P130 H = p130_zero();
  int64_t prev = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t e = (k < K - 1) ? ((int64_t)(k + 1) * C - 32) / 16 : ((int64_t)N + 15) / 16;
    const uint32_t* pp = partials.data() + (size_t)k * 8;
    const P130 hk = P130{{pp[0], pp[1], pp[2], pp[3], pp[4]}};
    if (k == 0) H = hk;
    else {
      const int64_t dd = e - prev;
      const P130 Rd = (dd == C / 16) ? rC : p130_pow(r, (uint32_t)dd);
      H = p130_carry(p130_add(p130_mul(H, Rd), hk));
    }
    prev = e;
  }
  const uint32_t s4[4] = {key.poly_s[0], key.poly_s[1], key.poly_s[2], key.poly_s[3]};
  p130_finish(tag, H, s4);
}

// sink of the host run of decode_lane: values by rank, and how often each rank was written
struct HostDecodeSink {
  static constexpr bool kAdditive = false;
  std::vector<uint32_t>* out;
  std::vector<int>* hits;
  void put(uint32_t local, uint32_t v, uint32_t term) {
    if (term) { (*out)[local] = v; ++(*hits)[local]; }
  }
  void put_masked(uint32_t local, uint32_t v) { put(local, v, 1); }
  void put_rank(uint32_t rank, uint32_t v) { (*out)[rank] = v; ++(*hits)[rank]; }
};

int main() {
  // 1. primitives vs host
  for (int it = 0; it < 20; ++it) {
    uint8_t k[32], n16[16], n8[8];
    hc::os_random(k, 32); hc::os_random(n16, 16); hc::os_random(n8, 8);
    uint32_t kw[8], nw[4], n8w[2];
    words(kw, k, 8); words(nw, n16, 4); words(n8w, n8, 2);
    uint8_t hb[32], db[32];
    hc::hsalsa20(hb, k, n16);
    uint32_t dw[8];
    hsalsa20(dw, kw, nw);
    bytes(db, dw, 8);
    CHECK(std::memcmp(hb, db, 32) == 0, "hsalsa20");
    uint8_t sb[64], dsb[64];
    hc::salsa20_block(sb, k, n8, 12345 + it);
    uint32_t sw[16];
    salsa20_block(sw, kw, n8w[0], n8w[1], 12345 + it);
    bytes(dsb, sw, 16);
    CHECK(std::memcmp(sb, dsb, 64) == 0, "salsa20");
    {  // the same block from the message's counter-independent prefix
      const SalsaPrefix pre = salsa20_prefix(kw, n8w[0], n8w[1]);
      uint32_t pw[16];
      salsa20_block(pw, pre, kw, n8w[0], n8w[1], (uint32_t)(12345 + it));
      CHECK(std::memcmp(pw, sw, 64) == 0, "salsa20 from prefix");
      salsa20_block(pw, pre, kw, n8w[0], n8w[1], 0xfffffff0u + (uint32_t)it);
      salsa20_block(sw, kw, n8w[0], n8w[1], (uint64_t)(0xfffffff0u + (uint32_t)it));
      CHECK(std::memcmp(pw, sw, 64) == 0, "salsa20 from prefix, large counter");
    }
    uint8_t m64[64];
    hc::os_random(m64, 64);
    uint8_t b2[24], db2[24];
    hc::blake2b(b2, 24, m64, 64);
    uint32_t mw[16], bw[6];
    words(mw, m64, 16);
    blake2b_192_64(bw, mw);
    bytes(db2, bw, 6);
    CHECK(std::memcmp(b2, db2, 24) == 0, "blake2b");
  }
  // 1b. device X25519 (radix 2^25.5 ladder) vs host
  for (int it = 0; it < 256; ++it) {
    uint8_t sc[32], pt[32], ho[32];
    hc::os_random(sc, 32);
    hc::os_random(pt, 32);
    if (it == 0) { std::memset(pt, 0, 32); pt[0] = 9; }
    if (it == 1) std::memset(pt, 0xff, 32);  // non-canonical u
    hc::x25519(ho, sc, pt);
    uint32_t sw[8], pw[8], dw[8];
    words(sw, sc, 8); words(pw, pt, 8);
    x25519(dw, sw, pw);
    uint8_t db[32];
    bytes(db, dw, 8);
    CHECK(std::memcmp(ho, db, 32) == 0, "x25519 it=%d", it);
  }
  // 1c. fixed-base X25519 (edwards25519 table) vs the host's scalarmult_base
  {
    static const uint32_t table[32 * 8 * kEdEntryWords] = {
#include "ed25519_base.inc"
    };
    for (int it = 0; it < 256; ++it) {
      uint8_t sc[32], ho[32];
      hc::os_random(sc, 32);
      if (it == 0) std::memset(sc, 0, 32);
      if (it == 1) std::memset(sc, 0xff, 32);
      if (it == 2) { std::memset(sc, 0x88, 32); }  // every digit at the carry border
      if (it == 3) { std::memset(sc, 0x77, 32); }
      hc::x25519_base(ho, sc);
      uint32_t sw[8], dw[8];
      words(sw, sc, 8);
      x25519_base(dw, sw, table);
      uint8_t db[32];
      bytes(db, dw, 8);
      CHECK(std::memcmp(ho, db, 32) == 0, "x25519_base it=%d", it);
      // ... and the pair with a shared inversion against the two separate routes
      uint8_t pt[32], hs[32];
      hc::os_random(pt, 32);
      hc::x25519(hs, sc, pt);
      uint32_t pw[8], ew[8], shw2[8];
      words(pw, pt, 8);
      x25519_seal_pair(ew, shw2, sw, pw, table);
      uint8_t eb[32], sb[32];
      bytes(eb, ew, 8);
      bytes(sb, shw2, 8);
      CHECK(std::memcmp(ho, eb, 32) == 0, "seal pair epk it=%d", it);
      CHECK(std::memcmp(hs, sb, 32) == 0, "seal pair shared it=%d", it);
    }
  }
  // 2. message key derivation vs host crypto_box_seal
  uint8_t pk[32], sk[32], esk[32], epk[32];
  hc::box_keypair(pk, sk);
  hc::os_random(esk, 32);
  hc::x25519_base(epk, esk);
  uint8_t shared[32];
  hc::x25519(shared, esk, pk);
  uint32_t shw[8], epkw[8], pkw[8];
  words(shw, shared, 8); words(epkw, epk, 8); words(pkw, pk, 8);
  MsgKey mk = derive(shw, epkw, pkw);
  // host: nonce, k, subkey, block0
  uint8_t nonce[24], kk[32], sub[32], blk0[64];
  hc::seal_nonce(nonce, epk, pk);
  hc::box_beforenm(kk, pk, esk);
  hc::hsalsa20(sub, kk, nonce);
  hc::salsa20_block(blk0, sub, nonce + 16, 0);
  uint8_t mkb[80];
  std::memcpy(mkb, &mk, 80);
  CHECK(std::memcmp(mkb, sub, 32) == 0, "subkey");
  CHECK(std::memcmp(mkb + 32, nonce + 16, 8) == 0, "nonce tail");
  CHECK(std::memcmp(mkb + 40, blk0, 32) == 0, "poly key");
  // 3. MAC emulation vs host poly1305 for several lengths
  for (uint32_t N : {0u, 1u, 15u, 16u, 17u, 100u, 16351u, 16352u, 16353u, 40000u, 100000u}) {
    std::vector<uint8_t> ct(N + 16);
    hc::os_random(ct.data(), ct.size());
    uint8_t tag[16];
    hc::poly1305(tag, ct.data(), N, blk0);
    uint32_t dt[4];
    emul_mac(dt, mk, ct.data(), N);
    uint8_t dtb[16];
    bytes(dtb, dt, 4);
    CHECK(std::memcmp(tag, dtb, 16) == 0, "poly1305 chunked N=%u", N);
  }
  // 4. matrix-core MAC formulation vs host poly1305 (segment-aligned, partial
  //    last blocks, single-chunk, multi-chunk, all-0xff bytes)
  for (uint32_t N : {0u, 1u, 15u, 16u, 17u, 100u, 1000u, 1024u, 1055u, 2047u, 16351u, 16352u,
                     16353u, 16368u, 32704u, 40000u, 65536u, 100000u, 100001u}) {
    for (int fill = 0; fill < 2; ++fill) {
      std::vector<uint8_t> ct(N + 16);
      if (fill) std::memset(ct.data(), 0xff, ct.size());
      else hc::os_random(ct.data(), ct.size());
      uint8_t tag[16];
      hc::poly1305(tag, ct.data(), N, blk0);
      uint32_t dt[4];
      emul_mac_mfma(dt, mk, ct.data(), N);
      uint8_t dtb[16];
      bytes(dtb, dt, 4);
      CHECK(std::memcmp(tag, dtb, 16) == 0, "poly1305 mfma N=%u fill=%d", N, fill);
    }
  }
  // 5. random lengths up to 2 MB (MFMA formulation)
  {
    uint32_t seedw[1];
    for (int it = 0; it < 300; ++it) {
      hc::os_random(reinterpret_cast<uint8_t*>(seedw), 4);
      uint32_t N = it < 150 ? seedw[0] % 2000000u : seedw[0] % 70000u;
      if (it % 7 == 0) N &= ~15u;
      if (it % 11 == 0) N = (N / kChunkBytes) * kChunkBytes + (uint32_t)(seedw[0] >> 24) * 4;
      std::vector<uint8_t> ct(N + 16);
      hc::os_random(ct.data(), ct.size());
      uint8_t tag[16];
      hc::poly1305(tag, ct.data(), N, blk0);
      uint32_t dt[4];
      emul_mac_mfma(dt, mk, ct.data(), N);
      uint8_t dtb[16];
      bytes(dtb, dt, 4);
      CHECK(std::memcmp(tag, dtb, 16) == 0, "poly1305 mfma random N=%u", N);
    }
  }
  // 6. the encode kernel's per-tile MAC: random tile borders (8 KiB .. 24 KiB tiles,
  //    as 8192 values of 1..3 bytes give), chunk-aligned and off-by-one borders
  {
    uint32_t seedw[2];
    for (int it = 0; it < 120; ++it) {
      hc::os_random(reinterpret_cast<uint8_t*>(seedw), 8);
      uint32_t N = it < 60 ? seedw[0] % 400000u : seedw[0] % 70000u;
      if (it % 7 == 0) N &= ~15u;
      if (it % 5 == 0) {  // within -40 .. +215 bytes of a chunk border
        const int64_t near = (int64_t)(N / kChunkBytes) * kChunkBytes + (int64_t)(seedw[0] >> 24) - 40;
        N = (uint32_t)std::max<int64_t>(1, near);
      }
      if (N == 0) N = 1;
      std::vector<uint8_t> ct(N + 16);
      if (it % 9 == 0) std::memset(ct.data(), 0xff, ct.size());
      else hc::os_random(ct.data(), ct.size());
      std::vector<uint32_t> cuts{0};
      uint32_t x = seedw[1];
      while (cuts.back() < N) {
        x = x * 1664525u + 1013904223u;
        uint32_t step = 8192u + (x >> 8) % 16385u;
        if (it % 4 == 1) step = kChunkBytes;                       // borders on the chunk grid
        if (it % 4 == 2 && cuts.size() == 1) step = kChunkBytes - 32;  // ... on the keystream grid
        if (it % 4 == 3) step = 8192u + ((x >> 8) % 3u) * 8192u + ((x >> 20) % 3u) - 1u;
        cuts.push_back(std::min(N, cuts.back() + step));
      }
      uint8_t tag[16];
      hc::poly1305(tag, ct.data(), N, blk0);
      uint32_t dt[4];
      emul_mac_fused(dt, mk, ct.data(), N, cuts);
      uint8_t dtb[16];
      bytes(dtb, dt, 4);
      CHECK(std::memcmp(tag, dtb, 16) == 0, "poly1305 fused tiles N=%u it=%d", N, it);
    }
  }
  // 7. the 24-bit Barrett reduction of the small-field share kernel: exhaustive over
  //    every sum it can see, for each modulus the parameter search accepts
  {
    int accepted = 0;
    for (uint32_t m : {2u, 3u, 13u, 101u, 241u, 251u, 257u, 433u, 521u, 769u, 1009u, 4093u, 8191u}) {
      for (int terms : {5, 7}) {
        const uint64_t wmax = (uint64_t)terms * (m - 1) * (m - 1);
        const Mod24 P = make_mod24(m, wmax);
        if (!P.c) continue;
        ++accepted;
        bool ok = true;
        for (uint64_t w = 0; w <= wmax && ok; ++w) ok = mod24((uint32_t)w, P) == (uint32_t)(w % m);
        CHECK(ok, "mod24 m=%u terms=%d (k=%u c=%u)", m, terms, P.k, P.c);
      }
    }
    CHECK(accepted >= 10, "mod24 parameter search accepted only %d cases", accepted);
    CHECK(make_mod24(433, 7ull * 432 * 432).c != 0 && make_mod24(241, 5ull * 240 * 240).c != 0,
          "mod24 must cover the benchmark fields");
  }
  // 7b. the double-precision reduction of the GEMM epilogue (quotient never too large,
  //     at most one too small): multiples of m and their neighbours up to 2^53, random
  //     values, for small, typical and the largest moduli; and the epilogue's varint
  //     length formula against the threshold count
  {
    uint64_t x = 0x9e3779b97f4a7c15ull;
    auto next = [&x] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (uint32_t m : {16u, 17u, 433u, 60013u, 746497u, 5038849u, 16777213u, (1u << 27) - 39, (1u << 28) - 57}) {
      const ModF64 P = make_modf64(m);
      bool ok = true;
      const uint64_t top = (1ull << 53) - 1;
      for (int it = 0; it < 400000 && ok; ++it) {
        const uint64_t r = next();
        uint64_t v;
        switch (it & 3) {
          case 0: v = r & top; break;
          case 1: v = ((r & top) / m) * m; break;                 // a multiple of m
          case 2: v = ((r & top) / m) * m + (m - 1); break;       // just below one
          default: v = top - (r % (4ull * m)); break;             // the top of the range
        }
        if (v > top) v = top;
        ok = modf64d((double)v, P) == (uint32_t)(v % m);
        if (!ok) std::printf("  v=%llu m=%u got %u\n", (unsigned long long)v, m, modf64d((double)v, P));
      }
      CHECK(ok, "modf64d m=%u", m);
    }
    bool ok = true;
    for (uint64_t o = 0; o < (1ull << 29) && ok; o += (o < 70000 ? 1 : 997)) {
      const uint32_t out = (uint32_t)o;
      const uint32_t len = (1406u - 37u * (uint32_t)__builtin_clz((out << 1) | 1u)) >> 8;
      const uint32_t ref = 1u + (out >= (1u << 6)) + (out >= (1u << 13)) + (out >= (1u << 20)) + (out >= (1u << 27));
      ok = len == ref;
    }
    for (int b = 0; b < 29 && ok; ++b)
      for (uint32_t out : {(1u << b) - 1, 1u << b, (1u << b) + 1}) {
        const uint32_t len = (1406u - 37u * (uint32_t)__builtin_clz((out << 1) | 1u)) >> 8;
        const uint32_t ref = 1u + (out >= (1u << 6)) + (out >= (1u << 13)) + (out >= (1u << 20)) + (out >= (1u << 27));
        ok = ok && len == ref;
      }
    CHECK(ok, "varint length from the leading-zero count");
  }
  // 7c. the GEMM's signed limb scheme: digits in int8, value recovered, and the fold of
  //     worst-case and random degree sums (exact integers) against 128-bit arithmetic
  {
    uint64_t x = 0x2545f4914f6cdd1dull;
    auto next = [&x] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (uint32_t m : {(1u << 21), 2097169u, 5038849u, 9999991u, (1u << 24) - (1u << 18) - 1}) {
      const int Kp = 4096;
      const LimbScheme sch = limb_scheme(m, Kp);
      CHECK(sch.limbs == 3 && sch.bits == 8, "limb scheme of m=%u", m);
      bool ok = true;
      for (int it = 0; it < 200000 && ok; ++it) {
        uint32_t v = (uint32_t)(next() % m);
        if (it < 8) v = (uint32_t[]){0u, 1u, m / 2, m / 2 + 1, m - 1, m / 2 - 1, 255u, 65535u}[it];
        int8_t d[4];
        limbs_of_value(v, m, sch, d);
        const int64_t back = (int64_t)d[0] + 256 * (int64_t)d[1] + 65536 * (int64_t)d[2];
        ok = ((back % (int64_t)m) + m) % m == v && (back == (int64_t)v || back == (int64_t)v - (int64_t)m);
      }
      CHECK(ok, "signed limbs of m=%u", m);
      const ModF64 P = make_modf64_signed(m, Kp);
      const int64_t top[5] = {(int64_t)Kp << 14, (int64_t)Kp << 15, 3 * ((int64_t)Kp << 14), (int64_t)Kp << 15,
                              (int64_t)Kp << 14};  // |acc_d| at most
      for (int it = 0; it < 200000 && ok; ++it) {
        int64_t a[5];
        for (int dgr = 0; dgr < 5; ++dgr) {
          const int mode = it < 64 ? (it >> dgr) & 1 : 2;  // all sign patterns of the extremes first
          a[dgr] = mode == 2 ? (int64_t)(next() % (2 * (uint64_t)top[dgr] + 1)) - top[dgr]
                             : (mode ? top[dgr] : -top[dgr]);
        }
        double s = P.off + (double)a[0];
        s = __builtin_fma((double)a[1], 256.0, s);
        s = __builtin_fma((double)a[2], 65536.0, s);
        s = __builtin_fma((double)a[3], 16777216.0, s);
        s = __builtin_fma((double)a[4], P.w4, s);
        __int128 ref = 0;
        for (int dgr = 4; dgr >= 0; --dgr) ref = ref * 256 + a[dgr];
        int64_t r = (int64_t)(ref % (__int128)m);
        if (r < 0) r += m;
        ok = s >= 0 && s < 0x1p53 && modf64d(s, P) == (uint32_t)r;
      }
      CHECK(ok, "signed-limb fold m=%u", m);
    }
  }
  // 7d. the generic varint decoder, lane by lane as the kernels call it (64 bytes a lane,
  //     the 8 bytes before it, terminator masks, ranks), against a plain decoder: codes of
  //     one to five bytes, negative values, values past the modulus, overlong and
  //     64-bit codes (the walk), for small and the largest moduli and for raw u32 output
  {
    using HostSink = HostDecodeSink;
    uint64_t x = 0x853c49e6748fea9bull;
    auto next = [&x] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (uint32_t m : {433u, 746497u, 5038849u, (1u << 27) - 39, 2147483647u, 0u}) {
      const ModParams mp = make_mod_params(m);
      for (int variant = 0; variant < 3; ++variant) {
        // variant 0: canonical values; 1: mixed lengths and signs; 2: with overlong / huge codes
        std::vector<uint8_t> msg;
        std::vector<uint32_t> want;
        const int count = 3000;
        for (int i = 0; i < count; ++i) {
          int64_t v;
          const uint64_t r = next();
          const uint64_t span = m ? m : 0xffffffffull;
          if (variant == 0) v = (int64_t)(r % span);
          else {
            const int bits = 1 + (int)((r >> 40) % (variant == 2 ? 62 : 31));
            v = (int64_t)(r & ((1ull << bits) - 1));
            if (m != 0 && (r >> 63)) v = -v;
            if (m == 0) v &= 0xffffffffll;
          }
          uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
          int pad = variant == 2 && (r >> 50) % 7 == 0 ? 1 + (int)((r >> 53) % 3) : 0;  // overlong: zero groups
          int len = 1;
          for (uint64_t t = z >> 7; t; t >>= 7) ++len;
          if (len + pad > 10) pad = 10 - len;  // ten bytes is the longest code the decoders take
          do {
            uint8_t b = z & 0x7f;
            z >>= 7;
            if (z || pad) b |= 0x80;
            msg.push_back(b);
          } while (z);
          while (pad--) msg.push_back(pad ? 0x80 : 0x00);
          uint32_t ref;
          if (m == 0) ref = (uint32_t)v;
          else {
            int64_t t = v % (int64_t)m;
            ref = (uint32_t)(t < 0 ? t + m : t);
          }
          want.push_back(ref);
        }
        const int64_t N = (int64_t)msg.size();
        msg.resize(msg.size() + 128, 0);
        std::vector<uint32_t> got(want.size(), 0xdeadbeefu);
        std::vector<int> hits(want.size(), 0);
        HostSink sink{&got, &hits};
        uint32_t rank = 0;
        bool bad = false;
        for (int64_t p0 = 0; p0 < N; p0 += 64) {
          uint32_t w[16];
          for (int q = 0; q < 16; ++q) {
            uint32_t word = 0;
            for (int b = 0; b < 4; ++b) {
              const int64_t pos = p0 + 4 * q + b;
              word |= (uint32_t)(pos < N ? msg[pos] : 0) << (8 * b);
            }
            w[q] = word;
          }
          auto word_at = [&](int64_t pos) {
            uint32_t word = 0;
            if (pos >= 0) std::memcpy(&word, &msg[pos], 4);
            return word;
          };
          const int hi = (int)std::min<int64_t>(64, N - p0);
          const uint64_t traw = term_mask64(w);
          const uint64_t tmask = traw & byte_range_mask(0, hi);
          bad |= decode_lane<false>(w, word_at(p0 - 8), word_at(p0 - 4), tmask, traw, rank, mp, msg.data(), p0, sink);
          rank += (uint32_t)__builtin_popcountll(tmask);
        }
        bool ok = rank == want.size() && !bad;
        for (size_t i = 0; i < want.size() && ok; ++i) ok = got[i] == want[i] && hits[i] == 1;
        CHECK(ok, "generic varint decode m=%u variant %d", m, variant);
      }
    }
  }
  // 8. the encode kernel's packed varint pairs against a plain zigzag-LEB128 encoder:
  //    every low value with a spread of high values, and the reverse
  {
    auto leb = [](uint32_t v, uint8_t (&out)[2]) {  // v < 2^13: one or two bytes
      const uint32_t z = v << 1;
      out[0] = (uint8_t)((z & 0x7f) | (z >= 128 ? 0x80 : 0));
      out[1] = (uint8_t)(z >> 7);
      return z >= 128 ? 2 : 1;
    };
    bool ok = true;
    for (uint32_t a = 0; a < 8192 && ok; ++a) {
      for (uint32_t b : {0u, 1u, 63u, 64u, 65u, 127u, 128u, 432u, 4095u, 8191u, (a * 2654435761u) >> 19}) {
        for (int swap = 0; swap < 2 && ok; ++swap) {
          const uint32_t lo = swap ? b : a, hi = swap ? a : b;
          uint32_t codes, two;
          varint_pair16(lo | (hi << 16), codes, two);
          uint8_t el[2], eh[2];
          const int nl = leb(lo, el), nh = leb(hi, eh);
          ok = ok && (two & 0xffffu) == (uint32_t)(nl - 1) && (two >> 16) == (uint32_t)(nh - 1);
          ok = ok && (codes & 0xffu) == el[0] && ((codes >> 8) & 0xffu) == el[1];
          ok = ok && ((codes >> 16) & 0xffu) == eh[0] && (codes >> 24) == eh[1];
          if (!ok) std::printf("  pair lo=%u hi=%u codes=%08x two=%08x\n", lo, hi, codes, two);
        }
      }
    }
    CHECK(ok, "varint_pair16 against zigzag LEB128");
  }
  // 9. the encode kernel's work units: every tile of every message exactly once, ends
  // together only where they are short, no unit outside the launch's grid
  {
    const int Ls[] = {1, 7, 2047, 2048, 2049, 8191, 8192, 8193, 10000, 10240, 16382, 25000,
                      65536, 65537, 70000, 150001};
    const int Ms[] = {1, 3, 4, 5, 64, 1000};
    for (int mac = 0; mac < 2; ++mac)
      for (int L : Ls)
        for (int M : Ms) {
          const int tiles = (L + kEncodeValues - 1) / kEncodeValues;
          std::vector<int> seen((size_t)tiles * M, 0);
          const unsigned grid = encode_grid(mac != 0, M, L);
          bool ok = true;
          for (unsigned b = 0; b < grid; ++b) {
            const EncodeUnit u0 = encode_unit(mac != 0, M, L, (int)b, 0);
            for (int w = 0; w < (u0.ends ? kWaves : 1); ++w) {
              const EncodeUnit u = encode_unit(mac != 0, M, L, (int)b, w);
              ok = ok && u.ends == u0.ends && u.tile >= 0 && u.tile < tiles && u.msg >= 0 && u.msg < M;
              if (u.ends) ok = ok && !mac && u.tile == tiles - 1 && L - u.tile * kEncodeValues <= kEncodeValues / kWaves;
              if (ok && !u.idle) ++seen[(size_t)u.tile * M + u.msg];
            }
          }
          for (int c : seen) ok = ok && c == 1;
          CHECK(ok, "encode work units");
        }
  }
  // 9b. the decode + sum kernels' workgroup order is a permutation of the grid
  {
    const unsigned dims[][3] = {{1, 1, 1}, {2, 728, 26}, {2, 19682, 1}, {3, 5, 7}, {7, 1, 1}, {8, 3, 2}, {163, 3, 26}};
    for (const auto& d : dims) {
      std::vector<int> seen((size_t)d[0] * d[1] * d[2], 0);
      bool ok = true;
      for (unsigned z = 0; z < d[2]; ++z)
        for (unsigned y = 0; y < d[1]; ++y)
          for (unsigned x = 0; x < d[0]; ++x) {
            const SumTileId id = sum_tile_of(d[0], d[1], d[2], x, y, z);
            ok = ok && id.t >= 0 && (unsigned)id.t < d[0] && id.r >= 0 && (unsigned)id.r < d[1] && id.g >= 0 &&
                 (unsigned)id.g < d[2];
            if (ok) ++seen[((size_t)id.g * d[1] + id.r) * d[0] + id.t];
          }
      for (int c : seen) ok = ok && c == 1;
      CHECK(ok, "decode + sum workgroup order");
    }
  }
  std::printf(failures ? "host_emul: %d FAILURES\n" : "host_emul: all ok\n", failures);
  return failures ? 1 : 0;
}
