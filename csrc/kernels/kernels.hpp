// Host-side launch API of the SDA HIP kernels (gfx950).
//
// All buffers are raw device pointers owned by the caller (PyTorch tensors in the
// Python engine); every launcher is asynchronous on the given stream and does no
// allocation or synchronisation, so a whole aggregation round can be captured
// into a hipGraph.
//
// Message model (shared by every kernel): a *message* is one sealed box
// (libsodium crypto_box_seal, reference sodium.rs:36-43) over the zigzag-varint
// encoding of a vector of L field values. Messages of one launch have a uniform
// value count L and live in a ciphertext arena at `ct + j*stride` laid out as
//   epk(32) | mac(16) | ct bytes (<= L*maxlen) | padding   (stride % 64 == 0).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sdagpu {

// Per-message stream state derived by the seal/open setup kernels.
struct MsgKey {
  uint32_t subkey[8];   // XSalsa20 subkey = HSalsa20(k, nonce[0:16])
  uint32_t nonce[2];    // nonce[16:24]
  uint32_t poly_r[4];   // keystream bytes 0..15
  uint32_t poly_s[4];   // keystream bytes 16..31
  uint32_t pad[2];
};
static_assert(sizeof(MsgKey) == 80, "MsgKey layout");

constexpr int kTileValues = 4096;    // values per byte-count tile (256 lanes x 16)
constexpr int kEncodeValues = 8192;  // values per encode tile = 2 count tiles (256 x 32)
constexpr int kChunkBytes = 16384;  // bytes per MAC / decrypt chunk (256 threads x 64)
constexpr int kSubBytes = 1024;     // terminator-count granularity (16 lanes x 64 B)
constexpr int kSubPerChunk = kChunkBytes / kSubBytes;
constexpr int kSumTile = 6144;      // elements per decode-sum tile (~11 KiB of varints at m = 433)

// Per-message Poly1305 tables (k_poly_powers), kPowWords u32 per message. The
// matrix-core MAC takes a 16 KiB chunk as 16 interleaved rows: row i = blocks
// i, i + 16, i + 32, ... (so 16 lanes read 256 contiguous bytes), K index
// 16 t + a = byte a of block i + 16 t; R = r^16.
//   [0, 1280)           chunk factors r^(4(255-t)), t < 256, 5 x 26-bit limbs (Horner lanes)
//   [kPowKsegOff, +5)   row constant without the pad bits: 128 sum W - 2^24 sum_d 2^(7d)
//   [kPowTabOff, ...)   int8 weight digits [kPolyDigits][kSegBytes]: 7-bit digit d of
//                       W(16 t + a) = 2^(8a) R^(63 - t) mod p
//   [kPowRowOff, +80)   row factors r^(16 - i), i < 16 (5 limbs each)
//   [kPowQOff, +325)    pad-bit prefixes 2^128 sum_{t' < T} R^(63 - t'), T = 0..64 (a
//                       whole row: entry 64; a row cut by a tile border: a difference)
constexpr int kSegBytes = 1024;     // MFMA MAC row: 64 blocks
constexpr int kPolyDigits = 19;     // 7-bit digits of a value < 2^133
constexpr int kPowKsegOff = 256 * 5;
constexpr int kPowTabOff = kPowKsegOff + 8;
constexpr int kPowRowOff = kPowTabOff + kPolyDigits * kSegBytes / 4;
constexpr int kPowQOff = kPowRowOff + 16 * 5;
constexpr int kPowWords = (kPowQOff + 65 * 5 + 7) / 8 * 8;

// Messages of at most kShortMaxChunks chunks (64 KiB) take the one-pass MAC
// (k_mac_short) with its own, small table: r^(t+1), t < 64, 5 limbs each.
constexpr int kShortMaxChunks = 4;
constexpr int kPowShortWords = 64 * 5;

// Error bits (device error word)
enum ErrBits : uint32_t {
  kErrBadKey = 1u,          // X25519 produced the all-zero point
  kErrMac = 2u,             // Poly1305 verification failed
  kErrMalformed = 4u,       // varint stream does not hold exactly L values
  kErrChaChaReject = 8u,    // rand-0.3 ChaCha mask hit a rejection (host fallback)
  kErrRange = 16u,          // value outside the expected modulus
};

struct RngKeyArg {
  uint32_t k[8];
};

// ---- keys.hip --------------------------------------------------------------
// Seal setup: esk from the device CSPRNG (purpose ephemeral, owner
// msg_owner_base + j), epk -> header, MsgKey for encryption. key_tables (may be null):
// per public key a fixed-base table of kKeyTableWords words (host: x25519_comb_table; zeros
// = none), used by the many-message form instead of the ladder.
constexpr int kKeyTableWords = 32 * 8 * 32;
void launch_seal_setup(int M, RngKeyArg rng, uint64_t msg_owner_base, const uint32_t* key_idx,
                       const uint32_t* pks, uint8_t* ct, uint64_t stride, MsgKey* keys,
                       uint32_t* err, uint32_t* gate, uint32_t gate_val, const uint32_t* key_tables,
                       hipStream_t s);
// Open setup: epk from header, X25519 with the recipient secret key.
void launch_open_setup(int M, const uint32_t* key_idx, const uint32_t* sks, const uint32_t* pks,
                       const uint8_t* ct, uint64_t stride, MsgKey* keys, uint32_t* err,
                       uint32_t* gate, uint32_t gate_val, hipStream_t s);
// Wave priority of the open-side setup and the Poly1305 table kernels (1 = top;
// default 0 = normal: neither is latency-critical) -- scheduling experiments.
void set_key_prio(int open_prio, int powers_prio);
// Dispatch gate: the setup kernels store gate_val to *gate (if non-null) when
// their first workgroup starts; k_gate_wait (one wave) polls for it, giving up
// after timeout_us. Orders a side-stream setup's dispatch before a main-stream
// grid launched right after it.
void launch_gate_wait(const uint32_t* gate, uint32_t val, uint32_t timeout_us, hipStream_t s);
// Standalone batched X25519 (tests / key generation): out[i] = X25519(sc[i], u[i]).
// X25519(scalar, 9) through the edwards25519 fixed-base table (test hook).
void launch_x25519_base(int N, const uint32_t* scalars, uint32_t* out, hipStream_t s);
// launch_seal_setup's kernel: -1 by message count (default), 0 two lanes per message
// (both ladders side by side: lowest latency), 1 one lane per message with the
// fixed-base table for the public key (least work)
void set_seal_many(int mode);
void launch_x25519(int N, const uint32_t* scalars, const uint32_t* points, uint32_t* out,
                   hipStream_t s);

// ---- share.hip -------------------------------------------------------------
enum MaskMode : int { kMaskNone = 0, kMaskFull = 1, kMaskChaCha = 2 };

// Additive sharing (client/src/crypto/sharing/additive.rs:32-51 semantics, canonical
// representatives) fused with masking and per-tile varint byte counts.
//   secrets  [P][D] int32 ; shares [n][P][D] (u16 if value_bytes==2 else u32)
//   cnt      [n][P][T] tile byte counts (T = ceil(D / kTileValues))
//   mask_out [P][D] (kMaskFull; the same element type as `shares`) and mask_cnt [P][T]
// mask_mode is kMaskNone or kMaskFull; ChaCha-masked participants mask first
// (launch_chacha_mask_apply) and share the masked vectors with kMaskNone.
void launch_share_additive(int P, int D, int n, uint32_t m, int value_bytes, const int32_t* secrets,
                           int mask_mode, RngKeyArg rng, uint64_t owner_base, void* shares,
                           uint32_t* cnt, void* mask_out, uint32_t* mask_cnt, hipStream_t s);

// Additive share kernel selection -- benchmarking switch: 1 (default) = three
// draws per word where m^3 < 2^32, else 16-bit halves; 2 = 16-bit halves; 0 = u32.
void set_share16(int mode);
// Packed-Shamir small-field kernel (k = 3, n = 8, t = 2 or 4, no mask; default
// on) -- benchmarking switch.
void set_pss48(int mode);

// Packed Shamir: shares = M . [s_1..s_k, r_1..r_t] mod p per batch (M: n x (k+t)
// host-computed from the tss FFT construction).
void launch_share_pss(int P, int D, int n, int k, int t, uint32_t p, int value_bytes,
                      const int32_t* secrets, const uint32_t* share_matrix, int mask_mode,
                      RngKeyArg rng, uint64_t owner_base, void* shares, uint32_t* cnt,
                      void* mask_out, uint32_t* mask_cnt, hipStream_t s);

// Tile byte counts for arbitrary canonical value vectors [M][L].
void launch_count(int M, int L, int value_bytes, const void* vals, uint32_t* cnt, hipStream_t s);

// ---- chacha_mask.hip -------------------------------------------------------
// ChaCha masks (client/src/crypto/masking/chacha.rs): rand-0.3 ChaChaRng streams,
// exact under rejected draws (a rejection shifts the rest of that participant's
// stream; fast kernels record it, gated repair kernels re-index the stream).
// seeds [P][seed_words] u32 from the round's CSPRNG:
void launch_chacha_seeds(int P, int seed_words, RngKeyArg rng, uint64_t owner_base, uint32_t* seeds,
                         hipStream_t s);
// u32 words of `scratch` both launches below need (contents need no initialisation)
size_t chacha_scratch_words(int P, int D);
// participants: masked[p][e] = (secrets[p][e] + gen_range(0, m)_e(seed_p)) mod m
void launch_chacha_mask_apply(int P, int D, uint32_t m, int seed_words, const uint32_t* seeds,
                              const int32_t* secrets, int32_t* masked, uint32_t* scratch,
                              uint32_t* err, hipStream_t s);
// recipient: out[e] = sum_p gen_range(0, m)_e(seed_p) mod m      (chacha.rs:56-77).
// part [groups][D] u32 slabs (groups = chacha_sum_groups(P, D)), fix [D] u64.
int chacha_sum_groups(int P, int D);
void launch_chacha_mask_sum(int P, int D, uint32_t m, int seed_words, const uint32_t* seeds,
                            uint32_t* out, uint32_t* part, int groups, uint32_t* scratch,
                            uint64_t* fix, uint32_t* err, hipStream_t s);
// Test hook: cap the rand-0.3 acceptance zone (draws at or above cap - cap % m are
// rejected) so that rejections, 1e-10 per draw at most in production, can be made
// frequent. ~0 = no cap. The host model has the same hook (crypto.hpp).
void set_chacha_zone_cap(uint64_t cap);

// ---- seal.hip --------------------------------------------------------------
// Segmented exclusive scan of rows [M][T] in place; totals[M] = row sums. With
// `err` non-null, a row whose sum differs from `expect` sets kErrMalformed.
void launch_segscan(int M, int T, uint32_t* data, uint32_t* totals, uint32_t expect, uint32_t* err,
                    hipStream_t s);
// Varint-encode + XSalsa20-encrypt tiles into the arena (ct bytes only). With
// `pows`, `pt_len` and zeroed `partials` [M][K][8] non-null,
// every tile also adds its share of the Poly1305 partials of the message's middle
// chunks (all but the first and the last) to `partials`; launch_mac_edges then
// supplies those two and launch_mac_final the tag.
// max_code_bytes: the longest varint the values can have (5 = any u32; the arena's slots
// are sized by the same bound): 32-bit values with at most 3 / 4 bytes get a kernel
// with a smaller LDS tile and more workgroups per CU.
void launch_encode_encrypt(int M, int L, int value_bytes, const void* vals,
                           const uint32_t* tile_off, const MsgKey* keys, uint8_t* ct,
                           uint64_t stride, const uint32_t* pows, const uint32_t* pt_len,
                           uint32_t* partials, int K, int max_code_bytes, hipStream_t s);
// Poly1305 partials of every message's first and last chunk only (per-lane Horner).
void launch_mac_edges(int M, int K, const MsgKey* keys, const uint32_t* pows, const uint8_t* ct,
                      uint64_t stride, const uint32_t* pt_len, uint32_t* partials, hipStream_t s);
// Poly1305 chunk partials (and, when decrypt!=0, in-place decryption plus
// varint-terminator counts per chunk).
// Per-message Poly1305 tables pows [M][kPowWords]: chunk factors, segment
// constant and weight digits of the matrix-core MAC (layout above).
// full == 0: Horner factors only (enough for messages of at most two chunks)
void launch_poly_powers(int M, const MsgKey* keys, uint32_t* pows, int full, hipStream_t s);
// With decrypt, term_cnt [M][K] (per chunk) and/or sub_cnt [M][K * kSubPerChunk]
// (per 1 KiB sub-chunk) receive terminator counts (either may be null).
void launch_mac_chunks(int M, int K, const MsgKey* keys, const uint32_t* pows, uint8_t* ct,
                       uint64_t stride, const uint32_t* pt_len, uint32_t* partials, int decrypt,
                       uint32_t* term_cnt, uint32_t* sub_cnt, hipStream_t s);
// One-pass Poly1305 of short messages (any length works; meant for at most
// kShortMaxChunks chunks): pows [M][kPowShortWords] from launch_poly_powers_short;
// verify == 0 writes the tag into the header, else compares (ok[j] may be null, a
// mismatch raises kErrMac). Reads the ciphertext: run it before the decryption.
void launch_poly_powers_short(int M, const MsgKey* keys, uint32_t* pows, hipStream_t s);
void launch_mac_short(int M, const MsgKey* keys, const uint32_t* pows, uint8_t* ct, uint64_t stride,
                      const uint32_t* pt_len, int verify, uint32_t* ok, uint32_t* err, hipStream_t s);
// In-place decryption + terminator counts alone (launch_mac_chunks without its MAC).
void launch_decrypt_count(int M, int K, const MsgKey* keys, uint8_t* ct, uint64_t stride,
                          const uint32_t* pt_len, uint32_t* term_cnt, uint32_t* sub_cnt,
                          hipStream_t s);
// Matrix-core Poly1305 segments (default on; 0 = per-lane Horner everywhere) --
// benchmarking switch.
void set_mac_mfma(int mode);
// Combine partials -> tag; mode 0 = write the header mac, 1 = verify (ok[j]).
void launch_mac_final(int M, int K, const MsgKey* keys, const uint32_t* pows, uint8_t* ct,
                      uint64_t stride, const uint32_t* pt_len, const uint32_t* partials, int verify,
                      uint32_t* ok, uint32_t* err, hipStream_t s);

// ---- open.hip --------------------------------------------------------------
// Decode the plaintext varint stream of each message into canonical values.
void launch_decode(int M, int K, int L, uint32_t m, int value_bytes, const uint8_t* pt,
                   uint64_t stride, const uint32_t* pt_len, const uint32_t* elem_start,
                   void* vals, uint32_t* err, hipStream_t s);
// Fused clerk decode + combine over rows R (clerks) x P participants, message
// j = r * P + p. pre [M][S] = exclusive sub-chunk terminator ranks (segscan of
// sub_cnt), totals [M]; tile_sub [M][T+1] scratch (T = ceil(L / kSumTile));
// part [G][R][L] scratch slabs (G = ceil(P / Pg); needs Pg * (m - 1) < 2^32 unless
// decode_sum_wide(m): then two words per entry and no bound on Pg);
// out [R][L] = sum_p values mod m.
void launch_locate_tiles(int M, int S, int L, const uint32_t* pre, const uint32_t* totals,
                         uint32_t* tile_sub, hipStream_t s);
// `redo` (may be null): one zeroed scratch word. With it and m <= 8192 the lean
// kernel (sums of zigzag codes, no per-element decode) runs first and the
// generic one only if a stream is not canonical (long or negative varints);
// needs Pg * 16383 < 2^32 as well.
// Moduli above 2^27 (past the lean kernels' four-byte codes) are summed in 64-bit
// accumulators: `part` then holds two words per sum, and a group may be any size.
inline bool decode_sum_wide(uint32_t m) { return m > (1u << 27); }
void launch_decode_sum(int R, int P, int Pg, int L, uint32_t m, const uint8_t* pt, uint64_t stride,
                       const uint32_t* pt_len, int S, const uint32_t* pre, const uint32_t* tile_sub,
                       uint32_t* part, uint32_t* out, int64_t* acc, uint32_t* err, uint32_t* redo,
                       hipStream_t s);  // acc != null: acc[r][l] += the sums instead of writing out
// Lean clerk decode (default on; 0 = generic kernel only) -- benchmarking switch.
void set_decode_lean(int mode);
// lean decode-sum accumulator layout: -1 padded rows by modulus (default), 0 never, 1 always
void set_decode_swz(int mode);
// lean decode-sum of three- and four-byte fields: 1 walks values (one LDS add per value),
// 0 adds byte by byte like the short-code kernel, -1 (default) the former for three-byte fields
void set_decode_long(int mode);
void set_encode_tile2(int on);
// Column sums mod m: out[g][l] = sum_r vals[g][r][l] mod m.
void launch_colsum(int G, int R, int L, uint32_t m, int value_bytes, const void* vals,
                   uint32_t* out, hipStream_t s);
// Packed Shamir reconstruction: out[b*k + s] = sum_i lag[s][i] * ys[i][b] mod p,
// truncated to D (batched.rs:68-99 + tss reconstruct).
void launch_pss_reconstruct(int B, int k, int nI, int D, uint32_t p, const uint32_t* lag,
                            const uint32_t* ys, uint32_t* out, hipStream_t s);
// out[e] = (a[e] - b[e]) mod m  (unmask, full.rs:54-67 / chacha.rs:79-93)
void launch_sub_mod(int D, uint32_t m, const uint32_t* a, const uint32_t* b, uint32_t* out,
                    hipStream_t s);

// ---- modgemm.hip -----------------------------------------------------------
// How field elements become int8 GEMM operands: `limbs` digits of `bits` bits -- 7:
// non-negative base-128 digits of the canonical value; 8: signed base-256 digits of the
// balanced residue (three limbs; 2^21 <= p < 2^24 - 2^18 and Kp <= 4096).
struct LimbScheme {
  int limbs, bits;
};
inline LimbScheme limb_scheme(uint32_t p, int Kp) {
  if (p < (1u << 21)) return LimbScheme{3, 7};
  // signed digits: the top one stays inside int8 for p / 2 + 128 + 2^15 <= 127 * 2^16; the
  // fold's sums (below K 2^40 each way) stay exact in doubles for K <= 4096
  if (p < (1u << 24) - (1u << 18) && Kp <= 4096) return LimbScheme{3, 8};
  return LimbScheme{4, 7};
}
// The limbs d[0 .. limbs) of one canonical value (host side: the fixed A operands).
inline void limbs_of_value(uint32_t x, uint32_t p, LimbScheme sch, int8_t* d) {
  if (sch.bits == 7) {
    for (int l = 0; l < sch.limbs; ++l) d[l] = (int8_t)((x >> (7 * l)) & 0x7f);
    return;
  }
  int32_t t = x > p / 2 ? (int32_t)x - (int32_t)p : (int32_t)x;
  for (int l = 0; l + 1 < sch.limbs; ++l) {
    d[l] = (int8_t)(t & 0xff);
    t = (t - d[l]) >> 8;
  }
  d[sch.limbs - 1] = (int8_t)t;
}
// C = A . B mod p (p < 2^28) on i8 MFMA, operands in limb_scheme(p, Kp) (`limbs` must be
// its limb count). A limbs [L][M][Kp], B limbs [L][batches][N][Kp] (b_plane = batches*N*Kp bytes between limb
// planes), C[z*ldc_z + m*ldc_m + n*ldc_n] written where that index < limit.
// cnt (may be null; zeroed by the caller): [M][batches][ceil(N / kTileValues)] varint
// bytes of the written elements, i.e. launch_count's result for C as M x batches
// messages of N values (the share GEMM: rows = clerks, batches = participants).
// a_frag (may be null): A in the fragment order of launch_a_fragments; with it, short
// K (Kp <= 256) and at least four row blocks the panel-resident kernel runs.
void launch_modgemm_i8(int M, int N, int Kp, int batches, int limbs, uint32_t p, const int8_t* A,
                       const int8_t* a_frag, const int8_t* B, int64_t b_plane, int value_bytes, void* C,
                       int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit, uint32_t* cnt,
                       hipStream_t s);
// A limbs [L][M][Kp] reordered into `out` (a_fragments_bytes(M, Kp, limbs) bytes: M
// rounded up to 64 rows): what each wave of the panel kernel loads is consecutive.
int64_t a_fragments_bytes(int M, int Kp, int limbs);
void launch_a_fragments(int M, int Kp, int limbs, const int8_t* A, int8_t* out, hipStream_t s);
// epilogue fold through the double-precision unit: 0 never (integer only), 1 for
// three-limb fields only, 2 for every field below 2^24 (default)
void set_gemm_fold_f64(int mode);
// -1 (default): the panel-resident kernel for short K with at least four row blocks;
// 0 never; 1 whenever Kp <= 256 (both need a_frag)
void set_gemm_panel(int mode);
// X limbs [L][P][B][Kp] of packed-Shamir inputs: secrets (canonical) then t draws.
void launch_pss_x_limbs(int P, int D, int B, int k, int t, int Kp, uint32_t p, const int32_t* secrets,
                        RngKeyArg rng, uint64_t owner_base, int8_t* X, hipStream_t s);
// Limbs of Y [R][N] (canonical values) transposed to [L][N][Kp].
void launch_limbs_t(int R, int N, int Kp, uint32_t p, const uint32_t* Y, int8_t* out, hipStream_t s);

}  // namespace sdagpu
