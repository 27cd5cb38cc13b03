// pybind11 bindings for the gfx950 kernels (`sda_amd._lib._sda_gpu`).
//
// Tensors cross the boundary as raw device pointers (tensor.data_ptr()) and the
// current HIP stream as an integer handle; shape/dtype/device validation is done
// in sda_amd/ops/gpu.py before any launch.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.hpp"

namespace py = pybind11;
using namespace sdagpu;

namespace {

template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

RngKeyArg rng_from(const std::vector<uint32_t>& k) {
  if (k.size() != 8) throw std::invalid_argument("rng key must be 8 x u32");
  RngKeyArg a;
  for (int i = 0; i < 8; ++i) a.k[i] = k[i];
  return a;
}

void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

PYBIND11_MODULE(_sda_gpu, m) {
  m.doc() = "SDA MI355X (gfx950) HIP kernels";
  m.attr("TILE_VALUES") = kTileValues;
  m.attr("CHUNK_BYTES") = kChunkBytes;
  m.attr("MSGKEY_BYTES") = (int)sizeof(MsgKey);
  m.attr("ERR_BAD_KEY") = (int)kErrBadKey;
  m.attr("ERR_MAC") = (int)kErrMac;
  m.attr("ERR_MALFORMED") = (int)kErrMalformed;
  m.attr("ERR_CHACHA_REJECT") = (int)kErrChaChaReject;
  m.attr("ERR_RANGE") = (int)kErrRange;

  m.def("device_info", []() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) throw std::runtime_error("no HIP device");
    py::dict d;
    d["name"] = std::string(p.name);
    d["gcn_arch"] = std::string(p.gcnArchName);
    d["cus"] = p.multiProcessorCount;
    d["lds_per_block"] = (long long)p.sharedMemPerBlock;
    d["total_mem"] = (long long)p.totalGlobalMem;
    return d;
  });

  m.def("seal_setup", [](int M, std::vector<uint32_t> rng, uint64_t owner_base, uintptr_t key_idx,
                         uintptr_t pks, uintptr_t ct, uint64_t stride, uintptr_t keys,
                         uintptr_t err, uintptr_t gate, uint32_t gate_val, uintptr_t key_tables,
                         uintptr_t stream) {
    launch_seal_setup(M, rng_from(rng), owner_base, P<const uint32_t>(key_idx),
                      P<const uint32_t>(pks), P<uint8_t>(ct), stride, P<MsgKey>(keys),
                      P<uint32_t>(err), P<uint32_t>(gate), gate_val, P<const uint32_t>(key_tables),
                      S(stream));
    check_launch("seal_setup");
  });
  m.def("open_setup", [](int M, uintptr_t key_idx, uintptr_t sks, uintptr_t pks, uintptr_t ct,
                         uint64_t stride, uintptr_t keys, uintptr_t err, uintptr_t gate,
                         uint32_t gate_val, uintptr_t stream) {
    launch_open_setup(M, P<const uint32_t>(key_idx), P<const uint32_t>(sks),
                      P<const uint32_t>(pks), P<const uint8_t>(ct), stride, P<MsgKey>(keys),
                      P<uint32_t>(err), P<uint32_t>(gate), gate_val, S(stream));
    check_launch("open_setup");
  });
  m.def("gate_wait", [](uintptr_t gate, uint32_t val, uint32_t timeout_us, uintptr_t stream) {
    if (gate == 0) throw std::invalid_argument("gate_wait: null gate");
    launch_gate_wait(P<const uint32_t>(gate), val, timeout_us, S(stream));
    check_launch("gate_wait");
  });
  m.def("x25519", [](int N, uintptr_t sc, uintptr_t pt, uintptr_t out, uintptr_t stream) {
    launch_x25519(N, P<const uint32_t>(sc), P<const uint32_t>(pt), P<uint32_t>(out), S(stream));
    check_launch("x25519");
  });
  m.def("share_additive",
        [](int Pn, int D, int n, uint32_t mod, int value_bytes, uintptr_t secrets, int mask_mode,
           std::vector<uint32_t> rng, uint64_t owner_base, uintptr_t shares, uintptr_t cnt,
           uintptr_t mask_out, uintptr_t mask_cnt, uintptr_t stream) {
          if (n < 1 || n > 256) throw std::invalid_argument("share_additive: n must be 1..256");
          if (mask_mode != kMaskNone && mask_mode != kMaskFull)
            throw std::invalid_argument("share_additive: mask mode none or full (ChaCha masks are "
                                        "applied first: chacha_mask_apply)");
          launch_share_additive(Pn, D, n, mod, value_bytes, P<const int32_t>(secrets), mask_mode,
                                rng_from(rng), owner_base, P<void>(shares), P<uint32_t>(cnt),
                                P<void>(mask_out), P<uint32_t>(mask_cnt), S(stream));
          check_launch("share_additive");
        });
  m.def("share_pss",
        [](int Pn, int D, int n, int k, int t, uint32_t prime, int value_bytes, uintptr_t secrets,
           uintptr_t matrix, int mask_mode, std::vector<uint32_t> rng, uint64_t owner_base,
           uintptr_t shares, uintptr_t cnt, uintptr_t mask_out, uintptr_t mask_cnt,
           uintptr_t stream) {
          if (k > 8 || t > 16 || n > 64)
            throw std::invalid_argument("share_pss: register kernel supports k<=8, t<=16, n<=64");
          if (mask_mode != kMaskNone && mask_mode != kMaskFull)
            throw std::invalid_argument("share_pss: mask mode none or full");
          launch_share_pss(Pn, D, n, k, t, prime, value_bytes, P<const int32_t>(secrets),
                           P<const uint32_t>(matrix), mask_mode, rng_from(rng), owner_base,
                           P<void>(shares), P<uint32_t>(cnt), P<void>(mask_out),
                           P<uint32_t>(mask_cnt), S(stream));
          check_launch("share_pss");
        });
  m.def("set_share16", &set_share16, "use the 16-bit-draw additive share kernel (benchmarking)");
  m.def("set_key_prio", &set_key_prio, "wave priority of open setup / Poly1305 tables (1 = top)");
  m.def("set_pss48", &set_pss48, "packed-Shamir small-field share kernel (benchmarking)");
  m.def("set_mac_mfma", &set_mac_mfma, "matrix-core Poly1305 segments (benchmarking; 0 = Horner)");
  m.def("count", [](int M, int L, int value_bytes, uintptr_t vals, uintptr_t cnt, uintptr_t stream) {
    launch_count(M, L, value_bytes, P<const void>(vals), P<uint32_t>(cnt), S(stream));
    check_launch("count");
  });
  m.def("chacha_seeds", [](int Pn, int seed_words, std::vector<uint32_t> rng, uint64_t owner_base,
                           uintptr_t seeds, uintptr_t stream) {
    if (seed_words < 1 || seed_words > 8) throw std::invalid_argument("chacha_seeds: 1..8 words");
    launch_chacha_seeds(Pn, seed_words, rng_from(rng), owner_base, P<uint32_t>(seeds), S(stream));
    check_launch("chacha_seeds");
  });
  m.def("chacha_scratch_words", &chacha_scratch_words);
  m.def("chacha_sum_groups", &chacha_sum_groups);
  m.def("set_chacha_zone_cap", &set_chacha_zone_cap,
        "test hook: cap the rand-0.3 acceptance zone (2^64 - 1 = none)");
  m.def("chacha_mask_apply", [](int Pn, int D, uint32_t mod, int seed_words, uintptr_t seeds,
                                uintptr_t secrets, uintptr_t masked, uintptr_t scratch,
                                uintptr_t err, uintptr_t stream) {
    if (mod < 2 || seed_words < 1 || seed_words > 8)
      throw std::invalid_argument("chacha_mask_apply: modulus >= 2, seeds of 1..8 words");
    launch_chacha_mask_apply(Pn, D, mod, seed_words, P<const uint32_t>(seeds),
                             P<const int32_t>(secrets), P<int32_t>(masked), P<uint32_t>(scratch),
                             P<uint32_t>(err), S(stream));
    check_launch("chacha_mask_apply");
  });
  m.def("chacha_mask_sum", [](int Pn, int D, uint32_t mod, int seed_words, uintptr_t seeds,
                              uintptr_t out, uintptr_t part, int groups, uintptr_t scratch,
                              uintptr_t fix, uintptr_t err, uintptr_t stream) {
    if (mod < 2 || seed_words < 1 || seed_words > 8 || groups < 1)
      throw std::invalid_argument("chacha_mask_sum: modulus >= 2, seeds of 1..8 words");
    launch_chacha_mask_sum(Pn, D, mod, seed_words, P<const uint32_t>(seeds), P<uint32_t>(out),
                           P<uint32_t>(part), groups, P<uint32_t>(scratch), P<uint64_t>(fix),
                           P<uint32_t>(err), S(stream));
    check_launch("chacha_mask_sum");
  });
  m.def("segscan", [](int M, int T, uintptr_t data, uintptr_t totals, uint32_t expect,
                      uintptr_t err, uintptr_t stream) {
    launch_segscan(M, T, P<uint32_t>(data), P<uint32_t>(totals), expect, P<uint32_t>(err), S(stream));
    check_launch("segscan");
  });
  m.def("encode_encrypt", [](int M, int L, int value_bytes, uintptr_t vals, uintptr_t tile_off,
                             uintptr_t keys, uintptr_t ct, uint64_t stride, uintptr_t pows,
                             uintptr_t pt_len, uintptr_t partials, int K, int max_code_bytes,
                             uintptr_t stream) {
    launch_encode_encrypt(M, L, value_bytes, P<const void>(vals), P<const uint32_t>(tile_off),
                          P<const MsgKey>(keys), P<uint8_t>(ct), stride, P<const uint32_t>(pows),
                          P<const uint32_t>(pt_len), P<uint32_t>(partials), K, max_code_bytes, S(stream));
    check_launch("encode_encrypt");
  });
  m.def("poly_powers", [](int M, uintptr_t keys, uintptr_t pows, int full, uintptr_t stream) {
    launch_poly_powers(M, P<const MsgKey>(keys), P<uint32_t>(pows), full, S(stream));
    check_launch("poly_powers");
  });
  m.def("mac_edges", [](int M, int K, uintptr_t keys, uintptr_t pows, uintptr_t ct, uint64_t stride,
                        uintptr_t pt_len, uintptr_t partials, uintptr_t stream) {
    launch_mac_edges(M, K, P<const MsgKey>(keys), P<const uint32_t>(pows), P<const uint8_t>(ct), stride,
                     P<const uint32_t>(pt_len), P<uint32_t>(partials), S(stream));
    check_launch("mac_edges");
  });
  m.def("mac_chunks", [](int M, int K, uintptr_t keys, uintptr_t pows, uintptr_t ct,
                         uint64_t stride, uintptr_t pt_len, uintptr_t partials, int decrypt,
                         uintptr_t term_cnt, uintptr_t sub_cnt, uintptr_t stream) {
    launch_mac_chunks(M, K, P<const MsgKey>(keys), P<const uint32_t>(pows), P<uint8_t>(ct), stride,
                      P<const uint32_t>(pt_len), P<uint32_t>(partials), decrypt,
                      P<uint32_t>(term_cnt), P<uint32_t>(sub_cnt), S(stream));
    check_launch("mac_chunks");
  });
  m.def("poly_powers_short", [](int M, uintptr_t keys, uintptr_t pows, uintptr_t stream) {
    launch_poly_powers_short(M, P<const MsgKey>(keys), P<uint32_t>(pows), S(stream));
    check_launch("poly_powers_short");
  });
  m.def("mac_short", [](int M, uintptr_t keys, uintptr_t pows, uintptr_t ct, uint64_t stride,
                        uintptr_t pt_len, int verify, uintptr_t ok, uintptr_t err, uintptr_t stream) {
    launch_mac_short(M, P<const MsgKey>(keys), P<const uint32_t>(pows), P<uint8_t>(ct), stride,
                     P<const uint32_t>(pt_len), verify, P<uint32_t>(ok), P<uint32_t>(err), S(stream));
    check_launch("mac_short");
  });
  m.def("decrypt_count", [](int M, int K, uintptr_t keys, uintptr_t ct, uint64_t stride,
                            uintptr_t pt_len, uintptr_t term_cnt, uintptr_t sub_cnt,
                            uintptr_t stream) {
    launch_decrypt_count(M, K, P<const MsgKey>(keys), P<uint8_t>(ct), stride,
                         P<const uint32_t>(pt_len), P<uint32_t>(term_cnt), P<uint32_t>(sub_cnt),
                         S(stream));
    check_launch("decrypt_count");
  });
  m.def("mac_final", [](int M, int K, uintptr_t keys, uintptr_t pows, uintptr_t ct, uint64_t stride,
                        uintptr_t pt_len, uintptr_t partials, int verify, uintptr_t ok,
                        uintptr_t err, uintptr_t stream) {
    launch_mac_final(M, K, P<const MsgKey>(keys), P<const uint32_t>(pows), P<uint8_t>(ct), stride,
                     P<const uint32_t>(pt_len), P<const uint32_t>(partials), verify,
                     P<uint32_t>(ok), P<uint32_t>(err), S(stream));
    check_launch("mac_final");
  });
  m.def("decode", [](int M, int K, int L, uint32_t mod, int value_bytes, uintptr_t pt,
                     uint64_t stride, uintptr_t pt_len, uintptr_t elem_start, uintptr_t vals,
                     uintptr_t err, uintptr_t stream) {
    launch_decode(M, K, L, mod, value_bytes, P<const uint8_t>(pt), stride,
                  P<const uint32_t>(pt_len), P<const uint32_t>(elem_start), P<void>(vals),
                  P<uint32_t>(err), S(stream));
    check_launch("decode");
  });
  m.attr("SUB_BYTES") = kSubBytes;
  m.attr("SUM_TILE") = kSumTile;
  m.attr("POW_WORDS") = kPowWords;
  m.attr("KEY_TABLE_WORDS") = kKeyTableWords;
  m.attr("POW_SHORT_WORDS") = kPowShortWords;
  m.attr("SHORT_MAX_CHUNKS") = kShortMaxChunks;
  m.def("locate_tiles", [](int M, int Sn, int L, uintptr_t pre, uintptr_t totals,
                           uintptr_t tile_sub, uintptr_t stream) {
    launch_locate_tiles(M, Sn, L, P<const uint32_t>(pre), P<const uint32_t>(totals),
                        P<uint32_t>(tile_sub), S(stream));
    check_launch("locate_tiles");
  });
  m.def("decode_sum", [](int R, int Pn, int Pg, int L, uint32_t mod, uintptr_t pt, uint64_t stride,
                         uintptr_t pt_len, int Sn, uintptr_t pre, uintptr_t tile_sub,
                         uintptr_t part, uintptr_t out, uintptr_t acc, uintptr_t err, uintptr_t redo,
                         uintptr_t stream) {
    if (mod == 0) throw std::invalid_argument("decode_sum: needs a modulus");
    if (out == 0 && acc == 0) throw std::invalid_argument("decode_sum: needs out or acc");
    if (!decode_sum_wide(mod) && (uint64_t)Pg * (mod - 1) > 0xffffffffull)
      throw std::invalid_argument("decode_sum: Pg * (m - 1) overflows the u32 accumulators");
    // lean kernels add zigzag codes: up to 14 bits (two bytes), 21 (three) or 28 (four)
    const uint64_t code_max = mod <= 8192u ? 16383ull
                              : 2ull * (mod - 1) < (1ull << 21) ? (1ull << 21) - 1 : (1ull << 28) - 1;
    if (redo != 0 && mod <= (1u << 27) && (uint64_t)Pg * code_max > 0xffffffffull)
      throw std::invalid_argument("decode_sum: Pg codes overflow the u32 accumulators");
    launch_decode_sum(R, Pn, Pg, L, mod, P<const uint8_t>(pt), stride, P<const uint32_t>(pt_len), Sn,
                      P<const uint32_t>(pre), P<const uint32_t>(tile_sub), P<uint32_t>(part),
                      P<uint32_t>(out), P<int64_t>(acc), P<uint32_t>(err), P<uint32_t>(redo), S(stream));
    check_launch("decode_sum");
  });
  m.def("set_decode_lean", &set_decode_lean);
  m.def("set_decode_swz", &set_decode_swz);
  m.def("set_decode_long", &set_decode_long);
  m.def("set_encode_tile2", &set_encode_tile2);
  m.def("set_seal_many", &set_seal_many);
  m.def("x25519_base", [](int N, uintptr_t sc, uintptr_t out, uintptr_t stream) {
    launch_x25519_base(N, P<const uint32_t>(sc), P<uint32_t>(out), S(stream));
    check_launch("x25519_base");
  });
  m.def("set_gemm_fold_f64", &set_gemm_fold_f64);
  m.def("set_gemm_panel", &set_gemm_panel);
  m.def("colsum", [](int G, int R, int L, uint32_t mod, int value_bytes, uintptr_t vals,
                     uintptr_t out, uintptr_t stream) {
    launch_colsum(G, R, L, mod, value_bytes, P<const void>(vals), P<uint32_t>(out), S(stream));
    check_launch("colsum");
  });
  m.def("pss_reconstruct", [](int B, int k, int nI, int D, uint32_t prime, uintptr_t lag,
                              uintptr_t ys, uintptr_t out, uintptr_t stream) {
    launch_pss_reconstruct(B, k, nI, D, prime, P<const uint32_t>(lag), P<const uint32_t>(ys),
                           P<uint32_t>(out), S(stream));
    check_launch("pss_reconstruct");
  });
  m.def("a_fragments_bytes", &a_fragments_bytes);
  m.def("a_fragments", [](int M, int Kp, int limbs, uintptr_t A, uintptr_t out, uintptr_t stream) {
    if (Kp % 64 != 0) throw std::invalid_argument("a_fragments: Kp must be a multiple of 64");
    launch_a_fragments(M, Kp, limbs, P<const int8_t>(A), P<int8_t>(out), S(stream));
    check_launch("a_fragments");
  });
  m.def("modgemm_i8", [](int M, int N, int Kp, int batches, int limbs, uint32_t prime,
                         uintptr_t A, uintptr_t a_frag, uintptr_t B, int64_t b_plane, int value_bytes, uintptr_t C,
                         int64_t ldc_z, int64_t ldc_m, int64_t ldc_n, int64_t limit,
                         uintptr_t cnt, uintptr_t stream) {
    if (Kp % 64 != 0) throw std::invalid_argument("modgemm_i8: Kp must be a multiple of 64");
    if (prime < 2 || prime >= (1u << 28)) throw std::invalid_argument("modgemm_i8: modulus must be in [2, 2^28)");
    if (limbs != limb_scheme(prime, Kp).limbs)
      throw std::invalid_argument("modgemm_i8: limb count does not match limb_scheme(prime, Kp)");
    if ((int64_t)Kp * 128 * 128 * limbs >= (int64_t)1 << 31)
      throw std::invalid_argument("modgemm_i8: K too large for int32 limb accumulators");
    launch_modgemm_i8(M, N, Kp, batches, limbs, prime, P<const int8_t>(A), P<const int8_t>(a_frag), P<const int8_t>(B), b_plane,
                      value_bytes, P<void>(C), ldc_z, ldc_m, ldc_n, limit, P<uint32_t>(cnt), S(stream));
    check_launch("modgemm_i8");
  });
  m.def("limb_scheme", [](uint32_t prime, int Kp) {
    const LimbScheme sch = limb_scheme(prime, Kp);
    return std::make_pair(sch.limbs, sch.bits);
  });
  m.def("pss_x_limbs", [](int Pn, int D, int B, int k, int t, int Kp, uint32_t prime,
                          uintptr_t secrets, std::vector<uint32_t> rng, uint64_t owner_base,
                          uintptr_t X, uintptr_t stream) {
    if (Kp % 64 != 0 || Kp < k + t) throw std::invalid_argument("pss_x_limbs: bad Kp");
    launch_pss_x_limbs(Pn, D, B, k, t, Kp, prime, P<const int32_t>(secrets), rng_from(rng),
                       owner_base, P<int8_t>(X), S(stream));
    check_launch("pss_x_limbs");
  });
  m.def("limbs_t", [](int R, int N, int Kp, uint32_t prime, uintptr_t Y, uintptr_t out,
                      uintptr_t stream) {
    if (Kp % 64 != 0 || Kp < R) throw std::invalid_argument("limbs_t: bad Kp");
    launch_limbs_t(R, N, Kp, prime, P<const uint32_t>(Y), P<int8_t>(out), S(stream));
    check_launch("limbs_t");
  });
  m.def("sub_mod", [](int D, uint32_t mod, uintptr_t a, uintptr_t b, uintptr_t out,
                      uintptr_t stream) {
    launch_sub_mod(D, mod, P<const uint32_t>(a), P<const uint32_t>(b), P<uint32_t>(out), S(stream));
    check_launch("sub_mod");
  });
}
