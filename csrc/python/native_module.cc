// pybind11 bindings of the host control plane (`sda_amd._lib._sda_native`).
//
// Part 1 (this file): crypto primitives and field / packed-Shamir math, used by
// the GPU engine (key generation, matrices) and as the bit-exact oracle in tests.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "sda/crypto.hpp"
#include "sda/field.hpp"

namespace py = pybind11;
using namespace sda;

namespace sda {
namespace crypto {
uint64_t sha512_round_constant(int i);
uint64_t sha512_iv(int i);
}  // namespace crypto
}  // namespace sda

namespace {

std::string as_str(const uint8_t* p, size_t n) { return std::string(reinterpret_cast<const char*>(p), n); }
const uint8_t* U(const std::string& s) { return reinterpret_cast<const uint8_t*>(s.data()); }
void need(const std::string& s, size_t n, const char* what) {
  if (s.size() != n) throw std::invalid_argument(std::string(what) + ": wrong length");
}

}  // namespace

void bind_control_plane(py::module_& m);  // control_bindings.cc

PYBIND11_MODULE(_sda_native, m) {
  m.doc() = "SDA host control plane + crypto (C++)";

  py::register_exception<SdaError>(m, "SdaNativeError");

  auto c = m.def_submodule("crypto", "host crypto primitives");
  c.def("random_bytes", [](size_t n) {
    std::string s(n, '\0');
    crypto::os_random(reinterpret_cast<uint8_t*>(&s[0]), n);
    return py::bytes(s);
  });
  c.def("sha512", [](py::bytes b) {
    std::string s = b;
    uint8_t out[64];
    crypto::sha512(U(s), s.size(), out);
    return py::bytes(as_str(out, 64));
  });
  c.def("sha512_round_constant", &crypto::sha512_round_constant);
  c.def("sha512_iv", &crypto::sha512_iv);
  c.def("blake2b", [](py::bytes b, size_t outlen, py::bytes key) {
    std::string s = b, k = key;
    uint8_t out[64];
    crypto::blake2b(out, outlen, U(s), s.size(), k.empty() ? nullptr : U(k), k.size());
    return py::bytes(as_str(out, outlen));
  }, py::arg("data"), py::arg("outlen") = 64, py::arg("key") = py::bytes(""));
  c.def("salsa20_block", [](py::bytes key, py::bytes nonce, uint64_t ctr) {
    std::string k = key, n = nonce;
    need(k, 32, "key"); need(n, 8, "nonce");
    uint8_t out[64];
    crypto::salsa20_block(out, U(k), U(n), ctr);
    return py::bytes(as_str(out, 64));
  });
  c.def("hsalsa20", [](py::bytes key, py::bytes in16) {
    std::string k = key, n = in16;
    need(k, 32, "key"); need(n, 16, "input");
    uint8_t out[32];
    crypto::hsalsa20(out, U(k), U(n));
    return py::bytes(as_str(out, 32));
  });
  c.def("xsalsa20_xor", [](py::bytes data, py::bytes nonce, py::bytes key, uint64_t ofs) {
    std::string d = data, n = nonce, k = key;
    need(n, 24, "nonce"); need(k, 32, "key");
    std::string out(d.size(), '\0');
    crypto::xsalsa20_xor(reinterpret_cast<uint8_t*>(&out[0]), U(d), d.size(), U(n), U(k), ofs);
    return py::bytes(out);
  }, py::arg("data"), py::arg("nonce"), py::arg("key"), py::arg("offset") = 0);
  c.def("chacha20_block_words", [](std::vector<uint32_t> in, int rounds) {
    if (in.size() != 16) throw std::invalid_argument("need 16 words");
    uint32_t out[16];
    crypto::chacha20_block_words(out, in.data(), rounds);
    return std::vector<uint32_t>(out, out + 16);
  }, py::arg("words"), py::arg("rounds") = 20);
  c.def("set_chacha_zone_cap", &crypto::set_chacha_zone_cap,
        "test hook: cap the rand-0.3 acceptance zone of ChaChaRng.gen_range (2^64 - 1 = none)");
  py::class_<crypto::ChaChaRng>(c, "ChaChaRng")
      .def(py::init([](std::vector<uint32_t> seed) {
        return new crypto::ChaChaRng(seed.data(), seed.size());
      }))
      .def("next_u32", &crypto::ChaChaRng::next_u32)
      .def("next_u64", &crypto::ChaChaRng::next_u64)
      .def("gen_range", &crypto::ChaChaRng::gen_range);
  c.def("poly1305", [](py::bytes msg, py::bytes key) {
    std::string d = msg, k = key;
    need(k, 32, "key");
    uint8_t tag[16];
    crypto::poly1305(tag, U(d), d.size(), U(k));
    return py::bytes(as_str(tag, 16));
  });
  c.def("x25519", [](py::bytes scalar, py::bytes point) {
    std::string a = scalar, b = point;
    need(a, 32, "scalar"); need(b, 32, "point");
    uint8_t out[32];
    bool ok = crypto::x25519(out, U(a), U(b));
    return py::make_tuple(py::bytes(as_str(out, 32)), ok);
  });
  c.def("x25519_base", [](py::bytes scalar) {
    std::string a = scalar;
    need(a, 32, "scalar");
    uint8_t out[32];
    crypto::x25519_base(out, U(a));
    return py::bytes(as_str(out, 32));
  });
  c.def("x25519_comb_tables", [](std::vector<std::string> pks) {
    // one table of kX25519CombTableWords little-endian words per key (zeros where the key
    // has none), and which keys got one
    std::string blob(pks.size() * crypto::kX25519CombTableWords * 4, '\0');
    std::vector<bool> ok(pks.size());
    for (size_t i = 0; i < pks.size(); ++i) {
      need(pks[i], 32, "public key");
      ok[i] = crypto::x25519_comb_table(
          reinterpret_cast<uint32_t*>(&blob[i * crypto::kX25519CombTableWords * 4]), U(pks[i]));
    }
    return py::make_tuple(py::bytes(blob), ok);
  });
  c.def("box_keypair", []() {
    uint8_t pk[32], sk[32];
    crypto::box_keypair(pk, sk);
    return py::make_tuple(py::bytes(as_str(pk, 32)), py::bytes(as_str(sk, 32)));
  });
  c.def("box_beforenm", [](py::bytes pk, py::bytes sk) {
    std::string a = pk, b = sk;
    need(a, 32, "pk"); need(b, 32, "sk");
    uint8_t k[32];
    if (!crypto::box_beforenm(k, U(a), U(b))) throw SdaError("box_beforenm: invalid key");
    return py::bytes(as_str(k, 32));
  });
  c.def("secretbox_easy", [](py::bytes msg, py::bytes nonce, py::bytes key) {
    std::string d = msg, n = nonce, k = key;
    need(n, 24, "nonce"); need(k, 32, "key");
    std::string out(d.size() + 16, '\0');
    crypto::secretbox_easy(reinterpret_cast<uint8_t*>(&out[0]), U(d), d.size(), U(n), U(k));
    return py::bytes(out);
  });
  c.def("seal_nonce", [](py::bytes epk, py::bytes pk) {
    std::string a = epk, b = pk;
    need(a, 32, "epk"); need(b, 32, "pk");
    uint8_t n[24];
    crypto::seal_nonce(n, U(a), U(b));
    return py::bytes(as_str(n, 24));
  });
  c.def("box_seal", [](py::bytes msg, py::bytes pk, py::object esk) {
    std::string d = msg, k = pk;
    need(k, 32, "pk");
    std::string e;
    const uint8_t* ep = nullptr;
    if (!esk.is_none()) { e = esk.cast<std::string>(); need(e, 32, "esk"); ep = U(e); }
    Bytes out = crypto::box_seal(U(d), d.size(), U(k), ep);
    return py::bytes(as_str(out.data(), out.size()));
  }, py::arg("msg"), py::arg("pk"), py::arg("esk") = py::none());
  c.def("box_seal_open", [](py::bytes ct, py::bytes pk, py::bytes sk) -> py::object {
    std::string d = ct, a = pk, b = sk;
    need(a, 32, "pk"); need(b, 32, "sk");
    Bytes out;
    if (!crypto::box_seal_open(out, U(d), d.size(), U(a), U(b))) return py::none();
    return py::bytes(as_str(out.data(), out.size()));
  });
  c.def("ed25519_keypair_from_seed", [](py::bytes seed) {
    std::string s = seed;
    need(s, 32, "seed");
    uint8_t pk[32], sk[64];
    crypto::ed25519_keypair_from_seed(pk, sk, U(s));
    return py::make_tuple(py::bytes(as_str(pk, 32)), py::bytes(as_str(sk, 64)));
  });
  c.def("ed25519_keypair", []() {
    uint8_t pk[32], sk[64];
    crypto::ed25519_keypair(pk, sk);
    return py::make_tuple(py::bytes(as_str(pk, 32)), py::bytes(as_str(sk, 64)));
  });
  c.def("ed25519_sign", [](py::bytes msg, py::bytes sk) {
    std::string d = msg, k = sk;
    need(k, 64, "sk");
    uint8_t sig[64];
    crypto::ed25519_sign(sig, U(d), d.size(), U(k));
    return py::bytes(as_str(sig, 64));
  });
  c.def("ed25519_verify", [](py::bytes sig, py::bytes msg, py::bytes pk) {
    std::string s = sig, d = msg, k = pk;
    if (s.size() != 64 || k.size() != 32) return false;
    return crypto::ed25519_verify(U(s), U(d), d.size(), U(k));
  });

  auto f = m.def_submodule("field", "prime field / packed Shamir");
  f.def("mod_pow", &mod_pow);
  f.def("mod_inv", &mod_inv);
  f.def("mult_order", &mult_order, py::arg("w"), py::arg("p"), py::arg("limit") = 1u << 22);
  py::class_<PackedShamirParams>(f, "PackedShamirParams")
      .def(py::init([](int k, int n, int t, int64_t p, int64_t ws, int64_t wn) {
             return PackedShamirParams{k, n, t, p, ws, wn};
           }),
           py::arg("secret_count"), py::arg("share_count"), py::arg("privacy_threshold"),
           py::arg("prime_modulus"), py::arg("omega_secrets"), py::arg("omega_shares"))
      .def_readonly("secret_count", &PackedShamirParams::secret_count)
      .def_readonly("share_count", &PackedShamirParams::share_count)
      .def_readonly("privacy_threshold", &PackedShamirParams::privacy_threshold)
      .def_readonly("prime_modulus", &PackedShamirParams::prime)
      .def_readonly("omega_secrets", &PackedShamirParams::omega_secrets)
      .def_readonly("omega_shares", &PackedShamirParams::omega_shares)
      .def("reconstruct_limit", &PackedShamirParams::reconstruct_limit)
      .def("validate", &PackedShamirParams::validate)
      .def("share_matrix", &PackedShamirParams::share_matrix)
      .def("lagrange_matrix", &PackedShamirParams::lagrange_matrix)
      .def("share", &PackedShamirParams::share)
      .def("reconstruct", &PackedShamirParams::reconstruct);
  f.def("pss_4_8_3", &pss_4_8_3);
  f.def("pss_4_26_3", &pss_4_26_3);
  f.def("pss_155_728_100", &pss_155_728_100);
  f.def("pss_155_19682_100", &pss_155_19682_100);

  bind_control_plane(m);
}
