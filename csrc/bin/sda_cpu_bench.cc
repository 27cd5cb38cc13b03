// Reference-equivalent CPU baseline for the headline metric (aggregated secret-shared elements/s).
//
// The reference publishes no numbers and cannot be built here (no Rust), so the
// comparison point is its algorithm, step for step, in C++ on the host:
//   participant  additive shares from the OS RNG, one draw per share value
//                (rand-0.3 OsRng gen_range: client/src/crypto/sharing/additive.rs:32-51),
//                Rust `%` for the last share, zigzag varints + one sealed box per
//                clerk (client/src/crypto/encryption/sodium.rs)
//   server       snapshot transpose (server/src/snapshot.rs:4-47)
//   clerk        open every box, element-wise sum, seal for the recipient
//                (client/src/clerk.rs:63-107)
//   recipient    open the n results, sum, positive() (client/src/receive.rs)
// `--rng chacha` swaps the per-value syscall for a buffered ChaCha20 stream and
// `--threads T` spreads participants / clerks over threads: a stronger CPU
// point than the reference itself, reported separately.
//
//   sda_cpu_bench [--participants P] [--dim D] [--clerks n] [--modulus m]
//                 [--rng os|chacha] [--threads T]
// Prints one JSON line: elements/s = P * D / end-to-end seconds.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sda/client.hpp"
#include "sda/crypto.hpp"

using namespace sda;
namespace cr = sda::crypto;

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
void parallel_for(size_t n, int threads, F f) {
  if (threads <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : ts) t.join();
}

}  // namespace

int main(int argc, char** argv) {
  size_t P = 10, D = 1000000, n = 3;
  int64_t m = 433;
  int threads = 1;
  std::string rng = "os";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) { std::fprintf(stderr, "%s needs a value\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "--participants") P = std::stoull(val());
    else if (a == "--dim") D = std::stoull(val());
    else if (a == "--clerks") n = std::stoull(val());
    else if (a == "--modulus") m = std::stoll(val());
    else if (a == "--threads") threads = std::stoi(val());
    else if (a == "--rng") rng = val();
    else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
  }
  // keys: n clerks + recipient
  std::vector<EncryptionKeypair> kp(n + 1);
  for (auto& k : kp) {
    cr::box_keypair(k.ek.sodium.data(), k.dk.sodium.data());
  }
  // participant inputs (not timed)
  std::vector<std::vector<int64_t>> secrets(P, std::vector<int64_t>(D));
  {
    uint32_t seed[8] = {1, 2, 3, 4, 5, 6, 7, 8};
    cr::ChaChaRng g(seed, 8);
    for (auto& v : secrets)
      for (auto& x : v) x = g.gen_range(0, m);
  }

  const double t0 = now();
  // ---- participants
  std::vector<std::vector<Encryption>> boxes(P, std::vector<Encryption>(n));
  parallel_for(P, threads, [&](size_t p) {
    std::vector<std::vector<int64_t>> shares(n, std::vector<int64_t>(D));
    uint32_t seed[8];
    for (auto& w : seed) w = cr::os_random_u32();
    cr::ChaChaRng g(seed, 8);
    for (size_t e = 0; e < D; ++e) {
      int64_t last = secrets[p][e];
      for (size_t c = 0; c + 1 < n; ++c) {
        const int64_t r = rng == "os" ? cr::os_random_range(m) : g.gen_range(0, m);
        shares[c][e] = r;
        last = (last - r) % m;
      }
      shares[n - 1][e] = last;
    }
    for (size_t c = 0; c < n; ++c) boxes[p][c] = encrypt_shares(kp[c].ek, shares[c]);
  });
  const double t1 = now();
  // ---- server: transpose P x n -> n x P
  std::vector<std::vector<Encryption>> jobs(n);
  for (size_t c = 0; c < n; ++c)
    for (size_t p = 0; p < P; ++p) jobs[c].push_back(std::move(boxes[p][c]));
  const double t2 = now();
  // ---- clerks
  std::vector<Encryption> results(n);
  parallel_for(n, threads, [&](size_t c) {
    std::vector<int64_t> acc(D, 0);
    for (auto& e : jobs[c]) {
      auto v = decrypt_shares(kp[c], e);
      for (size_t i = 0; i < D; ++i) acc[i] = (acc[i] + v[i]) % m;  // combine (clerk.rs)
    }
    results[c] = encrypt_shares(kp[n].ek, acc);
  });
  const double t3 = now();
  // ---- recipient
  std::vector<int64_t> out(D, 0);
  for (size_t c = 0; c < n; ++c) {
    auto v = decrypt_shares(kp[n], results[c]);
    for (size_t i = 0; i < D; ++i) out[i] = (out[i] + v[i]) % m;
  }
  for (auto& x : out) x = ((x % m) + m) % m;  // RecipientOutput::positive
  const double t4 = now();

  // verify
  bool ok = true;
  for (size_t i = 0; i < D && ok; ++i) {
    int64_t s = 0;
    for (size_t p = 0; p < P; ++p) s += secrets[p][i];
    ok = (s % m) == out[i];
  }
  const double total = t4 - t0;
  std::printf(
      "{\"metric\": \"aggregated secret-shared elements/sec\", \"value\": %.6g, "
      "\"unit\": \"elements/s\", \"participants\": %zu, \"dimension\": %zu, \"clerks\": %zu, "
      "\"modulus\": %lld, \"rng\": \"%s\", \"threads\": %d, \"seconds\": %.4f, "
      "\"stage_s\": {\"participate\": %.4f, \"snapshot\": %.4f, \"clerk\": %.4f, "
      "\"reveal\": %.4f}, \"correct\": %s}\n",
      (double)(P * D) / total, P, D, n, (long long)m, rng.c_str(), threads, total, t1 - t0,
      t2 - t1, t3 - t2, t4 - t3, ok ? "true" : "false");
  return ok ? 0 : 1;
}
