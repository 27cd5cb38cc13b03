// Host self-test for sanitizer builds (`make asan`, `make tsan`): exercises the
// C++ control plane without Python -- crypto round trips, the wire codec, every
// store backend, the in-process workflow with real client crypto (additive and
// packed Shamir, with and without masks), and the HTTP server under concurrent
// REST clients (the multithreaded part the reference ran without any locking
// analysis).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "sda/client.hpp"
#include "sda/crypto.hpp"
#include "sda/http.hpp"
#include "sda/log.hpp"
#include "sda/server.hpp"

using namespace sda;
namespace cr = sda::crypto;
namespace fs = std::filesystem;

namespace {

int g_fail = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

void test_crypto() {
  uint8_t pk[32], sk[32];
  cr::box_keypair(pk, sk);
  for (size_t n : {0u, 1u, 15u, 16u, 17u, 63u, 64u, 1000u, 70000u}) {
    Bytes m(n);
    cr::os_random(m.data(), n);
    Bytes c = cr::box_seal(m.data(), n, pk);
    CHECK(c.size() == n + 48);
    Bytes out;
    CHECK(cr::box_seal_open(out, c.data(), c.size(), pk, sk) && out == m);
    if (n) {
      c[48 + n / 2] ^= 1;
      CHECK(!cr::box_seal_open(out, c.data(), c.size(), pk, sk));
    }
  }
  uint8_t epk[32], esk[64], sig[64];
  cr::ed25519_keypair(epk, esk);
  const char* msg = "canonical json";
  cr::ed25519_sign(sig, reinterpret_cast<const uint8_t*>(msg), 14, esk);
  CHECK(cr::ed25519_verify(sig, reinterpret_cast<const uint8_t*>(msg), 14, epk));
  sig[3] ^= 4;
  CHECK(!cr::ed25519_verify(sig, reinterpret_cast<const uint8_t*>(msg), 14, epk));
}

void test_wire() {
  MemoryStore ks;
  Agent a = SdaClient::new_agent(ks);
  CHECK(wire::decode<Agent>(wire::encode(a)) == a);
  for (const char* bad : {"", "{", "[1,", "{\"id\":1}", "\"\\u12\"", "nul", "1e999999"}) {
    bool threw = false;
    try {
      (void)wire::decode<Agent>(bad);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }
}

LinearSecretSharingScheme additive(size_t n, int64_t m) {
  LinearSecretSharingScheme s;
  s.kind = LinearSecretSharingScheme::Kind::Additive;
  s.share_count = n;
  s.modulus = m;
  return s;
}

LinearSecretSharingScheme pss_483() {
  LinearSecretSharingScheme s;
  s.kind = LinearSecretSharingScheme::Kind::PackedShamir;
  s.secret_count = 3;
  s.share_count = 8;
  s.privacy_threshold_ = 4;
  s.modulus = 433;
  s.omega_secrets = 354;
  s.omega_shares = 150;
  return s;
}

// full_loop.rs equivalent over any service: 2 participants x [1,2,3,4] -> [2,4,6,8]
void full_loop(ServicePtr svc, LinearSecretSharingScheme sharing, LinearMaskingScheme::Kind mask) {
  auto store = [] { return std::make_shared<MemoryStore>(); };
  auto make = [&](StorePtr ks) {
    return std::make_unique<SdaClient>(SdaClient::new_agent(*ks), ks, svc);
  };
  auto rks = store();
  auto rp = make(rks);
  SdaClient& recipient = *rp;
  auto rkey = recipient.new_encryption_key();
  recipient.upload_agent();
  recipient.upload_encryption_key(rkey);
  Aggregation agg;
  agg.id = AggregationId::random();
  agg.title = "selftest";
  agg.vector_dimension = 4;
  agg.modulus = 433;
  agg.recipient = recipient.agent().id;
  agg.recipient_key = rkey;
  agg.masking_scheme.kind = mask;
  agg.masking_scheme.modulus = 433;
  agg.masking_scheme.dimension = 4;
  agg.masking_scheme.seed_bitsize = 128;
  agg.committee_sharing_scheme = sharing;
  recipient.upload_aggregation(agg);
  std::vector<std::unique_ptr<SdaClient>> clerks;
  for (int i = 0; i < 8; ++i) {
    clerks.push_back(make(store()));
    auto k = clerks.back()->new_encryption_key();
    clerks.back()->upload_agent();
    clerks.back()->upload_encryption_key(k);
  }
  recipient.begin_aggregation(agg.id);
  for (int i = 0; i < 2; ++i) {
    auto p = make(store());
    p->upload_agent();
    p->participate({1, 2, 3, 4}, agg.id);
  }
  recipient.end_aggregation(agg.id);
  recipient.run_chores(-1);
  for (auto& c : clerks) c->run_chores(-1);
  auto out = recipient.reveal_aggregation(agg.id).positive();
  CHECK((out.values == std::vector<int64_t>{2, 4, 6, 8}));
}

void test_stores_and_loops(const fs::path& tmp) {
  using K = LinearMaskingScheme::Kind;
  int run = 0;
  // a fresh server per loop: the committee is picked from every keyed agent
  auto fresh = [&](const std::string& kind) -> std::shared_ptr<SdaServerService> {
    const std::string dir = (tmp / (kind + std::to_string(run++))).string();
    if (kind == "memory") return new_memory_server();
    if (kind == "jfs") return new_jfs_server(dir);
    return new_document_server(dir);
  };
  for (const char* kind : {"memory", "jfs", "document"}) {
    full_loop(fresh(kind), additive(3, 433), K::None);
    full_loop(fresh(kind), additive(3, 433), K::Full);
    full_loop(fresh(kind), additive(3, 433), K::ChaCha);
    full_loop(fresh(kind), pss_483(), K::None);
    std::printf("  loops ok: %s\n", kind);
    std::fflush(stdout);
  }
}

void test_http(const fs::path& tmp) {
  auto srv = new_jfs_server((tmp / "http").string());
  auto handler = std::make_shared<SdaHttpHandler>(srv);
  HttpServer http([handler](const HttpRequest& r) { return handler->handle(r); }, 4);
  const int port = http.start("127.0.0.1:0");
  const std::string root = "http://127.0.0.1:" + std::to_string(port) + "/";
  // the full loop over REST
  full_loop(std::make_shared<SdaHttpClient>(root, std::make_shared<MemoryStore>()),
            additive(3, 433), LinearMaskingScheme::Kind::Full);
  // concurrent clients: distinct agents, shared server state
  std::atomic<int> ok{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&] {
      auto tokens = std::make_shared<MemoryStore>();
      auto cli = std::make_shared<SdaHttpClient>(root, tokens);
      MemoryStore ks;
      Agent a = SdaClient::new_agent(ks);
      cli->create_agent(a, a);
      bool good = true;
      for (int i = 0; i < 20; ++i) {
        auto got = cli->get_agent(a, a.id);
        good &= got && *got == a;
        good &= cli->ping().running;
      }
      if (good) ++ok;
    });
  for (auto& t : ts) t.join();
  CHECK(ok == 8);
  http.stop();
}

}  // namespace

int main() {
  set_log_level(1);
  const fs::path tmp = fs::temp_directory_path() / ("sda_selftest_" + std::to_string(::getpid()));
  fs::create_directories(tmp);
  std::setvbuf(stdout, nullptr, _IONBF, 0);
  std::printf("crypto\n");
  test_crypto();
  std::printf("wire\n");
  test_wire();
  std::printf("stores + full loops\n");
  test_stores_and_loops(tmp);
  std::printf("http\n");
  test_http(tmp);
  fs::remove_all(tmp);
  if (g_fail) {
    std::fprintf(stderr, "sda_selftest: %d checks failed\n", g_fail);
    return 1;
  }
  std::printf("sda_selftest: all ok\n");
  return 0;
}
