// `sda` -- the agent command line (reference cli/src/main.rs).
//
//   sda [-s SERVER] [-i IDENTITY] [--device cpu|gpu[:N]] [-v...] <command>
//     ping
//     agent create [-f|--force] | agent show | agent keys create | agent keys show
//     clerk [-o|--once] [--interval SECONDS]
//     aggregations (agg|aggs|aggregation)
//         create TITLE DIMENSION MODULUS KEY SHARE_COUNT [--id ID]
//                [--mask none|full|chacha] [--sharing add|shamir]
//         begin ID | end ID | reveal ID
//     participate ID VALUE...
//     participate-file ID FILE        one vector per line (bulk; one participation each)
//
// `--device gpu` runs the bulk cryptography of clerk / reveal / participate on an
// MI355X through libsda_device.so (loaded on demand; the wire format is
// unchanged, so GPU and CPU agents mix freely in one aggregation).
//
// Identity layout (cli/src/main.rs:99-124): IDENTITY (default `.sda`) holds the
// agent (alias `agent`) and the REST auth token; IDENTITY/keys holds the signing
// and encryption keypairs, one `<key id>.json` each.
//
// Deviations from the reference, all fixes: `--sharing shamir` works for the
// reference's named parameter sets (the reference leaves it unimplemented);
// `--mask chacha` expands over the vector dimension (the reference passes the
// share count); `agent keys show` lists the local keys.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "sda/client.hpp"
#include "sda/field.hpp"
#include "sda/http.hpp"
#include "sda/log.hpp"

using namespace sda;

namespace {

[[noreturn]] void usage(const std::string& why = "") {
  if (!why.empty()) std::fprintf(stderr, "error: %s\n\n", why.c_str());
  std::fprintf(stderr,
               "usage: sda [-s SERVER] [-i IDENTITY] [--device cpu|gpu[:N]] [-v...] <command>\n"
               "  ping                          check service availability\n"
               "  agent create [-f]             create (or reuse) and upload the local agent\n"
               "  agent show                    show the local agent\n"
               "  agent keys create|show        create+upload an encryption key / list keys\n"
               "  clerk [--once] [--interval S] run clerking jobs (loop every S s, default 300)\n"
               "  aggregations create TITLE DIMENSION MODULUS KEY SHARE_COUNT\n"
               "               [--id ID] [--mask none|full|chacha] [--sharing add|shamir]\n"
               "  aggregations begin|end|reveal ID\n"
               "  participate ID VALUE...       contribute a vector\n"
               "  participate-file ID FILE      contribute every line of FILE as a vector\n"
               "  --device gpu[:N]              clerk / reveal / participate on MI355X N\n");
  std::exit(2);
}

struct Args {
  std::vector<std::string> pos;
  std::vector<std::pair<std::string, std::string>> opts;  // --name value / flags ("")
  bool flag(const char* a, const char* b = nullptr) const {
    for (auto& o : opts)
      if (o.first == a || (b && o.first == b)) return true;
    return false;
  }
  std::string opt(const char* a, const char* b, const std::string& def) const {
    for (auto& o : opts)
      if (o.first == a || (b && o.first == b)) return o.second;
    return def;
  }
};

// Options that take a value (everything else starting with '-' is a flag,
// except negative numbers, which are values of `participate`).
bool takes_value(const std::string& o) {
  return o == "-s" || o == "--server" || o == "-i" || o == "--identity" || o == "--id" ||
         o == "--mask" || o == "--sharing" || o == "--interval" || o == "--device";
}

bool is_number(const std::string& s) {
  if (s.empty()) return false;
  size_t i = (s[0] == '-') ? 1 : 0;
  if (i == s.size()) return false;
  for (; i < s.size(); ++i)
    if (s[i] < '0' || s[i] > '9') return false;
  return true;
}

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s == "-h" || s == "--help") usage();
    if (s.size() > 1 && s[0] == '-' && !is_number(s)) {
      if (s.size() > 2 && s[1] != '-' && s.find_first_not_of('v', 1) == std::string::npos) {
        for (size_t k = 1; k < s.size(); ++k) a.opts.push_back({"-v", ""});  // -vvv
        continue;
      }
      auto eq = s.find('=');
      if (s.rfind("--", 0) == 0 && eq != std::string::npos) {
        a.opts.push_back({s.substr(0, eq), s.substr(eq + 1)});
      } else if (takes_value(s)) {
        if (i + 1 >= argc) usage("option " + s + " needs a value");
        a.opts.push_back({s, argv[++i]});
      } else {
        a.opts.push_back({s, ""});
      }
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

int verbosity(const Args& a) {
  int v = 0;
  for (auto& o : a.opts)
    if (o.first == "-v" || o.first == "--verbose") ++v;
  return v;
}

std::string fmt_values(const std::vector<int64_t>& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
  return s;
}

std::vector<std::string> list_key_ids(const std::string& dir) {
  std::vector<std::string> out;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.size() > 5 && n.compare(n.size() - 5, 5, ".json") == 0 && n.rfind("alias_", 0) != 0)
        out.push_back(n.substr(0, n.size() - 5));
    }
    closedir(d);
  }
  return out;
}

LinearSecretSharingScheme shamir_for(size_t share_count, int64_t modulus) {
  for (auto p : {pss_4_8_3(), pss_4_26_3(), pss_155_728_100(), pss_155_19682_100()}) {
    if ((size_t)p.share_count == share_count && (int64_t)p.prime == modulus) {
      LinearSecretSharingScheme s;
      s.kind = LinearSecretSharingScheme::Kind::PackedShamir;
      s.secret_count = p.secret_count;
      s.share_count = p.share_count;
      s.privacy_threshold_ = p.privacy_threshold;
      s.modulus = (int64_t)p.prime;
      s.omega_secrets = (int64_t)p.omega_secrets;
      s.omega_shares = (int64_t)p.omega_shares;
      return s;
    }
  }
  throw SdaError("no packed Shamir parameter set for " + std::to_string(share_count) +
                 " shares mod " + std::to_string(modulus) +
                 " (known: 8 or 26 shares mod 433, 728 mod 746497, 19682 mod 5038849)");
}

int run(const Args& a) {
  if (a.pos.empty()) usage("missing command");
  const std::string server_root = a.opt("-s", "--server", "http://localhost:8888");
  const std::string identity = a.opt("-i", "--identity", ".sda");
  log_debug("Using service at " + server_root);
  auto identity_store = std::make_shared<FileStore>(identity);
  auto keystore = std::make_shared<FileStore>(identity + "/keys");
  auto service = std::make_shared<SdaHttpClient>(server_root, identity_store);
  std::optional<Agent> agent = identity_store->get_aliased<Agent>("agent");
  const std::string& cmd = a.pos[0];
  auto need_agent = [&]() -> Agent {
    if (!agent) throw SdaError("Agent is needed. Maybe run \"sda agent create\" ?");
    return *agent;
  };
  auto arg = [&](size_t i, const char* what) -> const std::string& {
    if (a.pos.size() <= i) usage(std::string("missing ") + what);
    return a.pos[i];
  };
  // --device gpu[:N]: the roles' bulk cryptography on an MI355X
  DeviceBackendPtr device;
  const std::string dev = a.opt("--device", nullptr, "cpu");
  if (dev.rfind("gpu", 0) == 0) {
    int index = 0;
    if (dev.size() > 3) {
      if (dev[3] != ':' || !is_number(dev.substr(4))) usage("--device must be cpu, gpu or gpu:N");
      index = std::stoi(dev.substr(4));
    }
    device = load_device_backend("", index);
    log_info("Roles run on " + device->describe());
  } else if (dev != "cpu" && dev != "host") {
    usage("--device must be cpu, gpu or gpu:N");
  }

  if (cmd == "ping") {
    if (!service->ping().running) throw SdaError("Service may not be running");
    log_info("Service appears to be running");
    return 0;
  }
  if (cmd == "agent") {
    const std::string sub = arg(1, "agent subcommand");
    if (sub == "create") {
      Agent ag;
      if (agent && !a.flag("-f", "--force")) {
        log_warn("Using existing agent; use --force to create new");
        ag = *agent;
      } else {
        ag = SdaClient::new_agent(*keystore);
        identity_store->put_aliased("agent", ag.id.str(), ag);
        log_info("Created new agent with id " + ag.id.str());
      }
      SdaClient(ag, keystore, service).upload_agent();
      return 0;
    }
    if (sub == "show") {
      if (!agent) {
        log_warn("No local agent found");
      } else {
        log_info("Local agent is " + wire::encode(*agent));
        std::printf("%s\n", wire::encode(*agent).c_str());
      }
      return 0;
    }
    if (sub == "keys") {
      const std::string kc = arg(2, "keys subcommand");
      SdaClient client(need_agent(), keystore, service);
      if (kc == "create") {
        auto key = client.new_encryption_key();
        client.upload_encryption_key(key);
        log_info("Created and uploaded key: " + key.str());
        std::printf("%s\n", key.str().c_str());
        return 0;
      }
      if (kc == "show") {
        for (auto& id : list_key_ids(identity + "/keys")) {
          auto v = keystore->get_json(id);
          if (v && v->find("ek")) std::printf("%s\n", id.c_str());
        }
        return 0;
      }
      throw SdaError("Unknown subcommand " + kc);
    }
    throw SdaError("Unknown subcommand " + sub);
  }
  if (cmd == "clerk") {
    Agent ag = need_agent();
    service->ping();
    SdaClient client(ag, keystore, service);
    client.set_device_backend(device);
    const long interval = std::stol(a.opt("--interval", nullptr, "300"));
    for (;;) {
      log_debug("Polling for clerking job");
      client.run_chores(-1);
      if (a.flag("-o", "--once")) return 0;
      std::this_thread::sleep_for(std::chrono::seconds(interval));
    }
  }
  if (cmd == "aggregations" || cmd == "agg" || cmd == "aggs" || cmd == "aggregation") {
    Agent ag = need_agent();
    service->ping();
    SdaClient client(ag, keystore, service);
    client.set_device_backend(device);
    const std::string sub = arg(1, "aggregations subcommand");
    if (sub == "create") {
      Aggregation agg;
      agg.title = arg(2, "title");
      agg.vector_dimension = std::stoull(arg(3, "dimension"));
      agg.modulus = std::stoll(arg(4, "modulus"));
      agg.recipient = ag.id;
      agg.recipient_key = EncryptionKeyId::parse(arg(5, "key"));
      const size_t share_count = std::stoull(arg(6, "share_count"));
      const std::string id = a.opt("--id", nullptr, "");
      agg.id = id.empty() ? AggregationId::random() : AggregationId::parse(id);
      const std::string sharing = a.opt("--sharing", nullptr, "add");
      if (sharing == "add") {
        agg.committee_sharing_scheme.kind = LinearSecretSharingScheme::Kind::Additive;
        agg.committee_sharing_scheme.share_count = share_count;
        agg.committee_sharing_scheme.modulus = agg.modulus;
      } else if (sharing == "shamir") {
        agg.committee_sharing_scheme = shamir_for(share_count, agg.modulus);
      } else {
        usage("--sharing must be add or shamir");
      }
      const std::string mask = a.opt("--mask", nullptr, "none");
      if (mask == "none") {
        agg.masking_scheme.kind = LinearMaskingScheme::Kind::None;
      } else if (mask == "full") {
        agg.masking_scheme.kind = LinearMaskingScheme::Kind::Full;
        agg.masking_scheme.modulus = agg.modulus;
      } else if (mask == "chacha") {
        agg.masking_scheme.kind = LinearMaskingScheme::Kind::ChaCha;
        agg.masking_scheme.modulus = agg.modulus;
        agg.masking_scheme.dimension = agg.vector_dimension;
        agg.masking_scheme.seed_bitsize = 128;
      } else {
        usage("--mask must be none, full or chacha");
      }
      client.upload_aggregation(agg);
      log_info("aggregation created. id: " + agg.id.str());
      std::printf("%s\n", agg.id.str().c_str());
      return 0;
    }
    if (sub == "begin") {
      client.begin_aggregation(AggregationId::parse(arg(2, "aggregation id")));
      return 0;
    }
    if (sub == "end") {
      client.end_aggregation(AggregationId::parse(arg(2, "aggregation id")));
      return 0;
    }
    if (sub == "reveal") {
      auto out = client.reveal_aggregation(AggregationId::parse(arg(2, "aggregation id"))).positive();
      std::printf("result: RecipientOutput { modulus: %lld, values: [%s] }\n",
                  (long long)out.modulus, fmt_values(out.values).c_str());
      return 0;
    }
    throw SdaError("Unknown command " + sub);
  }
  if (cmd == "participate") {
    SdaClient client(need_agent(), keystore, service);
    const AggregationId id = AggregationId::parse(arg(1, "aggregation id"));
    std::vector<int64_t> values;
    for (size_t i = 2; i < a.pos.size(); ++i) {
      if (!is_number(a.pos[i])) usage("not an integer: " + a.pos[i]);
      values.push_back(std::stoll(a.pos[i]));
    }
    if (device) client.set_device_backend(device), client.participate_many({values}, id);
    else client.participate(values, id);
    return 0;
  }
  if (cmd == "participate-file") {
    SdaClient client(need_agent(), keystore, service);
    client.set_device_backend(device);
    const AggregationId id = AggregationId::parse(arg(1, "aggregation id"));
    std::ifstream in(arg(2, "file"));
    if (!in) throw SdaError("cannot read " + a.pos[2]);
    std::vector<std::vector<int64_t>> inputs;
    std::string line;
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::vector<int64_t> v;
      std::string tok;
      while (ls >> tok) {
        if (!tok.empty() && tok.back() == ',') tok.pop_back();
        if (!is_number(tok)) throw SdaError("not an integer: " + tok);
        v.push_back(std::stoll(tok));
      }
      if (!v.empty()) inputs.push_back(std::move(v));
    }
    client.participate_many(inputs, id);
    log_info("Uploaded " + std::to_string(inputs.size()) + " participations");
    return 0;
  }
  throw SdaError("Unknown command " + cmd);
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  set_log_level(4 + verbosity(a));  // info by default, like the reference
  try {
    return run(a);
  } catch (const std::exception& e) {
    log_error(e.what());
    return 1;
  }
}
