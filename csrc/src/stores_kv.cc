// Memory and JFS-layout stores (reference server/src/jfs_stores/*).
//
// Both run the same store logic over `Collection`s: std::map-backed in memory,
// or one `<id>.json` file per object (atomic write + rename) in the reference's
// directory layout:
//   DIR/agents/{agents,profiles,encryption_keys}/   DIR/auths/auth_tokens/
//   DIR/agg/{aggregations,committees,snapshots,snapshot_contents,snapshot_masks}/
//   DIR/agg/participations/<agg>/   DIR/jobs/{queue/<clerk>,results/<snap>,done/<clerk>}/
#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>
#include <sstream>

#include "sda/stores.hpp"

namespace sda {

namespace {

void mkdirs(const std::string& path) {
  std::string cur;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    cur = path.substr(0, j);
    if (!cur.empty()) {
      if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
        throw SdaError("store: cannot create directory " + cur);
    }
    i = j + 1;
  }
}

bool safe_id(const std::string& id) {
  if (id.empty() || id.size() > 200) return false;
  for (char c : id)
    if (!(std::isalnum((unsigned char)c) || c == '-' || c == '_')) return false;
  return true;
}

class MemCollection : public Collection {
 public:
  std::optional<std::string> get(const std::string& id) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(id);
    if (it == m_.end()) return std::nullopt;
    return it->second;
  }
  void put(const std::string& id, const std::string& json) override {
    std::lock_guard<std::mutex> g(mu_);
    m_[id] = json;
  }
  bool remove(const std::string& id) override {
    std::lock_guard<std::mutex> g(mu_);
    return m_.erase(id) > 0;
  }
  std::vector<std::pair<std::string, std::string>> all() override {
    std::lock_guard<std::mutex> g(mu_);
    return {m_.begin(), m_.end()};
  }
  std::optional<std::pair<std::string, std::string>> first() override {
    std::lock_guard<std::mutex> g(mu_);
    if (m_.empty()) return std::nullopt;
    return *m_.begin();
  }
  size_t count() override {
    std::lock_guard<std::mutex> g(mu_);
    return m_.size();
  }

 private:
  std::mutex mu_;
  std::map<std::string, std::string> m_;
};

class FileCollection : public Collection {
 public:
  explicit FileCollection(std::string dir) : dir_(std::move(dir)) { mkdirs(dir_); }
  std::optional<std::string> get(const std::string& id) override {
    if (!safe_id(id)) throw SdaError("store: invalid id " + id);
    std::ifstream f(path(id), std::ios::binary | std::ios::ate);
    if (!f) return std::nullopt;
    std::string text((size_t)std::max<std::streamoff>(0, f.tellg()), '\0');  // one read, no stream copy
    f.seekg(0);
    f.read(&text[0], (std::streamsize)text.size());
    text.resize((size_t)f.gcount());
    return text;
  }
  void put(const std::string& id, const std::string& json) override {
    if (!safe_id(id)) throw SdaError("store: invalid id " + id);
    std::string tmp = path(id) + ".tmp" + std::to_string(::getpid()) + "_" +
                      std::to_string(std::hash<std::string>{}(json) & 0xffff);
    {
      std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
      if (!f) throw SdaError("store: cannot write " + tmp);
      f << json;
    }
    if (std::rename(tmp.c_str(), path(id).c_str()) != 0) throw SdaError("store: rename failed");
  }
  bool remove(const std::string& id) override {
    if (!safe_id(id)) throw SdaError("store: invalid id " + id);
    return ::unlink(path(id).c_str()) == 0;
  }
  std::vector<std::pair<std::string, std::string>> all() override {
    std::vector<std::pair<std::string, std::string>> out;
    for (auto& id : ids()) {
      auto v = get(id);
      if (v) out.emplace_back(id, *v);
    }
    return out;
  }
  std::optional<std::pair<std::string, std::string>> first() override {
    for (auto& id : ids()) {
      auto v = get(id);
      if (v) return std::make_pair(id, std::move(*v));
    }
    return std::nullopt;
  }
  size_t count() override { return ids().size(); }

 private:
  std::string path(const std::string& id) const { return dir_ + "/" + id + ".json"; }
  std::vector<std::string> ids() {
    std::vector<std::string> out;
    DIR* d = ::opendir(dir_.c_str());
    if (!d) return out;
    while (dirent* e = ::readdir(d)) {
      std::string n = e->d_name;
      if (n.size() > 5 && n.compare(n.size() - 5, 5, ".json") == 0) out.push_back(n.substr(0, n.size() - 5));
    }
    ::closedir(d);
    std::sort(out.begin(), out.end());
    return out;
  }
  std::string dir_;
};

using CollFactory = std::function<std::shared_ptr<Collection>(const std::string& rel)>;

CollFactory mem_factory() {
  auto reg = std::make_shared<std::map<std::string, std::shared_ptr<Collection>>>();
  auto mu = std::make_shared<std::mutex>();
  return [reg, mu](const std::string& rel) {
    std::lock_guard<std::mutex> g(*mu);
    auto& c = (*reg)[rel];
    if (!c) c = make_mem_collection();
    return c;
  };
}
CollFactory file_factory(const std::string& root) {
  auto reg = std::make_shared<std::map<std::string, std::shared_ptr<Collection>>>();
  auto mu = std::make_shared<std::mutex>();
  return [root, reg, mu](const std::string& rel) {
    std::lock_guard<std::mutex> g(*mu);
    auto& c = (*reg)[rel];
    if (!c) c = make_file_collection(root + "/" + rel);
    return c;
  };
}

// jfs_stores/mod.rs:82-107 semantics
template <class T>
void create_with_id(Collection& c, const std::string& id, const T& obj) {
  std::string js = wire::encode(obj);
  auto prev = c.get(id);
  if (prev && json::Value::parse(*prev) != json::Value::parse(js)) throw SdaError("File already exists");
  c.put(id, js);
}
template <class T>
void update_with_id(Collection& c, const std::string& id, const T& obj) {
  if (!c.get(id)) throw SdaError("File not present");
  c.put(id, wire::encode(obj));
}
template <class T>
void upsert_with_id(Collection& c, const std::string& id, const T& obj) {
  c.put(id, wire::encode(obj));
}
template <class T>
std::optional<T> get_as(Collection& c, const std::string& id) {
  auto v = c.get(id);
  if (!v) return std::nullopt;
  return wire::decode<T>(*v);
}

// ---------------------------------------------------------------------------
class KvAgentsStore : public AgentsStore {
 public:
  explicit KvAgentsStore(CollFactory f)
      : agents_(f("agents/agents")), profiles_(f("agents/profiles")), keys_(f("agents/encryption_keys")) {}
  void create_agent(const Agent& a) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*agents_, a.id.str(), a);
  }
  std::optional<Agent> get_agent(const AgentId& id) override { return get_as<Agent>(*agents_, id.str()); }
  void upsert_profile(const Profile& p) override { upsert_with_id(*profiles_, p.owner.str(), p); }
  std::optional<Profile> get_profile(const AgentId& owner) override {
    return get_as<Profile>(*profiles_, owner.str());
  }
  void create_encryption_key(const SignedEncryptionKey& k) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*keys_, k.body.id.str(), k);
  }
  std::optional<SignedEncryptionKey> get_encryption_key(const EncryptionKeyId& id) override {
    return get_as<SignedEncryptionKey>(*keys_, id.str());
  }
  std::vector<ClerkCandidate> suggest_committee() override {
    std::map<AgentId, std::vector<EncryptionKeyId>> by_signer;
    for (auto& kv : keys_->all()) {
      auto k = wire::decode<SignedEncryptionKey>(kv.second);
      by_signer[k.signer].push_back(k.body.id);
    }
    std::vector<ClerkCandidate> out;
    for (auto& s : by_signer) out.push_back(ClerkCandidate{s.first, s.second});
    return out;
  }

 private:
  std::mutex mu_;
  std::shared_ptr<Collection> agents_, profiles_, keys_;
};

class KvAuthTokensStore : public AuthTokensStore {
 public:
  explicit KvAuthTokensStore(CollFactory f) : tokens_(f("auths/auth_tokens")) {}
  void upsert_auth_token(const AuthToken& t) override { upsert_with_id(*tokens_, t.id.str(), t); }
  std::optional<AuthToken> get_auth_token(const AgentId& id) override {
    return get_as<AuthToken>(*tokens_, id.str());
  }
  void delete_auth_token(const AgentId& id) override { tokens_->remove(id.str()); }

 private:
  std::shared_ptr<Collection> tokens_;
};

class KvAggregationsStore : public AggregationsStore {
 public:
  explicit KvAggregationsStore(CollFactory f)
      : f_(f), aggs_(f("agg/aggregations")), committees_(f("agg/committees")),
        snapshots_(f("agg/snapshots")), contents_(f("agg/snapshot_contents")),
        masks_(f("agg/snapshot_masks")) {}

  std::vector<AggregationId> list_aggregations(const std::optional<std::string>& filter,
                                               const std::optional<AgentId>& recipient) override {
    std::vector<AggregationId> out;
    for (auto& kv : aggs_->all()) {
      auto a = wire::decode<Aggregation>(kv.second);
      if (filter && a.title.find(*filter) == std::string::npos) continue;
      if (recipient && a.recipient != *recipient) continue;
      out.push_back(a.id);
    }
    return out;
  }
  void create_aggregation(const Aggregation& a) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*aggs_, a.id.str(), a);
  }
  std::optional<Aggregation> get_aggregation(const AggregationId& id) override {
    return get_as<Aggregation>(*aggs_, id.str());
  }
  void delete_aggregation(const AggregationId& id) override {
    std::lock_guard<std::mutex> g(mu_);
    aggs_->remove(id.str());
    committees_->remove(id.str());  // the reference leaves these behind
    auto parts = participations(id);
    for (auto& kv : parts->all()) parts->remove(kv.first);
  }
  std::optional<Committee> get_committee(const AggregationId& owner) override {
    return get_as<Committee>(*committees_, owner.str());
  }
  void create_committee(const Committee& c) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*committees_, c.aggregation.str(), c);
  }
  void create_participation(const Participation& p) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*participations(p.aggregation), p.id.str(), p);
  }
  void create_snapshot(const Snapshot& s) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*snapshots_, s.id.str(), s);
  }
  std::vector<SnapshotId> list_snapshots(const AggregationId& aggregation) override {
    std::vector<SnapshotId> out;
    for (auto& kv : snapshots_->all()) {
      auto s = wire::decode<Snapshot>(kv.second);
      if (s.aggregation == aggregation) out.push_back(s.id);
    }
    return out;
  }
  std::optional<Snapshot> get_snapshot(const AggregationId&, const SnapshotId& s) override {
    return get_as<Snapshot>(*snapshots_, s.str());
  }
  size_t count_participations(const AggregationId& aggregation) override {
    return participations(aggregation)->count();
  }
  void snapshot_participations(const AggregationId& aggregation, const SnapshotId& snapshot) override {
    std::lock_guard<std::mutex> g(mu_);
    json::Value ids = json::Value::array();
    for (auto& kv : participations(aggregation)->all()) ids.push(json::Value(kv.first));
    json::Value content = json::Value::object();
    content.set("participations", ids);  // SnapshotContent (jfs_stores/aggregations.rs:14-17)
    auto prev = contents_->get(snapshot.str());
    if (prev && json::Value::parse(*prev) != content) throw SdaError("File already exists");
    contents_->put(snapshot.str(), content.dump());
  }
  std::vector<Participation> snapped_participations(const AggregationId& aggregation,
                                                    const SnapshotId& snapshot) override {
    auto content = contents_->get(snapshot.str());
    if (!content) throw SdaError("snapshot content not found");
    auto parts = participations(aggregation);
    std::vector<Participation> out;
    const json::Value doc = json::Value::parse(*content);  // keep alive across the loop
    for (auto& id : doc.at("participations").as_array()) {
      auto p = get_as<Participation>(*parts, id.as_string());
      if (!p) throw SdaError("participation id=" + id.as_string() + " not found");
      out.push_back(std::move(*p));
    }
    return out;
  }
  size_t count_participations_snapshot(const AggregationId&, const SnapshotId& snapshot) override {
    auto content = contents_->get(snapshot.str());
    if (!content) return 0;
    return json::Value::parse(*content).at("participations").size();
  }
  void create_snapshot_mask(const SnapshotId& s, const std::vector<Encryption>& mask) override {
    json::Value arr = json::Value::array();
    for (auto& e : mask) arr.push(wire::to_json(e));
    auto prev = masks_->get(s.str());
    if (prev && json::Value::parse(*prev) != arr) throw SdaError("File already exists");
    masks_->put(s.str(), arr.dump());
  }
  std::optional<std::string> get_snapshot_mask_json(const SnapshotId& s) override {
    return masks_->get(s.str());
  }
  std::optional<std::vector<Encryption>> get_snapshot_mask(const SnapshotId& s) override {
    auto v = masks_->get(s.str());
    if (!v) return std::nullopt;
    std::vector<Encryption> out;
    const json::Value doc = json::Value::parse(*v);
    for (auto& e : doc.as_array()) out.push_back(wire::from_json<Encryption>(e));
    return out;
  }

 private:
  std::shared_ptr<Collection> participations(const AggregationId& a) {
    return f_("agg/participations/" + a.str());
  }
  std::mutex mu_;
  CollFactory f_;
  std::shared_ptr<Collection> aggs_, committees_, snapshots_, contents_, masks_;
};

class KvClerkingJobsStore : public ClerkingJobsStore {
 public:
  explicit KvClerkingJobsStore(CollFactory f) : f_(f) {}
  void enqueue_clerking_job(const ClerkingJob& j) override {
    std::lock_guard<std::mutex> g(mu_);
    create_with_id(*f_("jobs/queue/" + j.clerk.str()), j.id.str(), j);
  }
  std::optional<ClerkingJob> poll_clerking_job(const AgentId& clerk) override {
    auto head = f_("jobs/queue/" + clerk.str())->first();
    if (!head) return std::nullopt;
    return wire::decode<ClerkingJob>(head->second);
  }
  std::optional<ClerkingJob> get_clerking_job(const AgentId& clerk, const ClerkingJobId& job) override {
    return get_as<ClerkingJob>(*f_("jobs/queue/" + clerk.str()), job.str());
  }
  std::optional<std::string> poll_clerking_job_json(const AgentId& clerk) override {
    auto head = f_("jobs/queue/" + clerk.str())->first();
    if (!head) return std::nullopt;
    return std::move(head->second);
  }
  std::optional<ClerkingJob> get_clerking_job_head(const AgentId& clerk, const ClerkingJobId& job) override {
    auto text = f_("jobs/queue/" + clerk.str())->get(job.str());
    if (!text) return std::nullopt;
    if (auto view = wire::scan_clerking_job(*text)) return view->head;
    return wire::decode<ClerkingJob>(*text);
  }
  std::optional<std::string> get_result_json(const SnapshotId& snapshot, const ClerkingJobId& job) override {
    return f_("jobs/results/" + snapshot.str())->get(job.str());
  }
  void create_clerking_result(const ClerkingResult& r) override {
    // atomic queue -> done move (the reference's check-then-write was racy); the job
    // moves as the text it is stored as
    std::lock_guard<std::mutex> g(mu_);
    auto queue = f_("jobs/queue/" + r.clerk.str());
    auto text = queue->get(r.job.str());
    if (!text) throw SdaError("Job not found");
    auto view = wire::scan_clerking_job(*text);
    const SnapshotId snapshot = view ? view->head.snapshot : wire::decode<ClerkingJob>(*text).snapshot;
    upsert_with_id(*f_("jobs/results/" + snapshot.str()), r.job.str(), r);
    f_("jobs/done/" + r.clerk.str())->put(r.job.str(), *text);
    queue->remove(r.job.str());
  }
  std::vector<ClerkingJobId> list_results(const SnapshotId& snapshot) override {
    std::vector<ClerkingJobId> out;
    for (auto& kv : f_("jobs/results/" + snapshot.str())->all())
      out.push_back(wire::decode<ClerkingResult>(kv.second).job);
    return out;
  }
  std::optional<ClerkingResult> get_result(const SnapshotId& snapshot, const ClerkingJobId& job) override {
    return get_as<ClerkingResult>(*f_("jobs/results/" + snapshot.str()), job.str());
  }

 private:
  std::mutex mu_;
  CollFactory f_;
};

Stores make_kv_stores(CollFactory f) {
  Stores s;
  s.agents = std::make_shared<KvAgentsStore>(f);
  s.auth_tokens = std::make_shared<KvAuthTokensStore>(f);
  s.aggregations = std::make_shared<KvAggregationsStore>(f);
  s.clerking_jobs = std::make_shared<KvClerkingJobsStore>(f);
  return s;
}

}  // namespace

std::vector<std::vector<Encryption>> AggregationsStore::snapshot_clerk_jobs_data(
    const AggregationId& aggregation, const SnapshotId& snapshot, size_t clerks) {
  std::vector<std::vector<Encryption>> shares(clerks);
  auto parts = snapped_participations(aggregation, snapshot);
  for (auto& s : shares) s.reserve(parts.size());
  for (auto& p : parts) {
    for (size_t ix = 0; ix < p.clerk_encryptions.size() && ix < clerks; ++ix)
      shares[ix].push_back(std::move(p.clerk_encryptions[ix].second));
  }
  return shares;
}

std::optional<std::string> AggregationsStore::get_snapshot_mask_json(const SnapshotId& snapshot) {
  auto m = get_snapshot_mask(snapshot);
  if (!m) return std::nullopt;
  json::Value arr = json::Value::array();
  for (auto& e : *m) arr.push(wire::to_json(e));
  return arr.dump();
}
std::optional<std::string> ClerkingJobsStore::poll_clerking_job_json(const AgentId& clerk) {
  auto j = poll_clerking_job(clerk);
  if (!j) return std::nullopt;
  return wire::encode(*j);
}
std::optional<ClerkingJob> ClerkingJobsStore::get_clerking_job_head(const AgentId& clerk,
                                                                    const ClerkingJobId& job) {
  return get_clerking_job(clerk, job);
}
std::optional<std::string> ClerkingJobsStore::get_result_json(const SnapshotId& snapshot,
                                                              const ClerkingJobId& job) {
  auto r = get_result(snapshot, job);
  if (!r) return std::nullopt;
  return wire::encode(*r);
}

std::shared_ptr<Collection> make_mem_collection() { return std::make_shared<MemCollection>(); }
std::shared_ptr<Collection> make_file_collection(const std::string& dir) {
  return std::make_shared<FileCollection>(dir);
}

Stores make_memory_stores() { return make_kv_stores(mem_factory()); }
Stores make_jfs_stores(const std::string& dir) {
  mkdirs(dir);
  return make_kv_stores(file_factory(dir));
}

}  // namespace sda
