// Document store with the MongoDB data model of the reference's production
// backend (server-store-mongodb/src/*.rs), on a native embedded document engine.
//
// No MongoDB server or driver exists in this environment, so the engine here
// implements exactly the operations the reference DAO uses (server-store-mongodb/src/*.rs):
// unique `id` index, find/find_one by dotted-path equality, $set / $push /
// $pull / $addToSet updates with upsert, update_many, count, and the snapshot
// transpose pipeline ($match -> $unwind(includeArrayIndex) -> $group -> $sort).
// Documents persist one JSON file per document under DIR/<collection>/ when a
// directory is given (so a restarted sdad resumes), otherwise in memory.
//
// Collections / documents (as in the reference):
//   agents         {id, agent, profile, keys: [{id, body: SignedEncryptionKey}]}
//   auth_tokens    {id, token}
//   aggregations   {id, aggregation, committee}
//   participations {id, participation, snapshots: [SnapshotId]}
//   snapshots      {id, snapshot, mask}
//   clerking_jobs  {id, clerking_job, done, result}
#include <map>
#include <mutex>

#include "sda/stores.hpp"

namespace sda {

namespace {

using json::Value;

const Value* path_get(const Value& doc, const std::string& path) {
  const Value* cur = &doc;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('.', i);
    if (j == std::string::npos) j = path.size();
    if (!cur->is_object()) return nullptr;
    cur = cur->find(path.substr(i, j - i));
    if (!cur) return nullptr;
    i = j + 1;
  }
  return cur;
}

// Mongo equality semantics: a field equals v, or (for arrays) contains v.
bool matches(const Value& doc, const std::vector<std::pair<std::string, Value>>& filter) {
  for (auto& f : filter) {
    const Value* v = path_get(doc, f.first);
    if (!v) {
      if (!f.second.is_null()) return false;
      continue;
    }
    if (*v == f.second) continue;
    if (v->is_array()) {
      bool found = false;
      for (auto& e : v->as_array())
        if (e == f.second) { found = true; break; }
      if (found) continue;
    }
    return false;
  }
  return true;
}

class DocCollection {
 public:
  DocCollection(std::string name, const std::string& dir) : name_(std::move(name)) {
    if (!dir.empty()) {
      files_ = make_file_collection(dir + "/" + name_);
      for (auto& kv : files_->all()) docs_[kv.first] = Value::parse(kv.second);
    }
  }
  using Filter = std::vector<std::pair<std::string, Value>>;

  std::optional<Value> find_one(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : docs_)
      if (matches(kv.second, f)) return kv.second;
    return std::nullopt;
  }
  std::vector<Value> find(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Value> out;
    for (auto& kv : docs_)
      if (matches(kv.second, f)) out.push_back(kv.second);
    return out;
  }
  size_t count(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (auto& kv : docs_) n += matches(kv.second, f) ? 1 : 0;
    return n;
  }
  // {$set: fields} by id, optionally upserting (Dao::modisert_by_id / modify_by_id)
  bool set_by_id(const std::string& id, const Value::Object& fields, bool upsert) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = docs_.find(id);
    if (it == docs_.end()) {
      if (!upsert) return false;
      Value d = Value::object();
      d.set("id", Value(id));
      it = docs_.emplace(id, d).first;
    }
    for (auto& kv : fields) it->second.set(kv.first, kv.second);
    persist(id, it->second);
    return true;
  }
  // mutate with a callback under the lock (push / pull / addToSet)
  template <class F>
  bool update_by_id(const std::string& id, F fn) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = docs_.find(id);
    if (it == docs_.end()) return false;
    fn(it->second);
    persist(id, it->second);
    return true;
  }
  template <class F>
  size_t update_many(const Filter& f, F fn) {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (auto& kv : docs_) {
      if (!matches(kv.second, f)) continue;
      fn(kv.second);
      persist(kv.first, kv.second);
      ++n;
    }
    return n;
  }
  bool delete_one(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    if (files_) files_->remove(id);
    return docs_.erase(id) > 0;
  }

 private:
  void persist(const std::string& id, const Value& d) {
    if (files_) files_->put(id, d.dump());
  }
  std::string name_;
  std::mutex mu_;
  std::map<std::string, Value> docs_;
  std::shared_ptr<Collection> files_;
};

Value::Object fields(std::initializer_list<std::pair<std::string, Value>> l) {
  return Value::Object(l.begin(), l.end());
}

template <class T>
std::optional<T> field_as(const std::optional<Value>& doc, const char* name) {
  if (!doc) return std::nullopt;
  const Value* v = doc->find(name);
  if (!v || v->is_null()) return std::nullopt;
  return wire::from_json<T>(*v);
}

// ---------------------------------------------------------------------------
class DocAgentsStore : public AgentsStore {
 public:
  explicit DocAgentsStore(const std::string& dir) : c_("agents", dir) {}
  void ping() override {}
  void create_agent(const Agent& a) override {
    auto prev = c_.find_one({{"id", Value(a.id.str())}});
    if (prev && prev->find("agent") && !prev->at("agent").is_null() &&
        !(wire::from_json<Agent>(prev->at("agent")) == a))
      throw SdaError("Agent already exists");
    c_.set_by_id(a.id.str(), fields({{"agent", wire::to_json(a)}}), true);
  }
  std::optional<Agent> get_agent(const AgentId& id) override {
    return field_as<Agent>(c_.find_one({{"id", Value(id.str())}}), "agent");
  }
  void upsert_profile(const Profile& p) override {
    c_.set_by_id(p.owner.str(), fields({{"profile", wire::to_json(p)}}), false);
  }
  std::optional<Profile> get_profile(const AgentId& owner) override {
    return field_as<Profile>(c_.find_one({{"id", Value(owner.str())}}), "profile");
  }
  void create_encryption_key(const SignedEncryptionKey& k) override {
    const std::string kid = k.body.id.str();
    bool ok = c_.update_by_id(k.signer.str(), [&](Value& doc) {
      // $pull {keys: {id}} then $push {keys: {id, body}}
      Value keys = doc.find("keys") && doc.at("keys").is_array() ? doc.at("keys") : Value::array();
      Value out = Value::array();
      for (auto& e : keys.as_array())
        if (!(e.find("id") && e.at("id") == Value(kid))) out.push(e);
      Value lab = Value::object();
      lab.set("id", Value(kid));
      lab.set("body", wire::to_json(k));
      out.push(lab);
      doc.set("keys", out);
    });
    if (!ok) throw SdaError("Agent not found for encryption key");
  }
  std::optional<SignedEncryptionKey> get_encryption_key(const EncryptionKeyId& id) override {
    auto doc = c_.find_one({{"keys.id", Value(id.str())}});
    if (!doc) {
      // keys.id addresses elements of the keys array: scan
      for (auto& d : c_.find({})) {
        const Value* keys = d.find("keys");
        if (!keys || !keys->is_array()) continue;
        for (auto& e : keys->as_array())
          if (e.find("id") && e.at("id") == Value(id.str()))
            return wire::from_json<SignedEncryptionKey>(e.at("body"));
      }
      return std::nullopt;
    }
    for (auto& e : doc->at("keys").as_array())
      if (e.at("id") == Value(id.str())) return wire::from_json<SignedEncryptionKey>(e.at("body"));
    return std::nullopt;
  }
  std::vector<ClerkCandidate> suggest_committee() override {
    std::vector<ClerkCandidate> out;
    for (auto& d : c_.find({})) {
      const Value* keys = d.find("keys");
      if (!keys || !keys->is_array() || keys->size() == 0) continue;  // the reference suggests keyless agents here
      ClerkCandidate c;
      c.id = AgentId::parse(d.at("id").as_string());
      for (auto& e : keys->as_array()) c.keys.push_back(EncryptionKeyId::parse(e.at("id").as_string()));
      out.push_back(std::move(c));
    }
    return out;
  }

 private:
  DocCollection c_;
};

class DocAuthTokensStore : public AuthTokensStore {
 public:
  explicit DocAuthTokensStore(const std::string& dir) : c_("auth_tokens", dir) {}
  void upsert_auth_token(const AuthToken& t) override {
    c_.set_by_id(t.id.str(), fields({{"token", wire::to_json(t)}}), true);
  }
  std::optional<AuthToken> get_auth_token(const AgentId& id) override {
    return field_as<AuthToken>(c_.find_one({{"id", Value(id.str())}}), "token");
  }
  void delete_auth_token(const AgentId& id) override { c_.delete_one(id.str()); }

 private:
  DocCollection c_;
};

class DocAggregationsStore : public AggregationsStore {
 public:
  explicit DocAggregationsStore(const std::string& dir)
      : aggs_("aggregations", dir), parts_("participations", dir), snaps_("snapshots", dir) {}

  std::vector<AggregationId> list_aggregations(const std::optional<std::string>& filter,
                                               const std::optional<AgentId>& recipient) override {
    DocCollection::Filter f;
    if (recipient) f.emplace_back("aggregation.recipient", Value(recipient->str()));
    std::vector<AggregationId> out;
    for (auto& d : aggs_.find(f)) {
      auto a = wire::from_json<Aggregation>(d.at("aggregation"));
      if (filter && a.title.find(*filter) == std::string::npos) continue;  // $regex substring
      out.push_back(a.id);
    }
    return out;
  }
  void create_aggregation(const Aggregation& a) override {
    auto prev = aggs_.find_one({{"id", Value(a.id.str())}});
    if (prev && !(wire::from_json<Aggregation>(prev->at("aggregation")) == a))
      throw SdaError("Aggregation already exists");
    aggs_.set_by_id(a.id.str(), fields({{"aggregation", wire::to_json(a)}}), true);
  }
  std::optional<Aggregation> get_aggregation(const AggregationId& id) override {
    return field_as<Aggregation>(aggs_.find_one({{"id", Value(id.str())}}), "aggregation");
  }
  void delete_aggregation(const AggregationId& id) override { aggs_.delete_one(id.str()); }
  std::optional<Committee> get_committee(const AggregationId& id) override {
    return field_as<Committee>(aggs_.find_one({{"id", Value(id.str())}}), "committee");
  }
  void create_committee(const Committee& c) override {
    auto prev = get_committee(c.aggregation);
    if (prev && !(*prev == c)) throw SdaError("Committee already exists");
    if (!aggs_.set_by_id(c.aggregation.str(), fields({{"committee", wire::to_json(c)}}), false))
      throw SdaError("aggregation not found");
  }
  void create_participation(const Participation& p) override {
    auto prev = parts_.find_one({{"id", Value(p.id.str())}});
    if (prev && !(wire::from_json<Participation>(prev->at("participation")) == p))
      throw SdaError("Participation already exists");
    parts_.set_by_id(p.id.str(), fields({{"participation", wire::to_json(p)}}), true);
  }
  void create_snapshot(const Snapshot& s) override {
    snaps_.set_by_id(s.id.str(), fields({{"snapshot", wire::to_json(s)}}), true);
  }
  std::vector<SnapshotId> list_snapshots(const AggregationId& a) override {
    std::vector<SnapshotId> out;
    for (auto& d : snaps_.find({{"snapshot.aggregation", Value(a.str())}}))
      out.push_back(SnapshotId::parse(d.at("id").as_string()));
    return out;
  }
  std::optional<Snapshot> get_snapshot(const AggregationId&, const SnapshotId& s) override {
    return field_as<Snapshot>(snaps_.find_one({{"id", Value(s.str())}}), "snapshot");
  }
  size_t count_participations(const AggregationId& a) override {
    return parts_.count({{"participation.aggregation", Value(a.str())}});
  }
  void snapshot_participations(const AggregationId& a, const SnapshotId& s) override {
    parts_.update_many({{"participation.aggregation", Value(a.str())}}, [&](Value& doc) {
      Value snaps = doc.find("snapshots") && doc.at("snapshots").is_array() ? doc.at("snapshots")
                                                                            : Value::array();
      bool has = false;
      for (auto& e : snaps.as_array()) has |= (e == Value(s.str()));
      if (!has) snaps.push(Value(s.str()));  // $addToSet
      doc.set("snapshots", snaps);
    });
  }
  std::vector<Participation> snapped_participations(const AggregationId&, const SnapshotId& s) override {
    std::vector<Participation> out;
    for (auto& d : parts_.find({{"snapshots", Value(s.str())}}))
      out.push_back(wire::from_json<Participation>(d.at("participation")));
    return out;
  }
  size_t count_participations_snapshot(const AggregationId&, const SnapshotId& s) override {
    return parts_.count({{"snapshots", Value(s.str())}});
  }
  // $match {snapshots: s} -> $unwind(clerk_encryptions, includeArrayIndex clerk_id)
  //  -> $group by clerk_id (push) -> $sort by _id
  std::vector<std::vector<Encryption>> snapshot_clerk_jobs_data(const AggregationId&,
                                                                const SnapshotId& s,
                                                                size_t clerks) override {
    std::map<size_t, std::vector<Encryption>> groups;
    for (auto& d : parts_.find({{"snapshots", Value(s.str())}})) {
      const auto& ce = d.at("participation").at("clerk_encryptions").as_array();
      for (size_t i = 0; i < ce.size(); ++i)
        groups[i].push_back(wire::from_json<Encryption>(ce[i].as_array().at(1)));
    }
    std::vector<std::vector<Encryption>> out(clerks);
    for (auto& g : groups)
      if (g.first < clerks) out[g.first] = std::move(g.second);
    return out;
  }
  void create_snapshot_mask(const SnapshotId& s, const std::vector<Encryption>& mask) override {
    Value arr = Value::array();
    for (auto& e : mask) arr.push(wire::to_json(e));
    snaps_.set_by_id(s.str(), fields({{"mask", arr}}), false);
  }
  std::optional<std::vector<Encryption>> get_snapshot_mask(const SnapshotId& s) override {
    auto doc = snaps_.find_one({{"id", Value(s.str())}});
    if (!doc || !doc->find("mask") || doc->at("mask").is_null()) return std::nullopt;
    std::vector<Encryption> out;
    for (auto& e : doc->at("mask").as_array()) out.push_back(wire::from_json<Encryption>(e));
    return out;
  }

 private:
  DocCollection aggs_, parts_, snaps_;
};

class DocClerkingJobsStore : public ClerkingJobsStore {
 public:
  explicit DocClerkingJobsStore(const std::string& dir) : c_("clerking_jobs", dir) {}
  void enqueue_clerking_job(const ClerkingJob& j) override {
    c_.set_by_id(j.id.str(), fields({{"clerking_job", wire::to_json(j)}, {"done", Value(false)}}), true);
  }
  std::optional<ClerkingJob> poll_clerking_job(const AgentId& clerk) override {
    return field_as<ClerkingJob>(
        c_.find_one({{"done", Value(false)}, {"clerking_job.clerk", Value(clerk.str())}}), "clerking_job");
  }
  std::optional<ClerkingJob> get_clerking_job(const AgentId& clerk, const ClerkingJobId& job) override {
    // only pending jobs accept results (same as the JFS queue semantics)
    return field_as<ClerkingJob>(c_.find_one({{"clerking_job.clerk", Value(clerk.str())},
                                              {"id", Value(job.str())},
                                              {"done", Value(false)}}),
                                 "clerking_job");
  }
  void create_clerking_result(const ClerkingResult& r) override {
    if (!c_.update_by_id(r.job.str(), [&](Value& doc) {
          doc.set("result", wire::to_json(r));
          doc.set("done", Value(true));
        }))
      throw SdaError("Job not found");
  }
  std::vector<ClerkingJobId> list_results(const SnapshotId& s) override {
    std::vector<ClerkingJobId> out;
    for (auto& d : c_.find({{"clerking_job.snapshot", Value(s.str())}, {"done", Value(true)}}))
      out.push_back(ClerkingJobId::parse(d.at("id").as_string()));
    return out;
  }
  std::optional<ClerkingResult> get_result(const SnapshotId& s, const ClerkingJobId& job) override {
    return field_as<ClerkingResult>(
        c_.find_one({{"clerking_job.snapshot", Value(s.str())}, {"id", Value(job.str())}}), "result");
  }

 private:
  DocCollection c_;
};

}  // namespace

Stores make_document_stores(const std::string& dir) {
  Stores s;
  s.agents = std::make_shared<DocAgentsStore>(dir);
  s.auth_tokens = std::make_shared<DocAuthTokensStore>(dir);
  s.aggregations = std::make_shared<DocAggregationsStore>(dir);
  s.clerking_jobs = std::make_shared<DocClerkingJobsStore>(dir);
  return s;
}

}  // namespace sda
