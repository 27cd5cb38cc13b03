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
#include <algorithm>
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

// The string values a dotted path reaches in a document, Mongo style: arrays on
// the way are traversed element by element ("keys.id" reaches the id of every
// element of `keys`; "snapshots" reaches every snapshot id of the array).
void collect_strings(const Value& v, const std::vector<std::string>& parts, size_t i,
                     std::vector<std::string>& out) {
  if (v.is_array()) {
    for (auto& e : v.as_array()) collect_strings(e, parts, i, out);
    return;
  }
  if (i == parts.size()) {
    if (v.is_string()) out.push_back(v.as_string());
    return;
  }
  if (!v.is_object()) return;
  if (const Value* next = v.find(parts[i])) collect_strings(*next, parts, i + 1, out);
}

std::vector<std::string> split_path(const std::string& path) {
  std::vector<std::string> parts;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('.', i);
    if (j == std::string::npos) j = path.size();
    parts.push_back(path.substr(i, j - i));
    i = j + 1;
  }
  return parts;
}

// Mongo equality semantics: a field equals v, or (for arrays) contains v; a
// dotted path traverses arrays of sub-documents.
bool matches(const Value& doc, const std::vector<std::pair<std::string, Value>>& filter) {
  for (auto& f : filter) {
    const Value* v = path_get(doc, f.first);
    if (!v) {
      if (f.second.is_string()) {  // the path may run through an array of sub-documents
        std::vector<std::string> got;
        collect_strings(doc, split_path(f.first), 0, got);
        bool found = false;
        for (auto& g : got) found |= (g == f.second.as_string());
        if (found) continue;
        return false;
      }
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

// A collection with the unique `id` index of the reference DAO
// (server-store-mongodb/src/lib.rs: `ensure_index` on `id`) and secondary
// indexes on the string fields its queries filter on: find / count touch the
// documents an index names, not the whole collection.
class DocCollection {
 public:
  DocCollection(std::string name, const std::string& dir, std::vector<std::string> indexed = {})
      : name_(std::move(name)) {
    for (auto& f : indexed) index_[f];
    if (!dir.empty()) {
      files_ = make_file_collection(dir + "/" + name_);
      for (auto& kv : files_->all()) {
        auto it = docs_.emplace(kv.first, Value::parse(kv.second)).first;
        index_add(it->first, it->second);
      }
    }
  }
  using Filter = std::vector<std::pair<std::string, Value>>;

  std::optional<Value> find_one(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    std::optional<Value> out;
    scan(f, [&](const std::string&, const Value& d) {
      out = d;
      return false;
    });
    return out;
  }
  std::vector<Value> find(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Value> out;
    scan(f, [&](const std::string&, const Value& d) {
      out.push_back(d);
      return true;
    });
    return out;
  }
  size_t count(const Filter& f) {
    std::lock_guard<std::mutex> g(mu_);
    // a single indexed term: the index holds the answer
    if (f.size() == 1 && f[0].second.is_string()) {
      auto ix = index_.find(f[0].first);
      if (ix != index_.end()) return ix->second.count(f[0].second.as_string());
    }
    size_t n = 0;
    scan(f, [&](const std::string&, const Value&) {
      ++n;
      return true;
    });
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
    index_remove(id, it->second);
    for (auto& kv : fields) it->second.set(kv.first, kv.second);
    index_add(id, it->second);
    persist(id, it->second);
    return true;
  }
  // mutate with a callback under the lock (push / pull / addToSet)
  template <class F>
  bool update_by_id(const std::string& id, F fn) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = docs_.find(id);
    if (it == docs_.end()) return false;
    index_remove(id, it->second);
    fn(it->second);
    index_add(id, it->second);
    persist(id, it->second);
    return true;
  }
  template <class F>
  size_t update_many(const Filter& f, F fn) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> ids;
    scan(f, [&](const std::string& id, const Value&) {
      ids.push_back(id);
      return true;
    });
    for (auto& id : ids) {
      Value& d = docs_.at(id);
      index_remove(id, d);
      fn(d);
      index_add(id, d);
      persist(id, d);
    }
    return ids.size();
  }
  bool delete_one(const std::string& id) {
    std::lock_guard<std::mutex> g(mu_);
    if (files_) files_->remove(id);
    auto it = docs_.find(id);
    if (it == docs_.end()) return false;
    index_remove(id, it->second);
    docs_.erase(it);
    return true;
  }

 private:
  // Visit the documents matching `f` in id order until `visit` returns false.
  // Candidates come from the `id` term or the most selective indexed term.
  template <class V>
  void scan(const Filter& f, V visit) {
    for (auto& t : f)
      if (t.first == "id" && t.second.is_string()) {
        auto it = docs_.find(t.second.as_string());
        if (it != docs_.end() && matches(it->second, f)) visit(it->first, it->second);
        return;
      }
    const std::multimap<std::string, std::string>* best = nullptr;
    const std::string* key = nullptr;
    size_t best_n = 0;
    for (auto& t : f) {
      if (!t.second.is_string()) continue;
      auto ix = index_.find(t.first);
      if (ix == index_.end()) continue;
      size_t n = ix->second.count(t.second.as_string());
      if (!best || n < best_n) best = &ix->second, key = &t.second.as_string(), best_n = n;
    }
    if (best) {
      std::vector<std::string> ids;
      auto range = best->equal_range(*key);
      for (auto it = range.first; it != range.second; ++it) ids.push_back(it->second);
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      for (auto& id : ids) {
        auto it = docs_.find(id);
        if (it != docs_.end() && matches(it->second, f) && !visit(it->first, it->second)) return;
      }
      return;
    }
    for (auto& kv : docs_)
      if (matches(kv.second, f) && !visit(kv.first, kv.second)) return;
  }
  void index_add(const std::string& id, const Value& d) {
    for (auto& ix : index_) {
      std::vector<std::string> vals;
      collect_strings(d, split_path(ix.first), 0, vals);
      for (auto& v : vals) ix.second.emplace(v, id);
    }
  }
  void index_remove(const std::string& id, const Value& d) {
    for (auto& ix : index_) {
      std::vector<std::string> vals;
      collect_strings(d, split_path(ix.first), 0, vals);
      for (auto& v : vals) {
        auto range = ix.second.equal_range(v);
        for (auto it = range.first; it != range.second;) {
          if (it->second == id) it = ix.second.erase(it);
          else ++it;
        }
      }
    }
  }
  void persist(const std::string& id, const Value& d) {
    if (files_) files_->put(id, d.dump());
  }
  std::string name_;
  std::mutex mu_;
  std::map<std::string, Value> docs_;
  std::map<std::string, std::multimap<std::string, std::string>> index_;  // field -> value -> ids
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
  explicit DocAgentsStore(const std::string& dir) : c_("agents", dir, {"keys.id"}) {}
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
    auto doc = c_.find_one({{"keys.id", Value(id.str())}});  // indexed: the ids inside `keys`
    if (!doc) return std::nullopt;
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
      : aggs_("aggregations", dir, {"aggregation.recipient"}),
        parts_("participations", dir, {"participation.aggregation", "snapshots"}),
        snaps_("snapshots", dir, {"snapshot.aggregation"}) {}

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
  std::optional<std::string> get_snapshot_mask_json(const SnapshotId& s) override {
    auto doc = snaps_.find_one({{"id", Value(s.str())}});
    if (!doc || !doc->find("mask") || doc->at("mask").is_null()) return std::nullopt;
    return doc->at("mask").dump();
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
  explicit DocClerkingJobsStore(const std::string& dir)
      : c_("clerking_jobs", dir, {"clerking_job.clerk", "clerking_job.snapshot"}) {}
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
  // bulk forms: the stored sub-documents are dumped as they are, the boxes are
  // never decoded on the server
  std::optional<std::string> poll_clerking_job_json(const AgentId& clerk) override {
    auto doc = c_.find_one({{"done", Value(false)}, {"clerking_job.clerk", Value(clerk.str())}});
    if (!doc || !doc->find("clerking_job")) return std::nullopt;
    return doc->at("clerking_job").dump();
  }
  std::optional<ClerkingJob> get_clerking_job_head(const AgentId& clerk, const ClerkingJobId& job) override {
    auto doc = c_.find_one({{"clerking_job.clerk", Value(clerk.str())},
                            {"id", Value(job.str())},
                            {"done", Value(false)}});
    if (!doc) return std::nullopt;
    const Value& j = doc->at("clerking_job");
    ClerkingJob head;
    head.id = ClerkingJobId::parse(j.at("id").as_string());
    head.clerk = AgentId::parse(j.at("clerk").as_string());
    head.aggregation = AggregationId::parse(j.at("aggregation").as_string());
    head.snapshot = SnapshotId::parse(j.at("snapshot").as_string());
    return head;
  }
  std::optional<std::string> get_result_json(const SnapshotId& s, const ClerkingJobId& job) override {
    auto doc = c_.find_one({{"clerking_job.snapshot", Value(s.str())}, {"id", Value(job.str())}});
    if (!doc || !doc->find("result") || doc->at("result").is_null()) return std::nullopt;
    return doc->at("result").dump();
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
