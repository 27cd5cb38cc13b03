// Server store interfaces and implementations.
//
// Interfaces mirror server/src/stores.rs:4-120. Three backends:
//   * memory    -- std::map collections (tests, ephemeral servers)
//   * JFS       -- one `<id>.json` per object with the reference's directory
//                  layout (server/src/lib.rs:34-45 + jfs_stores/*), so an `sdad
//                  --jfs DIR` state directory is interchangeable
//   * document  -- the MongoDB data model of server-store-mongodb (collections of
//                  documents with embedded committee / snapshot tags / done flags,
//                  snapshot transpose as an unwind-group pipeline) on a native
//                  embedded document engine persisted as JSON files
// All stores are internally locked (the reference's JFS store had no locking,
// server/src/jfs_stores/), so the multithreaded HTTP server is race-free.
#pragma once

#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "sda/protocol.hpp"

namespace sda {

class AgentsStore {
 public:
  virtual ~AgentsStore() = default;
  virtual void ping() {}
  virtual void create_agent(const Agent& agent) = 0;
  virtual std::optional<Agent> get_agent(const AgentId& id) = 0;
  virtual void upsert_profile(const Profile& profile) = 0;
  virtual std::optional<Profile> get_profile(const AgentId& owner) = 0;
  virtual void create_encryption_key(const SignedEncryptionKey& key) = 0;
  virtual std::optional<SignedEncryptionKey> get_encryption_key(const EncryptionKeyId& key) = 0;
  // every key-holding agent, keys grouped per signer, sorted by signer id
  virtual std::vector<ClerkCandidate> suggest_committee() = 0;
};

class AuthTokensStore {
 public:
  virtual ~AuthTokensStore() = default;
  virtual void ping() {}
  virtual void upsert_auth_token(const AuthToken& token) = 0;
  virtual std::optional<AuthToken> get_auth_token(const AgentId& id) = 0;
  virtual void delete_auth_token(const AgentId& id) = 0;
};

class AggregationsStore {
 public:
  virtual ~AggregationsStore() = default;
  virtual void ping() {}
  virtual std::vector<AggregationId> list_aggregations(const std::optional<std::string>& filter,
                                                       const std::optional<AgentId>& recipient) = 0;
  virtual void create_aggregation(const Aggregation& aggregation) = 0;
  virtual std::optional<Aggregation> get_aggregation(const AggregationId& id) = 0;
  virtual void delete_aggregation(const AggregationId& id) = 0;
  virtual std::optional<Committee> get_committee(const AggregationId& owner) = 0;
  virtual void create_committee(const Committee& committee) = 0;
  virtual void create_participation(const Participation& participation) = 0;
  virtual void create_snapshot(const Snapshot& snapshot) = 0;
  virtual std::vector<SnapshotId> list_snapshots(const AggregationId& aggregation) = 0;
  virtual std::optional<Snapshot> get_snapshot(const AggregationId& aggregation,
                                               const SnapshotId& snapshot) = 0;
  virtual size_t count_participations(const AggregationId& aggregation) = 0;
  virtual void snapshot_participations(const AggregationId& aggregation,
                                       const SnapshotId& snapshot) = 0;
  virtual std::vector<Participation> snapped_participations(const AggregationId& aggregation,
                                                            const SnapshotId& snapshot) = 0;
  virtual size_t count_participations_snapshot(const AggregationId& aggregation,
                                               const SnapshotId& snapshot) {
    return snapped_participations(aggregation, snapshot).size();
  }
  // Transpose P x n participations into n per-clerk lists (stores.rs:86-101).
  virtual std::vector<std::vector<Encryption>> snapshot_clerk_jobs_data(
      const AggregationId& aggregation, const SnapshotId& snapshot, size_t clerks);
  virtual void create_snapshot_mask(const SnapshotId& snapshot, const std::vector<Encryption>& mask) = 0;
  virtual std::optional<std::vector<Encryption>> get_snapshot_mask(const SnapshotId& snapshot) = 0;
  // The mask boxes as the JSON text of the array (stores that hold text return
  // it as stored; the default encodes get_snapshot_mask()).
  virtual std::optional<std::string> get_snapshot_mask_json(const SnapshotId& snapshot);
};

class ClerkingJobsStore {
 public:
  virtual ~ClerkingJobsStore() = default;
  virtual void ping() {}
  virtual void enqueue_clerking_job(const ClerkingJob& job) = 0;
  virtual std::optional<ClerkingJob> poll_clerking_job(const AgentId& clerk) = 0;
  virtual std::optional<ClerkingJob> get_clerking_job(const AgentId& clerk,
                                                      const ClerkingJobId& job) = 0;
  virtual void create_clerking_result(const ClerkingResult& result) = 0;
  virtual std::vector<ClerkingJobId> list_results(const SnapshotId& snapshot) = 0;
  virtual std::optional<ClerkingResult> get_result(const SnapshotId& snapshot,
                                                   const ClerkingJobId& job) = 0;
  // Bulk forms. A job holds a sealed box per participation: serving it as the
  // text the store holds, and reading only its head for the result ACL, keeps
  // the server from decoding and re-encoding hundreds of megabytes per request.
  // Defaults go through the struct forms.
  virtual std::optional<std::string> poll_clerking_job_json(const AgentId& clerk);
  virtual std::optional<ClerkingJob> get_clerking_job_head(const AgentId& clerk,
                                                           const ClerkingJobId& job);  // may lack the boxes
  virtual std::optional<std::string> get_result_json(const SnapshotId& snapshot,
                                                     const ClerkingJobId& job);
};

struct Stores {
  std::shared_ptr<AgentsStore> agents;
  std::shared_ptr<AuthTokensStore> auth_tokens;
  std::shared_ptr<AggregationsStore> aggregations;
  std::shared_ptr<ClerkingJobsStore> clerking_jobs;
};

Stores make_memory_stores();
Stores make_jfs_stores(const std::string& dir);
// `dir` empty = purely in-memory document engine.
Stores make_document_stores(const std::string& dir);

// ---- key/value collection (JFS semantics) used by the memory/JFS backends ----
class Collection {
 public:
  virtual ~Collection() = default;
  virtual std::optional<std::string> get(const std::string& id) = 0;
  virtual void put(const std::string& id, const std::string& json) = 0;
  virtual bool remove(const std::string& id) = 0;
  // all (id, json) sorted by id (jfs::Store::all is a BTreeMap)
  virtual std::vector<std::pair<std::string, std::string>> all() = 0;
  // the entry with the smallest id (what `all().front()` is), without copying the rest
  virtual std::optional<std::pair<std::string, std::string>> first() {
    auto a = all();
    if (a.empty()) return std::nullopt;
    return std::move(a.front());
  }
  virtual size_t count() = 0;
};
std::shared_ptr<Collection> make_mem_collection();
std::shared_ptr<Collection> make_file_collection(const std::string& dir);

}  // namespace sda
