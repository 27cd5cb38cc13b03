// The SDA server: workflow, ACL, snapshot (reference server/src/server.rs,
// server/src/snapshot.rs, server/src/lib.rs).
#pragma once

#include <memory>
#include <string>

#include "sda/service.hpp"
#include "sda/stores.hpp"

namespace sda {

// Store pass-through plus the server-side logic (server.rs:5-191).
class SdaServer {
 public:
  explicit SdaServer(Stores stores) : s_(std::move(stores)) {}

  Pong ping();
  void create_agent(const Agent& agent);
  std::optional<Agent> get_agent(const AgentId& id);
  void upsert_profile(const Profile& profile);
  std::optional<Profile> get_profile(const AgentId& owner);
  void create_encryption_key(const SignedEncryptionKey& key);
  std::optional<SignedEncryptionKey> get_encryption_key(const EncryptionKeyId& id);
  std::vector<AggregationId> list_aggregations(const std::optional<std::string>& filter,
                                               const std::optional<AgentId>& recipient);
  std::optional<Aggregation> get_aggregation(const AggregationId& id);
  std::optional<Committee> get_committee(const AggregationId& id);
  void create_aggregation(const Aggregation& a);
  void delete_aggregation(const AggregationId& id);
  std::vector<ClerkCandidate> suggest_committee(const AggregationId& id);
  void create_committee(const Committee& c);
  void create_participation(const Participation& p);
  std::optional<AggregationStatus> get_aggregation_status(const AggregationId& id);
  void create_snapshot(const Snapshot& s);  // snapshot.rs:4-47
  std::optional<ClerkingJob> poll_clerking_job(const AgentId& clerk);
  std::optional<ClerkingJob> get_clerking_job(const AgentId& clerk, const ClerkingJobId& job);
  // bulk forms (see ClerkingJobsStore): the job as stored text, its head only
  std::optional<std::string> poll_clerking_job_json(const AgentId& clerk);
  std::optional<ClerkingJob> get_clerking_job_head(const AgentId& clerk, const ClerkingJobId& job);
  void create_clerking_result(const ClerkingResult& r);
  std::optional<SnapshotResult> get_snapshot_result(const AggregationId& a, const SnapshotId& s);
  std::optional<std::string> get_snapshot_result_json(const AggregationId& a, const SnapshotId& s);
  // auth (server.rs:171-190)
  void upsert_auth_token(const AuthToken& token);
  Agent check_auth_token(const AuthToken& token);  // throws InvalidCredentials
  void delete_auth_token(const AgentId& agent);

  const Stores& stores() const { return s_; }

 private:
  Stores s_;
};

// SdaService over an in-process SdaServer, with the reference's ACL
// (server.rs:193-361): recipient-only / owner-only operations raise
// PermissionDenied.
class SdaServerService : public SdaService {
 public:
  explicit SdaServerService(std::shared_ptr<SdaServer> server) : srv_(std::move(server)) {}
  SdaServer& server() { return *srv_; }
  std::shared_ptr<SdaServer> server_ptr() { return srv_; }

  Pong ping() override;
  void create_agent(const Agent& caller, const Agent& agent) override;
  std::optional<Agent> get_agent(const Agent& caller, const AgentId& agent) override;
  void upsert_profile(const Agent& caller, const Profile& profile) override;
  std::optional<Profile> get_profile(const Agent& caller, const AgentId& owner) override;
  void create_encryption_key(const Agent& caller, const SignedEncryptionKey& key) override;
  std::optional<SignedEncryptionKey> get_encryption_key(const Agent& caller,
                                                        const EncryptionKeyId& key) override;
  std::vector<AggregationId> list_aggregations(const Agent& caller,
                                               const std::optional<std::string>& filter,
                                               const std::optional<AgentId>& recipient) override;
  std::optional<Aggregation> get_aggregation(const Agent& caller, const AggregationId& a) override;
  std::optional<Committee> get_committee(const Agent& caller, const AggregationId& a) override;
  void create_participation(const Agent& caller, const Participation& p) override;
  std::optional<ClerkingJob> get_clerking_job(const Agent& caller, const AgentId& clerk) override;
  std::optional<std::string> get_clerking_job_json(const Agent& caller, const AgentId& clerk) override;
  std::optional<std::string> get_snapshot_result_json(const Agent& caller, const AggregationId& a,
                                                      const SnapshotId& s) override;
  void create_clerking_result(const Agent& caller, const ClerkingResult& r) override;
  void create_aggregation(const Agent& caller, const Aggregation& a) override;
  void delete_aggregation(const Agent& caller, const AggregationId& a) override;
  std::vector<ClerkCandidate> suggest_committee(const Agent& caller, const AggregationId& a) override;
  void create_committee(const Agent& caller, const Committee& c) override;
  std::optional<AggregationStatus> get_aggregation_status(const Agent& caller,
                                                          const AggregationId& a) override;
  void create_snapshot(const Agent& caller, const Snapshot& s) override;
  std::optional<SnapshotResult> get_snapshot_result(const Agent& caller, const AggregationId& a,
                                                    const SnapshotId& s) override;

 private:
  Aggregation require_aggregation(const AggregationId& a);
  std::shared_ptr<SdaServer> srv_;
};

// Factories (server/src/lib.rs:34-45 + server-store-mongodb/src/lib.rs:64-84)
std::shared_ptr<SdaServerService> new_memory_server();
std::shared_ptr<SdaServerService> new_jfs_server(const std::string& dir);
std::shared_ptr<SdaServerService> new_document_server(const std::string& dir);

}  // namespace sda
