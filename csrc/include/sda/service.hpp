// The SdaService interface (reference protocol/src/methods.rs:13-112).
//
// Two implementations, exactly like the reference's central seam:
//   * SdaServerService (in-process, server.hpp) -- the real workflow + ACL
//   * SdaHttpClient   (http.hpp)              -- the same API over REST
// Client logic (client.hpp) only ever holds a `std::shared_ptr<SdaService>`.
// Every method takes the calling agent; `std::optional` = Option; errors are
// SdaError exceptions with the reference kinds.
#pragma once

#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "sda/protocol.hpp"

namespace sda {

class SdaService {
 public:
  virtual ~SdaService() = default;
  // SdaBaseService
  virtual Pong ping() = 0;
  // SdaAgentService
  virtual void create_agent(const Agent& caller, const Agent& agent) = 0;
  virtual std::optional<Agent> get_agent(const Agent& caller, const AgentId& agent) = 0;
  virtual void upsert_profile(const Agent& caller, const Profile& profile) = 0;
  virtual std::optional<Profile> get_profile(const Agent& caller, const AgentId& owner) = 0;
  virtual void create_encryption_key(const Agent& caller, const SignedEncryptionKey& key) = 0;
  virtual std::optional<SignedEncryptionKey> get_encryption_key(const Agent& caller,
                                                                const EncryptionKeyId& key) = 0;
  // SdaAggregationService
  virtual std::vector<AggregationId> list_aggregations(const Agent& caller,
                                                       const std::optional<std::string>& filter,
                                                       const std::optional<AgentId>& recipient) = 0;
  virtual std::optional<Aggregation> get_aggregation(const Agent& caller,
                                                     const AggregationId& aggregation) = 0;
  virtual std::optional<Committee> get_committee(const Agent& caller,
                                                 const AggregationId& owner) = 0;
  // SdaParticipationService
  virtual void create_participation(const Agent& caller, const Participation& participation) = 0;
  // SdaClerkingService
  virtual std::optional<ClerkingJob> get_clerking_job(const Agent& caller, const AgentId& clerk) = 0;
  virtual void create_clerking_result(const Agent& caller, const ClerkingResult& result) = 0;
  // SdaRecipientService
  virtual void create_aggregation(const Agent& caller, const Aggregation& aggregation) = 0;
  virtual void delete_aggregation(const Agent& caller, const AggregationId& aggregation) = 0;
  virtual std::vector<ClerkCandidate> suggest_committee(const Agent& caller,
                                                        const AggregationId& aggregation) = 0;
  virtual void create_committee(const Agent& caller, const Committee& committee) = 0;
  virtual std::optional<AggregationStatus> get_aggregation_status(const Agent& caller,
                                                                  const AggregationId& aggregation) = 0;
  virtual void create_snapshot(const Agent& caller, const Snapshot& snapshot) = 0;
  virtual std::optional<SnapshotResult> get_snapshot_result(const Agent& caller,
                                                            const AggregationId& aggregation,
                                                            const SnapshotId& snapshot) = 0;

  // The two bulk downloads as the JSON text of their responses (a clerking job
  // holds a sealed box per participation, a snapshot result a mask box per
  // participation). Implementations that hold or receive the text anyway (the
  // server's stores, the REST client) return it without building the structs;
  // `wire::scan_*` then locates the payloads in place. Defaults encode the
  // struct forms.
  virtual std::optional<std::string> get_clerking_job_json(const Agent& caller, const AgentId& clerk) {
    auto j = get_clerking_job(caller, clerk);
    if (!j) return std::nullopt;
    return wire::encode(*j);
  }
  virtual std::optional<std::string> get_snapshot_result_json(const Agent& caller,
                                                              const AggregationId& aggregation,
                                                              const SnapshotId& snapshot) {
    auto r = get_snapshot_result(caller, aggregation, snapshot);
    if (!r) return std::nullopt;
    return wire::encode(*r);
  }
};

using ServicePtr = std::shared_ptr<SdaService>;

}  // namespace sda
