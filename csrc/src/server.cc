// SDA server workflow + ACL (reference server/src/server.rs, snapshot.rs).
#include "sda/server.hpp"

#include "sda/log.hpp"

namespace sda {

// ---- SdaServer ----------------------------------------------------------------
Pong SdaServer::ping() {
  s_.agents->ping();
  return Pong{true};
}
void SdaServer::create_agent(const Agent& a) { s_.agents->create_agent(a); }
std::optional<Agent> SdaServer::get_agent(const AgentId& id) { return s_.agents->get_agent(id); }
void SdaServer::upsert_profile(const Profile& p) { s_.agents->upsert_profile(p); }
std::optional<Profile> SdaServer::get_profile(const AgentId& o) { return s_.agents->get_profile(o); }
void SdaServer::create_encryption_key(const SignedEncryptionKey& k) { s_.agents->create_encryption_key(k); }
std::optional<SignedEncryptionKey> SdaServer::get_encryption_key(const EncryptionKeyId& id) {
  return s_.agents->get_encryption_key(id);
}
std::vector<AggregationId> SdaServer::list_aggregations(const std::optional<std::string>& filter,
                                                        const std::optional<AgentId>& recipient) {
  return s_.aggregations->list_aggregations(filter, recipient);
}
std::optional<Aggregation> SdaServer::get_aggregation(const AggregationId& id) {
  return s_.aggregations->get_aggregation(id);
}
std::optional<Committee> SdaServer::get_committee(const AggregationId& id) {
  return s_.aggregations->get_committee(id);
}
void SdaServer::create_aggregation(const Aggregation& a) { s_.aggregations->create_aggregation(a); }
void SdaServer::delete_aggregation(const AggregationId& id) { s_.aggregations->delete_aggregation(id); }

std::vector<ClerkCandidate> SdaServer::suggest_committee(const AggregationId& id) {
  if (!s_.aggregations->get_aggregation(id)) throw SdaError("aggregation not found");
  return s_.agents->suggest_committee();
}

void SdaServer::create_committee(const Committee& c) {
  auto agg = s_.aggregations->get_aggregation(c.aggregation);
  if (!agg) throw SdaError("aggregation not found");
  if (agg->committee_sharing_scheme.output_size() != c.clerks_and_keys.size())
    throw SdaError::invalid("Expected " + std::to_string(agg->committee_sharing_scheme.output_size()) +
                            " clerks in the committee, found " +
                            std::to_string(c.clerks_and_keys.size()) + " instead");
  s_.aggregations->create_committee(c);
}

void SdaServer::create_participation(const Participation& p) { s_.aggregations->create_participation(p); }

std::optional<AggregationStatus> SdaServer::get_aggregation_status(const AggregationId& id) {
  auto agg = s_.aggregations->get_aggregation(id);
  if (!agg) return std::nullopt;
  AggregationStatus st;
  st.aggregation = id;
  for (auto& sid : s_.aggregations->list_snapshots(id)) {
    size_t results = s_.clerking_jobs->list_results(sid).size();
    st.snapshots.push_back(SnapshotStatus{
        sid, results, results >= agg->committee_sharing_scheme.reconstruction_threshold()});
  }
  st.number_of_participations = s_.aggregations->count_participations(id);
  return st;
}

void SdaServer::create_snapshot(const Snapshot& snapshot) {
  auto agg = s_.aggregations->get_aggregation(snapshot.aggregation);
  if (!agg) throw SdaError("lost aggregation");
  log_debug("Snapshot participations");
  s_.aggregations->snapshot_participations(snapshot.aggregation, snapshot.id);
  auto committee = s_.aggregations->get_committee(snapshot.aggregation);
  if (!committee) throw SdaError("lost committee");
  log_debug("Transposing encryptions");
  auto per_clerk = s_.aggregations->snapshot_clerk_jobs_data(snapshot.aggregation, snapshot.id,
                                                             committee->clerks_and_keys.size());
  log_debug("Creating clerking jobs");
  for (size_t i = 0; i < committee->clerks_and_keys.size(); ++i) {
    ClerkingJob job;
    job.id = ClerkingJobId::random();
    job.clerk = committee->clerks_and_keys[i].first;
    job.aggregation = snapshot.aggregation;
    job.snapshot = snapshot.id;
    job.encryptions = std::move(per_clerk[i]);
    s_.clerking_jobs->enqueue_clerking_job(job);
  }
  log_debug("Create snapshot");
  s_.aggregations->create_snapshot(snapshot);
  if (agg->masking_scheme.has_mask()) {
    log_debug("Creating masking data");
    std::vector<Encryption> masks;
    for (auto& p : s_.aggregations->snapped_participations(snapshot.aggregation, snapshot.id)) {
      if (!p.recipient_encryption) throw SdaError("participation should have had a recipient encryption");
      masks.push_back(std::move(*p.recipient_encryption));
    }
    s_.aggregations->create_snapshot_mask(snapshot.id, masks);
  }
  log_debug("Done snapshot");
}

std::optional<ClerkingJob> SdaServer::poll_clerking_job(const AgentId& clerk) {
  return s_.clerking_jobs->poll_clerking_job(clerk);
}
std::optional<ClerkingJob> SdaServer::get_clerking_job(const AgentId& clerk, const ClerkingJobId& job) {
  return s_.clerking_jobs->get_clerking_job(clerk, job);
}
std::optional<std::string> SdaServer::poll_clerking_job_json(const AgentId& clerk) {
  return s_.clerking_jobs->poll_clerking_job_json(clerk);
}
std::optional<ClerkingJob> SdaServer::get_clerking_job_head(const AgentId& clerk, const ClerkingJobId& job) {
  return s_.clerking_jobs->get_clerking_job_head(clerk, job);
}
void SdaServer::create_clerking_result(const ClerkingResult& r) { s_.clerking_jobs->create_clerking_result(r); }

std::optional<SnapshotResult> SdaServer::get_snapshot_result(const AggregationId& a, const SnapshotId& s) {
  SnapshotResult r;
  r.snapshot = s;
  for (auto& job : s_.clerking_jobs->list_results(s)) {
    auto res = s_.clerking_jobs->get_result(s, job);
    if (!res) throw SdaError("inconsistent storage");
    r.clerk_encryptions.push_back(std::move(*res));
  }
  r.number_of_participations = s_.aggregations->count_participations_snapshot(a, s);
  r.recipient_encryptions = s_.aggregations->get_snapshot_mask(s);
  return r;
}

// The same document assembled from the stores' text: the mask boxes (one per
// participation) and the results are spliced in as they are stored.
std::optional<std::string> SdaServer::get_snapshot_result_json(const AggregationId& a, const SnapshotId& s) {
  std::string out = "{\"snapshot\":" + wire::to_json(s).dump() + ",\"number_of_participations\":" +
                    std::to_string(s_.aggregations->count_participations_snapshot(a, s)) +
                    ",\"clerk_encryptions\":[";
  bool first = true;
  for (auto& job : s_.clerking_jobs->list_results(s)) {
    auto res = s_.clerking_jobs->get_result_json(s, job);
    if (!res) throw SdaError("inconsistent storage");
    if (!first) out.push_back(',');
    first = false;
    out += *res;
  }
  out += "],\"recipient_encryptions\":";
  auto masks = s_.aggregations->get_snapshot_mask_json(s);
  out += masks ? *masks : std::string("null");
  out.push_back('}');
  return out;
}

void SdaServer::upsert_auth_token(const AuthToken& t) { s_.auth_tokens->upsert_auth_token(t); }
Agent SdaServer::check_auth_token(const AuthToken& t) {
  auto db = s_.auth_tokens->get_auth_token(t.id);
  if (db && *db == t) {
    auto agent = s_.agents->get_agent(t.id);
    if (!agent) throw SdaError("Agent not found");
    return *agent;
  }
  throw SdaError::invalid_credentials();
}
void SdaServer::delete_auth_token(const AgentId& a) { s_.auth_tokens->delete_auth_token(a); }

// ---- SdaServerService (ACL) ----------------------------------------------------
namespace {
void acl_agent_is(const Agent& caller, const AgentId& id) {
  if (caller.id != id) throw SdaError::permission_denied();
}
}  // namespace

Aggregation SdaServerService::require_aggregation(const AggregationId& a) {
  auto agg = srv_->get_aggregation(a);
  if (!agg) throw SdaError("No aggregation found");
  return *agg;
}

Pong SdaServerService::ping() { return srv_->ping(); }
void SdaServerService::create_agent(const Agent& caller, const Agent& agent) {
  acl_agent_is(caller, agent.id);
  srv_->create_agent(agent);
}
std::optional<Agent> SdaServerService::get_agent(const Agent&, const AgentId& a) { return srv_->get_agent(a); }
void SdaServerService::upsert_profile(const Agent& caller, const Profile& p) {
  acl_agent_is(caller, p.owner);
  srv_->upsert_profile(p);
}
std::optional<Profile> SdaServerService::get_profile(const Agent&, const AgentId& o) { return srv_->get_profile(o); }
void SdaServerService::create_encryption_key(const Agent& caller, const SignedEncryptionKey& k) {
  acl_agent_is(caller, k.signer);
  srv_->create_encryption_key(k);
}
std::optional<SignedEncryptionKey> SdaServerService::get_encryption_key(const Agent&, const EncryptionKeyId& k) {
  return srv_->get_encryption_key(k);
}
std::vector<AggregationId> SdaServerService::list_aggregations(const Agent&, const std::optional<std::string>& f,
                                                               const std::optional<AgentId>& r) {
  return srv_->list_aggregations(f, r);
}
std::optional<Aggregation> SdaServerService::get_aggregation(const Agent&, const AggregationId& a) {
  return srv_->get_aggregation(a);
}
std::optional<Committee> SdaServerService::get_committee(const Agent&, const AggregationId& a) {
  return srv_->get_committee(a);
}
void SdaServerService::create_participation(const Agent& caller, const Participation& p) {
  acl_agent_is(caller, p.participant);
  srv_->create_participation(p);
}
std::optional<ClerkingJob> SdaServerService::get_clerking_job(const Agent& caller, const AgentId& clerk) {
  acl_agent_is(caller, clerk);
  return srv_->poll_clerking_job(clerk);
}
std::optional<std::string> SdaServerService::get_clerking_job_json(const Agent& caller, const AgentId& clerk) {
  acl_agent_is(caller, clerk);
  return srv_->poll_clerking_job_json(clerk);
}
void SdaServerService::create_clerking_result(const Agent& caller, const ClerkingResult& r) {
  // re-fetch the job by (clerk, job) so a forged clerk id cannot be used (server.rs:351-360);
  // only its head is read
  auto job = srv_->get_clerking_job_head(r.clerk, r.job);
  if (!job) throw SdaError("Job not found");
  acl_agent_is(caller, job->clerk);
  srv_->create_clerking_result(r);
}
void SdaServerService::create_aggregation(const Agent& caller, const Aggregation& a) {
  acl_agent_is(caller, a.recipient);
  srv_->create_aggregation(a);
}
void SdaServerService::delete_aggregation(const Agent& caller, const AggregationId& a) {
  acl_agent_is(caller, require_aggregation(a).recipient);
  srv_->delete_aggregation(a);
}
std::vector<ClerkCandidate> SdaServerService::suggest_committee(const Agent& caller, const AggregationId& a) {
  acl_agent_is(caller, require_aggregation(a).recipient);
  return srv_->suggest_committee(a);
}
void SdaServerService::create_committee(const Agent& caller, const Committee& c) {
  acl_agent_is(caller, require_aggregation(c.aggregation).recipient);
  srv_->create_committee(c);
}
std::optional<AggregationStatus> SdaServerService::get_aggregation_status(const Agent& caller,
                                                                          const AggregationId& a) {
  acl_agent_is(caller, require_aggregation(a).recipient);
  return srv_->get_aggregation_status(a);
}
void SdaServerService::create_snapshot(const Agent& caller, const Snapshot& s) {
  acl_agent_is(caller, require_aggregation(s.aggregation).recipient);
  srv_->create_snapshot(s);
}
std::optional<SnapshotResult> SdaServerService::get_snapshot_result(const Agent& caller, const AggregationId& a,
                                                                    const SnapshotId& s) {
  acl_agent_is(caller, require_aggregation(a).recipient);
  // the snapshot must belong to this aggregation (the reference has a FIXME here)
  auto snap = srv_->stores().aggregations->get_snapshot(a, s);
  if (!snap || snap->aggregation != a) return std::nullopt;
  return srv_->get_snapshot_result(a, s);
}

std::optional<std::string> SdaServerService::get_snapshot_result_json(const Agent& caller,
                                                                     const AggregationId& a,
                                                                     const SnapshotId& s) {
  acl_agent_is(caller, require_aggregation(a).recipient);
  auto snap = srv_->stores().aggregations->get_snapshot(a, s);
  if (!snap || snap->aggregation != a) return std::nullopt;
  return srv_->get_snapshot_result_json(a, s);
}

std::shared_ptr<SdaServerService> new_memory_server() {
  return std::make_shared<SdaServerService>(std::make_shared<SdaServer>(make_memory_stores()));
}
std::shared_ptr<SdaServerService> new_jfs_server(const std::string& dir) {
  return std::make_shared<SdaServerService>(std::make_shared<SdaServer>(make_jfs_stores(dir)));
}
std::shared_ptr<SdaServerService> new_document_server(const std::string& dir) {
  return std::make_shared<SdaServerService>(std::make_shared<SdaServer>(make_document_stores(dir)));
}

}  // namespace sda
