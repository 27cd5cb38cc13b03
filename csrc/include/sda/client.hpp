// SDA client: agent roles over any SdaService (reference client/src/*.rs).
//
//   Maintenance   new_agent / upload_agent / new_encryption_key / upload_encryption_key
//   Participating new_participation / upload_participation / participate
//   Clerking      clerk_once / run_chores
//   Receiving     upload_aggregation / begin_aggregation / end_aggregation / reveal_aggregation
//
// The crypto module mirrors client/src/crypto/*: sodium sealed boxes over zigzag
// varints, Ed25519 signed key export, masking (None / Full / rand-0.3 ChaCha),
// additive sharing with the reference's Rust-`%` semantics, packed Shamir via
// the share / Lagrange matrices (field.hpp).
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "sda/device_backend.hpp"
#include "sda/service.hpp"

namespace sda {

// ---- client storage (client-store/src/{store,file}.rs) ------------------------
class Store {
 public:
  virtual ~Store() = default;
  virtual void put_json(const std::string& id, const json::Value& v) = 0;
  virtual std::optional<json::Value> get_json(const std::string& id) = 0;

  template <class T>
  void put(const std::string& id, const T& obj) { put_json(id, wire::to_json(obj)); }
  template <class T>
  std::optional<T> get(const std::string& id) {
    auto v = get_json(id);
    if (!v) return std::nullopt;
    return wire::from_json<T>(*v);
  }
  void define_alias(const std::string& alias, const std::string& id) {
    put_json("alias_" + alias, json::Value(id));
  }
  std::optional<std::string> resolve_alias(const std::string& alias) {
    auto v = get_json("alias_" + alias);
    if (!v) return std::nullopt;
    return v->as_string();
  }
  template <class T>
  void put_aliased(const std::string& alias, const std::string& id, const T& obj) {
    define_alias(alias, id);
    put(id, obj);
  }
  template <class T>
  std::optional<T> get_aliased(const std::string& alias) {
    auto id = resolve_alias(alias);
    if (!id) return std::nullopt;
    return get<T>(*id);
  }
  // client-http/src/tokenstore.rs: existing `auth_token` or 32 random alphanumerics
  std::string auth_token();
};

// One `<id>.json` per object in a directory (jfs layout of the reference CLI).
class FileStore : public Store {
 public:
  explicit FileStore(const std::string& dir);
  void put_json(const std::string& id, const json::Value& v) override;
  std::optional<json::Value> get_json(const std::string& id) override;
  const std::string& dir() const { return dir_; }

 private:
  std::string dir_;
  std::mutex mu_;
};

class MemoryStore : public Store {
 public:
  void put_json(const std::string& id, const json::Value& v) override;
  std::optional<json::Value> get_json(const std::string& id) override;

 private:
  std::mutex mu_;
  std::map<std::string, json::Value> m_;
};

using StorePtr = std::shared_ptr<Store>;

// ---- masking / sharing / encryption engines ---------------------------------
// Values use the reference's i64 representation and Rust `%` semantics.
struct MaskResult {
  std::vector<int64_t> mask;            // recipient payload (mask or ChaCha seed words)
  std::vector<int64_t> masked_secrets;  // committee payload
};
MaskResult mask_secrets(const LinearMaskingScheme& s, const std::vector<int64_t>& secrets);
std::vector<int64_t> combine_masks(const LinearMaskingScheme& s,
                                   const std::vector<std::vector<int64_t>>& masks);
std::vector<int64_t> unmask(const LinearMaskingScheme& s, const std::vector<int64_t>& mask,
                            const std::vector<int64_t>& masked);

// clerk-major shares: out[clerk][batch]
std::vector<std::vector<int64_t>> generate_shares(const LinearSecretSharingScheme& s,
                                                  const std::vector<int64_t>& secrets);
std::vector<int64_t> combine_shares(const LinearSecretSharingScheme& s,
                                    const std::vector<std::vector<int64_t>>& shares);
std::vector<int64_t> reconstruct_secrets(const LinearSecretSharingScheme& s, uint64_t dimension,
                                         const std::vector<std::pair<size_t, std::vector<int64_t>>>& indexed);

Bytes varint_encode(const std::vector<int64_t>& values);
std::vector<int64_t> varint_decode(const Bytes& bytes);  // throws on a dangling byte
Encryption encrypt_shares(const EncryptionKey& ek, const std::vector<int64_t>& shares);
std::vector<int64_t> decrypt_shares(const EncryptionKeypair& kp, const Encryption& e);

// RecipientOutput (receive.rs:8-21)
struct RecipientOutput {
  int64_t modulus = 0;
  std::vector<int64_t> values;
  RecipientOutput positive() const;
};

// ---- SdaClient ----------------------------------------------------------------
class SdaClient {
 public:
  SdaClient(Agent agent, StorePtr keystore, ServicePtr service)
      : agent_(std::move(agent)), keystore_(std::move(keystore)), service_(std::move(service)) {}

  // profile.rs:11-17 -- random id + fresh Ed25519 key stored in the keystore
  static Agent new_agent(Store& keystore);

  const Agent& agent() const { return agent_; }
  SdaService& service() { return *service_; }
  ServicePtr service_ptr() const { return service_; }
  StorePtr keystore() const { return keystore_; }

  // Maintenance
  void upload_agent();
  EncryptionKeyId new_encryption_key();
  void upload_encryption_key(const EncryptionKeyId& key);
  std::optional<SignedEncryptionKey> sign_export(const EncryptionKeyId& key);

  // GPU execution of the roles' bulk cryptography (sda/device_backend.hpp): the
  // clerk's open + combine + seal, the recipient's open + reconstruct + unmask and
  // bulk participation run on the device; aggregations the device cannot take
  // (see device_supports) use the host engines. Null = host only.
  void set_device_backend(DeviceBackendPtr backend) { device_ = std::move(backend); }
  DeviceBackendPtr device_backend() const { return device_; }
  // The reason `agg` stays on the host engines, or "" when the device takes it.
  static std::string device_unsupported(const Aggregation& agg);

  // Participating
  Participation new_participation(const std::vector<int64_t>& input, const AggregationId& agg);
  void upload_participation(const Participation& p);
  void participate(const std::vector<int64_t>& input, const AggregationId& agg);
  // Many input vectors contributed by this agent, one participation each
  // (participate.rs:37-113 per vector; keys fetched and verified once).
  std::vector<Participation> new_participations(const std::vector<std::vector<int64_t>>& inputs,
                                                const AggregationId& agg);
  void participate_many(const std::vector<std::vector<int64_t>>& inputs, const AggregationId& agg);

  // Clerking
  bool clerk_once();
  void run_chores(long max_iterations);
  ClerkingResult process_clerking_job(const ClerkingJob& job);
  // The same over box sources (`job.encryptions` is not read): the boxes may
  // still be base64 text inside the job's JSON.
  ClerkingResult process_clerking_boxes(const ClerkingJob& job, const std::vector<BoxSource>& boxes);

  // Receiving
  void upload_aggregation(const Aggregation& a);
  void begin_aggregation(const AggregationId& a);
  void end_aggregation(const AggregationId& a);
  RecipientOutput reveal_aggregation(const AggregationId& a);

  // Wall-clock milliseconds of the last clerk_once / reveal_aggregation:
  // "fetch" (service calls: HTTP, JSON, base64), "process" (the cryptography),
  // "post" (result upload).
  std::map<std::string, double> role_timings() const { return role_timings_; }

  // signing.rs:107-131, with the result cached per (agent, key) (reference FIXME)
  bool signature_is_valid(const Agent& signer, const SignedEncryptionKey& key);

 private:
  EncryptionKey verified_key(const AgentId& owner, const EncryptionKeyId& key, const char* what);
  Agent agent_;
  StorePtr keystore_;
  ServicePtr service_;
  std::mutex cache_mu_;
  std::map<std::string, bool> verify_cache_;
  DeviceBackendPtr device_;
  std::map<std::string, double> role_timings_;
};

}  // namespace sda
