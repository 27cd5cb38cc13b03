// SDA protocol: resources, scheme enums, service interface and wire format.
//
// Mirrors the reference `sda-protocol` crate:
//   resources  protocol/src/resources.rs:12-188
//   schemes    protocol/src/crypto.rs:7-188
//   helpers    protocol/src/helpers.rs (Signed, Labelled, Binary, uuid ids)
//   methods    protocol/src/methods.rs:13-112 (the SdaService traits)
// JSON follows serde 0.9 derive conventions: structs are objects in declaration
// order, newtype enum variants are externally tagged ({"Sodium": ...}), unit
// variants are bare strings ("None", "Sodium"), tuples are arrays, Option::None
// is null, ids are hyphenated UUID strings, byte arrays are padded base64.
#pragma once

#include <array>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "sda/common.hpp"
#include "sda/json.hpp"

namespace sda {

// ---- typed UUID ids --------------------------------------------------------
template <class Tag>
struct Id {
  Uuid uuid;
  static Id random() { return Id{Uuid::random()}; }
  static Id parse(const std::string& s) { return Id{Uuid::parse(s)}; }
  std::string str() const { return uuid.str(); }
  bool operator==(const Id& o) const { return uuid == o.uuid; }
  bool operator!=(const Id& o) const { return !(uuid == o.uuid); }
  bool operator<(const Id& o) const { return uuid < o.uuid; }
};
struct VerificationKeyTag {};
struct AgentTag {};
struct EncryptionKeyTag {};
struct AggregationTag {};
struct ParticipationTag {};
struct SnapshotTag {};
struct ClerkingJobTag {};
using VerificationKeyId = Id<VerificationKeyTag>;
using AgentId = Id<AgentTag>;
using EncryptionKeyId = Id<EncryptionKeyTag>;
using AggregationId = Id<AggregationTag>;
using ParticipationId = Id<ParticipationTag>;
using SnapshotId = Id<SnapshotTag>;
using ClerkingJobId = Id<ClerkingJobTag>;

template <size_t N>
using ByteArray = std::array<uint8_t, N>;  // B8 / B32 / B64

// ---- crypto value enums (single Sodium variant each) -----------------------
struct Encryption {        // Encryption::Sodium(Binary)
  Bytes sodium;
  bool operator==(const Encryption& o) const { return sodium == o.sodium; }
};
struct EncryptionKey {     // EncryptionKey::Sodium(B32)
  ByteArray<32> sodium{};
  bool operator==(const EncryptionKey& o) const { return sodium == o.sodium; }
};
struct DecryptionKey {     // client-side keystore
  ByteArray<32> sodium{};
  bool operator==(const DecryptionKey& o) const { return sodium == o.sodium; }
};
struct Signature {         // Signature::Sodium(B64)
  ByteArray<64> sodium{};
  bool operator==(const Signature& o) const { return sodium == o.sodium; }
};
struct SigningKey {        // SigningKey::Sodium(B64)
  ByteArray<64> sodium{};
  bool operator==(const SigningKey& o) const { return sodium == o.sodium; }
};
struct VerificationKey {   // VerificationKey::Sodium(B32)
  ByteArray<32> sodium{};
  bool operator==(const VerificationKey& o) const { return sodium == o.sodium; }
};

// ---- schemes -----------------------------------------------------------------
struct LinearMaskingScheme {
  enum class Kind { None, Full, ChaCha } kind = Kind::None;
  int64_t modulus = 0;
  uint64_t dimension = 0;
  uint64_t seed_bitsize = 0;
  bool has_mask() const { return kind != Kind::None; }
  bool operator==(const LinearMaskingScheme& o) const {
    return kind == o.kind && modulus == o.modulus && dimension == o.dimension &&
           seed_bitsize == o.seed_bitsize;
  }
  static LinearMaskingScheme none() { return {}; }
  static LinearMaskingScheme full(int64_t m) { return {Kind::Full, m, 0, 0}; }
  static LinearMaskingScheme chacha(int64_t m, uint64_t dim, uint64_t bits) {
    return {Kind::ChaCha, m, dim, bits};
  }
};

struct LinearSecretSharingScheme {
  enum class Kind { Additive, PackedShamir } kind = Kind::Additive;
  uint64_t share_count = 0;
  int64_t modulus = 0;  // Additive modulus / PackedShamir prime_modulus
  uint64_t secret_count = 0;
  uint64_t privacy_threshold_ = 0;
  int64_t omega_secrets = 0;
  int64_t omega_shares = 0;

  static LinearSecretSharingScheme additive(uint64_t n, int64_t m) {
    LinearSecretSharingScheme s;
    s.kind = Kind::Additive;
    s.share_count = n;
    s.modulus = m;
    return s;
  }
  static LinearSecretSharingScheme packed_shamir(uint64_t k, uint64_t n, uint64_t t, int64_t p,
                                                 int64_t ws, int64_t wn) {
    LinearSecretSharingScheme s;
    s.kind = Kind::PackedShamir;
    s.secret_count = k;
    s.share_count = n;
    s.privacy_threshold_ = t;
    s.modulus = p;
    s.omega_secrets = ws;
    s.omega_shares = wn;
    return s;
  }
  // crypto.rs:101-155
  uint64_t input_size() const { return kind == Kind::Additive ? 1 : secret_count; }
  uint64_t output_size() const { return share_count; }
  uint64_t privacy_threshold() const {
    return kind == Kind::Additive ? share_count - 1 : privacy_threshold_;
  }
  uint64_t reconstruction_threshold() const {
    return kind == Kind::Additive ? share_count : privacy_threshold_ + secret_count;
  }
  bool operator==(const LinearSecretSharingScheme& o) const {
    return kind == o.kind && share_count == o.share_count && modulus == o.modulus &&
           secret_count == o.secret_count && privacy_threshold_ == o.privacy_threshold_ &&
           omega_secrets == o.omega_secrets && omega_shares == o.omega_shares;
  }
};

struct AdditiveEncryptionScheme {  // only Sodium
  uint64_t batch_size() const { return 1; }
  bool operator==(const AdditiveEncryptionScheme&) const { return true; }
};

// ---- resources ---------------------------------------------------------------
struct LabelledVerificationKey {
  VerificationKeyId id;
  VerificationKey body;
  bool operator==(const LabelledVerificationKey& o) const { return id == o.id && body == o.body; }
};

struct Agent {
  AgentId id;
  LabelledVerificationKey verification_key;
  bool operator==(const Agent& o) const { return id == o.id && verification_key == o.verification_key; }
};

struct Profile {
  AgentId owner;
  std::optional<std::string> name, twitter_id, keybase_id, website;
  bool operator==(const Profile& o) const {
    return owner == o.owner && name == o.name && twitter_id == o.twitter_id &&
           keybase_id == o.keybase_id && website == o.website;
  }
};

struct LabelledEncryptionKey {
  EncryptionKeyId id;
  EncryptionKey body;
  bool operator==(const LabelledEncryptionKey& o) const { return id == o.id && body == o.body; }
};

struct SignedEncryptionKey {  // Signed<Labelled<EncryptionKeyId, EncryptionKey>>
  Signature signature;
  AgentId signer;
  LabelledEncryptionKey body;
  const EncryptionKeyId& id() const { return body.id; }
  bool operator==(const SignedEncryptionKey& o) const {
    return signature == o.signature && signer == o.signer && body == o.body;
  }
};

struct Aggregation {
  AggregationId id;
  std::string title;
  uint64_t vector_dimension = 0;
  int64_t modulus = 0;
  AgentId recipient;
  EncryptionKeyId recipient_key;
  LinearMaskingScheme masking_scheme;
  LinearSecretSharingScheme committee_sharing_scheme;
  AdditiveEncryptionScheme recipient_encryption_scheme;
  AdditiveEncryptionScheme committee_encryption_scheme;
  bool operator==(const Aggregation& o) const {
    return id == o.id && title == o.title && vector_dimension == o.vector_dimension &&
           modulus == o.modulus && recipient == o.recipient && recipient_key == o.recipient_key &&
           masking_scheme == o.masking_scheme &&
           committee_sharing_scheme == o.committee_sharing_scheme;
  }
};

struct ClerkCandidate {
  AgentId id;
  std::vector<EncryptionKeyId> keys;
};

struct Committee {
  AggregationId aggregation;
  std::vector<std::pair<AgentId, EncryptionKeyId>> clerks_and_keys;
  bool operator==(const Committee& o) const {
    return aggregation == o.aggregation && clerks_and_keys == o.clerks_and_keys;
  }
};

struct Participation {
  ParticipationId id;
  AgentId participant;
  AggregationId aggregation;
  std::optional<Encryption> recipient_encryption;
  std::vector<std::pair<AgentId, Encryption>> clerk_encryptions;
  bool operator==(const Participation& o) const {
    return id == o.id && participant == o.participant && aggregation == o.aggregation &&
           recipient_encryption == o.recipient_encryption &&
           clerk_encryptions == o.clerk_encryptions;
  }
};

struct Snapshot {
  SnapshotId id;
  AggregationId aggregation;
  bool operator==(const Snapshot& o) const { return id == o.id && aggregation == o.aggregation; }
};

struct ClerkingJob {
  ClerkingJobId id;
  AgentId clerk;
  AggregationId aggregation;
  SnapshotId snapshot;
  std::vector<Encryption> encryptions;
  bool operator==(const ClerkingJob& o) const {
    return id == o.id && clerk == o.clerk && aggregation == o.aggregation &&
           snapshot == o.snapshot && encryptions == o.encryptions;
  }
};

struct ClerkingResult {
  ClerkingJobId job;
  AgentId clerk;
  Encryption encryption;
  bool operator==(const ClerkingResult& o) const {
    return job == o.job && clerk == o.clerk && encryption == o.encryption;
  }
};

struct SnapshotStatus {
  SnapshotId id;
  uint64_t number_of_clerking_results = 0;
  bool result_ready = false;
  bool operator==(const SnapshotStatus& o) const {
    return id == o.id && number_of_clerking_results == o.number_of_clerking_results &&
           result_ready == o.result_ready;
  }
};

struct AggregationStatus {
  AggregationId aggregation;
  uint64_t number_of_participations = 0;
  std::vector<SnapshotStatus> snapshots;
};

struct SnapshotResult {
  SnapshotId snapshot;
  uint64_t number_of_participations = 0;
  std::vector<ClerkingResult> clerk_encryptions;
  std::optional<std::vector<Encryption>> recipient_encryptions;
};

struct Pong {
  bool running = false;
};

// Labelled<AgentId, String>  (server/src/stores.rs:8)
struct AuthToken {
  AgentId id;
  std::string body;
  bool operator==(const AuthToken& o) const { return id == o.id && body == o.body; }
};

// client keystore entries (client/src/crypto/encryption/mod.rs:7-17, signing/mod.rs:21-25)
struct EncryptionKeypair {
  EncryptionKey ek;
  DecryptionKey dk;
};
struct SignatureKeypair {
  VerificationKey vk;
  SigningKey sk;
};

// ---- JSON codecs ---------------------------------------------------------------
namespace wire {
using json::Value;

template <class Tag>
Value to_json(const Id<Tag>& id) { return Value(id.str()); }
template <class T>
T id_from(const Value& v) {
  return T::parse(v.as_string());
}

Value to_json(const Encryption&);
Value to_json(const EncryptionKey&);
Value to_json(const DecryptionKey&);
Value to_json(const Signature&);
Value to_json(const SigningKey&);
Value to_json(const VerificationKey&);
Value to_json(const LinearMaskingScheme&);
Value to_json(const LinearSecretSharingScheme&);
Value to_json(const AdditiveEncryptionScheme&);
Value to_json(const LabelledVerificationKey&);
Value to_json(const LabelledEncryptionKey&);
Value to_json(const Agent&);
Value to_json(const Profile&);
Value to_json(const SignedEncryptionKey&);
Value to_json(const Aggregation&);
Value to_json(const ClerkCandidate&);
Value to_json(const Committee&);
Value to_json(const Participation&);
Value to_json(const Snapshot&);
Value to_json(const ClerkingJob&);
Value to_json(const ClerkingResult&);
Value to_json(const SnapshotStatus&);
Value to_json(const AggregationStatus&);
Value to_json(const SnapshotResult&);
Value to_json(const Pong&);
Value to_json(const AuthToken&);
Value to_json(const EncryptionKeypair&);
Value to_json(const SignatureKeypair&);

template <class T>
T from_json(const Value& v);

template <class T>
std::string encode(const T& x) { return to_json(x).dump(); }
template <class T>
T decode(const std::string& s) { return from_json<T>(Value::parse(s)); }

// Zero-copy views of the bulk downloads (wire_views.cc): where each base64
// payload sits inside the response text. nullopt = the text is not in the plain
// shape serde_json emits; use decode<>() instead.
struct TextSpan {
  size_t off = 0, len = 0;
};
struct ClerkingJobView {
  ClerkingJob head;             // `encryptions` left empty
  std::vector<TextSpan> boxes;  // base64 of encryptions[i]
};
struct SnapshotResultView {
  struct Result {
    ClerkingJobId job;
    AgentId clerk;
    TextSpan box;
  };
  SnapshotId snapshot;
  uint64_t number_of_participations = 0;
  std::vector<Result> results;
  bool has_masks = false;
  std::vector<TextSpan> masks;
};
std::optional<ClerkingJobView> scan_clerking_job(const std::string& text);
std::optional<SnapshotResultView> scan_snapshot_result(const std::string& text);

// Canonical bytes for signing (helpers.rs:130-142): compact JSON.
template <class T>
Bytes canonical(const T& x) {
  std::string s = encode(x);
  return Bytes(s.begin(), s.end());
}
}  // namespace wire

}  // namespace sda
