// JSON wire codecs for the SDA protocol resources (see sda/protocol.hpp).
#include "sda/protocol.hpp"

namespace sda {
namespace wire {

namespace {

template <size_t N>
Value b64(const ByteArray<N>& a) { return Value(base64_encode(a.data(), N)); }

template <size_t N>
ByteArray<N> b64_fixed(const Value& v) {
  Bytes b = base64_decode_fixed(v.as_string(), N);
  ByteArray<N> out;
  std::copy(b.begin(), b.end(), out.begin());
  return out;
}

// {"Sodium": <payload>}
const Value& sodium_payload(const Value& v) {
  if (!v.is_object() || v.size() != 1 || !v.has("Sodium"))
    throw SdaError("json: expected {\"Sodium\": ...}");
  return v.at("Sodium");
}
Value sodium(Value payload) {
  Value o = Value::object();
  o.set("Sodium", std::move(payload));
  return o;
}

Value opt_str(const std::optional<std::string>& s) { return s ? Value(*s) : Value(nullptr); }
std::optional<std::string> opt_str_from(const Value* v) {
  if (!v || v->is_null()) return std::nullopt;
  return v->as_string();
}

// unit-or-newtype enum variant name + payload
std::pair<std::string, const Value*> variant(const Value& v) {
  if (v.is_string()) return {v.as_string(), nullptr};
  if (v.is_object() && v.size() == 1) {
    auto& kv = v.as_object()[0];
    return {kv.first, &kv.second};
  }
  throw SdaError("json: expected an enum variant");
}

}  // namespace

Value to_json(const Encryption& e) { return sodium(Value(base64_encode(e.sodium))); }
Value to_json(const EncryptionKey& k) { return sodium(b64(k.sodium)); }
Value to_json(const DecryptionKey& k) { return sodium(b64(k.sodium)); }
Value to_json(const Signature& s) { return sodium(b64(s.sodium)); }
Value to_json(const SigningKey& s) { return sodium(b64(s.sodium)); }
Value to_json(const VerificationKey& k) { return sodium(b64(k.sodium)); }

template <> Encryption from_json<Encryption>(const Value& v) {
  return Encryption{base64_decode(sodium_payload(v).as_string())};
}
template <> EncryptionKey from_json<EncryptionKey>(const Value& v) {
  return EncryptionKey{b64_fixed<32>(sodium_payload(v))};
}
template <> DecryptionKey from_json<DecryptionKey>(const Value& v) {
  return DecryptionKey{b64_fixed<32>(sodium_payload(v))};
}
template <> Signature from_json<Signature>(const Value& v) {
  return Signature{b64_fixed<64>(sodium_payload(v))};
}
template <> SigningKey from_json<SigningKey>(const Value& v) {
  return SigningKey{b64_fixed<64>(sodium_payload(v))};
}
template <> VerificationKey from_json<VerificationKey>(const Value& v) {
  return VerificationKey{b64_fixed<32>(sodium_payload(v))};
}

Value to_json(const LinearMaskingScheme& s) {
  switch (s.kind) {
    case LinearMaskingScheme::Kind::None: return Value("None");
    case LinearMaskingScheme::Kind::Full: {
      Value inner = Value::object();
      inner.set("modulus", Value((long long)s.modulus));
      Value o = Value::object();
      o.set("Full", inner);
      return o;
    }
    case LinearMaskingScheme::Kind::ChaCha: {
      Value inner = Value::object();
      inner.set("modulus", Value((long long)s.modulus));
      inner.set("dimension", Value((unsigned long long)s.dimension));
      inner.set("seed_bitsize", Value((unsigned long long)s.seed_bitsize));
      Value o = Value::object();
      o.set("ChaCha", inner);
      return o;
    }
  }
  return Value();
}
template <> LinearMaskingScheme from_json<LinearMaskingScheme>(const Value& v) {
  auto [name, p] = variant(v);
  if (name == "None") return LinearMaskingScheme::none();
  if (!p) throw SdaError("json: masking scheme `" + name + "` needs fields");
  if (name == "Full") return LinearMaskingScheme::full(p->at("modulus").as_i64());
  if (name == "ChaCha")
    return LinearMaskingScheme::chacha(p->at("modulus").as_i64(), p->at("dimension").as_u64(),
                                       p->at("seed_bitsize").as_u64());
  throw SdaError("json: unknown masking scheme `" + name + "`");
}

Value to_json(const LinearSecretSharingScheme& s) {
  Value inner = Value::object();
  Value o = Value::object();
  if (s.kind == LinearSecretSharingScheme::Kind::Additive) {
    inner.set("share_count", Value((unsigned long long)s.share_count));
    inner.set("modulus", Value((long long)s.modulus));
    o.set("Additive", inner);
  } else {
    inner.set("secret_count", Value((unsigned long long)s.secret_count));
    inner.set("share_count", Value((unsigned long long)s.share_count));
    inner.set("privacy_threshold", Value((unsigned long long)s.privacy_threshold_));
    inner.set("prime_modulus", Value((long long)s.modulus));
    inner.set("omega_secrets", Value((long long)s.omega_secrets));
    inner.set("omega_shares", Value((long long)s.omega_shares));
    o.set("PackedShamir", inner);
  }
  return o;
}
template <> LinearSecretSharingScheme from_json<LinearSecretSharingScheme>(const Value& v) {
  auto [name, p] = variant(v);
  if (!p) throw SdaError("json: sharing scheme `" + name + "` needs fields");
  if (name == "Additive")
    return LinearSecretSharingScheme::additive(p->at("share_count").as_u64(), p->at("modulus").as_i64());
  if (name == "PackedShamir")
    return LinearSecretSharingScheme::packed_shamir(
        p->at("secret_count").as_u64(), p->at("share_count").as_u64(),
        p->at("privacy_threshold").as_u64(), p->at("prime_modulus").as_i64(),
        p->at("omega_secrets").as_i64(), p->at("omega_shares").as_i64());
  throw SdaError("json: unknown sharing scheme `" + name + "`");
}

Value to_json(const AdditiveEncryptionScheme&) { return Value("Sodium"); }
template <> AdditiveEncryptionScheme from_json<AdditiveEncryptionScheme>(const Value& v) {
  auto [name, p] = variant(v);
  (void)p;
  if (name != "Sodium") throw SdaError("json: unknown encryption scheme `" + name + "`");
  return {};
}

Value to_json(const LabelledVerificationKey& l) {
  Value o = Value::object();
  o.set("id", to_json(l.id));
  o.set("body", to_json(l.body));
  return o;
}
template <> LabelledVerificationKey from_json<LabelledVerificationKey>(const Value& v) {
  return {id_from<VerificationKeyId>(v.at("id")), from_json<VerificationKey>(v.at("body"))};
}
Value to_json(const LabelledEncryptionKey& l) {
  Value o = Value::object();
  o.set("id", to_json(l.id));
  o.set("body", to_json(l.body));
  return o;
}
template <> LabelledEncryptionKey from_json<LabelledEncryptionKey>(const Value& v) {
  return {id_from<EncryptionKeyId>(v.at("id")), from_json<EncryptionKey>(v.at("body"))};
}

Value to_json(const Agent& a) {
  Value o = Value::object();
  o.set("id", to_json(a.id));
  o.set("verification_key", to_json(a.verification_key));
  return o;
}
template <> Agent from_json<Agent>(const Value& v) {
  return {id_from<AgentId>(v.at("id")), from_json<LabelledVerificationKey>(v.at("verification_key"))};
}

Value to_json(const Profile& p) {
  Value o = Value::object();
  o.set("owner", to_json(p.owner));
  o.set("name", opt_str(p.name));
  o.set("twitter_id", opt_str(p.twitter_id));
  o.set("keybase_id", opt_str(p.keybase_id));
  o.set("website", opt_str(p.website));
  return o;
}
template <> Profile from_json<Profile>(const Value& v) {
  Profile p;
  p.owner = id_from<AgentId>(v.at("owner"));
  p.name = opt_str_from(v.find("name"));
  p.twitter_id = opt_str_from(v.find("twitter_id"));
  p.keybase_id = opt_str_from(v.find("keybase_id"));
  p.website = opt_str_from(v.find("website"));
  return p;
}

Value to_json(const SignedEncryptionKey& k) {
  Value o = Value::object();
  o.set("signature", to_json(k.signature));
  o.set("signer", to_json(k.signer));
  o.set("body", to_json(k.body));
  return o;
}
template <> SignedEncryptionKey from_json<SignedEncryptionKey>(const Value& v) {
  return {from_json<Signature>(v.at("signature")), id_from<AgentId>(v.at("signer")),
          from_json<LabelledEncryptionKey>(v.at("body"))};
}

Value to_json(const Aggregation& a) {
  Value o = Value::object();
  o.set("id", to_json(a.id));
  o.set("title", Value(a.title));
  o.set("vector_dimension", Value((unsigned long long)a.vector_dimension));
  o.set("modulus", Value((long long)a.modulus));
  o.set("recipient", to_json(a.recipient));
  o.set("recipient_key", to_json(a.recipient_key));
  o.set("masking_scheme", to_json(a.masking_scheme));
  o.set("committee_sharing_scheme", to_json(a.committee_sharing_scheme));
  o.set("recipient_encryption_scheme", to_json(a.recipient_encryption_scheme));
  o.set("committee_encryption_scheme", to_json(a.committee_encryption_scheme));
  return o;
}
template <> Aggregation from_json<Aggregation>(const Value& v) {
  Aggregation a;
  a.id = id_from<AggregationId>(v.at("id"));
  a.title = v.at("title").as_string();
  a.vector_dimension = v.at("vector_dimension").as_u64();
  a.modulus = v.at("modulus").as_i64();
  a.recipient = id_from<AgentId>(v.at("recipient"));
  a.recipient_key = id_from<EncryptionKeyId>(v.at("recipient_key"));
  a.masking_scheme = from_json<LinearMaskingScheme>(v.at("masking_scheme"));
  a.committee_sharing_scheme = from_json<LinearSecretSharingScheme>(v.at("committee_sharing_scheme"));
  a.recipient_encryption_scheme = from_json<AdditiveEncryptionScheme>(v.at("recipient_encryption_scheme"));
  a.committee_encryption_scheme = from_json<AdditiveEncryptionScheme>(v.at("committee_encryption_scheme"));
  return a;
}

Value to_json(const ClerkCandidate& c) {
  Value o = Value::object();
  o.set("id", to_json(c.id));
  Value keys = Value::array();
  for (auto& k : c.keys) keys.push(to_json(k));
  o.set("keys", keys);
  return o;
}
template <> ClerkCandidate from_json<ClerkCandidate>(const Value& v) {
  ClerkCandidate c;
  c.id = id_from<AgentId>(v.at("id"));
  for (auto& k : v.at("keys").as_array()) c.keys.push_back(id_from<EncryptionKeyId>(k));
  return c;
}

Value to_json(const Committee& c) {
  Value o = Value::object();
  o.set("aggregation", to_json(c.aggregation));
  Value list = Value::array();
  for (auto& ck : c.clerks_and_keys) {
    Value pair = Value::array();
    pair.push(to_json(ck.first));
    pair.push(to_json(ck.second));
    list.push(pair);
  }
  o.set("clerks_and_keys", list);
  return o;
}
template <> Committee from_json<Committee>(const Value& v) {
  Committee c;
  c.aggregation = id_from<AggregationId>(v.at("aggregation"));
  for (auto& p : v.at("clerks_and_keys").as_array()) {
    auto& a = p.as_array();
    if (a.size() != 2) throw SdaError("json: expected a (clerk, key) pair");
    c.clerks_and_keys.emplace_back(id_from<AgentId>(a[0]), id_from<EncryptionKeyId>(a[1]));
  }
  return c;
}

Value to_json(const Participation& p) {
  Value o = Value::object();
  o.set("id", to_json(p.id));
  o.set("participant", to_json(p.participant));
  o.set("aggregation", to_json(p.aggregation));
  o.set("recipient_encryption", p.recipient_encryption ? to_json(*p.recipient_encryption) : Value(nullptr));
  Value list = Value::array();
  for (auto& ce : p.clerk_encryptions) {
    Value pair = Value::array();
    pair.push(to_json(ce.first));
    pair.push(to_json(ce.second));
    list.push(pair);
  }
  o.set("clerk_encryptions", list);
  return o;
}
template <> Participation from_json<Participation>(const Value& v) {
  Participation p;
  p.id = id_from<ParticipationId>(v.at("id"));
  p.participant = id_from<AgentId>(v.at("participant"));
  p.aggregation = id_from<AggregationId>(v.at("aggregation"));
  const Value* re = v.find("recipient_encryption");
  if (re && !re->is_null()) p.recipient_encryption = from_json<Encryption>(*re);
  for (auto& pair : v.at("clerk_encryptions").as_array()) {
    auto& a = pair.as_array();
    if (a.size() != 2) throw SdaError("json: expected a (clerk, encryption) pair");
    p.clerk_encryptions.emplace_back(id_from<AgentId>(a[0]), from_json<Encryption>(a[1]));
  }
  return p;
}

Value to_json(const Snapshot& s) {
  Value o = Value::object();
  o.set("id", to_json(s.id));
  o.set("aggregation", to_json(s.aggregation));
  return o;
}
template <> Snapshot from_json<Snapshot>(const Value& v) {
  return {id_from<SnapshotId>(v.at("id")), id_from<AggregationId>(v.at("aggregation"))};
}

Value to_json(const ClerkingJob& j) {
  Value o = Value::object();
  o.set("id", to_json(j.id));
  o.set("clerk", to_json(j.clerk));
  o.set("aggregation", to_json(j.aggregation));
  o.set("snapshot", to_json(j.snapshot));
  Value list = Value::array();
  for (auto& e : j.encryptions) list.push(to_json(e));
  o.set("encryptions", list);
  return o;
}
template <> ClerkingJob from_json<ClerkingJob>(const Value& v) {
  ClerkingJob j;
  j.id = id_from<ClerkingJobId>(v.at("id"));
  j.clerk = id_from<AgentId>(v.at("clerk"));
  j.aggregation = id_from<AggregationId>(v.at("aggregation"));
  j.snapshot = id_from<SnapshotId>(v.at("snapshot"));
  for (auto& e : v.at("encryptions").as_array()) j.encryptions.push_back(from_json<Encryption>(e));
  return j;
}

Value to_json(const ClerkingResult& r) {
  Value o = Value::object();
  o.set("job", to_json(r.job));
  o.set("clerk", to_json(r.clerk));
  o.set("encryption", to_json(r.encryption));
  return o;
}
template <> ClerkingResult from_json<ClerkingResult>(const Value& v) {
  return {id_from<ClerkingJobId>(v.at("job")), id_from<AgentId>(v.at("clerk")),
          from_json<Encryption>(v.at("encryption"))};
}

Value to_json(const SnapshotStatus& s) {
  Value o = Value::object();
  o.set("id", to_json(s.id));
  o.set("number_of_clerking_results", Value((unsigned long long)s.number_of_clerking_results));
  o.set("result_ready", Value(s.result_ready));
  return o;
}
template <> SnapshotStatus from_json<SnapshotStatus>(const Value& v) {
  return {id_from<SnapshotId>(v.at("id")), v.at("number_of_clerking_results").as_u64(),
          v.at("result_ready").as_bool()};
}

Value to_json(const AggregationStatus& s) {
  Value o = Value::object();
  o.set("aggregation", to_json(s.aggregation));
  o.set("number_of_participations", Value((unsigned long long)s.number_of_participations));
  Value list = Value::array();
  for (auto& x : s.snapshots) list.push(to_json(x));
  o.set("snapshots", list);
  return o;
}
template <> AggregationStatus from_json<AggregationStatus>(const Value& v) {
  AggregationStatus s;
  s.aggregation = id_from<AggregationId>(v.at("aggregation"));
  s.number_of_participations = v.at("number_of_participations").as_u64();
  for (auto& x : v.at("snapshots").as_array()) s.snapshots.push_back(from_json<SnapshotStatus>(x));
  return s;
}

Value to_json(const SnapshotResult& r) {
  Value o = Value::object();
  o.set("snapshot", to_json(r.snapshot));
  o.set("number_of_participations", Value((unsigned long long)r.number_of_participations));
  Value list = Value::array();
  for (auto& x : r.clerk_encryptions) list.push(to_json(x));
  o.set("clerk_encryptions", list);
  if (r.recipient_encryptions) {
    Value re = Value::array();
    for (auto& e : *r.recipient_encryptions) re.push(to_json(e));
    o.set("recipient_encryptions", re);
  } else {
    o.set("recipient_encryptions", Value(nullptr));
  }
  return o;
}
template <> SnapshotResult from_json<SnapshotResult>(const Value& v) {
  SnapshotResult r;
  r.snapshot = id_from<SnapshotId>(v.at("snapshot"));
  r.number_of_participations = v.at("number_of_participations").as_u64();
  for (auto& x : v.at("clerk_encryptions").as_array()) r.clerk_encryptions.push_back(from_json<ClerkingResult>(x));
  const Value* re = v.find("recipient_encryptions");
  if (re && !re->is_null()) {
    std::vector<Encryption> es;
    for (auto& e : re->as_array()) es.push_back(from_json<Encryption>(e));
    r.recipient_encryptions = std::move(es);
  }
  return r;
}

Value to_json(const Pong& p) {
  Value o = Value::object();
  o.set("running", Value(p.running));
  return o;
}
template <> Pong from_json<Pong>(const Value& v) { return Pong{v.at("running").as_bool()}; }

Value to_json(const AuthToken& t) {
  Value o = Value::object();
  o.set("id", to_json(t.id));
  o.set("body", Value(t.body));
  return o;
}
template <> AuthToken from_json<AuthToken>(const Value& v) {
  return {id_from<AgentId>(v.at("id")), v.at("body").as_string()};
}

Value to_json(const EncryptionKeypair& k) {
  Value o = Value::object();
  o.set("ek", to_json(k.ek));
  o.set("dk", to_json(k.dk));
  return o;
}
template <> EncryptionKeypair from_json<EncryptionKeypair>(const Value& v) {
  return {from_json<EncryptionKey>(v.at("ek")), from_json<DecryptionKey>(v.at("dk"))};
}
Value to_json(const SignatureKeypair& k) {
  Value o = Value::object();
  o.set("vk", to_json(k.vk));
  o.set("sk", to_json(k.sk));
  return o;
}
template <> SignatureKeypair from_json<SignatureKeypair>(const Value& v) {
  return {from_json<VerificationKey>(v.at("vk")), from_json<SigningKey>(v.at("sk"))};
}

}  // namespace wire
}  // namespace sda
