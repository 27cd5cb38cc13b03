// SDA client roles and crypto engines (reference client/src/*.rs).
#include "sda/client.hpp"

#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <thread>

#include "sda/crypto.hpp"
#include "sda/field.hpp"
#include "sda/log.hpp"

namespace sda {

namespace cr = crypto;

// ---- stores -------------------------------------------------------------------
static void mkdirs(const std::string& path) {
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    std::string cur = path.substr(0, j);
    if (!cur.empty() && ::mkdir(cur.c_str(), 0700) != 0 && errno != EEXIST)
      throw SdaError("Storage error: cannot create " + cur);
    i = j + 1;
  }
}

std::string Store::auth_token() {
  if (auto v = get_json("auth_token")) return v->as_string();
  static const char* alnum = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
  std::string tok;
  while (tok.size() < 32) {
    uint8_t b;
    cr::os_random(&b, 1);
    if (b < 248) tok.push_back(alnum[b % 62]);  // unbiased: 248 = 4 * 62
  }
  put_json("auth_token", json::Value(tok));
  return tok;
}

FileStore::FileStore(const std::string& dir) : dir_(dir) { mkdirs(dir_); }

void FileStore::put_json(const std::string& id, const json::Value& v) {
  std::lock_guard<std::mutex> g(mu_);
  std::string path = dir_ + "/" + id + ".json";
  std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp, std::ios::trunc);
    if (!f) throw SdaError("Storage error: cannot write " + path);
    f << v.dump();
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw SdaError("Storage error: rename failed");
}

std::optional<json::Value> FileStore::get_json(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  std::ifstream f(dir_ + "/" + id + ".json");
  if (!f) return std::nullopt;
  std::stringstream ss;
  ss << f.rdbuf();
  return json::Value::parse(ss.str());
}

void MemoryStore::put_json(const std::string& id, const json::Value& v) {
  std::lock_guard<std::mutex> g(mu_);
  m_[id] = v;
}
std::optional<json::Value> MemoryStore::get_json(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(id);
  if (it == m_.end()) return std::nullopt;
  return it->second;
}

// ---- masking (client/src/crypto/masking/*.rs) ----------------------------------
MaskResult mask_secrets(const LinearMaskingScheme& s, const std::vector<int64_t>& secrets) {
  MaskResult r;
  switch (s.kind) {
    case LinearMaskingScheme::Kind::None:
      r.masked_secrets = secrets;
      break;
    case LinearMaskingScheme::Kind::Full:
      for (int64_t x : secrets) {
        int64_t m = cr::os_random_range(s.modulus);
        r.mask.push_back(m);
        r.masked_secrets.push_back((x + m) % s.modulus);
      }
      break;
    case LinearMaskingScheme::Kind::ChaCha: {
      if (s.dimension != secrets.size()) throw SdaError("ChaCha mask dimension mismatch");
      size_t words = (s.seed_bitsize + 31) / 32;
      std::vector<uint32_t> seed(words);
      for (auto& w : seed) w = cr::os_random_u32();
      cr::ChaChaRng rng(seed.data(), seed.size());
      for (int64_t x : secrets) r.masked_secrets.push_back((x + rng.gen_range(0, s.modulus)) % s.modulus);
      for (uint32_t w : seed) r.mask.push_back((int64_t)w);
      break;
    }
  }
  return r;
}

std::vector<int64_t> combine_masks(const LinearMaskingScheme& s,
                                   const std::vector<std::vector<int64_t>>& masks) {
  switch (s.kind) {
    case LinearMaskingScheme::Kind::None:
      for (auto& m : masks)
        if (!m.empty()) throw SdaError("unexpected mask for the None scheme");
      return {};
    case LinearMaskingScheme::Kind::Full: {
      size_t dim = masks.empty() ? 0 : masks[0].size();
      std::vector<int64_t> out(dim, 0);
      for (auto& m : masks) {
        if (m.size() != dim) throw SdaError("mask dimension mismatch");
        for (size_t i = 0; i < dim; ++i) out[i] = (out[i] + m[i]) % s.modulus;
      }
      return out;
    }
    case LinearMaskingScheme::Kind::ChaCha: {
      std::vector<int64_t> out(s.dimension, 0);
      for (auto& seed64 : masks) {
        std::vector<uint32_t> seed;
        for (int64_t w : seed64) seed.push_back((uint32_t)w);
        cr::ChaChaRng rng(seed.data(), seed.size());
        for (size_t i = 0; i < s.dimension; ++i) out[i] = (out[i] + rng.gen_range(0, s.modulus)) % s.modulus;
      }
      return out;
    }
  }
  return {};
}

std::vector<int64_t> unmask(const LinearMaskingScheme& s, const std::vector<int64_t>& mask,
                            const std::vector<int64_t>& masked) {
  if (s.kind == LinearMaskingScheme::Kind::None) {
    if (!mask.empty()) throw SdaError("unexpected mask for the None scheme");
    return masked;
  }
  if (mask.size() != masked.size()) throw SdaError("mask / output dimension mismatch");
  std::vector<int64_t> out(masked.size());
  for (size_t i = 0; i < masked.size(); ++i) out[i] = (masked[i] - mask[i]) % s.modulus;
  return out;
}

// ---- sharing (client/src/crypto/sharing/*.rs) ----------------------------------
static PackedShamirParams pss_params(const LinearSecretSharingScheme& s) {
  return PackedShamirParams{(int)s.secret_count, (int)s.share_count, (int)s.privacy_threshold_,
                            s.modulus, s.omega_secrets, s.omega_shares};
}

std::vector<std::vector<int64_t>> generate_shares(const LinearSecretSharingScheme& s,
                                                  const std::vector<int64_t>& secrets) {
  const size_t n = s.output_size(), k = s.input_size();
  const size_t batches = (secrets.size() + k - 1) / k;
  std::vector<std::vector<int64_t>> out(n);
  for (auto& v : out) v.reserve(batches);
  if (s.kind == LinearSecretSharingScheme::Kind::Additive) {
    if (n < 1) throw SdaError("additive sharing needs at least one share");
    for (int64_t secret : secrets) {
      int64_t last = secret;
      for (size_t c = 0; c + 1 < n; ++c) {
        int64_t r = cr::os_random_range(s.modulus);
        out[c].push_back(r);
        last = (last - r) % s.modulus;  // Rust truncated remainder (additive.rs:47)
      }
      out[n - 1].push_back(last);
    }
    return out;
  }
  PackedShamirParams p = pss_params(s);
  p.validate();
  std::vector<int64_t> batch(k), rnd(p.privacy_threshold);
  for (size_t b = 0; b < batches; ++b) {
    for (size_t j = 0; j < k; ++j) {
      size_t e = b * k + j;
      batch[j] = e < secrets.size() ? secrets[e] : 0;  // zero padding (batched.rs:37-43)
    }
    for (auto& r : rnd) r = cr::os_random_range(p.prime);
    auto shares = p.share(batch, rnd);
    for (size_t c = 0; c < n; ++c) out[c].push_back(shares[c]);
  }
  return out;
}

std::vector<int64_t> combine_shares(const LinearSecretSharingScheme& s,
                                    const std::vector<std::vector<int64_t>>& shares) {
  size_t dim = shares.empty() ? 0 : shares[0].size();
  std::vector<int64_t> out(dim, 0);
  for (auto& v : shares) {
    if (v.size() != dim) throw SdaError("Wrong dimension");
    for (size_t i = 0; i < dim; ++i) out[i] = (out[i] + v[i]) % s.modulus;
  }
  return out;
}

std::vector<int64_t> reconstruct_secrets(const LinearSecretSharingScheme& s, uint64_t dimension,
                                         const std::vector<std::pair<size_t, std::vector<int64_t>>>& indexed) {
  if (s.kind == LinearSecretSharingScheme::Kind::Additive) {
    size_t dim = indexed.empty() ? 0 : indexed[0].second.size();
    std::vector<int64_t> out(dim, 0);
    for (auto& is : indexed) {
      if (is.second.size() != dim) throw SdaError("Mismatching dimension");
      for (size_t i = 0; i < dim; ++i) out[i] = (out[i] + is.second[i]) % s.modulus;
    }
    return out;
  }
  PackedShamirParams p = pss_params(s);
  if ((int)indexed.size() < p.reconstruct_limit()) throw SdaError("Not enough shares to reconstruct");
  std::vector<int> idx;
  for (auto& is : indexed) idx.push_back((int)is.first);
  const size_t k = s.secret_count;
  const size_t batches = (dimension + k - 1) / k;
  auto L = p.lagrange_matrix(idx);
  std::vector<int64_t> out;
  out.reserve(batches * k);
  for (size_t b = 0; b < batches; ++b) {
    for (size_t sidx = 0; sidx < k; ++sidx) {
      unsigned __int128 acc = 0;
      for (size_t i = 0; i < idx.size(); ++i) {
        if (indexed[i].second.size() <= b) throw SdaError("Mismatching dimension");
        acc += (unsigned __int128)L[sidx * idx.size() + i] * canon(indexed[i].second[b], p.prime);
      }
      out.push_back((int64_t)(uint64_t)(acc % (uint64_t)p.prime));
    }
  }
  out.resize(dimension);  // drop padding (batched.rs:94)
  return out;
}

// ---- encryption (client/src/crypto/encryption/sodium.rs) ------------------------
Bytes varint_encode(const std::vector<int64_t>& values) {
  Bytes out;
  out.reserve(values.size() * 2);
  for (int64_t v : values) {
    uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
    while (z >= 0x80) {
      out.push_back((uint8_t)(z | 0x80));
      z >>= 7;
    }
    out.push_back((uint8_t)z);
  }
  return out;
}

std::vector<int64_t> varint_decode(const Bytes& bytes) {
  std::vector<int64_t> out;
  uint64_t z = 0;
  int shift = 0;
  for (uint8_t b : bytes) {
    if (shift < 64) z |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) {
      out.push_back((int64_t)((z >> 1) ^ (~(z & 1) + 1)));
      z = 0;
      shift = 0;
    }
  }
  if (shift) throw SdaError("Sodium decryption failure: truncated varint");
  return out;
}

Encryption encrypt_shares(const EncryptionKey& ek, const std::vector<int64_t>& shares) {
  Bytes pt = varint_encode(shares);
  return Encryption{cr::box_seal(pt.data(), pt.size(), ek.sodium.data())};
}

std::vector<int64_t> decrypt_shares(const EncryptionKeypair& kp, const Encryption& e) {
  Bytes pt;
  if (!cr::box_seal_open(pt, e.sodium.data(), e.sodium.size(), kp.ek.sodium.data(), kp.dk.sodium.data()))
    throw SdaError("Sodium decryption failure");
  return varint_decode(pt);
}

RecipientOutput RecipientOutput::positive() const {
  RecipientOutput r{modulus, values};
  for (auto& v : r.values)
    if (v < 0) v += modulus;
  return r;
}

// ---- SdaClient --------------------------------------------------------------------
Agent SdaClient::new_agent(Store& keystore) {
  uint8_t pk[32], sk[64];
  cr::ed25519_keypair(pk, sk);
  SignatureKeypair kp;
  std::copy(pk, pk + 32, kp.vk.sodium.begin());
  std::copy(sk, sk + 64, kp.sk.sodium.begin());
  secure_zero(sk, sizeof(sk));
  Agent a;
  a.id = AgentId::random();
  a.verification_key.id = VerificationKeyId::random();
  a.verification_key.body = kp.vk;
  keystore.put(a.verification_key.id.str(), kp);
  return a;
}

void SdaClient::upload_agent() { service_->create_agent(agent_, agent_); }

EncryptionKeyId SdaClient::new_encryption_key() {
  EncryptionKeypair kp;
  cr::box_keypair(kp.ek.sodium.data(), kp.dk.sodium.data());
  EncryptionKeyId id = EncryptionKeyId::random();
  keystore_->put(id.str(), kp);
  return id;
}

std::optional<SignedEncryptionKey> SdaClient::sign_export(const EncryptionKeyId& key) {
  auto kp = keystore_->get<EncryptionKeypair>(key.str());
  if (!kp) return std::nullopt;
  auto skp = keystore_->get<SignatureKeypair>(agent_.verification_key.id.str());
  if (!skp) return std::nullopt;
  SignedEncryptionKey sk;
  sk.body = LabelledEncryptionKey{key, kp->ek};
  sk.signer = agent_.id;
  Bytes msg = wire::canonical(sk.body);  // compact JSON of Labelled{id, body}
  cr::ed25519_sign(sk.signature.sodium.data(), msg.data(), msg.size(), skp->sk.sodium.data());
  return sk;
}

void SdaClient::upload_encryption_key(const EncryptionKeyId& key) {
  auto signed_key = sign_export(key);
  if (!signed_key) throw SdaError("Could not sign encryption key");
  service_->create_encryption_key(agent_, *signed_key);
}

bool SdaClient::signature_is_valid(const Agent& signer, const SignedEncryptionKey& key) {
  if (key.signer != signer.id) throw SdaError("Agent differs from claimed signer");
  Bytes msg = wire::canonical(key.body);
  std::string cache_key = signer.id.str() + "|" + base64_encode(key.signature.sodium.data(), 64) + "|" +
                          base64_encode(signer.verification_key.body.sodium.data(), 32) + "|" +
                          std::string(msg.begin(), msg.end());
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    auto it = verify_cache_.find(cache_key);
    if (it != verify_cache_.end()) return it->second;
  }
  bool ok = cr::ed25519_verify(key.signature.sodium.data(), msg.data(), msg.size(),
                               signer.verification_key.body.sodium.data());
  std::lock_guard<std::mutex> g(cache_mu_);
  verify_cache_[cache_key] = ok;
  return ok;
}

EncryptionKey SdaClient::verified_key(const AgentId& owner, const EncryptionKeyId& key, const char* what) {
  auto sk = service_->get_encryption_key(agent_, key);
  if (!sk) throw SdaError(std::string("Unknown ") + what + " encryption key");
  auto a = service_->get_agent(agent_, owner);
  if (!a) throw SdaError(std::string("Unknown ") + what);
  if (!signature_is_valid(*a, *sk))
    throw SdaError(std::string("Signature verification failed for ") + what + " key");
  return sk->body.body;
}

Participation SdaClient::new_participation(const std::vector<int64_t>& input, const AggregationId& agg_id) {
  auto agg = service_->get_aggregation(agent_, agg_id);
  if (!agg) throw SdaError("Could not find aggregation");
  if (input.size() != agg->vector_dimension) throw SdaError("The input length does not match the aggregation.");
  auto committee = service_->get_committee(agent_, agg_id);
  if (!committee) throw SdaError("Could not find committee");
  MaskResult mr = mask_secrets(agg->masking_scheme, input);
  Participation p;
  if (!mr.mask.empty()) {
    EncryptionKey ek = verified_key(agg->recipient, agg->recipient_key, "recipient");
    p.recipient_encryption = encrypt_shares(ek, mr.mask);
  }
  auto shares = generate_shares(agg->committee_sharing_scheme, mr.masked_secrets);
  if (shares.size() != committee->clerks_and_keys.size())
    throw SdaError("committee size does not match the sharing scheme");
  // participate.rs:82-101: one sealed box per clerk. Keys are fetched and verified
  // in order; the n seals are independent and run side by side.
  std::vector<EncryptionKey> eks;
  for (size_t i = 0; i < shares.size(); ++i) {
    const auto& ck = committee->clerks_and_keys[i];
    eks.push_back(verified_key(ck.first, ck.second, "clerk"));
  }
  std::vector<Encryption> sealed(shares.size());
  const bool threaded = shares.size() > 1 && !shares[0].empty() && shares[0].size() * shares.size() >= 4096;
  if (threaded) {
    std::vector<std::thread> workers;
    const size_t nthreads = std::min<size_t>({shares.size(), (size_t)8,
                                              (size_t)std::max(1u, std::thread::hardware_concurrency())});
    for (size_t tid = 0; tid < nthreads; ++tid)
      workers.emplace_back([&, tid] {
        for (size_t i = tid; i < shares.size(); i += nthreads) sealed[i] = encrypt_shares(eks[i], shares[i]);
      });
    for (auto& w : workers) w.join();
  } else {
    for (size_t i = 0; i < shares.size(); ++i) sealed[i] = encrypt_shares(eks[i], shares[i]);
  }
  for (size_t i = 0; i < shares.size(); ++i)
    p.clerk_encryptions.emplace_back(committee->clerks_and_keys[i].first, std::move(sealed[i]));
  p.id = ParticipationId::random();
  p.participant = agent_.id;
  p.aggregation = agg->id;
  return p;
}

void SdaClient::upload_participation(const Participation& p) { service_->create_participation(agent_, p); }

std::string SdaClient::device_unsupported(const Aggregation& agg) {
  const auto& sh = agg.committee_sharing_scheme;
  const auto& mk = agg.masking_scheme;
  if (sh.modulus < 2 || sh.modulus >= ((int64_t)1 << 31)) return "the modulus does not fit 31 bits";
  if (agg.vector_dimension == 0 || agg.vector_dimension > ((uint64_t)1 << 30)) return "vector dimension out of range";
  if (mk.has_mask() && mk.modulus != sh.modulus) return "masking and sharing moduli differ";
  if (mk.kind == LinearMaskingScheme::Kind::ChaCha) {
    if (mk.seed_bitsize == 0 || mk.seed_bitsize > 256) return "ChaCha seeds of up to 256 bits";
    if (mk.dimension != agg.vector_dimension) return "ChaCha mask dimension differs from the vector dimension";
  }
  if (sh.kind == LinearSecretSharingScheme::Kind::Additive) {
    if (sh.share_count < 1 || sh.share_count > 256) return "additive sharing with 1..256 clerks";
  } else {
    const bool big = sh.secret_count > 8 || sh.privacy_threshold_ > 16 || sh.share_count > 64;
    if (big && sh.modulus >= ((int64_t)1 << 28)) return "large packed-Shamir sets need a modulus below 2^28";
    if (sh.secret_count + sh.privacy_threshold_ > 4096) return "packed-Shamir degree too large";
  }
  return "";
}

std::vector<Participation> SdaClient::new_participations(const std::vector<std::vector<int64_t>>& inputs,
                                                         const AggregationId& agg_id) {
  auto agg = service_->get_aggregation(agent_, agg_id);
  if (!agg) throw SdaError("Could not find aggregation");
  std::string why = device_ ? device_unsupported(*agg) : "no GPU backend";
  if (!why.empty()) {
    if (device_) log_warn("participate: host engines (" + why + ")");
    std::vector<Participation> out;
    for (auto& v : inputs) out.push_back(new_participation(v, agg_id));
    return out;
  }
  for (auto& v : inputs)
    if (v.size() != agg->vector_dimension) throw SdaError("The input length does not match the aggregation.");
  auto committee = service_->get_committee(agent_, agg_id);
  if (!committee) throw SdaError("Could not find committee");
  if (committee->clerks_and_keys.size() != agg->committee_sharing_scheme.output_size())
    throw SdaError("committee size does not match the sharing scheme");
  std::vector<EncryptionKey> clerk_keys;
  for (auto& ck : committee->clerks_and_keys) clerk_keys.push_back(verified_key(ck.first, ck.second, "clerk"));
  std::optional<EncryptionKey> rk;
  if (agg->masking_scheme.has_mask()) rk = verified_key(agg->recipient, agg->recipient_key, "recipient");
  DeviceParticipations dp = device_->participate_many(*agg, clerk_keys, rk ? &*rk : nullptr, inputs);
  std::vector<Participation> out(inputs.size());
  for (size_t i = 0; i < inputs.size(); ++i) {
    Participation& p = out[i];
    p.id = ParticipationId::random();
    p.participant = agent_.id;
    p.aggregation = agg->id;
    if (rk) p.recipient_encryption = std::move(dp.mask_boxes[i]);
    for (size_t c = 0; c < clerk_keys.size(); ++c)
      p.clerk_encryptions.emplace_back(committee->clerks_and_keys[c].first, std::move(dp.clerk_boxes[i][c]));
  }
  return out;
}

void SdaClient::participate_many(const std::vector<std::vector<int64_t>>& inputs, const AggregationId& agg) {
  for (auto& p : new_participations(inputs, agg)) upload_participation(p);
}

void SdaClient::participate(const std::vector<int64_t>& input, const AggregationId& agg) {
  upload_participation(new_participation(input, agg));
}

namespace {
double ms_since(std::chrono::steady_clock::time_point& t0) {
  auto t1 = std::chrono::steady_clock::now();
  double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  t0 = t1;
  return ms;
}
}  // namespace

bool SdaClient::clerk_once() {
  auto t = std::chrono::steady_clock::now();
  // the job as JSON text: its boxes are decoded from where they sit in the text
  auto text = service_->get_clerking_job_json(agent_, agent_.id);
  if (!text) return false;
  role_timings_.clear();
  ClerkingResult r;
  if (auto view = wire::scan_clerking_job(*text)) {
    role_timings_["fetch"] = ms_since(t);
    std::vector<BoxSource> boxes;
    boxes.reserve(view->boxes.size());
    for (auto& sp : view->boxes) boxes.push_back(box_source_base64(text->data() + sp.off, sp.len));
    r = process_clerking_boxes(view->head, boxes);
  } else {
    ClerkingJob job = wire::decode<ClerkingJob>(*text);
    role_timings_["fetch"] = ms_since(t);
    r = process_clerking_job(job);
  }
  role_timings_["process"] = ms_since(t);
  service_->create_clerking_result(agent_, r);
  role_timings_["post"] = ms_since(t);
  return true;
}

void SdaClient::run_chores(long max_iterations) {
  if (max_iterations < 0) {
    while (clerk_once()) {
    }
  } else {
    for (long i = 0; i < max_iterations; ++i)
      if (!clerk_once()) break;
  }
}

ClerkingResult SdaClient::process_clerking_job(const ClerkingJob& job) {
  std::vector<BoxSource> boxes;
  boxes.reserve(job.encryptions.size());
  for (auto& e : job.encryptions) boxes.push_back(box_source(e));
  return process_clerking_boxes(job, boxes);
}

namespace {
// A box materialised from its source (the host engines take owned bytes).
Encryption materialise(const BoxSource& src) {
  Encryption e;
  e.sodium.resize(src.max_len);
  size_t n = src.fill(e.sodium.data(), e.sodium.size());
  if (n > e.sodium.size()) throw SdaError("Sodium decryption failure: box longer than announced");
  e.sodium.resize(n);
  return e;
}
}  // namespace

ClerkingResult SdaClient::process_clerking_boxes(const ClerkingJob& job, const std::vector<BoxSource>& boxes) {
  auto agg = service_->get_aggregation(agent_, job.aggregation);
  if (!agg) throw SdaError("Unknown aggregation");
  auto committee = service_->get_committee(agent_, job.aggregation);
  if (!committee) throw SdaError("Unknown committee");
  std::optional<EncryptionKeyId> own;
  for (auto& ck : committee->clerks_and_keys)
    if (ck.first == agent_.id) { own = ck.second; break; }
  if (!own) throw SdaError("Could not find own encryption key in keyset");
  auto kp = keystore_->get<EncryptionKeypair>(own->str());
  if (!kp) throw SdaError("Could not load keypair for decryption");
  if (device_) {
    std::string why = device_unsupported(*agg);
    if (why.empty()) {
      const auto& sh = agg->committee_sharing_scheme;
      const size_t values = (agg->vector_dimension + sh.input_size() - 1) / sh.input_size();
      EncryptionKey ek = verified_key(agg->recipient, agg->recipient_key, "recipient");
      return ClerkingResult{job.id, job.clerk, device_->clerk_combine(sh, values, *kp, boxes, ek)};
    }
    log_warn("clerk: host engines (" + why + ")");
  }
  // clerk.rs:79-86: open every box and fold it into a running sum. The boxes are
  // independent, so a few threads each fold a share of them (the reference's
  // `(a + b) % m` per element; partial sums are folded the same way).
  const int64_t m = agg->committee_sharing_scheme.modulus;
  const size_t nthreads = std::max<size_t>(1, std::min<size_t>({boxes.size() / 4, (size_t)8,
                                          (size_t)std::max(1u, std::thread::hardware_concurrency())}));
  std::vector<std::vector<int64_t>> partial(nthreads);
  std::vector<std::string> failure(nthreads);
  auto fold = [&](size_t tid) {
    try {
      std::vector<int64_t>& acc = partial[tid];
      bool first = true;
      for (size_t j = tid; j < boxes.size(); j += nthreads) {
        std::vector<int64_t> part = decrypt_shares(*kp, materialise(boxes[j]));
        if (first) {
          acc.assign(part.size(), 0);
          first = false;
        }
        if (part.size() != acc.size()) throw SdaError("Wrong dimension");
        for (size_t i = 0; i < part.size(); ++i) acc[i] = (acc[i] + part[i]) % m;
      }
    } catch (const std::exception& e) {
      failure[tid] = e.what();
      if (failure[tid].empty()) failure[tid] = "clerking failed";
    }
  };
  std::vector<std::thread> workers;
  for (size_t tid = 1; tid < nthreads; ++tid) workers.emplace_back(fold, tid);
  fold(0);
  for (auto& w : workers) w.join();
  for (auto& f : failure)
    if (!f.empty()) throw SdaError(f);
  std::vector<int64_t> combined = boxes.empty() ? std::vector<int64_t>{} : partial[0];
  for (size_t tid = 1; tid < nthreads; ++tid) {
    if (partial[tid].size() != combined.size()) throw SdaError("Wrong dimension");
    for (size_t i = 0; i < combined.size(); ++i) combined[i] = (combined[i] + partial[tid][i]) % m;
  }
  EncryptionKey ek = verified_key(agg->recipient, agg->recipient_key, "recipient");
  return ClerkingResult{job.id, job.clerk, encrypt_shares(ek, combined)};
}

void SdaClient::upload_aggregation(const Aggregation& a) { service_->create_aggregation(agent_, a); }

void SdaClient::begin_aggregation(const AggregationId& id) {
  auto agg = service_->get_aggregation(agent_, id);
  if (!agg) throw SdaError("Unknown aggregation, " + id.str());
  auto candidates = service_->suggest_committee(agent_, id);
  Committee c;
  c.aggregation = id;
  for (auto& cand : candidates) {
    if (c.clerks_and_keys.size() >= agg->committee_sharing_scheme.output_size()) break;
    if (cand.keys.empty()) continue;
    c.clerks_and_keys.emplace_back(cand.id, cand.keys[0]);
  }
  service_->create_committee(agent_, c);
}

void SdaClient::end_aggregation(const AggregationId& id) {
  auto status = service_->get_aggregation_status(agent_, id);
  if (!status) throw SdaError("Unknown aggregation");
  if (!status->snapshots.empty()) return;  // idempotent (receive.rs:68-70)
  service_->create_snapshot(agent_, Snapshot{SnapshotId::random(), id});
}

RecipientOutput SdaClient::reveal_aggregation(const AggregationId& id) {
  auto t = std::chrono::steady_clock::now();
  struct Stamp {  // "process" = everything after the fetch, however the function returns
    SdaClient& c;
    std::chrono::steady_clock::time_point& t;
    ~Stamp() { c.role_timings_["process"] = ms_since(t); }
  } stamp{*this, t};
  role_timings_.clear();
  auto agg = service_->get_aggregation(agent_, id);
  if (!agg) throw SdaError("Unknown aggregation, " + id.str());
  auto committee = service_->get_committee(agent_, id);
  if (!committee) throw SdaError("Unknown committee, " + id.str());
  auto status = service_->get_aggregation_status(agent_, id);
  if (!status) throw SdaError("Unknown aggregation");
  const SnapshotStatus* snap = nullptr;
  for (auto& s : status->snapshots)
    if (s.result_ready) { snap = &s; break; }
  if (!snap) throw SdaError("Aggregation not ready");
  // the result as JSON text: the boxes are decoded from where they sit in it
  auto text = service_->get_snapshot_result_json(agent_, id, snap->id);
  if (!text) throw SdaError("Missing aggregation result");
  std::vector<std::pair<AgentId, BoxSource>> by_clerk;
  std::vector<BoxSource> masks;
  bool has_masks = false;
  std::optional<SnapshotResult> owned;  // backs the sources when the text is not in the plain shape
  if (auto view = wire::scan_snapshot_result(*text)) {
    for (auto& r : view->results)
      by_clerk.emplace_back(r.clerk, box_source_base64(text->data() + r.box.off, r.box.len));
    has_masks = view->has_masks;
    for (auto& sp : view->masks) masks.push_back(box_source_base64(text->data() + sp.off, sp.len));
  } else {
    owned = wire::decode<SnapshotResult>(*text);
    for (auto& cr_ : owned->clerk_encryptions) by_clerk.emplace_back(cr_.clerk, box_source(cr_.encryption));
    has_masks = owned->recipient_encryptions.has_value();
    if (has_masks)
      for (auto& e : *owned->recipient_encryptions) masks.push_back(box_source(e));
  }
  role_timings_["fetch"] = ms_since(t);
  auto kp = keystore_->get<EncryptionKeypair>(agg->recipient_key.str());
  if (!kp) throw SdaError("Could not load keypair for decryption");
  // receive.rs:127-138: each result's clerk -> its committee index
  std::vector<std::pair<size_t, BoxSource>> results;
  for (auto& cb : by_clerk) {
    size_t idx = committee->clerks_and_keys.size();
    for (size_t i = 0; i < committee->clerks_and_keys.size(); ++i)
      if (committee->clerks_and_keys[i].first == cb.first) { idx = i; break; }
    if (idx == committee->clerks_and_keys.size()) throw SdaError("Missing clerk, " + cb.first.str());
    results.emplace_back(idx, cb.second);
  }
  if (device_) {
    std::string why = device_unsupported(*agg);
    if (why.empty()) return RecipientOutput{agg->modulus, device_->reveal(*agg, *kp, results, masks)};
    log_warn("reveal: host engines (" + why + ")");
  }
  std::vector<int64_t> mask;
  if (has_masks) {
    std::vector<std::vector<int64_t>> opened;
    for (auto& src : masks) opened.push_back(decrypt_shares(*kp, materialise(src)));
    mask = combine_masks(agg->masking_scheme, opened);
  }
  std::vector<std::pair<size_t, std::vector<int64_t>>> indexed;
  for (auto& r : results) indexed.emplace_back(r.first, decrypt_shares(*kp, materialise(r.second)));
  auto masked = reconstruct_secrets(agg->committee_sharing_scheme, agg->vector_dimension, indexed);
  return RecipientOutput{agg->modulus, unmask(agg->masking_scheme, mask, masked)};
}

}  // namespace sda
