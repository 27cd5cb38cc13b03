// Packed Shamir secret sharing as share / Lagrange matrices (see field.hpp).
#include <algorithm>
#include <set>

#include "sda/field.hpp"

namespace sda {

uint64_t mod_pow(uint64_t b, uint64_t e, uint64_t p) {
  unsigned __int128 r = 1, x = b % p;
  while (e) {
    if (e & 1) r = (r * x) % p;
    x = (x * x) % p;
    e >>= 1;
  }
  return (uint64_t)r;
}

uint64_t mod_inv(uint64_t a, uint64_t p) {
  if (a % p == 0) throw SdaError::invalid("mod_inv of zero");
  return mod_pow(a, p - 2, p);
}

uint64_t mult_order(uint64_t w, uint64_t p, uint64_t limit) {
  uint64_t x = w % p;
  for (uint64_t k = 1; k <= limit; ++k) {
    if (x == 1) return k;
    x = (uint64_t)((unsigned __int128)x * w % p);
  }
  return 0;
}

namespace {

inline uint64_t mul(uint64_t a, uint64_t b, uint64_t p) { return (uint64_t)((unsigned __int128)a * b % p); }
inline uint64_t sub(uint64_t a, uint64_t b, uint64_t p) { return a >= b ? a - b : a + p - b; }

// v[i] <- 1 / v[i] for non-zero v[i] (one field inversion: Montgomery's trick).
void batch_invert(std::vector<uint64_t>& v, uint64_t p) {
  std::vector<uint64_t> pre(v.size() + 1, 1);
  for (size_t i = 0; i < v.size(); ++i) pre[i + 1] = mul(pre[i], v[i], p);
  uint64_t inv = mod_inv(pre[v.size()], p);
  for (size_t i = v.size(); i-- > 0;) {
    const uint64_t vi = v[i];
    v[i] = mul(inv, pre[i], p);
    inv = mul(inv, vi, p);
  }
}

// Lagrange interpolation in barycentric form: l_j(x) = l(x) w_j / (x - x_j) with
// l(x) = prod_i (x - x_i) and w_j = 1 / prod_{i != j} (x_j - x_i). The weights cost
// O(N^2) multiplications once -- or O(N) when the nodes are all the N-th roots of
// unity, where prod_{i != j} (x_j - x_i) = N x_j^(N-1) = N / x_j (the full share
// point set {1, w_n, .., w_n^n} and the secret point set of the tss parameter sets)
// -- and a row of basis values O(N). (Evaluating every l_j(x) by its own product,
// as before, was O(N^2) per point: minutes for the 19,682-share set.)
class Barycentric {
 public:
  Barycentric(std::vector<uint64_t> nodes, uint64_t p) : x_(std::move(nodes)), p_(p), w_(x_.size()) {
    const size_t N = x_.size();
    bool roots = N >= 2;
    if (roots) {  // every node an N-th root of unity (they are distinct: validate())
      for (size_t i = 0; i < N && roots; ++i) roots = mod_pow(x_[i], N, p) == 1;
    }
    if (roots) {
      const uint64_t invN = mod_inv(N % p, p);
      for (size_t j = 0; j < N; ++j) w_[j] = mul(x_[j], invN, p);
    } else {
      for (size_t j = 0; j < N; ++j) {
        uint64_t d = 1;
        for (size_t i = 0; i < N; ++i)
          if (i != j) d = mul(d, sub(x_[j], x_[i], p), p);
        w_[j] = d;
      }
      batch_invert(w_, p);
    }
  }
  // out[j] = l_j(x) for every node j; x must not be a node.
  void row(uint64_t x, std::vector<uint64_t>& out) const {
    const size_t N = x_.size();
    out.resize(N);
    uint64_t l = 1;
    for (size_t j = 0; j < N; ++j) {
      out[j] = sub(x, x_[j], p_);
      if (out[j] == 0) throw SdaError::invalid("packed shamir: evaluation point is a node");
      l = mul(l, out[j], p_);
    }
    batch_invert(out, p_);
    for (size_t j = 0; j < N; ++j) out[j] = mul(mul(l, w_[j], p_), out[j], p_);
  }

 private:
  std::vector<uint64_t> x_;
  uint64_t p_;
  std::vector<uint64_t> w_;
};

}  // namespace

void PackedShamirParams::validate() const {
  if (secret_count < 1 || share_count < 1 || privacy_threshold < 0)
    throw SdaError::invalid("packed shamir: counts must be positive");
  if (prime < 3 || prime >= (1LL << 31))
    throw SdaError::invalid("packed shamir: prime must be in [3, 2^31)");
  if (reconstruct_limit() > share_count)
    throw SdaError::invalid("packed shamir: t + k must not exceed the share count");
  const uint64_t p = (uint64_t)prime;
  std::set<uint64_t> sec, sh;
  for (int j = 0; j <= reconstruct_limit(); ++j) sec.insert(mod_pow(omega_secrets, j, p));
  if ((int)sec.size() != reconstruct_limit() + 1)
    throw SdaError::invalid("packed shamir: omega_secrets powers are not distinct");
  for (int i = 0; i <= share_count; ++i) sh.insert(mod_pow(omega_shares, i, p));
  if ((int)sh.size() != share_count + 1)
    throw SdaError::invalid("packed shamir: omega_shares powers are not distinct");
  for (int i = 1; i <= share_count; ++i) {
    uint64_t x = mod_pow(omega_shares, i, p);
    for (int j = 0; j <= secret_count; ++j)
      if (x == mod_pow(omega_secrets, j, p))
        throw SdaError::invalid("packed shamir: a share point coincides with a secret point");
  }
}

std::vector<uint32_t> PackedShamirParams::share_matrix() const {
  validate();
  const uint64_t p = (uint64_t)prime;
  const int K = reconstruct_limit();
  std::vector<uint64_t> nodes(K + 1);
  for (int j = 0; j <= K; ++j) nodes[j] = mod_pow(omega_secrets, j, p);
  std::vector<uint32_t> M((size_t)share_count * K);
  const Barycentric basis(nodes, p);
  std::vector<uint64_t> row;
  for (int c = 0; c < share_count; ++c) {
    basis.row(mod_pow(omega_shares, c + 1, p), row);
    for (int j = 1; j <= K; ++j) M[(size_t)c * K + (j - 1)] = (uint32_t)row[j];
  }
  return M;
}

std::vector<uint32_t> PackedShamirParams::lagrange_matrix(const std::vector<int>& indices) const {
  validate();
  const uint64_t p = (uint64_t)prime;
  if ((int)indices.size() < reconstruct_limit())
    throw SdaError::invalid("Not enough shares to reconstruct");
  std::set<int> uniq(indices.begin(), indices.end());
  if (uniq.size() != indices.size()) throw SdaError::invalid("duplicate share indices");
  std::vector<uint64_t> nodes;
  nodes.push_back(1);
  for (int i : indices) {
    if (i < 0 || i >= share_count) throw SdaError::invalid("share index out of range");
    nodes.push_back(mod_pow(omega_shares, i + 1, p));
  }
  std::vector<uint32_t> L((size_t)secret_count * indices.size());
  const Barycentric basis(nodes, p);
  std::vector<uint64_t> row;
  for (int s = 0; s < secret_count; ++s) {
    basis.row(mod_pow(omega_secrets, s + 1, p), row);
    for (size_t i = 0; i < indices.size(); ++i) L[(size_t)s * indices.size() + i] = (uint32_t)row[i + 1];
  }
  return L;
}

std::vector<int64_t> PackedShamirParams::share(const std::vector<int64_t>& secrets,
                                               const std::vector<int64_t>& randomness) const {
  if ((int)secrets.size() != secret_count || (int)randomness.size() != privacy_threshold)
    throw SdaError::invalid("packed shamir share: wrong input sizes");
  const uint64_t p = (uint64_t)prime;
  const int K = reconstruct_limit();
  auto M = share_matrix();
  std::vector<uint64_t> v(K);
  for (int j = 0; j < secret_count; ++j) v[j] = canon(secrets[j], prime);
  for (int d = 0; d < privacy_threshold; ++d) v[secret_count + d] = canon(randomness[d], prime);
  std::vector<int64_t> out(share_count);
  for (int c = 0; c < share_count; ++c) {
    unsigned __int128 acc = 0;
    for (int j = 0; j < K; ++j) acc += (unsigned __int128)M[(size_t)c * K + j] * v[j];
    out[c] = (int64_t)(uint64_t)(acc % p);
  }
  return out;
}

std::vector<int64_t> PackedShamirParams::reconstruct(const std::vector<int>& indices,
                                                     const std::vector<int64_t>& shares) const {
  if (indices.size() != shares.size()) throw SdaError::invalid("Inputs must have same length");
  const uint64_t p = (uint64_t)prime;
  auto L = lagrange_matrix(indices);
  std::vector<int64_t> out(secret_count);
  for (int s = 0; s < secret_count; ++s) {
    unsigned __int128 acc = 0;
    for (size_t i = 0; i < indices.size(); ++i)
      acc += (unsigned __int128)L[(size_t)s * indices.size() + i] * canon(shares[i], prime);
    out[s] = (int64_t)(uint64_t)(acc % p);
  }
  return out;
}

PackedShamirParams pss_4_8_3() { return {3, 8, 4, 433, 354, 150}; }
PackedShamirParams pss_4_26_3() { return {3, 26, 4, 433, 354, 17}; }
PackedShamirParams pss_155_728_100() { return {100, 728, 155, 746497, 95660, 610121}; }
PackedShamirParams pss_155_19682_100() { return {100, 19682, 155, 5038849, 4318906, 1814687}; }

}  // namespace sda
