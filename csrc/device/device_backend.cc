// The client roles' bulk cryptography on an MI355X (see sda/device_backend.hpp).
//
// Wire-format sealed boxes are staged into a pinned host arena of fixed-stride
// slots (base64 text is decoded straight into its slot by a few host threads),
// cross PCIe in one copy, and are then processed by the same gfx950 kernels the
// simulation engine uses (csrc/kernels): X25519 key agreement, matrix-core
// Poly1305 verify fused with XSalsa20 decryption, varint decode fused with the
// modular sum, the share kernels, varint encode fused with encryption.
//
// Reference roles: client/src/clerk.rs:63-107, client/src/receive.rs:80-157,
// client/src/participate.rs:37-113.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "../kernels/kernels.hpp"
#include "sda/crypto.hpp"
#include "sda/device_backend.hpp"
#include "sda/field.hpp"

namespace sda {
namespace {

using namespace sdagpu;
using Clock = std::chrono::steady_clock;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw SdaError(std::string("GPU backend: ") + what + ": " + hipGetErrorString(e));
}
#define HIP_OK(x) hip_ok((x), #x)

void launched(const char* what) { hip_ok(hipGetLastError(), what); }

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- shapes (the same rules as the engine's arena: sda_amd/ops/sealed.py) ------
constexpr size_t kSealOverhead = 48;

int varint_max_len(uint64_t modulus) {
  if (modulus == 0) return 5;  // any u32
  uint64_t z = 2 * (modulus - 1);
  int n = 1;
  while (z >= 128) {
    z >>= 7;
    ++n;
  }
  return n;
}
size_t slot_stride(size_t L, uint64_t modulus) {
  return round_up(kSealOverhead + round_up(L * varint_max_len(modulus), 16), 64);
}
int chunks_for(size_t max_pt) { return (int)((max_pt + 32 + kChunkBytes - 1) / kChunkBytes); }
int tiles(size_t L) { return (int)((L + kTileValues - 1) / kTileValues); }
int sum_tiles(size_t L) { return (int)((L + kSumTile - 1) / kSumTile); }

// most participants one decode-sum accumulator may add up (64-bit accumulators above 2^27)
uint64_t decode_sum_group_limit(uint64_t m) {
  if (m > (1ull << 27)) return 1ull << 30;
  const uint64_t per = m <= 8192 ? 16383 : 2 * (m - 1) < (1ull << 21) ? (1ull << 21) - 1 : (1ull << 28) - 1;
  return std::max<uint64_t>(1, 0xffffffffull / per);
}
int decode_group_size(int P, int tiles_x_rows, uint64_t limit) {
  auto cdiv = [](int a, int b) { return (a + b - 1) / b; };
  int groups = std::max(cdiv(4096, tiles_x_rows), std::min(cdiv(10000, tiles_x_rows), P / 40));
  groups = std::max(1, std::min(P, groups));
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cdiv(P, groups), limit));
}

// ---- device / pinned memory with reuse across calls --------------------------------
class Pool {
 public:
  ~Pool() { release(); }
  void* get(size_t bytes) {
    size_t cls = size_class(bytes);
    auto it = free_.find(cls);
    if (it != free_.end()) {
      void* p = it->second;
      free_.erase(it);
      return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess) {  // give the cached blocks back and try once more
      (void)hipGetLastError();
      release();
      HIP_OK(hipMalloc(&p, cls));
    }
    sizes_[p] = cls;
    return p;
  }
  void put(void* p) {
    if (p) free_.emplace(sizes_[p], p);
  }
  void release() {
    for (auto& kv : free_) {
      (void)hipFree(kv.second);
      sizes_.erase(kv.second);
    }
    free_.clear();
  }

 private:
  static size_t size_class(size_t b) {
    if (b <= 4096) return 4096;
    if (b >= (64u << 20)) return round_up(b, 64u << 20);
    size_t c = 4096;
    while (c < b) c <<= 1;
    return c;
  }
  std::multimap<size_t, void*> free_;
  std::map<void*, size_t> sizes_;
};

// Buffers of one call: returned to the pool when the call ends.
class Lease {
 public:
  explicit Lease(Pool& pool) : pool_(pool) {}
  ~Lease() {
    for (void* p : held_) pool_.put(p);
  }
  template <class T>
  T* take(size_t count) {
    void* p = pool_.get(std::max<size_t>(1, count) * sizeof(T));
    held_.push_back(p);
    return static_cast<T*>(p);
  }

 private:
  Pool& pool_;
  std::vector<void*> held_;
};

class Pinned {
 public:
  ~Pinned() {
    if (p_) (void)hipHostFree(p_);
  }
  uint8_t* get(size_t bytes) {
    if (bytes > cap_) {
      if (p_) (void)hipHostFree(p_);
      p_ = nullptr;
      cap_ = 0;
      size_t want = round_up(bytes + bytes / 4, 1u << 20);
      HIP_OK(hipHostMalloc(&p_, want, hipHostMallocDefault));
      cap_ = want;
    }
    return static_cast<uint8_t*>(p_);
  }

 private:
  void* p_ = nullptr;
  size_t cap_ = 0;
};

struct Arena {
  int M = 0;
  size_t L = 0;
  uint32_t modulus = 0;
  size_t stride = 0;
  int K = 0;
  uint8_t* ct = nullptr;       // device [M][stride]
  uint32_t* pt_len = nullptr;  // device [M]
};

struct Keys {
  MsgKey* keys = nullptr;
  uint32_t* pows = nullptr;
};

void words_of(const uint8_t in[32], uint32_t out[8]) { std::memcpy(out, in, 32); }

RngKeyArg fresh_rng_key() {
  RngKeyArg k;
  crypto::os_random(reinterpret_cast<uint8_t*>(k.k), sizeof(k.k));
  return k;
}

std::string describe_error(uint32_t e) {
  std::string s;
  auto add = [&](const char* t) { s += (s.empty() ? "" : ", ") + std::string(t); };
  if (e & kErrBadKey) add("bad public key");
  if (e & kErrMac) add("MAC verification failed");
  if (e & kErrMalformed) add("malformed varint stream");
  if (e & kErrChaChaReject) add("ChaCha mask rejection");
  if (e & kErrRange) add("value out of range");
  return s;
}

class Backend final : public DeviceBackend {
 public:
  explicit Backend(int device) : device_(device) {
    HIP_OK(hipSetDevice(device_));
    hipDeviceProp_t p;
    HIP_OK(hipGetDeviceProperties(&p, device_));
    name_ = std::string(p.name) + " (" + p.gcnArchName + ")";
    if (std::string(p.gcnArchName).rfind("gfx950", 0) != 0)
      throw SdaError("GPU backend: the kernels are built for gfx950, this device is " +
                     std::string(p.gcnArchName));
    HIP_OK(hipStreamCreate(&s_));
  }
  ~Backend() override {
    (void)hipSetDevice(device_);
    (void)hipStreamSynchronize(s_);
    pool_.release();
    (void)hipStreamDestroy(s_);
  }

  std::string describe() const override { return "HIP device " + std::to_string(device_) + ": " + name_; }
  std::map<std::string, double> last_timings() const override {
    std::lock_guard<std::mutex> g(mu_);
    return timings_;
  }

  Encryption clerk_combine(const LinearSecretSharingScheme& sharing, size_t values,
                           const EncryptionKeypair& own, const std::vector<BoxSource>& boxes,
                           const EncryptionKey& recipient) override;
  std::vector<int64_t> reveal(const Aggregation& agg, const EncryptionKeypair& own,
                              const std::vector<std::pair<size_t, BoxSource>>& results,
                              const std::vector<BoxSource>& masks) override;
  DeviceParticipations participate_many(const Aggregation& agg,
                                        const std::vector<EncryptionKey>& clerk_keys,
                                        const EncryptionKey* recipient_key,
                                        const std::vector<std::vector<int64_t>>& inputs) override;

 private:
  // ---- timing ----
  struct Timer {
    Backend& b;
    Clock::time_point t0 = Clock::now();
    explicit Timer(Backend& bk) : b(bk) { b.timings_.clear(); }
    void mark(const char* stage) {
      auto t1 = Clock::now();
      b.timings_[stage] += std::chrono::duration<double, std::milli>(t1 - t0).count();
      t0 = t1;
    }
  };
  void sync() { HIP_OK(hipStreamSynchronize(s_)); }

  static uint32_t field_modulus(int64_t m) {
    if (m < 2 || m >= (int64_t)1 << 31)
      throw SdaError("GPU backend: modulus must be in [2, 2^31)");
    return (uint32_t)m;
  }

  // ---- staging ----
  Arena upload(Lease& mem, const std::vector<const BoxSource*>& boxes, size_t L, uint32_t modulus);
  std::vector<Encryption> download(const Arena& a);

  // ---- kernel sequences (the order and shapes of sda_amd/ops/sealed.py) ----
  Keys open_setup(Lease& mem, const Arena& a, const uint32_t* key_idx, const uint32_t* sks,
                  const uint32_t* pks, uint32_t* err);
  Keys seal_setup(Lease& mem, const Arena& a, const uint32_t* key_idx, const uint32_t* pks,
                  uint64_t owner_base, const RngKeyArg& rng, uint32_t* err);
  void tables(Lease& mem, const Arena& a, Keys& k);
  void verify_decrypt(Lease& mem, const Arena& a, const Keys& k, uint32_t* term, uint32_t* pre,
                      uint32_t* err);
  void open_sum(Lease& mem, const Arena& a, const Keys& k, int rows, uint32_t* out, uint32_t* err);
  void open_data(Lease& mem, const Arena& a, const Keys& k, uint32_t* out, uint32_t* err);
  void seal_data(Lease& mem, const Arena& a, const Keys& k, const void* values, int value_bytes,
                 uint32_t* cnt, uint32_t* err);
  Arena new_arena(Lease& mem, int M, size_t L, uint32_t modulus);
  void check(uint32_t* err_dev, const char* what);

  template <class T>
  T* to_device(Lease& mem, const std::vector<T>& host) {
    T* d = mem.take<T>(host.size());
    if (!host.empty())
      HIP_OK(hipMemcpyAsync(d, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice, s_));
    return d;
  }
  uint32_t* zeros(Lease& mem, size_t count) {
    uint32_t* d = mem.take<uint32_t>(count);
    HIP_OK(hipMemsetAsync(d, 0, std::max<size_t>(1, count) * sizeof(uint32_t), s_));
    return d;
  }
  uint32_t* key_words(Lease& mem, const std::vector<const uint8_t*>& keys32) {
    std::vector<uint32_t> w(8 * keys32.size());
    for (size_t i = 0; i < keys32.size(); ++i) words_of(keys32[i], &w[8 * i]);
    uint32_t* d = to_device(mem, w);
    sync();  // `w` is pageable host memory going out of scope
    return d;
  }

  int device_;
  std::string name_;
  hipStream_t s_ = nullptr;
  Pool pool_;
  Pinned pinned_in_, pinned_out_;
  mutable std::mutex mu_;     // one role call at a time per backend
  std::map<std::string, double> timings_;
};

// -------------------------------------------------------------------- staging ----
Arena Backend::upload(Lease& mem, const std::vector<const BoxSource*>& boxes, size_t L,
                      uint32_t modulus) {
  const int M = (int)boxes.size();
  size_t max_len = kSealOverhead;
  for (auto* b : boxes) max_len = std::max(max_len, b->max_len);
  Arena a;
  a.M = M;
  a.L = L;
  a.modulus = modulus;
  a.stride = std::max(slot_stride(L, modulus),
                      round_up(kSealOverhead + round_up(max_len - kSealOverhead, 16), 64));
  a.K = chunks_for(std::max(max_len - kSealOverhead, L * (size_t)varint_max_len(modulus)));
  uint8_t* host = pinned_in_.get((size_t)M * a.stride + (size_t)M * sizeof(uint32_t));
  uint32_t* lens = reinterpret_cast<uint32_t*>(host + (size_t)M * a.stride);
  // decode / copy the boxes into their slots on a few threads
  std::atomic<int> next{0};
  std::atomic<int> bad{-1};
  auto work = [&]() {
    for (;;) {
      int j = next.fetch_add(1);
      if (j >= M) return;
      uint8_t* slot = host + (size_t)j * a.stride;
      size_t n = 0;
      try {
        n = boxes[j]->fill(slot, a.stride);
      } catch (const std::exception&) {
        bad.store(j);
        n = 0;
      }
      if (n < kSealOverhead || n > a.stride) {
        bad.store(j);
        n = kSealOverhead;
      }
      lens[j] = (uint32_t)(n - kSealOverhead);
      // the kernels read whole 64-byte lines of a slot: no stale bytes behind the box
      size_t end = std::min(a.stride, round_up(n, 64) + 64);
      std::memset(slot + n, 0, end - n);
    }
  };
  unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 8u);
  nt = std::min<unsigned>(nt, std::max(1, M / 4));
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (bad.load() >= 0)
    throw SdaError("Sodium decryption failure: box " + std::to_string(bad.load()) +
                   " is not a sealed box");
  a.ct = mem.take<uint8_t>((size_t)M * a.stride);
  a.pt_len = mem.take<uint32_t>(M);
  HIP_OK(hipMemcpyAsync(a.ct, host, (size_t)M * a.stride, hipMemcpyHostToDevice, s_));
  HIP_OK(hipMemcpyAsync(a.pt_len, lens, (size_t)M * sizeof(uint32_t), hipMemcpyHostToDevice, s_));
  sync();  // the pinned arena is reused (or regrown) by the next upload of this call
  return a;
}

std::vector<Encryption> Backend::download(const Arena& a) {
  const size_t bytes = (size_t)a.M * a.stride;
  uint8_t* host = pinned_out_.get(bytes + (size_t)a.M * sizeof(uint32_t));
  uint32_t* lens = reinterpret_cast<uint32_t*>(host + bytes);
  HIP_OK(hipMemcpyAsync(host, a.ct, bytes, hipMemcpyDeviceToHost, s_));
  HIP_OK(hipMemcpyAsync(lens, a.pt_len, (size_t)a.M * sizeof(uint32_t), hipMemcpyDeviceToHost, s_));
  sync();
  std::vector<Encryption> out(a.M);
  for (int j = 0; j < a.M; ++j) {
    size_t n = kSealOverhead + lens[j];
    if (n > a.stride) throw SdaError("GPU backend: sealed box longer than its slot");
    const uint8_t* slot = host + (size_t)j * a.stride;
    out[j].sodium.assign(slot, slot + n);
  }
  return out;
}

Arena Backend::new_arena(Lease& mem, int M, size_t L, uint32_t modulus) {
  Arena a;
  a.M = M;
  a.L = L;
  a.modulus = modulus;
  a.stride = slot_stride(L, modulus);
  a.K = chunks_for(L * (size_t)varint_max_len(modulus));
  a.ct = mem.take<uint8_t>((size_t)M * a.stride);
  a.pt_len = zeros(mem, M);
  return a;
}

void Backend::check(uint32_t* err_dev, const char* what) {
  uint32_t e = 0;
  HIP_OK(hipMemcpyAsync(&e, err_dev, sizeof(e), hipMemcpyDeviceToHost, s_));
  sync();
  if (e & (kErrMac | kErrBadKey)) throw SdaError(std::string("Sodium decryption failure (") + what + ": " + describe_error(e) + ")");
  if (e) throw SdaError(std::string("GPU backend: ") + what + ": " + describe_error(e));
}

// ------------------------------------------------------------ kernel sequences ----
// Poly1305 tables of a key set: the one-pass form (r^1 .. r^64) for boxes of at most
// kShortMaxChunks chunks, the chunked MAC's 26 KB per box otherwise.
static bool short_boxes(const Arena& a) { return a.K <= kShortMaxChunks; }

void Backend::tables(Lease& mem, const Arena& a, Keys& k) {
  if (short_boxes(a)) {
    k.pows = mem.take<uint32_t>((size_t)a.M * kPowShortWords);
    launch_poly_powers_short(a.M, k.keys, k.pows, s_);
    launched("poly_powers_short");
  } else {
    k.pows = mem.take<uint32_t>((size_t)a.M * kPowWords);
    launch_poly_powers(a.M, k.keys, k.pows, 1, s_);
    launched("poly_powers");
  }
}

// Tag check, then in-place decryption with terminator counts (per chunk / sub-chunk).
void Backend::verify_decrypt(Lease& mem, const Arena& a, const Keys& k, uint32_t* term,
                             uint32_t* pre, uint32_t* err) {
  const int M = a.M, K = a.K;
  if (short_boxes(a)) {
    launch_mac_short(M, k.keys, k.pows, a.ct, a.stride, a.pt_len, 1, nullptr, err, s_);
    launched("mac_short");
    launch_decrypt_count(M, K, k.keys, a.ct, a.stride, a.pt_len, term, pre, s_);
    launched("decrypt_count");
    return;
  }
  uint32_t* partials = mem.take<uint32_t>((size_t)M * K * 8);
  launch_mac_chunks(M, K, k.keys, k.pows, a.ct, a.stride, a.pt_len, partials, 1, term, pre, s_);
  launched("mac_chunks");
  launch_mac_final(M, K, k.keys, k.pows, a.ct, a.stride, a.pt_len, partials, 1, nullptr, err, s_);
  launched("mac_final");
}

Keys Backend::open_setup(Lease& mem, const Arena& a, const uint32_t* key_idx, const uint32_t* sks,
                         const uint32_t* pks, uint32_t* err) {
  Keys k;
  k.keys = mem.take<MsgKey>(a.M);
  launch_open_setup(a.M, key_idx, sks, pks, a.ct, a.stride, k.keys, err, nullptr, 0, s_);
  launched("open_setup");
  tables(mem, a, k);
  return k;
}

Keys Backend::seal_setup(Lease& mem, const Arena& a, const uint32_t* key_idx, const uint32_t* pks,
                         uint64_t owner_base, const RngKeyArg& rng, uint32_t* err) {
  Keys k;
  k.keys = mem.take<MsgKey>(a.M);
  launch_seal_setup(a.M, rng, owner_base, key_idx, pks, a.ct, a.stride, k.keys, err, nullptr, 0, nullptr,
                    s_);
  launched("seal_setup");
  tables(mem, a, k);
  return k;
}

void Backend::open_sum(Lease& mem, const Arena& a, const Keys& k, int rows, uint32_t* out,
                       uint32_t* err) {
  const int M = a.M, K = a.K, P = M / rows;
  const int S = K * kSubPerChunk;
  const int L = (int)a.L;
  uint32_t* pre = mem.take<uint32_t>((size_t)M * S);
  verify_decrypt(mem, a, k, nullptr, pre, err);
  uint32_t* totals = mem.take<uint32_t>(M);
  launch_segscan(M, S, pre, totals, (uint32_t)L, err, s_);  // exactly L values per box
  launched("segscan");
  const int T = sum_tiles(L);
  uint32_t* tile_sub = mem.take<uint32_t>((size_t)M * (T + 1));
  launch_locate_tiles(M, S, L, pre, totals, tile_sub, s_);
  launched("locate_tiles");
  const int Pg = decode_group_size(P, T * rows, decode_sum_group_limit(a.modulus));
  const int G = (P + Pg - 1) / Pg;
  uint32_t* part = mem.take<uint32_t>((size_t)G * rows * L * (decode_sum_wide((uint32_t)a.modulus) ? 2 : 1));
  uint32_t* redo = zeros(mem, 1);
  launch_decode_sum(rows, P, Pg, L, a.modulus, a.ct, a.stride, a.pt_len, S, pre, tile_sub, part, out,
                    nullptr, err, redo, s_);
  launched("decode_sum");
}

void Backend::open_data(Lease& mem, const Arena& a, const Keys& k, uint32_t* out, uint32_t* err) {
  const int M = a.M, K = a.K, L = (int)a.L;
  uint32_t* term = mem.take<uint32_t>((size_t)M * K);
  verify_decrypt(mem, a, k, term, nullptr, err);
  uint32_t* totals = mem.take<uint32_t>(M);
  launch_segscan(M, K, term, totals, (uint32_t)L, err, s_);
  launched("segscan");
  launch_decode(M, K, L, a.modulus, 4, a.ct, a.stride, a.pt_len, term, out, err, s_);
  launched("decode");
}

void Backend::seal_data(Lease& mem, const Arena& a, const Keys& k, const void* values,
                        int value_bytes, uint32_t* cnt, uint32_t* err) {
  const int M = a.M, K = a.K, L = (int)a.L;
  const int T = tiles(L);
  if (!cnt) {
    cnt = mem.take<uint32_t>((size_t)M * T);
    launch_count(M, L, value_bytes, values, cnt, s_);
    launched("count");
  }
  launch_segscan(M, T, cnt, a.pt_len, 0, nullptr, s_);  // tile byte offsets; pt_len = totals
  launched("segscan");
  launch_encode_encrypt(M, L, value_bytes, values, cnt, k.keys, a.ct, a.stride, nullptr, nullptr,
                        nullptr, 0, varint_max_len(a.modulus), s_);
  launched("encode_encrypt");
  if (short_boxes(a)) {
    launch_mac_short(M, k.keys, k.pows, a.ct, a.stride, a.pt_len, 0, nullptr, err, s_);
    launched("mac_short");
    return;
  }
  uint32_t* partials = mem.take<uint32_t>((size_t)M * K * 8);
  launch_mac_chunks(M, K, k.keys, k.pows, a.ct, a.stride, a.pt_len, partials, 0, nullptr, nullptr, s_);
  launched("mac_chunks");
  launch_mac_final(M, K, k.keys, k.pows, a.ct, a.stride, a.pt_len, partials, 0, nullptr, err, s_);
  launched("mac_final");
}

// ---------------------------------------------------------------------- clerk ----
Encryption Backend::clerk_combine(const LinearSecretSharingScheme& sharing, size_t values,
                                  const EncryptionKeypair& own, const std::vector<BoxSource>& boxes,
                                  const EncryptionKey& recipient) {
  std::lock_guard<std::mutex> g(mu_);
  HIP_OK(hipSetDevice(device_));
  const uint32_t m = field_modulus(sharing.modulus);
  if (values == 0 || values > (size_t)1 << 30) throw SdaError("GPU backend: bad share count per box");
  Timer t(*this);
  Lease mem(pool_);
  uint32_t* err = zeros(mem, 1);
  uint32_t* combined = mem.take<uint32_t>(values);
  if (boxes.empty()) {  // combiner.rs:15-29 over no participants: zeros
    HIP_OK(hipMemsetAsync(combined, 0, values * sizeof(uint32_t), s_));
  } else {
    std::vector<const BoxSource*> src;
    for (auto& b : boxes) src.push_back(&b);
    Arena in = upload(mem, src, values, m);
    t.mark("stage+h2d");
    uint32_t* kidx = zeros(mem, in.M);
    uint32_t* sks = key_words(mem, {own.dk.sodium.data()});
    uint32_t* pks = key_words(mem, {own.ek.sodium.data()});
    Keys ko = open_setup(mem, in, kidx, sks, pks, err);
    open_sum(mem, in, ko, 1, combined, err);
    HIP_OK(hipMemsetAsync(sks, 0, 32, s_));  // the secret key does not linger in the pool
  }
  // clerk.rs:99-100: seal the combined shares for the recipient
  Arena res = new_arena(mem, 1, values, m);
  uint32_t* kidx_r = zeros(mem, 1);
  uint32_t* pks_r = key_words(mem, {recipient.sodium.data()});
  Keys ks = seal_setup(mem, res, kidx_r, pks_r, 0, fresh_rng_key(), err);
  seal_data(mem, res, ks, combined, 4, nullptr, err);
  check(err, "clerking job");
  t.mark("gpu");
  Encryption out = download(res)[0];
  t.mark("d2h");
  return out;
}

// ------------------------------------------------------------------ recipient ----
std::vector<int64_t> Backend::reveal(const Aggregation& agg, const EncryptionKeypair& own,
                                     const std::vector<std::pair<size_t, BoxSource>>& results,
                                     const std::vector<BoxSource>& masks) {
  std::lock_guard<std::mutex> g(mu_);
  HIP_OK(hipSetDevice(device_));
  const auto& sh = agg.committee_sharing_scheme;
  const auto& mk = agg.masking_scheme;
  const uint32_t m = field_modulus(sh.modulus);
  if (mk.has_mask() && mk.modulus != sh.modulus)
    throw SdaError("GPU backend: masking and sharing moduli differ");
  const size_t D = agg.vector_dimension;
  const size_t k = sh.input_size();
  const size_t B = (D + k - 1) / k;
  if (D == 0 || D > (size_t)1 << 30) throw SdaError("GPU backend: bad vector dimension");
  if (results.size() < sh.reconstruction_threshold()) throw SdaError("Not enough shares to reconstruct");
  Timer t(*this);
  Lease mem(pool_);
  uint32_t* err = zeros(mem, 1);
  uint32_t* sks = key_words(mem, {own.dk.sodium.data()});
  uint32_t* pks = key_words(mem, {own.ek.sodium.data()});

  // ---- the clerks' results (receive.rs:127-144)
  std::vector<const BoxSource*> src;
  for (auto& r : results) src.push_back(&r.second);
  Arena res = upload(mem, src, B, m);
  t.mark("stage+h2d");
  uint32_t* kidx = zeros(mem, res.M);
  Keys ko = open_setup(mem, res, kidx, sks, pks, err);
  uint32_t* masked = mem.take<uint32_t>(B * k);
  if (sh.kind == LinearSecretSharingScheme::Kind::Additive) {
    open_sum(mem, res, ko, 1, masked, err);  // the reconstruction is the sum of the n results
  } else {
    const int nI = (int)results.size();
    uint32_t* ys = mem.take<uint32_t>((size_t)nI * B);
    open_data(mem, res, ko, ys, err);
    PackedShamirParams p{(int)sh.secret_count, (int)sh.share_count, (int)sh.privacy_threshold_,
                         sh.modulus, sh.omega_secrets, sh.omega_shares};
    p.validate();
    std::vector<int> idx;
    for (auto& r : results) idx.push_back((int)r.first);
    std::vector<uint32_t> lag = p.lagrange_matrix(idx);  // k x nI
    if (lag.size() * sizeof(uint32_t) <= 48 * 1024) {
      uint32_t* dlag = to_device(mem, lag);
      launch_pss_reconstruct((int)B, (int)k, nI, (int)D, m, dlag, ys, masked, s_);
      launched("pss_reconstruct");
      sync();
    } else {
      // large committees: the Lagrange matrix times the results on the int8 matrix cores
      if (m >= (1u << 28)) throw SdaError("GPU backend: packed-Shamir modulus too large for the limb GEMM");
      const int Kp = (nI + 63) / 64 * 64;
      const LimbScheme sch = limb_scheme(m, Kp);
      const int limbs = sch.limbs;
      std::vector<int8_t> A((size_t)limbs * k * Kp, 0);
      for (size_t s = 0; s < k; ++s)
        for (int i = 0; i < nI; ++i) {
          int8_t d[4];
          limbs_of_value(lag[s * nI + i], m, sch, d);
          for (int l = 0; l < limbs; ++l) A[((size_t)l * k + s) * Kp + i] = d[l];
        }
      int8_t* dA = to_device(mem, A);
      int8_t* X = mem.take<int8_t>((size_t)limbs * B * Kp);
      launch_limbs_t(nI, (int)B, Kp, m, ys, X, s_);
      launched("limbs_t");
      launch_modgemm_i8((int)k, (int)B, Kp, 1, limbs, m, dA, nullptr, X, (int64_t)B * Kp, 4, masked, 0, 1,
                        (int64_t)k, (int64_t)D, nullptr, s_);
      launched("modgemm_i8");
      sync();
    }
  }

  // ---- the participants' masks (receive.rs:102-118)
  uint32_t* out = masked;
  if (mk.has_mask()) {
    if (masks.empty()) throw SdaError("Missing mask encryptions");
    std::vector<const BoxSource*> msrc;
    for (auto& b : masks) msrc.push_back(&b);
    uint32_t* mask_sum = mem.take<uint32_t>(D);
    if (mk.kind == LinearMaskingScheme::Kind::Full) {
      Arena ma = upload(mem, msrc, D, m);
      uint32_t* kidx_m = zeros(mem, ma.M);
      Keys km = open_setup(mem, ma, kidx_m, sks, pks, err);
      open_sum(mem, ma, km, 1, mask_sum, err);
    } else {
      if (mk.dimension != D) throw SdaError("ChaCha mask dimension mismatch");
      const int w = (int)((mk.seed_bitsize + 31) / 32);
      if (w < 1 || w > 8) throw SdaError("GPU backend: ChaCha seeds of 1..8 words");
      Arena ma = upload(mem, msrc, (size_t)w, 0);
      uint32_t* kidx_m = zeros(mem, ma.M);
      Keys km = open_setup(mem, ma, kidx_m, sks, pks, err);
      uint32_t* seeds = mem.take<uint32_t>((size_t)ma.M * w);
      open_data(mem, ma, km, seeds, err);
      const int groups = chacha_sum_groups(ma.M, (int)D);
      uint32_t* part = mem.take<uint32_t>((size_t)groups * D);
      uint32_t* scratch = mem.take<uint32_t>(chacha_scratch_words(ma.M, (int)D));
      uint64_t* fix = mem.take<uint64_t>(D);
      launch_chacha_mask_sum(ma.M, (int)D, m, w, seeds, mask_sum, part, groups, scratch, fix, err, s_);
      launched("chacha_mask_sum");
    }
    out = mem.take<uint32_t>(D);
    launch_sub_mod((int)D, m, masked, mask_sum, out, s_);
    launched("sub_mod");
  }
  HIP_OK(hipMemsetAsync(sks, 0, 32, s_));
  check(err, "reveal");
  t.mark("gpu");
  std::vector<uint32_t> host(D);
  HIP_OK(hipMemcpyAsync(host.data(), out, D * sizeof(uint32_t), hipMemcpyDeviceToHost, s_));
  sync();
  std::vector<int64_t> values(host.begin(), host.end());
  t.mark("d2h");
  return values;
}

// ---------------------------------------------------------------- participants ----
DeviceParticipations Backend::participate_many(const Aggregation& agg,
                                               const std::vector<EncryptionKey>& clerk_keys,
                                               const EncryptionKey* recipient_key,
                                               const std::vector<std::vector<int64_t>>& inputs) {
  std::lock_guard<std::mutex> g(mu_);
  HIP_OK(hipSetDevice(device_));
  const auto& sh = agg.committee_sharing_scheme;
  const auto& mk = agg.masking_scheme;
  const uint32_t m = field_modulus(sh.modulus);
  if (mk.has_mask() && mk.modulus != sh.modulus)
    throw SdaError("GPU backend: masking and sharing moduli differ");
  if (mk.has_mask() && !recipient_key) throw SdaError("GPU backend: masked scheme without a recipient key");
  const size_t D = agg.vector_dimension;
  const int n = (int)sh.output_size();
  const size_t k = sh.input_size();
  const size_t B = (D + k - 1) / k;
  const bool pss = sh.kind == LinearSecretSharingScheme::Kind::PackedShamir;
  const int t_priv = (int)sh.privacy_threshold_;
  if ((int)clerk_keys.size() != n) throw SdaError("committee size does not match the sharing scheme");
  if (D == 0 || D > (size_t)1 << 30) throw SdaError("GPU backend: bad vector dimension");
  if (n < 1 || (n > 256 && !pss)) throw SdaError("GPU backend: additive sharing with 1..256 clerks");
  const bool big = pss && (k > 8 || t_priv > 16 || n > 64);
  if (big && m >= (1u << 28)) throw SdaError("GPU backend: packed-Shamir modulus too large for the limb GEMM");
  int mask_mode = kMaskNone, seed_words = 0;
  if (mk.kind == LinearMaskingScheme::Kind::Full) mask_mode = kMaskFull;
  if (mk.kind == LinearMaskingScheme::Kind::ChaCha) {
    mask_mode = kMaskChaCha;
    if (mk.dimension != D) throw SdaError("ChaCha mask dimension mismatch");
    seed_words = (int)((mk.seed_bitsize + 31) / 32);
    if (seed_words < 1 || seed_words > 8) throw SdaError("GPU backend: ChaCha seeds of 1..8 words");
  }
  for (auto& v : inputs)
    if (v.size() != D) throw SdaError("The input length does not match the aggregation.");

  PackedShamirParams pp;
  std::vector<uint32_t> share_matrix;
  if (pss) {
    pp = PackedShamirParams{(int)k, n, t_priv, sh.modulus, sh.omega_secrets, sh.omega_shares};
    pp.validate();
    share_matrix = pp.share_matrix();  // n x (k + t)
  }
  const int value_bytes = (pss && big) ? 4 : (m <= 65536 ? 2 : 4);
  const size_t stride = slot_stride(B, m);

  // participants per wave: arenas, shares and tables within about half of the free memory
  size_t free_b = 0, total_b = 0;
  HIP_OK(hipMemGetInfo(&free_b, &total_b));
  auto table_bytes = [&](size_t L) {
    return (size_t)4 * (chunks_for(L * (size_t)varint_max_len(m)) <= kShortMaxChunks ? kPowShortWords : kPowWords);
  };
  size_t per_p = (size_t)n * (stride + B * value_bytes + table_bytes(B) + 256) + D * 4 * 2 +
                 (mask_mode == kMaskFull ? slot_stride(D, m) + D * 4 + table_bytes(D) : 0) +
                 (big ? (size_t)(m < (1u << 21) ? 3 : 4) * B * ((k + t_priv + 63) / 64 * 64) : 0);
  size_t wave = std::max<size_t>(1, std::min<size_t>(inputs.size(), (free_b / 2) / std::max<size_t>(1, per_p)));

  DeviceParticipations out;
  out.clerk_boxes.resize(inputs.size());
  if (mask_mode != kMaskNone) out.mask_boxes.resize(inputs.size());
  Timer t(*this);
  for (size_t first = 0; first < inputs.size(); first += wave) {
    const int P = (int)std::min(wave, inputs.size() - first);
    Lease mem(pool_);
    uint32_t* err = zeros(mem, 1);
    // inputs -> canonical int32 on the device
    int32_t* host = reinterpret_cast<int32_t*>(pinned_in_.get((size_t)P * D * 4));
    for (int p = 0; p < P; ++p) {
      const auto& v = inputs[first + p];
      int32_t* row = host + (size_t)p * D;
      for (size_t e = 0; e < D; ++e) row[e] = (int32_t)canon(v[e], (int64_t)m);
    }
    int32_t* secrets = mem.take<int32_t>((size_t)P * D);
    HIP_OK(hipMemcpyAsync(secrets, host, (size_t)P * D * 4, hipMemcpyHostToDevice, s_));
    sync();  // the pinned buffer is rewritten by the next wave
    t.mark("stage");
    const RngKeyArg rng = fresh_rng_key();
    void* shares = mem.take<uint8_t>((size_t)n * P * B * value_bytes);
    uint32_t* cnt = mem.take<uint32_t>((size_t)n * P * tiles(B));
    // full masks in the shares' storage type (32-bit ahead of the limb GEMM)
    const int mask_bytes = (pss && big) ? 4 : value_bytes;
    void* mask_out = mask_mode == kMaskFull ? mem.take<uint8_t>((size_t)P * D * mask_bytes) : nullptr;
    uint32_t* mask_cnt = mask_mode == kMaskFull ? mem.take<uint32_t>((size_t)P * tiles(D)) : nullptr;
    uint32_t* seeds = mask_mode == kMaskChaCha ? mem.take<uint32_t>((size_t)P * seed_words) : nullptr;
    bool have_mask_cnt = mask_mode == kMaskFull;
    int share_mode = mask_mode;
    if (mask_mode == kMaskChaCha) {
      // chacha.rs:29-45 as a pre-pass: fresh seeds, masked = secret + the seed's stream;
      // the shares then come from the unmasked fast kernels
      launch_chacha_seeds(P, seed_words, rng, 0, seeds, s_);
      launched("chacha_seeds");
      int32_t* msk = mem.take<int32_t>((size_t)P * D);
      uint32_t* scratch = mem.take<uint32_t>(chacha_scratch_words(P, (int)D));
      launch_chacha_mask_apply(P, (int)D, m, seed_words, seeds, secrets, msk, scratch, err, s_);
      launched("chacha_mask_apply");
      secrets = msk;
      share_mode = kMaskNone;
    }
    if (!pss) {
      launch_share_additive(P, (int)D, n, m, value_bytes, secrets, share_mode, rng, 0, shares, cnt,
                            mask_out, mask_cnt, s_);
      launched("share_additive");
    } else if (!big) {
      uint32_t* dM = to_device(mem, share_matrix);
      launch_share_pss(P, (int)D, n, (int)k, t_priv, m, value_bytes, secrets, dM, share_mode, rng, 0,
                       shares, cnt, mask_out, nullptr, s_);
      launched("share_pss");
      have_mask_cnt = false;  // packed batches do not align with the mask tiles: recounted
      sync();
    } else {
      const int32_t* masked = secrets;
      if (share_mode == kMaskFull) {
        int32_t* msk = mem.take<int32_t>((size_t)P * D);
        uint32_t* c1 = mem.take<uint32_t>((size_t)P * tiles(D));
        launch_share_additive(P, (int)D, 1, m, 4, secrets, kMaskFull, rng, 0, msk, c1, mask_out,
                              mask_cnt, s_);
        launched("mask_secrets");
        masked = msk;
      }
      const int K = (int)k + t_priv;
      const int Kp = (K + 63) / 64 * 64;
      const LimbScheme sch = limb_scheme(m, Kp);
      const int limbs = sch.limbs;
      std::vector<int8_t> A((size_t)limbs * n * Kp, 0);
      for (int c = 0; c < n; ++c)
        for (int j = 0; j < K; ++j) {
          int8_t d[4];
          limbs_of_value(share_matrix[(size_t)c * K + j], m, sch, d);
          for (int l = 0; l < limbs; ++l) A[((size_t)l * n + c) * Kp + j] = d[l];
        }
      int8_t* dA = to_device(mem, A);
      int8_t* dAf = mem.take<int8_t>((size_t)a_fragments_bytes(n, Kp, limbs));
      launch_a_fragments(n, Kp, limbs, dA, dAf, s_);
      int8_t* X = mem.take<int8_t>((size_t)limbs * P * B * Kp);
      launch_pss_x_limbs(P, (int)D, (int)B, (int)k, t_priv, Kp, m, masked, rng, 0, X, s_);
      launched("pss_x_limbs");
      // the boxes' varint bytes come out of the GEMM epilogue (cnt zeroed first; this
      // backend never runs inside a captured graph)
      HIP_OK(hipMemsetAsync(cnt, 0, (size_t)n * P * tiles(B) * sizeof(uint32_t), s_));
      launch_modgemm_i8(n, (int)B, Kp, P, limbs, m, dA, dAf, X, (int64_t)P * B * Kp, value_bytes, shares,
                        (int64_t)B, (int64_t)P * B, 1, (int64_t)n * P * B, cnt, s_);
      launched("modgemm_i8");
      sync();
    }
    // ---- seal: slot c * P + p = participant p's box for clerk c (participate.rs:82-101)
    Arena arena = new_arena(mem, n * P, B, m);
    std::vector<uint32_t> kidx((size_t)n * P);
    for (int c = 0; c < n; ++c) std::fill(kidx.begin() + (size_t)c * P, kidx.begin() + (size_t)(c + 1) * P, (uint32_t)c);
    uint32_t* dkidx = to_device(mem, kidx);
    std::vector<const uint8_t*> kp;
    for (auto& ck : clerk_keys) kp.push_back(ck.sodium.data());
    uint32_t* pks = key_words(mem, kp);
    Keys ks = seal_setup(mem, arena, dkidx, pks, 0, rng, err);
    seal_data(mem, arena, ks, shares, value_bytes, cnt, err);
    Arena marena;
    if (mask_mode != kMaskNone) {
      const bool full = mask_mode == kMaskFull;
      marena = new_arena(mem, P, full ? D : (size_t)seed_words, full ? m : 0);
      uint32_t* kidx_m = zeros(mem, P);
      uint32_t* pks_r = key_words(mem, {recipient_key->sodium.data()});
      Keys km = seal_setup(mem, marena, kidx_m, pks_r, (uint64_t)n * P, rng, err);
      seal_data(mem, marena, km, full ? (const void*)mask_out : (const void*)seeds,
                full ? mask_bytes : 4, have_mask_cnt ? mask_cnt : nullptr, err);
    }
    check(err, "participate");
    t.mark("gpu");
    std::vector<Encryption> boxes = download(arena);
    for (int p = 0; p < P; ++p) {
      auto& row = out.clerk_boxes[first + p];
      row.resize(n);
      for (int c = 0; c < n; ++c) row[c] = std::move(boxes[(size_t)c * P + p]);
    }
    if (mask_mode != kMaskNone) {
      std::vector<Encryption> mb = download(marena);
      for (int p = 0; p < P; ++p) out.mask_boxes[first + p] = std::move(mb[p]);
    }
    t.mark("d2h");
  }
  return out;
}

}  // namespace

extern "C" DeviceBackend* sda_device_backend_create(int device_index, char* err, size_t err_len) {
  try {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
      (void)hipGetLastError();
      throw SdaError("no HIP device is visible to this process");
    }
    if (device_index < 0 || device_index >= count)
      throw SdaError("device index " + std::to_string(device_index) + " out of range (" +
                     std::to_string(count) + " visible)");
    return new Backend(device_index);
  } catch (const std::exception& e) {
    if (err && err_len) {
      std::strncpy(err, e.what(), err_len - 1);
      err[err_len - 1] = 0;
    }
    return nullptr;
  }
}

}  // namespace sda
