// Zero-copy views of the two bulk downloads of the REST API.
//
// A `ClerkingJob` (protocol/src/resources.rs:127-139) carries one sealed box per
// participation and a `SnapshotResult` (protocol/src/resources.rs:178-188) one
// mask box per participation: hundreds of megabytes of base64 inside one JSON
// document. Parsing such a document into a `json::Value` tree and then into
// `Encryption` structs copies every payload twice before the first byte is
// decrypted. The views below walk the text once at memchr speed and record
// where each payload *is*; the roles then base64-decode every box straight into
// its staging slot (pinned memory for the GPU backend).
//
// Only the plain shape serde_json emits is accepted (no escapes inside the
// strings of interest); anything else makes `scan_*` return nullopt and the
// caller falls back to the full codec, so the views never change what is
// accepted or rejected.
#include <cstring>

#include "sda/protocol.hpp"

namespace sda {
namespace wire {
namespace {

struct NotPlain {};  // the text is outside the plain shape: fall back to the full codec

class Skimmer {
 public:
  explicit Skimmer(const std::string& t) : p_(t.data()), n_(t.size()) {}

  void ws() {
    while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\n' || p_[i_] == '\r' || p_[i_] == '\t')) ++i_;
  }
  char peek() {
    ws();
    if (i_ >= n_) throw NotPlain{};
    return p_[i_];
  }
  void expect(char c) {
    if (peek() != c) throw NotPlain{};
    ++i_;
  }
  bool accept(char c) {
    if (peek() != c) return false;
    ++i_;
    return true;
  }
  // A string without escapes, as a span of the text.
  TextSpan string_span() {
    expect('"');
    const char* q = static_cast<const char*>(std::memchr(p_ + i_, '"', n_ - i_));
    if (!q) throw NotPlain{};
    size_t off = i_, len = (size_t)(q - (p_ + i_));
    if (std::memchr(p_ + off, '\\', len)) throw NotPlain{};
    i_ = off + len + 1;
    return TextSpan{off, len};
  }
  std::string string() {
    TextSpan s = string_span();
    return std::string(p_ + s.off, s.len);
  }
  uint64_t u64() {
    ws();
    size_t s = i_;
    uint64_t v = 0;
    while (i_ < n_ && p_[i_] >= '0' && p_[i_] <= '9') {
      if (v > (UINT64_MAX - 9) / 10) throw NotPlain{};
      v = v * 10 + (uint64_t)(p_[i_++] - '0');
    }
    if (i_ == s) throw NotPlain{};
    return v;
  }
  bool null() {
    ws();
    if (n_ - i_ >= 4 && std::memcmp(p_ + i_, "null", 4) == 0) {
      i_ += 4;
      return true;
    }
    return false;
  }
  void end() {
    ws();
    if (i_ != n_) throw NotPlain{};
  }
  // {"Sodium":"<base64>"} -> the base64 span
  TextSpan sodium() {
    expect('{');
    if (string() != "Sodium") throw NotPlain{};
    expect(':');
    TextSpan s = string_span();
    expect('}');
    return s;
  }
  // Walks the members of an object: f(key) must consume the value.
  template <class F>
  void object(F&& f) {
    expect('{');
    if (accept('}')) return;
    for (;;) {
      std::string key = string();
      expect(':');
      f(key);
      if (accept(',')) continue;
      expect('}');
      return;
    }
  }
  template <class F>
  void array(F&& f) {
    expect('[');
    if (accept(']')) return;
    for (;;) {
      f();
      if (accept(',')) continue;
      expect(']');
      return;
    }
  }

 private:
  const char* p_;
  size_t n_;
  size_t i_ = 0;
};

}  // namespace

std::optional<ClerkingJobView> scan_clerking_job(const std::string& text) {
  try {
    ClerkingJobView v;
    Skimmer s(text);
    int seen = 0;
    s.object([&](const std::string& key) {
      if (key == "id") v.head.id = ClerkingJobId::parse(s.string()), seen |= 1;
      else if (key == "clerk") v.head.clerk = AgentId::parse(s.string()), seen |= 2;
      else if (key == "aggregation") v.head.aggregation = AggregationId::parse(s.string()), seen |= 4;
      else if (key == "snapshot") v.head.snapshot = SnapshotId::parse(s.string()), seen |= 8;
      else if (key == "encryptions") {
        s.array([&] { v.boxes.push_back(s.sodium()); });
        seen |= 16;
      } else throw NotPlain{};
    });
    s.end();
    if (seen != 31) return std::nullopt;
    return v;
  } catch (const NotPlain&) {
    return std::nullopt;
  } catch (const SdaError&) {  // an unparseable id: let the full codec report it
    return std::nullopt;
  }
}

std::optional<SnapshotResultView> scan_snapshot_result(const std::string& text) {
  try {
    SnapshotResultView v;
    Skimmer s(text);
    int seen = 0;
    s.object([&](const std::string& key) {
      if (key == "snapshot") v.snapshot = SnapshotId::parse(s.string()), seen |= 1;
      else if (key == "number_of_participations") v.number_of_participations = s.u64(), seen |= 2;
      else if (key == "clerk_encryptions") {
        s.array([&] {
          SnapshotResultView::Result r;
          int got = 0;
          s.object([&](const std::string& k) {
            if (k == "job") r.job = ClerkingJobId::parse(s.string()), got |= 1;
            else if (k == "clerk") r.clerk = AgentId::parse(s.string()), got |= 2;
            else if (k == "encryption") r.box = s.sodium(), got |= 4;
            else throw NotPlain{};
          });
          if (got != 7) throw NotPlain{};
          v.results.push_back(r);
        });
        seen |= 4;
      } else if (key == "recipient_encryptions") {
        if (!s.null()) {
          v.has_masks = true;
          s.array([&] { v.masks.push_back(s.sodium()); });
        }
        seen |= 8;
      } else throw NotPlain{};
    });
    s.end();
    if (seen != 15) return std::nullopt;
    return v;
  } catch (const NotPlain&) {
    return std::nullopt;
  } catch (const SdaError&) {
    return std::nullopt;
  }
}

}  // namespace wire
}  // namespace sda
