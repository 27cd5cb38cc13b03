// Minimal JSON value + parser + compact serializer with serde_json 0.9 output
// conventions (declaration-ordered objects, compact separators, `\uXXXX` only
// for control characters). This reproduces the reference wire format exactly
// (protocol/src/helpers.rs:130-142: the signed bytes of a key are the compact
// JSON of the labelled body, so field order and escaping must match).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "sda/common.hpp"

namespace sda {
namespace json {

class Value {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Value>;
  using Object = std::vector<std::pair<std::string, Value>>;

  Value() : type_(Type::Null) {}
  Value(std::nullptr_t) : type_(Type::Null) {}
  Value(bool b) : type_(Type::Bool), b_(b) {}
  Value(int v) : type_(Type::Int), i_(v), neg_(v < 0) {}
  Value(long v) : type_(Type::Int), i_(v), neg_(v < 0) {}
  Value(long long v) : type_(Type::Int), i_(v), neg_(v < 0) {}
  Value(unsigned v) : type_(Type::Int), i_((long long)v), neg_(false) {}
  Value(unsigned long v) : type_(Type::Int), u_(v), unsigned_(true) {}
  Value(unsigned long long v) : type_(Type::Int), u_(v), unsigned_(true) {}
  Value(double d) : type_(Type::Double), d_(d) {}
  Value(const char* s) : type_(Type::String), s_(s) {}
  Value(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Value(Array a) : type_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Value(Object o) : type_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Value array() { return Value(Array{}); }
  static Value object() { return Value(Object{}); }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_i64() const;
  uint64_t as_u64() const;
  double as_double() const;
  const std::string& as_string() const;
  const Array& as_array() const;
  Array& as_array();
  const Object& as_object() const;
  Object& as_object();

  // object helpers
  const Value* find(const std::string& key) const;
  const Value& at(const std::string& key) const;  // throws if missing
  Value& set(const std::string& key, Value v);     // append or replace
  bool has(const std::string& key) const { return find(key) != nullptr; }
  // array helpers
  void push(Value v) { as_array().push_back(std::move(v)); }
  size_t size() const;

  std::string dump() const;
  void dump_to(std::string& out) const;
  static Value parse(const std::string& text);

  bool operator==(const Value& o) const;
  bool operator!=(const Value& o) const { return !(*this == o); }

 private:
  Type type_;
  bool b_ = false;
  long long i_ = 0;
  unsigned long long u_ = 0;
  bool unsigned_ = false;
  bool neg_ = false;
  double d_ = 0;
  std::string s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

std::string escape_string(const std::string& s);

}  // namespace json

// ---- base64 (RFC 4648 standard alphabet, padded) ---------------------------
std::string base64_encode(const uint8_t* p, size_t n);
inline std::string base64_encode(const Bytes& b) { return base64_encode(b.data(), b.size()); }
// Strict padded decode (data-encoding `base64::decode`).
Bytes base64_decode(const std::string& s);
// In-place forms for bulk payloads: encode `n` bytes to `out` (room for
// (n + 2) / 3 * 4 symbols; returns the count); the decoded length of a padded
// string; decode into `dst` (returns the decoded length; when that exceeds
// `cap` nothing is written). All three throw SdaError like `base64_decode`.
size_t base64_encode_into(const uint8_t* p, size_t n, char* out);
size_t base64_decoded_len(const char* s, size_t n);
size_t base64_decode_into(const char* s, size_t n, uint8_t* dst, size_t cap);
// Decode the first `encode_nopad_len(size)` characters without padding
// (protocol/src/byte_arrays.rs:14-21: B8/B32/B64 tolerate the padding).
Bytes base64_decode_fixed(const std::string& s, size_t size);

// ---- UUIDv4 ----------------------------------------------------------------
struct Uuid {
  uint8_t b[16] = {0};
  static Uuid random();
  static Uuid parse(const std::string& s);  // hyphenated or simple hex; throws
  std::string str() const;                  // lowercase hyphenated
  bool operator==(const Uuid& o) const;
  bool operator!=(const Uuid& o) const { return !(*this == o); }
  bool operator<(const Uuid& o) const;
};

}  // namespace sda
