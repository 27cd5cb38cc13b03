// JSON codec, base64 and UUIDs (see sda/json.hpp).
#include "sda/json.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>

#include "sda/crypto.hpp"

namespace sda {
namespace json {

namespace {
[[noreturn]] void type_error(const char* want) {
  throw SdaError(std::string("json: expected ") + want);
}
}  // namespace

bool Value::as_bool() const {
  if (type_ != Type::Bool) type_error("bool");
  return b_;
}
int64_t Value::as_i64() const {
  if (type_ != Type::Int) type_error("integer");
  if (unsigned_) {
    if (u_ > (unsigned long long)INT64_MAX) type_error("i64");
    return (int64_t)u_;
  }
  return i_;
}
uint64_t Value::as_u64() const {
  if (type_ != Type::Int) type_error("integer");
  if (unsigned_) return u_;
  if (i_ < 0) type_error("unsigned integer");
  return (uint64_t)i_;
}
double Value::as_double() const {
  if (type_ == Type::Double) return d_;
  if (type_ == Type::Int) return unsigned_ ? (double)u_ : (double)i_;
  type_error("number");
}
const std::string& Value::as_string() const {
  if (type_ != Type::String) type_error("string");
  return s_;
}
const Value::Array& Value::as_array() const {
  if (type_ != Type::Array) type_error("array");
  return *a_;
}
Value::Array& Value::as_array() {
  if (type_ != Type::Array) type_error("array");
  return *a_;
}
const Value::Object& Value::as_object() const {
  if (type_ != Type::Object) type_error("object");
  return *o_;
}
Value::Object& Value::as_object() {
  if (type_ != Type::Object) type_error("object");
  return *o_;
}
const Value* Value::find(const std::string& key) const {
  if (type_ != Type::Object) return nullptr;
  for (auto& kv : *o_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}
const Value& Value::at(const std::string& key) const {
  const Value* v = find(key);
  if (!v) throw SdaError("json: missing field `" + key + "`");
  return *v;
}
Value& Value::set(const std::string& key, Value v) {
  auto& o = as_object();
  for (auto& kv : o)
    if (kv.first == key) {
      kv.second = std::move(v);
      return kv.second;
    }
  o.emplace_back(key, std::move(v));
  return o.back().second;
}
size_t Value::size() const {
  if (type_ == Type::Array) return a_->size();
  if (type_ == Type::Object) return o_->size();
  return 0;
}

bool Value::operator==(const Value& o) const {
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::Int:
      if (unsigned_ || o.unsigned_) {
        if ((!unsigned_ && i_ < 0) || (!o.unsigned_ && o.i_ < 0)) return false;
        return as_u64() == o.as_u64();
      }
      return i_ == o.i_;
    case Type::Double: return d_ == o.d_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: return *o_ == *o.o_;
  }
  return false;
}

namespace {
// Bytes a string cannot hold verbatim: '"', '\\' and control characters. Long
// strings (base64 payloads of megabytes) are copied in whole runs between them.
struct PlainTable {
  bool special[256];
  PlainTable() {
    for (int c = 0; c < 256; ++c) special[c] = c < 0x20 || c == '"' || c == '\\';
  }
};
const PlainTable kPlain;

inline size_t plain_run(const char* p, size_t n) {
  size_t i = 0;
  while (i < n && !kPlain.special[(unsigned char)p[i]]) ++i;
  return i;
}

void escape_into(std::string& out, const std::string& s) {
  out.push_back('"');
  const char* p = s.data();
  size_t n = s.size(), i = 0;
  while (i < n) {
    size_t run = plain_run(p + i, n - i);
    out.append(p + i, run);
    i += run;
    if (i >= n) break;
    unsigned char c = (unsigned char)p[i++];
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default: {
        char buf[8];
        std::snprintf(buf, sizeof(buf), "\\u%04x", c);
        out += buf;
      }
    }
  }
  out.push_back('"');
}
}  // namespace

std::string escape_string(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  escape_into(out, s);
  return out;
}

void Value::dump_to(std::string& out) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += unsigned_ ? std::to_string(u_) : std::to_string(i_); break;
    case Type::Double: {
      if (!std::isfinite(d_)) { out += "null"; break; }
      char buf[64];
      std::snprintf(buf, sizeof(buf), "%.17g", d_);
      out += buf;
      if (!std::strpbrk(buf, ".eE")) out += ".0";
      break;
    }
    case Type::String: escape_into(out, s_); break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        v.dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (auto& kv : *o_) {
        if (!first) out.push_back(',');
        first = false;
        escape_into(out, kv.first);
        out.push_back(':');
        kv.second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

namespace {
// Lower bound of the dumped size (payload strings dominate): one allocation
// instead of a doubling chain over hundreds of megabytes.
size_t dump_estimate(const Value& v) {
  switch (v.type()) {
    case Value::Type::String: return v.as_string().size() + 2;
    case Value::Type::Array: {
      size_t n = 2;
      for (auto& x : v.as_array()) n += dump_estimate(x) + 1;
      return n;
    }
    case Value::Type::Object: {
      size_t n = 2;
      for (auto& kv : v.as_object()) n += kv.first.size() + 4 + dump_estimate(kv.second);
      return n;
    }
    default: return 8;
  }
}
}  // namespace

std::string Value::dump() const {
  std::string s;
  s.reserve(dump_estimate(*this));
  dump_to(s);
  return s;
}

// ---- parser ----------------------------------------------------------------
namespace {

struct Parser {
  const std::string& t;
  size_t i = 0;
  int depth = 0;
  explicit Parser(const std::string& text) : t(text) {}

  [[noreturn]] void fail(const char* msg) {
    throw SdaError(std::string("json parse error: ") + msg + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if (t.compare(i, n, s) == 0) { i += n; return true; }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out.push_back((char)cp);
    else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      out.push_back((char)(0xE0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    if (i + 4 > t.size()) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = t[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (t[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      // whole runs of plain bytes at once (payload strings are megabytes long)
      size_t run = plain_run(t.data() + i, t.size() - i);
      if (run) {
        if (out.empty()) out.reserve(run);
        out.append(t.data() + i, run);
        i += run;
      }
      if (i >= t.size()) fail("unterminated string");
      char c = t[i++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (i >= t.size()) fail("bad escape");
      char e = t[i++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00) {
            if (!(i + 1 < t.size() && t[i] == '\\' && t[i + 1] == 'u')) fail("lone surrogate");
            i += 2;
            uint32_t lo = hex4();
            if (lo < 0xDC00 || lo >= 0xE000) fail("bad surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Value number() {
    size_t s = i;
    bool neg = false;
    if (t[i] == '-') { neg = true; ++i; }
    if (i >= t.size() || !std::isdigit((unsigned char)t[i])) fail("bad number");
    while (i < t.size() && std::isdigit((unsigned char)t[i])) ++i;
    bool is_float = false;
    if (i < t.size() && t[i] == '.') {
      is_float = true;
      ++i;
      while (i < t.size() && std::isdigit((unsigned char)t[i])) ++i;
    }
    if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
      is_float = true;
      ++i;
      if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
      while (i < t.size() && std::isdigit((unsigned char)t[i])) ++i;
    }
    std::string num = t.substr(s, i - s);
    if (is_float) return Value(std::stod(num));
    errno = 0;
    if (neg) {
      long long v = std::strtoll(num.c_str(), nullptr, 10);
      if (errno == ERANGE) return Value(std::stod(num));
      return Value(v);
    }
    unsigned long long v = std::strtoull(num.c_str(), nullptr, 10);
    if (errno == ERANGE) return Value(std::stod(num));
    if (v <= (unsigned long long)INT64_MAX) return Value((long long)v);
    return Value(v);
  }
  Value value() {
    if (++depth > 512) fail("nesting too deep");
    ws();
    if (i >= t.size()) fail("unexpected end");
    Value out;
    char c = t[i];
    if (c == '{') {
      ++i;
      Value::Object o;
      ws();
      if (i < t.size() && t[i] == '}') { ++i; }
      else {
        while (true) {
          ws();
          std::string k = str();
          ws();
          if (i >= t.size() || t[i] != ':') fail("expected ':'");
          ++i;
          o.emplace_back(std::move(k), value());
          ws();
          if (i < t.size() && t[i] == ',') { ++i; continue; }
          if (i < t.size() && t[i] == '}') { ++i; break; }
          fail("expected ',' or '}'");
        }
      }
      out = Value(std::move(o));
    } else if (c == '[') {
      ++i;
      Value::Array a;
      ws();
      if (i < t.size() && t[i] == ']') { ++i; }
      else {
        while (true) {
          a.push_back(value());
          ws();
          if (i < t.size() && t[i] == ',') { ++i; continue; }
          if (i < t.size() && t[i] == ']') { ++i; break; }
          fail("expected ',' or ']'");
        }
      }
      out = Value(std::move(a));
    } else if (c == '"') {
      out = Value(str());
    } else if (lit("true")) {
      out = Value(true);
    } else if (lit("false")) {
      out = Value(false);
    } else if (lit("null")) {
      out = Value(nullptr);
    } else {
      out = number();
    }
    --depth;
    return out;
  }
};

}  // namespace

Value Value::parse(const std::string& text) {
  Parser p(text);
  Value v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

}  // namespace json

// ---- base64 ------------------------------------------------------------------
// Table-driven, four symbols (three bytes) per step: sealed boxes of megabytes
// cross the REST API as base64 strings, so this codec is on the data path of
// every role.
static const char* kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

namespace {
struct B64Tables {
  uint8_t val[256];  // 0..63, or 0xff for a symbol outside the alphabet
  B64Tables() {
    std::memset(val, 0xff, sizeof(val));
    for (int i = 0; i < 64; ++i) val[(uint8_t)kB64[i]] = (uint8_t)i;
  }
};
const B64Tables& b64_tables() {
  static const B64Tables t;
  return t;
}
}  // namespace

size_t base64_encode_into(const uint8_t* p, size_t n, char* out) {
  char* o = out;
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = ((uint32_t)p[i] << 16) | ((uint32_t)p[i + 1] << 8) | p[i + 2];
    o[0] = kB64[v >> 18];
    o[1] = kB64[(v >> 12) & 63];
    o[2] = kB64[(v >> 6) & 63];
    o[3] = kB64[v & 63];
    o += 4;
  }
  if (n - i == 1) {
    uint32_t v = (uint32_t)p[i] << 16;
    o[0] = kB64[v >> 18];
    o[1] = kB64[(v >> 12) & 63];
    o[2] = o[3] = '=';
    o += 4;
  } else if (n - i == 2) {
    uint32_t v = ((uint32_t)p[i] << 16) | ((uint32_t)p[i + 1] << 8);
    o[0] = kB64[v >> 18];
    o[1] = kB64[(v >> 12) & 63];
    o[2] = kB64[(v >> 6) & 63];
    o[3] = '=';
    o += 4;
  }
  return (size_t)(o - out);
}

std::string base64_encode(const uint8_t* p, size_t n) {
  std::string out((n + 2) / 3 * 4, '\0');
  base64_encode_into(p, n, &out[0]);
  return out;
}

// Unpadded decode of `len` symbols into `dst` (room for len * 3 / 4 bytes).
static size_t decode_nopad_into(const char* s, size_t len, uint8_t* dst) {
  const uint8_t* T = b64_tables().val;
  if (len % 4 == 1) throw SdaError("Base64 decoding error: invalid length");
  uint8_t* o = dst;
  size_t i = 0;
  uint32_t bad = 0;
  for (; i + 4 <= len; i += 4) {
    uint32_t a = T[(uint8_t)s[i]], b = T[(uint8_t)s[i + 1]], c = T[(uint8_t)s[i + 2]],
             d = T[(uint8_t)s[i + 3]];
    bad |= a | b | c | d;  // 0xff marks a foreign symbol: bit 7 survives the OR
    uint32_t v = (a << 18) | (b << 12) | (c << 6) | d;
    o[0] = (uint8_t)(v >> 16);
    o[1] = (uint8_t)(v >> 8);
    o[2] = (uint8_t)v;
    o += 3;
  }
  if (bad & 0x80) throw SdaError("Base64 decoding error: invalid symbol");
  size_t rest = len - i;
  if (rest) {  // 2 or 3 symbols: 1 or 2 bytes, trailing bits must be zero
    uint32_t a = T[(uint8_t)s[i]], b = T[(uint8_t)s[i + 1]], c = rest == 3 ? T[(uint8_t)s[i + 2]] : 0;
    if ((a | b | c) & 0x80) throw SdaError("Base64 decoding error: invalid symbol");
    uint32_t v = (a << 18) | (b << 12) | (c << 6);
    *o++ = (uint8_t)(v >> 16);
    if (rest == 3) *o++ = (uint8_t)(v >> 8);
    if (v & (rest == 3 ? 0xffu : 0xffffu))
      throw SdaError("Base64 decoding error: non-zero trailing bits");
  }
  return (size_t)(o - dst);
}

size_t base64_decoded_len(const char* s, size_t n) {
  if (n % 4 != 0) throw SdaError("Base64 decoding error: invalid length");
  size_t pad = 0;
  while (pad < 2 && n > pad && s[n - 1 - pad] == '=') ++pad;
  return n / 4 * 3 - pad;
}

size_t base64_decode_into(const char* s, size_t n, uint8_t* dst, size_t cap) {
  size_t want = base64_decoded_len(s, n);
  if (want > cap) return want;  // does not fit: nothing written
  size_t len = n;
  while (len > 0 && n - len < 2 && s[len - 1] == '=') --len;
  return decode_nopad_into(s, len, dst);
}

static Bytes decode_nopad(const std::string& s, size_t len) {
  Bytes out(len * 3 / 4 + 3);
  out.resize(decode_nopad_into(s.data(), len, out.data()));
  return out;
}

Bytes base64_decode(const std::string& s) {
  if (s.size() % 4 != 0) throw SdaError("Base64 decoding error: invalid length");
  size_t len = s.size();
  size_t pad = 0;
  while (pad < 2 && len > 0 && s[len - 1] == '=') { --len; ++pad; }
  return decode_nopad(s, len);
}

Bytes base64_decode_fixed(const std::string& s, size_t size) {
  size_t nopad = (size * 8 + 5) / 6;
  if (s.size() < nopad) throw SdaError("Base64 decoding error: too short");
  Bytes b = decode_nopad(s, nopad);
  if (b.size() != size) throw SdaError("Base64 decoding error: wrong size");
  return b;
}

// ---- UUID --------------------------------------------------------------------
Uuid Uuid::random() {
  Uuid u;
  crypto::os_random(u.b, 16);
  u.b[6] = (u.b[6] & 0x0f) | 0x40;  // version 4
  u.b[8] = (u.b[8] & 0x3f) | 0x80;  // RFC 4122 variant
  return u;
}

Uuid Uuid::parse(const std::string& s) {
  std::string hex;
  if (s.size() == 36) {
    if (s[8] != '-' || s[13] != '-' || s[18] != '-' || s[23] != '-')
      throw SdaError("unparseable uuid " + s);
    for (size_t i = 0; i < s.size(); ++i)
      if (i != 8 && i != 13 && i != 18 && i != 23) hex.push_back(s[i]);
  } else if (s.size() == 32) {
    hex = s;
  } else {
    throw SdaError("unparseable uuid " + s);
  }
  Uuid u;
  try {
    Bytes b = from_hex(hex);
    std::memcpy(u.b, b.data(), 16);
  } catch (const SdaError&) {
    throw SdaError("unparseable uuid " + s);
  }
  return u;
}

std::string Uuid::str() const {
  std::string h = to_hex(b, 16);
  return h.substr(0, 8) + "-" + h.substr(8, 4) + "-" + h.substr(12, 4) + "-" + h.substr(16, 4) +
         "-" + h.substr(20, 12);
}
bool Uuid::operator==(const Uuid& o) const { return std::memcmp(b, o.b, 16) == 0; }
bool Uuid::operator<(const Uuid& o) const { return std::memcmp(b, o.b, 16) < 0; }

}  // namespace sda
