// Common types for the SDA MI355X framework (host side).
//
// Error kinds mirror the reference's `SdaError` (protocol/src/lib.rs:21-41):
// PermissionDenied, InvalidCredentials, Invalid(String), plus a generic kind
// for everything the reference reports as a free-form error string.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace sda {

using Bytes = std::vector<uint8_t>;

enum class ErrorKind : int {
  Other = 0,
  PermissionDenied = 1,
  InvalidCredentials = 2,
  Invalid = 3,
};

class SdaError : public std::runtime_error {
 public:
  SdaError(ErrorKind kind, const std::string& msg)
      : std::runtime_error(msg), kind_(kind) {}
  explicit SdaError(const std::string& msg)
      : std::runtime_error(msg), kind_(ErrorKind::Other) {}
  ErrorKind kind() const { return kind_; }

  static SdaError permission_denied() {
    return SdaError(ErrorKind::PermissionDenied, "permission denied");
  }
  static SdaError invalid_credentials() {
    return SdaError(ErrorKind::InvalidCredentials, "invalid credentials");
  }
  static SdaError invalid(const std::string& s) {
    return SdaError(ErrorKind::Invalid, s);
  }

 private:
  ErrorKind kind_;
};

inline std::string to_hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}
inline std::string to_hex(const Bytes& b) { return to_hex(b.data(), b.size()); }

Bytes from_hex(const std::string& s);

// Secure wipe that the optimizer may not drop.
void secure_zero(void* p, size_t n);

}  // namespace sda
