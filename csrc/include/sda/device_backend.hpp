// GPU execution of the client roles' bulk cryptography.
//
// The three data-heavy loops of the reference client are
//   clerk      open P sealed boxes, combine, seal the sum   (client/src/clerk.rs:79-100)
//   recipient  open n results + P mask boxes, reconstruct, unmask
//                                                           (client/src/receive.rs:102-152)
//   participant mask, share, seal n boxes (+ the mask box)  (client/src/participate.rs:53-101)
// `DeviceBackend` is the seam through which `SdaClient` hands those loops to an
// MI355X: wire-format sealed boxes in, wire-format sealed boxes (or the
// revealed vector) out. Everything else of a role -- fetching the job, the
// committee, key verification, posting the result -- stays in `SdaClient`, so
// a GPU clerk is indistinguishable on the wire from the reference's.
//
// The implementation lives in `libsda_device.so` (csrc/device/, built with
// hipcc, holds the gfx950 kernels); host-only programs load it on demand with
// `load_device_backend()`, so the control plane has no link-time dependency on
// the HIP runtime.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "sda/protocol.hpp"

namespace sda {

// A sealed box that is written straight into a staging slot: `fill(dst, cap)`
// stores at most `cap` bytes of wire-format box (epk | mac | ciphertext) at
// `dst` and returns the box's length (a length above `cap` means "does not
// fit"; nothing usable was written). `max_len` bounds the length up front.
struct BoxSource {
  size_t max_len = 0;
  std::function<size_t(uint8_t* dst, size_t cap)> fill;
};

// Sources over owned boxes (the struct path) ...
BoxSource box_source(const Encryption& e);
// ... and over padded base64 text that is decoded in place (the REST path:
// the text is a span of the response body; no intermediate copy).
BoxSource box_source_base64(const char* text, size_t len);

struct DeviceParticipations {
  // [participant][clerk], and one mask box per participant when the scheme masks
  std::vector<std::vector<Encryption>> clerk_boxes;
  std::vector<Encryption> mask_boxes;
};

class DeviceBackend {
 public:
  virtual ~DeviceBackend() = default;
  virtual std::string describe() const = 0;

  // Clerk: every box holds `values` shares for `own`; returns the sum mod the
  // sharing modulus sealed for `recipient`. Throws SdaError on a box that does
  // not authenticate or does not hold exactly `values` varints.
  virtual Encryption clerk_combine(const LinearSecretSharingScheme& sharing, size_t values,
                                   const EncryptionKeypair& own,
                                   const std::vector<BoxSource>& boxes,
                                   const EncryptionKey& recipient) = 0;

  // Recipient: `results` = (committee index, box) of the clerks that answered,
  // `masks` = the participants' mask boxes (empty without a mask). Returns the
  // aggregate in [0, modulus).
  virtual std::vector<int64_t> reveal(const Aggregation& agg, const EncryptionKeypair& own,
                                      const std::vector<std::pair<size_t, BoxSource>>& results,
                                      const std::vector<BoxSource>& masks) = 0;

  // Participants in bulk: one participation's worth of boxes per input vector.
  virtual DeviceParticipations participate_many(const Aggregation& agg,
                                                const std::vector<EncryptionKey>& clerk_keys,
                                                const EncryptionKey* recipient_key,
                                                const std::vector<std::vector<int64_t>>& inputs) = 0;

  // Wall-clock milliseconds of the last call's stages ("stage", "h2d", "gpu", "d2h", ...).
  virtual std::map<std::string, double> last_timings() const = 0;
};

using DeviceBackendPtr = std::shared_ptr<DeviceBackend>;

// dlopen `path` (default: `libsda_device.so` next to this program / module, or
// $SDA_DEVICE_LIB) and create its backend on GPU `device_index`. Throws
// SdaError with the loader's message when the library or a GPU is missing.
DeviceBackendPtr load_device_backend(const std::string& path = "", int device_index = 0);

// Exported by libsda_device.so.
extern "C" DeviceBackend* sda_device_backend_create(int device_index, char* err, size_t err_len);

}  // namespace sda
