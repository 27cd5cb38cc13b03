// Run-time loading of the GPU backend (see sda/device_backend.hpp) and the box
// sources that feed its staging slots.
#include <dlfcn.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "sda/device_backend.hpp"

namespace sda {

BoxSource box_source(const Encryption& e) {
  const Bytes* b = &e.sodium;
  return BoxSource{b->size(), [b](uint8_t* dst, size_t cap) {
                     if (b->size() <= cap && !b->empty()) std::memcpy(dst, b->data(), b->size());
                     return b->size();
                   }};
}

BoxSource box_source_base64(const char* text, size_t len) {
  return BoxSource{len / 4 * 3, [text, len](uint8_t* dst, size_t cap) {
                     return base64_decode_into(text, len, dst, cap);
                   }};
}

namespace {

std::string dir_of(const std::string& path) {
  auto slash = path.rfind('/');
  return slash == std::string::npos ? "." : path.substr(0, slash);
}

// Candidates: $SDA_DEVICE_LIB, the directory of the shared object or program
// this code was linked into (sda_amd/_lib for the Python module), its parent
// (sda_amd/_lib/bin/sda -> sda_amd/_lib).
std::vector<std::string> candidates() {
  std::vector<std::string> out;
  if (const char* env = std::getenv("SDA_DEVICE_LIB"))
    if (*env) out.push_back(env);
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&candidates), &info) && info.dli_fname) {
    std::string d = dir_of(info.dli_fname);
    out.push_back(d + "/libsda_device.so");
    out.push_back(d + "/../libsda_device.so");
  }
  char exe[4096];
  ssize_t n = ::readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  if (n > 0) {
    exe[n] = 0;
    std::string d = dir_of(exe);
    out.push_back(d + "/libsda_device.so");
    out.push_back(d + "/../libsda_device.so");
  }
  return out;
}

}  // namespace

DeviceBackendPtr load_device_backend(const std::string& path, int device_index) {
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  std::vector<std::string> paths = path.empty() ? candidates() : std::vector<std::string>{path};
  void* lib = nullptr;
  std::string tried;
  for (auto& p : paths) {
    if (::access(p.c_str(), R_OK) != 0) {
      tried += "\n  " + p + ": not found";
      continue;
    }
    lib = ::dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (lib) break;
    const char* e = ::dlerror();
    tried += "\n  " + p + ": " + (e ? e : "dlopen failed");
  }
  if (!lib) throw SdaError("GPU backend: cannot load libsda_device.so:" + tried);
  using Create = DeviceBackend* (*)(int, char*, size_t);
  auto create = reinterpret_cast<Create>(::dlsym(lib, "sda_device_backend_create"));
  if (!create) throw SdaError("GPU backend: libsda_device.so has no sda_device_backend_create");
  char err[512] = {0};
  DeviceBackend* b = create(device_index, err, sizeof(err));
  if (!b) throw SdaError(std::string("GPU backend: ") + (err[0] ? err : "creation failed"));
  // the library stays loaded for the life of the process (its code objects are
  // registered with the HIP runtime)
  return DeviceBackendPtr(b);
}

}  // namespace sda
