// Sealed-box key setup kernels: one lane per message runs the X25519 ladder(s),
// the BLAKE2b-192 nonce and the HSalsa20 derivations of libsodium's
// crypto_box_seal / crypto_box_seal_open (reference sodium.rs:43,78).
//
// These are latency-bound (a 255-step ladder per lane) but tiny in count
// (one per message), so the engine runs them on a side stream concurrently with
// the bandwidth-bound share/encode kernels.
#include "device_crypto.hpp"
#include "kernels.hpp"

namespace sdagpu {
namespace {

// ---- dispatch gate -----------------------------------------------------------
// The X25519 setup kernels need ~150 VGPRs per wave. Launched on the side stream
// at the same moment as a full-chip main-stream grid (the share kernel fills
// every SIMD's register file), their workgroups only become resident once that
// grid drains, and the first encrypt then waits on them (measured: 0.9 ms alone,
// 4.9 ms next to the share kernel). So the setup kernel's first lane posts a
// token when it is dispatched, and the main stream runs `k_gate_wait` -- one
// wave polling the token, bounded by a timeout -- before its big grid: the
// setup waves are resident first and run concurrently at their own latency.
SDA_DEV void signal_dispatched(uint32_t* gate, uint32_t val) {
  if (gate != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(gate, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) k_gate_wait(const uint32_t* gate, uint32_t val,
                                                  uint64_t timeout_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();  // constant-rate (100 MHz) counter
  while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != val) {
    if (wall_clock64() - t0 > timeout_ticks) break;  // never wait unboundedly
    __builtin_amdgcn_s_sleep(2);
  }
}

SDA_DEV void derive_msg_key(MsgKey& out, const uint32_t (&shared)[8], const uint32_t (&epk)[8],
                            const uint32_t (&pk)[8]) {
  const uint32_t zero4[4] = {0, 0, 0, 0};
  uint32_t k[8];
  hsalsa20(k, shared, zero4);  // crypto_box_beforenm
  uint32_t msg[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { msg[i] = epk[i]; msg[8 + i] = pk[i]; }
  uint32_t nonce[6];
  blake2b_192_64(nonce, msg);
  const uint32_t n4[4] = {nonce[0], nonce[1], nonce[2], nonce[3]};
  uint32_t sub[8];
  hsalsa20(sub, k, n4);
  uint32_t b0[16];
  salsa20_block(b0, sub, nonce[4], nonce[5], 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) out.subkey[i] = sub[i];
  out.nonce[0] = nonce[4];
  out.nonce[1] = nonce[5];
#pragma unroll
  for (int i = 0; i < 4; ++i) { out.poly_r[i] = b0[i]; out.poly_s[i] = b0[4 + i]; }
  out.pad[0] = out.pad[1] = 0;
}

// (j + 1) 256^i B of edwards25519 as y+x, y-x, 2dxy (x25519_base's table, 32 KB)
__device__ const uint32_t g_ed_base[32 * 8 * kEdEntryWords] = {
#include "ed25519_base.inc"
};

// Setup kernels run beside full-chip grids: 4 ladder waves per workgroup pack
// them onto a quarter as many CUs (a ~150-VGPR ladder wave costs its CU one of
// the neighbouring grid's workgroups; measured on the round timeline).
constexpr int kSetupBlock = 256;

// Two lanes per message: the even lane computes epk = esk . 9, the odd lane the
// shared point esk . pk -- the two ladders are independent, so running them side
// by side halves the setup latency (one ladder per lane is ~1.7 ms whatever the
// message count, and a round's first encode waits on these keys). The results
// meet through a lane shuffle; the even lane derives the message key.
__global__ void __launch_bounds__(kSetupBlock) k_seal_setup(int M, RngKeyArg rng, uint64_t owner_base,
                                                   const uint32_t* __restrict__ key_idx,
                                                   const uint32_t* __restrict__ pks, uint8_t* ct,
                                                   uint64_t stride, MsgKey* keys, uint32_t* err,
                                                   uint32_t* gate, uint32_t gate_val) {
  signal_dispatched(gate, gate_val);
  // Latency-bound ladders sharing SIMDs with the main stream's full-chip grids:
  // top wave priority, so the arbiter issues them first and they finish at
  // close to their stand-alone latency (the first encrypt waits on them).
  __builtin_amdgcn_s_setprio(3);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = t >> 1, role = t & 1;
  const bool live = j < M;
  const int jj = live ? j : M - 1;  // both lanes of a pair stay in the shuffle
  RngKey rk;
#pragma unroll
  for (int i = 0; i < 8; ++i) rk.k[i] = rng.k[i];
  uint32_t w[16];
  rng_block(w, rk, stream_id(kPurposeEphemeral, owner_base + (uint64_t)jj), 0);
  uint32_t esk[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) esk[i] = w[i];
  uint32_t pk[8];
  const uint32_t* pkp = pks + 8 * (size_t)key_idx[jj];
#pragma unroll
  for (int i = 0; i < 8; ++i) pk[i] = pkp[i];
  uint32_t u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = role ? pk[i] : (i == 0 ? 9u : 0u);
  uint32_t r[8];
  x25519(r, esk, u);
  uint32_t other[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) other[i] = __shfl_xor(r[i], 1, 64);
  if (!live || role) return;
  const uint32_t(&epk)[8] = r;
  const uint32_t(&shared)[8] = other;
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc |= shared[i];
  if (acc == 0) atomicOr(err, kErrBadKey);
  MsgKey mk;
  derive_msg_key(mk, shared, epk, pk);
  keys[j] = mk;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ct + (size_t)j * stride);
#pragma unroll
  for (int i = 0; i < 8; ++i) hdr[i] = epk[i];
}

// The many-message form (hundreds of thousands of boxes: the many-clerk committees):
// the launch runs for many rounds of resident waves, so what counts is the work per
// message, not one ladder's latency. One lane per message; its ephemeral public key
// comes from the fixed-base table (a fifth of a ladder's multiplications), only the
// shared point needs the ladder.
__global__ void __launch_bounds__(kSetupBlock) k_seal_setup_many(int M, RngKeyArg rng, uint64_t owner_base,
                                                        const uint32_t* __restrict__ key_idx,
                                                        const uint32_t* __restrict__ pks, uint8_t* ct,
                                                        uint64_t stride, MsgKey* keys, uint32_t* err,
                                                        uint32_t* gate, uint32_t gate_val,
                                                        const uint32_t* __restrict__ key_tables) {
  signal_dispatched(gate, gate_val);
  __builtin_amdgcn_s_setprio(3);  // see k_seal_setup
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= M) return;
  RngKey rk;
#pragma unroll
  for (int i = 0; i < 8; ++i) rk.k[i] = rng.k[i];
  uint32_t w[16];
  rng_block(w, rk, stream_id(kPurposeEphemeral, owner_base + (uint64_t)j), 0);
  uint32_t esk[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) esk[i] = w[i];
  uint32_t pk[8];
  const uint32_t* pkp = pks + 8 * (size_t)key_idx[j];
#pragma unroll
  for (int i = 0; i < 8; ++i) pk[i] = pkp[i];
  uint32_t epk[8], shared[8];
  // a key with a fixed-base table of its own (word 30 of an entry marks one): no ladder
  const uint32_t* kt = key_tables ? key_tables + (size_t)key_idx[j] * (32 * 8 * kEdEntryWords) : nullptr;
  if (kt != nullptr && kt[30] != 0) x25519_seal_pair_tables(epk, shared, esk, g_ed_base, kt);
  else x25519_seal_pair(epk, shared, esk, pk, g_ed_base);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc |= shared[i];
  if (acc == 0) atomicOr(err, kErrBadKey);
  MsgKey mk;
  derive_msg_key(mk, shared, epk, pk);
  keys[j] = mk;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ct + (size_t)j * stride);
#pragma unroll
  for (int i = 0; i < 8; ++i) hdr[i] = epk[i];
}

__global__ void __launch_bounds__(64) k_x25519_base(int N, const uint32_t* __restrict__ sc, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  uint32_t a[8], o[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) a[w] = sc[8 * (size_t)i + w];
  x25519_base(o, a, g_ed_base);
#pragma unroll
  for (int w = 0; w < 8; ++w) out[8 * (size_t)i + w] = o[w];
}

__global__ void __launch_bounds__(kSetupBlock) k_open_setup(int M, const uint32_t* __restrict__ key_idx,
                                                   const uint32_t* __restrict__ sks,
                                                   const uint32_t* __restrict__ pks,
                                                   const uint8_t* ct, uint64_t stride,
                                                   MsgKey* keys, uint32_t* err,
                                                   uint32_t* gate, uint32_t gate_val, int prio) {
  signal_dispatched(gate, gate_val);
  if (prio) __builtin_amdgcn_s_setprio(3);  // see k_seal_setup
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= M) return;
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(ct + (size_t)j * stride);
  uint32_t epk[8], sk[8], pk[8];
  const size_t kix = key_idx[j];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    epk[i] = hdr[i];
    sk[i] = sks[8 * kix + i];
    pk[i] = pks[8 * kix + i];
  }
  uint32_t shared[8];
  x25519(shared, sk, epk);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc |= shared[i];
  if (acc == 0) atomicOr(err, kErrBadKey);
  MsgKey mk;
  derive_msg_key(mk, shared, epk, pk);
  keys[j] = mk;
}

__global__ void __launch_bounds__(64) k_x25519(int N, const uint32_t* __restrict__ sc,
                                               const uint32_t* __restrict__ pt, uint32_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  uint32_t a[8], b[8], o[8];
#pragma unroll
  for (int w = 0; w < 8; ++w) { a[w] = sc[8 * (size_t)i + w]; b[w] = pt[8 * (size_t)i + w]; }
  x25519(o, a, b);
#pragma unroll
  for (int w = 0; w < 8; ++w) out[8 * (size_t)i + w] = o[w];
}

}  // namespace

static int g_seal_many = -1;  // -1: by message count; 0 / 1: force the pair / many-message form
void set_seal_many(int mode) { g_seal_many = mode; }
static int g_open_prio = 0;
int g_powers_prio = 0;
void set_key_prio(int open_prio, int powers_prio) {
  g_open_prio = open_prio;
  g_powers_prio = powers_prio;
}

void launch_seal_setup(int M, RngKeyArg rng, uint64_t owner_base, const uint32_t* key_idx,
                       const uint32_t* pks, uint8_t* ct, uint64_t stride, MsgKey* keys,
                       uint32_t* err, uint32_t* gate, uint32_t gate_val, const uint32_t* key_tables,
                       hipStream_t s) {
  if (M <= 0) return;
  // a launch of several rounds of resident waves (~200k lanes at three ladder waves
  // per SIMD) is bound by its work, not by a ladder's latency
  const bool many = g_seal_many < 0 ? M >= 65536 : g_seal_many != 0;
  if (many) {
    hipLaunchKernelGGL(k_seal_setup_many, dim3((unsigned)((M + kSetupBlock - 1) / kSetupBlock)),
                       dim3(kSetupBlock), 0, s, M, rng, owner_base, key_idx, pks, ct, stride, keys,
                       err, gate, gate_val, key_tables);
    return;
  }
  const int64_t threads = 2 * (int64_t)M;
  hipLaunchKernelGGL(k_seal_setup, dim3((unsigned)((threads + kSetupBlock - 1) / kSetupBlock)),
                     dim3(kSetupBlock), 0, s, M, rng,
                     owner_base, key_idx, pks, ct, stride, keys, err, gate, gate_val);
}

void launch_open_setup(int M, const uint32_t* key_idx, const uint32_t* sks, const uint32_t* pks,
                       const uint8_t* ct, uint64_t stride, MsgKey* keys, uint32_t* err,
                       uint32_t* gate, uint32_t gate_val, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_open_setup, dim3((M + kSetupBlock - 1) / kSetupBlock), dim3(kSetupBlock), 0, s,
                     M, key_idx, sks, pks, ct,
                     stride, keys, err, gate, gate_val, g_open_prio);
}

void launch_gate_wait(const uint32_t* gate, uint32_t val, uint32_t timeout_us, hipStream_t s) {
  hipLaunchKernelGGL(k_gate_wait, dim3(1), dim3(64), 0, s, gate, val,
                     (uint64_t)timeout_us * 100);
}

void launch_x25519_base(int N, const uint32_t* scalars, uint32_t* out, hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(k_x25519_base, dim3((N + 63) / 64), dim3(64), 0, s, N, scalars, out);
}

void launch_x25519(int N, const uint32_t* scalars, const uint32_t* points, uint32_t* out,
                   hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(k_x25519, dim3((N + 63) / 64), dim3(64), 0, s, N, scalars, points, out);
}

}  // namespace sdagpu
