// VALU throughput micro-benchmark (gfx950): wave-instructions per cycle per CU
// for the integer ops the SDA kernels lean on. Each thread runs 8 independent
// chains of one op; enough waves to fill every SIMD.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

#define CHAINS(OP)                                                        \
  _Pragma("unroll") for (int c = 0; c < 8; ++c) { OP; }

template <int K>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, uint32_t seed) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    a[c] = seed * (threadIdx.x + 1) + c;
    b[c] = seed ^ (c * 0x9e3779b9u) ^ threadIdx.x;
  }
  for (int i = 0; i < kIters; ++i) {
    if constexpr (K == 0) { CHAINS(a[c] = a[c] + b[c]) }
    if constexpr (K == 1) { CHAINS(a[c] = a[c] * b[c]) }                               // v_mul_lo_u32
    if constexpr (K == 2) { CHAINS(a[c] = __umulhi(a[c], b[c]) + 1) }                  // v_mul_hi_u32 (+add)
    if constexpr (K == 3) { CHAINS(a[c] = __builtin_amdgcn_alignbit(a[c], a[c], 7) ^ b[c]) }
    if constexpr (K == 4) { CHAINS(a[c] = (a[c] & 0xffffffu) * (b[c] & 0xffffu)) }     // v_mul_u32_u24
    if constexpr (K == 5) {                                                            // v_mad_u64_u32
      CHAINS(uint64_t p = (uint64_t)a[c] * b[c] + a[c]; a[c] = (uint32_t)(p >> 32) ^ (uint32_t)p)
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) r ^= a[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int K>
void run(const char* name, double ops_per_inner) {
  const int blocks = 256 * 8;  // 8 blocks per CU
  uint32_t* out;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(256), 0, 0, out, 12345u);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(256), 0, 0, out, 777u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double waves = blocks * 4.0;
  const double winsts = waves * kIters * 8 * ops_per_inner;
  // per CU per ns
  printf("%-28s %8.3f ms  %7.2f wave-inst/ns/CU (x 2.4 GHz -> %.2f per cycle per CU)\n", name, ms,
         winsts / (ms * 1e6) / 256, winsts / (ms * 1e6) / 256 / 2.4);
  (void)hipFree(out);
}

int main() {
  run<0>("v_add_u32", 1);
  run<1>("v_mul_lo_u32", 1);
  run<2>("v_mul_hi_u32 + v_add", 2);
  run<3>("v_alignbit + v_xor", 2);
  run<4>("v_mul_u32_u24 (+2 and)", 3);
  run<5>("v_mad_u64_u32 (+xor)", 2);
  return 0;
}
