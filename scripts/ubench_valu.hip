// VALU throughput micro-benchmark (gfx950): wave-instructions per cycle per CU
// for the integer ops the SDA kernels lean on. Each thread runs 8 independent
// chains of one op; enough waves to fill every SIMD.
//   hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops scripts/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
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
    if constexpr (K == 6) { CHAINS(a[c] = a[c] ^ b[c]) }
    if constexpr (K == 7) { CHAINS(a[c] = (a[c] >> 5) & 0x7fu; a[c] += b[c]) }         // v_bfe_u32 + add
    if constexpr (K == 8) { CHAINS(a[c] = __builtin_amdgcn_alignbit(a[c], a[c], 7)) }  // rotate alone
    if constexpr (K == 9) { CHAINS(a[c] = (a[c] ^ b[c]) + (uint32_t)i) }               // v_xad_u32
    if constexpr (K == 10) { CHAINS(a[c] = a[c] + b[c] + (uint32_t)i) }                // v_add3_u32
    if constexpr (K == 11) { CHAINS(a[c] = (a[c] & b[c]) | (uint32_t)i) }              // v_and_or_b32
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

// One Salsa20/20 block per lane per iteration (the XSalsa20 keystream's inner loop).
__global__ void __launch_bounds__(256) k_salsa(uint32_t* out, uint32_t seed, int iters) {
  uint32_t in[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) in[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[i];
#define QR(a, b, c, d)                                   \
  x[b] ^= __builtin_amdgcn_alignbit(x[a] + x[d], x[a] + x[d], 25); \
  x[c] ^= __builtin_amdgcn_alignbit(x[b] + x[a], x[b] + x[a], 23); \
  x[d] ^= __builtin_amdgcn_alignbit(x[c] + x[b], x[c] + x[b], 19); \
  x[a] ^= __builtin_amdgcn_alignbit(x[d] + x[c], x[d] + x[c], 14);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      QR(0, 4, 8, 12) QR(5, 9, 13, 1) QR(10, 14, 2, 6) QR(15, 3, 7, 11)
      QR(0, 1, 2, 3) QR(5, 6, 7, 4) QR(10, 11, 8, 9) QR(15, 12, 13, 14)
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i] + in[i];
    in[8] += 1;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// LDS atomic adds: every lane adds at stride-`stride` ranks (decode-sum's access shape).
__global__ void __launch_bounds__(256) k_dsadd(uint32_t* out, int stride, int iters) {
  __shared__ uint32_t acc[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) acc[i] = 0;
  __syncthreads();
  uint32_t base = ((threadIdx.x & 63) * stride + (threadIdx.x >> 6) * 17) & 4095u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) atomicAdd(&acc[(base + u * 3 + it) & 8191u], (uint32_t)u + 1u);
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = acc[threadIdx.x];
}

// Scatter shapes of the decode-sum accumulate: every lane walks ranks starting at a
// pseudo-random base (lanes ~34 ranks apart with data-dependent jitter), MODE 0 =
// ds_add_u32 on all lanes, 1 = ds_add_u32 with about half the lanes masked off
// per instruction, 2 = plain ds_write_b32, 3 = ds_add_u32 at consecutive ranks
// (lane l -> base + l: conflict-free reference).
template <int MODE>
__global__ void __launch_bounds__(256) k_scatter(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint32_t acc[8192];
  for (int i = threadIdx.x; i < 8192; i += 256) acc[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t h = (threadIdx.x + 1) * 0x9e3779b9u ^ seed;
  h ^= h >> 15; h *= 0x85ebca6bu; h ^= h >> 13;
  uint32_t base = (lane * 34u + (h & 15u)) & 4095u;  // ~34 apart, +-8 jitter
  if (MODE == 3) base = lane;
  uint32_t m = h;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t idx = (base + (uint32_t)u + (uint32_t)it * 7u) & 8191u;
      if (MODE == 0 || MODE == 3) atomicAdd(&acc[idx], (uint32_t)u + 1u);
      if (MODE == 1) { if ((m >> u) & 1u) atomicAdd(&acc[idx], (uint32_t)u + 1u); }
      if (MODE == 2) acc[idx] = (uint32_t)u + m;
    }
    m = m * 1664525u + 1013904223u;
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = acc[threadIdx.x];
}

template <typename F>
float time_ms(F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipEventRecord(e0);
  launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  {
    const int blocks = 256 * 8, iters = 512;
    uint32_t* out;
    (void)hipMalloc(&out, blocks * 256 * 4);
    float ms = time_ms([&] { hipLaunchKernelGGL(k_salsa, dim3(blocks), dim3(256), 0, 0, out, 5u, iters); });
    const double blk = (double)blocks * 256 * iters;
    printf("salsa20/20 core              %8.3f ms  %.3e blocks/s  (%.1f GB/s of keystream; 960 ARX ops/block -> %.3e lane-ops/s)\n",
           ms, blk / (ms * 1e-3), blk * 64 / (ms * 1e-3) / 1e9, blk * 960 / (ms * 1e-3));
    for (int stride : {1, 32, 34, 35, 37}) {
      const int it2 = 2048;
      float m2 = time_ms([&] { hipLaunchKernelGGL(k_dsadd, dim3(blocks), dim3(256), 0, 0, out, stride, it2); });
      const double adds = (double)blocks * 256 * it2 * 16;
      printf("ds_add_u32 stride %-2d          %8.3f ms  %.3e lane-adds/s  (%.2f wave-inst/cycle/CU at 2.4 GHz)\n",
             stride, m2, adds / (m2 * 1e-3), adds / 64 / (m2 * 1e-3) / 256 / 2.4e9);
    }
    {
      const int it3 = 2048;
      const char* names[4] = {"ds_add scatter (all lanes)", "ds_add scatter (half lanes)",
                              "ds_write_b32 scatter", "ds_add consecutive ranks"};
      float t[4];
      t[0] = time_ms([&] { hipLaunchKernelGGL(k_scatter<0>, dim3(blocks), dim3(256), 0, 0, out, it3, 1u); });
      t[1] = time_ms([&] { hipLaunchKernelGGL(k_scatter<1>, dim3(blocks), dim3(256), 0, 0, out, it3, 1u); });
      t[2] = time_ms([&] { hipLaunchKernelGGL(k_scatter<2>, dim3(blocks), dim3(256), 0, 0, out, it3, 1u); });
      t[3] = time_ms([&] { hipLaunchKernelGGL(k_scatter<3>, dim3(blocks), dim3(256), 0, 0, out, it3, 1u); });
      for (int i = 0; i < 4; ++i) {
        const double winst = (double)blocks * 4 * it3 * 16;
        printf("%-28s %8.3f ms  %.2f cycles per wave-instruction per CU (2.4 GHz)\n", names[i], t[i],
               t[i] * 1e-3 * 2.4e9 * 256 / winst);
      }
    }
    (void)hipFree(out);
  }
  run<0>("v_add_u32", 1);
  run<1>("v_mul_lo_u32", 1);
  run<2>("v_mul_hi_u32 + v_add", 2);
  run<3>("v_alignbit + v_xor", 2);
  run<4>("v_mul_u32_u24 (+2 and)", 3);
  run<5>("v_mad_u64_u32 (+xor)", 2);
  run<6>("v_xor_b32", 1);
  run<7>("v_bfe_u32 + v_add", 2);
  run<8>("v_alignbit (rotate)", 1);
  run<9>("v_xad_u32", 1);
  run<10>("v_add3_u32", 1);
  run<11>("v_and_or_b32", 1);
  return 0;
}
