// Do the matrix pipe and the VALU of one SIMD work at the same time for two different
// waves (gfx950)? One 512-thread workgroup per CU (waves w and w + 4 share a SIMD); every
// wave runs `iters` rounds of either 16 independent i8 MFMAs (16x16x64, 16 cycles each)
// or 64 independent integer multiply-adds (4 cycles each): 256 cycles of its pipe a round.
//   mm: all eight waves MFMA       vv: all eight VALU
//   mv: waves 0-3 MFMA, 4-7 VALU   m-: waves 0-3 MFMA, 4-7 idle   -v: waves 4-7 VALU only
//   M: the same pipe time in 32x32x32 MFMAs   l: xor-add instead of 64-bit multiply-add   d: double fma
// If the pipes overlap, mv takes as long as m- and -v; if not, as long as their sum.
//   hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops scripts/ubench_mfma_valu.hip -o /tmp/ubench_mv && /tmp/ubench_mv
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kIters = 2000;

__device__ __forceinline__ void mfma_rounds(int iters, uint32_t* out) {
  v4i a = {1, 2, 3, (int)threadIdx.x}, b = {5, 6, 7, 8};
  v4i acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = v4i{c, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[c], 0, 0, 0);
  }
  int r = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) r ^= acc[c][0] ^ acc[c][3];
  out[blockIdx.x * 512 + threadIdx.x] = (uint32_t)r;
}

// the same pipe time in 32x32x32 MFMAs (32 cycles each): 8 a round
__device__ __forceinline__ void mfma32_rounds(int iters, uint32_t* out) {
  v4i a = {1, 2, 3, (int)threadIdx.x}, b = {5, 6, 7, 8};
  v16i acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[c][e] = c + e;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[c], 0, 0, 0);
  }
  int r = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) r ^= acc[c][0] ^ acc[c][15];
  out[blockIdx.x * 512 + threadIdx.x] = (uint32_t)r;
}

// 64 independent single-cycle-class integer ops a round (v_xad_u32 / v_add3_u32)
__device__ __forceinline__ void valu_light_rounds(int iters, uint32_t* out, uint32_t seed) {
  uint32_t a[16], b = seed ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = seed * (threadIdx.x + 1) + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = (a[c] ^ b) + (uint32_t)i;
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) r ^= a[c];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

// 64 independent double-precision fused multiply-adds a round
__device__ __forceinline__ void valu_f64_rounds(int iters, uint32_t* out, uint32_t seed) {
  double a[16], b = 1.0 + 1e-9 * (double)(seed ^ threadIdx.x);
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = (double)(seed * (threadIdx.x + 1) + c);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = __builtin_fma(a[c], b, 0.5);
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) r += a[c];
  out[blockIdx.x * 512 + threadIdx.x] = (uint32_t)(int64_t)r;
}

__device__ __forceinline__ void valu_rounds(int iters, uint32_t* out, uint32_t seed) {
  uint32_t a[16], b = seed ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = seed * (threadIdx.x + 1) + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = a[c] * b + (uint32_t)i;  // v_mad_u32_u24-free: v_mul_lo + add or v_mad_u64
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) r ^= a[c];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

// role of waves 0-3 / 4-7: 0 idle, 1 MFMA 16x16x64, 2 VALU multiply-add, 3 MFMA 32x32x32, 4 VALU xor-add, 5 VALU double fma
__global__ void __launch_bounds__(512) k_mix(int lo, int hi, int iters, uint32_t* out, uint32_t seed) {
  __shared__ int pad[30000];  // one workgroup per CU
  if (seed == 0xdeadbeefu) pad[threadIdx.x] = 1;
  const int role = (threadIdx.x >> 6) < 4 ? lo : hi;
  if (role == 1) mfma_rounds(iters, out);
  else if (role == 2) valu_rounds(iters, out, seed);
  else if (role == 3) mfma32_rounds(iters, out);
  else if (role == 4) valu_light_rounds(iters, out, seed);
  else if (role == 5) valu_f64_rounds(iters, out, seed);
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 256 * 512 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const struct { const char* name; int lo, hi; } cases[] = {
      {"mm", 1, 1}, {"vv", 2, 2}, {"mv", 1, 2}, {"m-", 1, 0}, {"-v", 0, 2},
      {"M-", 3, 0}, {"Mv", 3, 2}, {"-l", 0, 4}, {"ml", 1, 4}, {"Ml", 3, 4}, {"ll", 4, 4},
      {"-d", 0, 5}, {"md", 1, 5}, {"dd", 5, 5}};
  for (const auto& c : cases) {
    hipLaunchKernelGGL(k_mix, dim3(256), dim3(512), 0, 0, c.lo, c.hi, kIters, out, 1u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mix, dim3(256), dim3(512), 0, 0, c.lo, c.hi, kIters, out, 2u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // a wave's pipe time: kIters * 256 cycles
    printf("%s  %.3f ms  (%.0f cycles per round at 2.4 GHz; one wave's pipe work is 256)\n", c.name, ms,
           ms * 1e-3 * 2.4e9 / kIters);
  }
  return 0;
}
