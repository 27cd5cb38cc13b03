// Micro-benchmark: issue rate of the integer / fp64 multiply forms used by the
// Poly1305 and GF(2^255-19) kernels (v_mad_u64_u32, v_mul_lo/hi_u32,
// v_mul_u32_u24, v_fma_f64, plain v_add_u32 as the full-rate reference).
// Build: hipcc -O3 --offload-arch=gfx950 int_mul_rates.hip -o int_mul_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;
constexpr int kChains = 8;  // independent accumulators per lane (ILP)

__global__ void k_add(uint32_t* out, uint32_t s) {
  uint32_t a[kChains];
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = a[c] + (a[c] ^ s);
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mad64(uint64_t* out, uint64_t s) {
  uint64_t a[kChains];
  uint32_t b[kChains];
  for (int c = 0; c < kChains; ++c) { a[c] = threadIdx.x + c; b[c] = s + c; }
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = (uint64_t)b[c] * (uint32_t)(a[c] >> 7) + a[c];
  uint64_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mullo(uint32_t* out, uint32_t s) {
  uint32_t a[kChains];
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = a[c] * (s + c);
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mul24(uint32_t* out, uint32_t s) {
  uint32_t a[kChains];
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = __umul24(a[c], s + c) + c;
  uint32_t r = 0;
  for (int c = 0; c < kChains; ++c) r ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma64(double* out, double s) {
  double a[kChains];
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
  for (int i = 0; i < kIters; ++i)
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = fma(a[c], s, 0.5);
  double r = 0;
  for (int c = 0; c < kChains; ++c) r += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <class K, class T>
void run(const char* name, K kern, T* buf, T arg) {
  const int blocks = 256 * 8, threads = 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, arg);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, arg);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double ops = 5.0 * blocks * threads * (double)kIters * kChains;
  std::printf("%-8s %8.2f Gop/s (lane-ops)  %6.3f ms\n", name, ops / (ms * 1e-3) / 1e9, ms / 5);
}

int main() {
  void* buf;
  hipMalloc(&buf, 256 * 8 * 256 * 8);
  run("add", k_add, (uint32_t*)buf, 3u);
  run("mullo", k_mullo, (uint32_t*)buf, 3u);
  run("mul24", k_mul24, (uint32_t*)buf, 3u);
  run("mad64", k_mad64, (uint64_t*)buf, (uint64_t)3);
  run("fma64", k_fma64, (double*)buf, 1.0000001);
  hipFree(buf);
  return 0;
}
