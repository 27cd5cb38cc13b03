// Workgroup-level reductions / scans for 256-thread (4 x wave64) blocks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_crypto.hpp"

namespace sdagpu {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

SDA_DEV uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Inclusive wave prefix sum.
SDA_DEV uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
// Block sum; result valid in every thread. `scratch` holds kWaves words.
SDA_DEV uint32_t block_sum(uint32_t v, uint32_t* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) t += scratch[i];
  return t;
}
// Block exclusive scan; returns the exclusive prefix, *total = block sum.
SDA_DEV uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
  uint32_t inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 63) scratch[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    uint32_t s = scratch[i];
    if (i < w) base += s;
    tot += s;
  }
  *total = tot;
  return base + inc - v;
}

}  // namespace sdagpu
