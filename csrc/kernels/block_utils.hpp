// Workgroup-level reductions / scans for 256-thread (4 x wave64) blocks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_crypto.hpp"

namespace sdagpu {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// Cross-lane moves on the VALU (DPP), not through LDS: a ds_bpermute queues behind
// every LDS instruction the wave has in flight (the decode kernel's 64 accumulator
// adds, the MAC kernels' digit-sum adds) and its result has to be waited for.
// `old` is what a lane without a source (or in a masked row) receives.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_move(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xf, false);
}
constexpr int kDppRowShr = 0x110;     // row_shr:n = kDppRowShr + n (rows of 16 lanes)
constexpr int kDppWaveShr1 = 0x138;   // lane l <- lane l - 1 over the whole wave
constexpr int kDppBcast15 = 0x142;    // lane 15 of a row -> the next row
constexpr int kDppBcast31 = 0x143;    // lane 31 -> lanes 32..63

// Inclusive prefix sum within each row of 16 lanes (lane 15 of a row: the row's sum).
__device__ __forceinline__ uint32_t row16_incl_scan(uint32_t v) {
  v += dpp_move<kDppRowShr + 1>(0u, v);
  v += dpp_move<kDppRowShr + 2>(0u, v);
  v += dpp_move<kDppRowShr + 4>(0u, v);
  v += dpp_move<kDppRowShr + 8>(0u, v);
  return v;
}
// Inclusive wave prefix sum.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v = row16_incl_scan(v);
  v += dpp_move<kDppBcast15, 0xa>(0u, v);  // rows 1 and 3 += sums of rows 0 and 2
  v += dpp_move<kDppBcast31, 0xc>(0u, v);  // rows 2 and 3 += sum of rows 0 and 1
  return v;
}
// Value of lane `l` on every lane (wave-uniform).
__device__ __forceinline__ uint32_t wave_read_lane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
// Lane l gets lane l - 1's value, lane 0 gets `first`.
__device__ __forceinline__ uint32_t wave_shift_up1(uint32_t v, uint32_t first) {
  return dpp_move<kDppWaveShr1>(first, v);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  return wave_read_lane(wave_incl_scan(v), 63);
}
// Block sum; result valid in every thread. `scratch` holds kWaves words.
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* scratch) {
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
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
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
