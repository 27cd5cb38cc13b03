// How much of the encode kernel's time is its data movement, and which lane <-> value layout
// moves it fastest (gfx950)? A workgroup of 256 threads turns a tile of 8192 32-bit values into
// 8192 three-byte codes in LDS (byte stores, as the encoder's), runs `rounds` double rounds of
// Salsa-like add-rotate-xor work per 64 bytes on the tile, and stores its 24 KiB with 16-byte
// writes. No cryptography here: the codes are fixed-length and the "keystream" is a stand-in with
// the instruction mix of the real one.
//   layout 0: a lane owns 32 consecutive values (8 x 16-byte loads 128 bytes apart from the
//             next lane's; byte stores 96 bytes apart: 4 of the 32 LDS banks)
//   layout 1: a lane owns 8 groups of 4 consecutive values, group q = values 256 q + 4 lane of
//             its wave's 2048 (loads coalesced; byte stores 12 bytes apart: all banks)
//   hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops scripts/ubench_scatter.hip -o /tmp/ubench_scatter && /tmp/ubench_scatter
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int kBlock = 256;
constexpr int kTile = 8192;          // values per workgroup
constexpr int kTileBytes = 3 * kTile;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }

template <int kLayout>
__global__ void __launch_bounds__(kBlock) k_tile(const uint32_t* __restrict__ vals, uint8_t* __restrict__ out,
                                                 int rounds, int stores) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTileBytes + 128];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t* src = vals + (size_t)blockIdx.x * kTile;
  uint32_t v[32];
  if constexpr (kLayout == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(src + tid * 32);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 d = p[q];
      v[4 * q] = d.x; v[4 * q + 1] = d.y; v[4 * q + 2] = d.z; v[4 * q + 3] = d.w;
    }
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(src + wave * 2048 + lane * 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 d = p[q * 64];
      v[4 * q] = d.x; v[4 * q + 1] = d.y; v[4 * q + 2] = d.z; v[4 * q + 3] = d.w;
    }
  }
  if (stores) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t pos = kLayout == 0 ? 96u * tid + 3u * i
                                        : 6144u * wave + 768u * (i >> 2) + 12u * lane + 3u * (i & 3);
      const uint32_t z = v[i] << 1;
      lds[pos] = (uint8_t)(z | 0x80u);
      lds[pos + 1] = (uint8_t)((z >> 7) | 0x80u);
      lds[pos + 2] = (uint8_t)(z >> 14);
    }
  } else {
    // no scatter: keep the loads alive
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) x ^= v[i];
    if (x == 0x12345678u) lds[tid] = 1;
  }
  __syncthreads();
  // 384 blocks of 64 bytes over 256 threads, as in the encoder
  for (int blk = tid; blk < kTileBytes / 64; blk += kBlock) {
    uint4* q = reinterpret_cast<uint4*>(lds + 64 * blk);
    uint32_t w[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) w[u] = 0x9e3779b9u * (blk + u + 1);
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint32_t &a = w[c], &b = w[4 + ((c + h) & 3)], &cc = w[8 + ((c + 2 * h) & 3)], &d = w[12 + ((c + 3 * h) & 3)];
          b ^= rotl(a + d, 7);
          cc ^= rotl(b + a, 9);
          d ^= rotl(cc + b, 13);
          a ^= rotl(d + cc, 18);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint4 d = q[u];
      d.x ^= w[4 * u]; d.y ^= w[4 * u + 1]; d.z ^= w[4 * u + 2]; d.w ^= w[4 * u + 3];
      q[u] = d;
    }
  }
  __syncthreads();
  uint8_t* dst = out + (size_t)blockIdx.x * kTileBytes;
  for (int c = 16 * tid; c < kTileBytes; c += 16 * kBlock)
    *reinterpret_cast<uint4*>(dst + c) = *reinterpret_cast<const uint4*>(lds + c);
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 122000;  // ~1e9 values, 3 GB out
  uint32_t* vals;
  uint8_t* out;
  (void)hipMalloc(&vals, (size_t)tiles * kTile * 4);
  (void)hipMalloc(&out, (size_t)tiles * kTileBytes);
  (void)hipMemset(vals, 0x5a, (size_t)tiles * kTile * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rounds : {0, 10}) {
    for (int stores : {0, 1}) {
      for (int layout : {0, 1}) {
        float best = 1e9f;
        for (int rep = 0; rep < 4; ++rep) {
          (void)hipEventRecord(e0);
          if (layout == 0) hipLaunchKernelGGL(k_tile<0>, dim3(tiles), dim3(kBlock), 0, 0, vals, out, rounds, stores);
          else hipLaunchKernelGGL(k_tile<1>, dim3(tiles), dim3(kBlock), 0, 0, vals, out, rounds, stores);
          (void)hipEventRecord(e1);
          (void)hipEventSynchronize(e1);
          float ms = 0;
          (void)hipEventElapsedTime(&ms, e0, e1);
          if (rep > 0 && ms < best) best = ms;
        }
        printf("double rounds %2d  byte scatter %d  layout %d: %.3f ms  (%.2f TB/s in + out)\n", rounds, stores, layout,
               best, (double)tiles * (kTile * 4 + kTileBytes) / best / 1e9);
        fflush(stdout);
      }
    }
  }
  return 0;
}
