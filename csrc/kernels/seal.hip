// Sealed-box bulk kernels: varint encode + XSalsa20 encrypt, and the parallel
// Poly1305 MAC (optionally fused with in-place decryption + varint terminator
// counting for the clerk/recipient side).
//
// Reference: sodium.rs:36-43 (encode each share with zigzag LEB128, then
// sealedbox::seal) and sodium.rs:78-89 (open, then decode until exhausted).
//
// Parallel Poly1305: a message is cut into 16 KiB chunks aligned to the keystream
// (chunk k covers keystream bytes [kC, (k+1)C), i.e. message bytes
// [kC-32, (k+1)C-32)). A middle chunk is 1024 full blocks, taken as 16 interleaved
// rows (row i = blocks i, i + 16, i + 32, ...: the 16 lanes of an MFMA operand
// group read 256 contiguous bytes) of an int8 GEMM against the message's weight
// digits on the matrix cores (v_mfma_i32_16x16x64_i8; the algebra is in
// device_crypto.hpp, poly_seg_value); a message's first and last chunk (message
// start, partial final block) are summed by per-lane Horner over 4 blocks. Row
// values are placed by r^(16 - i), Horner lane sums by r^(4(255-t)), and a
// per-message pass chains the chunk partials with r^(C/16).
#include "block_utils.hpp"
#include "device_crypto.hpp"
#include "encode_units.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));  // one i8 MFMA operand fragment (16 bytes)

constexpr int kValuesPerLane = kEncodeValues / kBlock;  // 32

// Index of a message's last chunk (chunk k covers message bytes [kC - 32, (k+1)C - 32)).
SDA_DEV int last_chunk(uint32_t N) { return (int)(((int64_t)N + 31) / kChunkBytes); }

// 16 bytes from an address that is only aligned to the value type: message rows
// start at j * L values, which is 16-byte aligned only for some L. The target's
// unaligned access mode (the HSA default) lets this be one global_load_dwordx4.
struct __attribute__((packed, aligned(1))) Vec16 {
  uint4 v;
};

template <typename VT>
SDA_DEV void load_values(uint32_t (&v)[kValuesPerLane], const VT* src, int e0, int L) {
  if (e0 + kValuesPerLane <= L) {
    const Vec16* p = reinterpret_cast<const Vec16*>(src + e0);
    if constexpr (sizeof(VT) == 1) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint4 d = p[q].v;
        const uint32_t ws[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int b = 0; b < 4; ++b) v[16 * q + 4 * u + b] = (ws[u] >> (8 * b)) & 0xffu;
        }
      }
    } else if constexpr (sizeof(VT) == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 d = p[q].v;
        const uint32_t ws[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[8 * q + 2 * u] = ws[u] & 0xffffu;
          v[8 * q + 2 * u + 1] = ws[u] >> 16;
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 d = p[q].v;
        v[4 * q] = d.x; v[4 * q + 1] = d.y; v[4 * q + 2] = d.z; v[4 * q + 3] = d.w;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) v[i] = (e0 + i < L) ? (uint32_t)src[e0 + i] : 0u;
  }
}

// One block per (tile of kEncodeValues values, message): lanes varint-encode 32
// values each into LDS at scanned offsets, every lane then XORs (about) one
// 64-byte XSalsa20 block in place, and the tile is stored with 16-byte writes
// (byte writes only at the two tile edges shared with neighbouring tiles).
//
// MAC: while the ciphertext is still in LDS the block adds the tile's share of the
// Poly1305 partials of the message's middle chunks (the first and the last chunk
// are k_mac_horner's). Poly1305 is linear in the message bytes, so a 16 KiB chunk
// cut by tile borders is the sum of what each tile sees of it, with the bytes
// outside the tile read as zero; a block's pad bit 2^128 belongs to the tile that
// holds the block's first byte. LDS index x is keystream byte 64 b0 + x, i.e. the
// 16-byte Poly1305 blocks sit on 16-byte LDS boundaries. Rows are interleaved (row
// i = blocks i, i + 16, ... of the chunk; tables: kernels.hpp), so the 16 lanes of
// an MFMA operand group read 256 contiguous bytes:
//   row value  = (sum_pos u_pos W(pos) + row constant + pad bits of the owned blocks)
//   chunk part = sum_i row value_i * r^(16 - i)     (relative to the chunk's end, as
//                                                    k_mac_chunks' middle chunks are)
// kMaxB: the longest code the caller's values can have (u8 / u16 storage: 3, or 2 for
// 16-bit values below 2^13; u32: 3 for values below 2^20, 4 below 2^27, else 5). It sizes
// the tile's LDS -- 16 / 24 / 32 / 40 KB, i.e. eight / six / four / three workgroups a CU; the issue-bound kernel ran at 57 % of its
// VALU peak with three -- and a value past the bound (a caller's error: the slots of
// the arena are sized by the same bound) is encoded as zero rather than overrun it.
template <typename VT, bool MAC, int kMaxB>
__global__ void __launch_bounds__(kBlock)
    k_encode_encrypt(int L, int M, const VT* __restrict__ vals, const uint32_t* __restrict__ tile_off,
                     const MsgKey* __restrict__ keys, uint8_t* __restrict__ ct, uint64_t stride,
                     const uint32_t* __restrict__ pows, const uint32_t* __restrict__ pt_len,
                     uint32_t* __restrict__ partials, int K) {
  static_assert(kMaxB >= 2 && kMaxB <= 5 && (sizeof(VT) > 2 || kMaxB <= 3) &&
                (kMaxB > 2 || (sizeof(VT) == 2 && !MAC)), "code length bound");
  constexpr uint32_t kBound = kMaxB == 5 ? 0xffffffffu : (1u << (7 * kMaxB - 1)) - 1u;  // largest value
  // Five-byte codes: the tile goes through LDS in two passes, the first two waves' values and
  // then the other two's (all four waves on the keystream and the stores of either pass), so
  // that LDS holds half a tile, 21 KB instead of 41, and five workgroups fit a CU instead of
  // three: 4.45 -> 4.03 ms for 1000 boxes of a million values below 2^31. Not for four-byte
  // codes (33 KB, four workgroups a CU in one pass): the extra barriers and the passes with two
  // waves scattering cost what the fifth workgroup gives (1.07 against 1.10 ms).
  constexpr int kPasses = (!MAC && kMaxB >= 5) ? 2 : 1;
  constexpr int kPassWaves = kWaves / kPasses;
  // a wave's part of the tile where the waves work on their own (below)
  constexpr int kWaveBytes = kEncodeValues / kWaves * kMaxB + 128;  // as a tile: room for the offset in the first block
  __shared__ __attribute__((aligned(16))) uint8_t tile[kPassWaves * kWaveBytes];
  __shared__ uint32_t scratch[kWaves];
  // chunks a tile can touch: its bytes span at most 2 + (tile bytes - 2) / chunk bytes
  constexpr int kSlots = sizeof(VT) <= 2 ? 3 : 4;
  __shared__ int32_t cacc[MAC ? kSlots : 1][16][kPolyDigits + 1];
  if constexpr (MAC) {
    int32_t* flat = &cacc[0][0][0];
    for (int i = threadIdx.x; i < kSlots * 16 * (kPolyDigits + 1); i += kBlock) flat[i] = 0;
  }
  const int T = (L + kTileValues - 1) / kTileValues;  // count tiles per message
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  // Workgroup -> (tile, message): first every message's whole tiles, then the ends
  // (encode_units.hpp). Workgroups go round-robin over the 8 XCDs; with the tile index fastest
  // in the grid, messages of two tiles -- a whole one and a short end, the boxes of
  // the many-clerk rounds -- sent every whole tile to the even XCDs and every end to the odd
  // ones, which then stood idle: the kernel took as long as half the chip needs for the whole
  // tiles (3.0 ps a value for boxes of 10,000 values, 2.2 for boxes of ten whole tiles).
  // Short ends: where a message's end has no more than a wave's 2048 values, a workgroup takes
  // the ends of four messages, a wave each, instead of keeping an LDS tile and four wave slots
  // busy with one or two waves at work (another 6 %: 2.45 -> 2.30 ps). `un` threads numbered
  // `tid` work on one tile: the workgroup's 256, or a wave's 64.
  const EncodeUnit unit = encode_unit(MAC, M, L, (int)blockIdx.x, wave);
  const bool ends = unit.ends, idle = unit.idle;  // block-uniform; a wave without a message: no values, stores nothing
  const int t = unit.tile, j = unit.msg;
  const int tid = ends ? lane : (int)threadIdx.x;
  const int un = ends ? 64 : kBlock;
  uint8_t* lds = ends ? tile + (wave % kPassWaves) * kWaveBytes : tile;
  const int Lv = idle ? t * kEncodeValues : L;  // the values this unit sees
  const int e0 = t * kEncodeValues + tid * kValuesPerLane;
  const VT* src = vals + (size_t)j * L;
  // the tile's offset and the message's key: uniform loads, asked for here so that they arrive
  // with the values instead of each costing the workgroup a memory latency of its own later
  const uint32_t a_tile = tile_off[(size_t)j * T + t * (kEncodeValues / kTileValues)];
  const MsgKey key = keys[j];
  // full: all 32 values present (the lane's values are then in registers); a tile's
  // last lane with values takes the rolled loops below, straight from memory, and
  // the lanes past the message's end (most of a short message's last tile) nothing
  const bool full = e0 + kValuesPerLane <= Lv;
  // The message's last values, fewer than a lane's 32: spread one by one over the lanes from the
  // first one without its 32 on, which have nothing else to do (more than one each only where
  // that lane sits at the very end of a tile). Lanes are scanned in order, so the bytes land
  // where they belong. One lane walking up to 31 values through two rolled loops of dependent
  // loads kept its whole workgroup, LDS tile and all, on the CU for ~20 us: as long as a full
  // tile takes, for every box whose length is no multiple of 32.
  int eg = e0, nv = kValuesPerLane;
  if (!full) {
    const int left = Lv - t * kEncodeValues;     // this tile's values (< kEncodeValues here)
    const int tl = left / kValuesPerLane;        // first lane without its 32: tid >= tl
    const int nt = left - tl * kValuesPerLane;   // 0..31 values for lanes tl..un-1
    const int c = (nt + (un - tl) - 1) / (un - tl);
    const int r = tid - tl;
    eg = t * kEncodeValues + tl * kValuesPerLane + r * c;
    nv = max(0, min(c, nt - r * c));
  }
  uint32_t v[kValuesPerLane];            // the lane's values (u8 / u32 storage)
  uint32_t pr[kValuesPerLane / 2] = {};  // u16 storage: the lane's values as pairs, as loaded
  // Fast lanes (all 32 values present and < 2^13, i.e. 1- or 2-byte varints of
  // non-negative values) encode branch-free; other lanes take the generic path.
  bool fast;
  // Middle lanes (all 32 values present and < 2^27: varints of up to four bytes, the
  // large packed-Shamir fields) encode branch-free too, 32-bit arithmetic only.
  bool mid = false;
  bool mid3 = false;  // ... all < 2^20: at most three bytes (fields below 2^20, u16 storage)
  uint32_t my_bytes = 0;
  if constexpr (sizeof(VT) == 2) {
    // u16 pairs stay packed: both halves of a dword are handled by one
    // instruction (v < 2^13, so no step carries from the low half into the high)
    uint32_t orp = 0;
    if (full) {
      const Vec16* p = reinterpret_cast<const Vec16*>(src + e0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 d = p[q].v;
        pr[4 * q] = d.x; pr[4 * q + 1] = d.y; pr[4 * q + 2] = d.z; pr[4 * q + 3] = d.w;
      }
#pragma unroll
      for (int k = 0; k < kValuesPerLane / 2; ++k) orp |= pr[k];
    }
    if (kMaxB == 2 && (orp & 0xe000e000u) != 0u) {  // past the bound: never with canonical values
#pragma unroll
      for (int k = 0; k < kValuesPerLane / 2; ++k) pr[k] = 0;
      orp = 0;
    }
    fast = full && (orp & 0xe000e000u) == 0u;
    if (fast) {
      my_bytes = kValuesPerLane;  // + one per value >= 64 (bit 15 of half + 0x7fc0)
#pragma unroll
      for (int k = 0; k < kValuesPerLane / 2; ++k)
        my_bytes += (uint32_t)__popc((pr[k] + 0x7fc07fc0u) & 0x80008000u);
    }
    mid = mid3 = !fast && full;
  } else {
    uint32_t orv = 0;
    if (full) {
      load_values<VT>(v, src, e0, L);
#pragma unroll
      for (int i = 0; i < kValuesPerLane; ++i) orv |= v[i];
      if (kMaxB < 5 && orv > kBound) {  // never with canonical values
#pragma unroll
        for (int i = 0; i < kValuesPerLane; ++i) v[i] = 0;
        orv = 0;
      }
    }
    fast = full && orv < 8192u;
    if (fast) {
#pragma unroll
      for (int i = 0; i < kValuesPerLane; ++i) my_bytes += 1u + (v[i] >= 64u);
    }
    mid = !fast && full && (kMaxB < 5 || orv < (1u << 27));
    mid3 = mid && (kMaxB == 3 || orv < (1u << 20));
  }
  // value i of the lane on the generic paths
  auto val = [&](int i) -> uint32_t {
    if constexpr (sizeof(VT) == 2) return (pr[i >> 1] >> (16 * (i & 1))) & 0xffffu;
    else return v[i];
  };
  if (mid3) {
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint32_t z = val(i) << 1;
      my_bytes += 1u + (z >= (1u << 7)) + (z >= (1u << 14));
    }
  } else if (mid) {
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint32_t z = val(i) << 1;
      my_bytes += 1u + (z >= (1u << 7)) + (z >= (1u << 14)) + (z >= (1u << 21));
    }
  } else if (kMaxB == 5 && !fast && full) {
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint64_t z = (uint64_t)val(i) << 1;
      my_bytes += 1u + (z >= (1ull << 7)) + (z >= (1ull << 14)) + (z >= (1ull << 21)) + (z >= (1ull << 28));
    }
  } else if (!fast) {
#pragma unroll 1
    for (int i = 0; i < nv; ++i) {
      const uint32_t x = (uint32_t)src[eg + i];
      const uint64_t z = (uint64_t)(x > kBound ? 0u : x) << 1;
      my_bytes += 1u + (z >= (1ull << 7)) + (z >= (1ull << 14)) + (z >= (1ull << 21)) + (z >= (1ull << 28));
    }
  }
  // byte offsets within the tile: a scan over the wave, and over the waves before it where
  // the workgroup shares the tile
  const uint32_t inc = wave_incl_scan(my_bytes);
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  uint32_t wsum[kWaves], before = 0;  // the waves' bytes; those of the waves before this one
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    wsum[i] = scratch[i];
    if (i < wave) before += wsum[i];
  }
#pragma unroll 1
  for (int pass = 0; pass < kPasses; ++pass) {
  // `mine`: this wave's values are in this pass (wave-uniform); `work`: it takes part in the
  // pass's keystream and stores (a wave on its own message end: only in its own pass)
  const bool mine = kPasses == 1 || wave / kPassWaves == pass;
  const bool work = !ends || mine;
  uint32_t pass_before = 0, pass_bytes = 0;  // of the shared tile: bytes before this pass, and in it
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    if (i < pass * kPassWaves) pass_before += wsum[i];
    else if (i < (pass + 1) * kPassWaves) pass_bytes += wsum[i];
  }
  const uint32_t a = ends ? a_tile : a_tile + pass_before;  // message byte where this pass's bytes begin
  const uint32_t tile_bytes = ends ? wsum[wave] : pass_bytes;
  const uint32_t b0 = (32u + a) >> 6;
  const uint32_t base = 32u + a - 64u * b0;  // LDS index of message byte `a`
  uint32_t pos = base + (ends ? 0u : before - pass_before) + inc - my_bytes;
  if (mine) {
  if constexpr (kPasses > 1) {
    // keeps the compiler from computing every code byte of both passes ahead of the loop
    // (256 registers and one wave a SIMD): the values "change" here
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) asm volatile("" : "+v"(v[i]));
  }
  if (fast) {
    if constexpr (sizeof(VT) == 2) {
      // Per pair: both 16-bit codes (byte 0 = low 7 bits of z = 2 v plus the
      // continuation flag, byte 1 = z >> 7) by packed shifts and masks, then byte
      // stores (unaligned 16-bit LDS stores work but measured at about half the
      // rate of two byte stores). A one-byte value's second byte (zero) is
      // overwritten by the next value of the lane (same lane, LDS program order);
      // the lane's last value stores exactly its length.
#pragma unroll
      for (int k = 0; k < kValuesPerLane / 2; ++k) {
        uint32_t c2, f;  // both 16-bit codes; bit 16 h: value h takes two bytes
        varint_pair16(pr[k], c2, f);
        lds[pos + 2 * k] = (uint8_t)c2;
        lds[pos + 2 * k + 1] = (uint8_t)(c2 >> 8);
        pos += f & 0xffffu;
        lds[pos + 2 * k + 1] = (uint8_t)(c2 >> 16);
        if (k + 1 < kValuesPerLane / 2 || (f >> 16)) lds[pos + 2 * k + 2] = (uint8_t)(c2 >> 24);
        pos += f >> 16;
      }
    } else {
      // each value stores both candidate bytes and the next value overwrites the
      // second one when the varint was a single byte
#pragma unroll
      for (int i = 0; i < kValuesPerLane; ++i) {
        const uint32_t z = v[i] << 1;
        const uint32_t l2 = v[i] >= 64u;
        lds[pos] = (uint8_t)((z & 0x7fu) | (l2 << 7));
        if (i + 1 < kValuesPerLane || l2) lds[pos + 1] = (uint8_t)(z >> 7);
        pos += 1u + l2;
      }
    }
  } else if (mid3) {
    // as below, three candidate bytes
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint32_t z = val(i) << 1;
      const uint32_t l1 = z >= (1u << 7), l2 = z >= (1u << 14);
      lds[pos] = (uint8_t)((z & 0x7fu) | (l1 << 7));
      if (i + 1 < kValuesPerLane || l1) lds[pos + 1] = (uint8_t)(((z >> 7) & 0x7fu) | (l2 << 7));
      if (i + 2 < kValuesPerLane || l2) lds[pos + 2] = (uint8_t)(z >> 14);
      pos += 1u + l1 + l2;
    }
  } else if (mid) {
    // every value stores its four candidate bytes; what lies past its length is
    // overwritten by the following values of the lane (each at least one byte), so
    // byte k is stored unconditionally only where k more values follow
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint32_t z = val(i) << 1;
      const uint32_t l1 = z >= (1u << 7), l2 = z >= (1u << 14), l3 = z >= (1u << 21);
      lds[pos] = (uint8_t)((z & 0x7fu) | (l1 << 7));
      if (i + 1 < kValuesPerLane || l1) lds[pos + 1] = (uint8_t)(((z >> 7) & 0x7fu) | (l2 << 7));
      if (i + 2 < kValuesPerLane || l2) lds[pos + 2] = (uint8_t)(((z >> 14) & 0x7fu) | (l3 << 7));
      if (i + 3 < kValuesPerLane || l3) lds[pos + 3] = (uint8_t)(z >> 21);
      pos += 1u + l1 + l2 + l3;
    }
  } else if (kMaxB == 5 && full) {
#pragma unroll
    for (int i = 0; i < kValuesPerLane; ++i) {
      const uint64_t z = (uint64_t)val(i) << 1;
      const uint32_t len = 1u + (z >= (1ull << 7)) + (z >= (1ull << 14)) + (z >= (1ull << 21)) + (z >= (1ull << 28));
#pragma unroll
      for (int q = 0; q < 5; ++q)
        if ((uint32_t)q < len)
          lds[pos + q] = (uint8_t)(((z >> (7 * q)) & 0x7f) | ((uint32_t)q + 1 < len ? 0x80u : 0u));
      pos += len;
    }
  } else {
#pragma unroll 1
    for (int i = 0; i < nv; ++i) {
      const uint32_t x = (uint32_t)src[eg + i];
      const uint64_t z = (uint64_t)(x > kBound ? 0u : x) << 1;
      const uint32_t len = 1u + (z >= (1ull << 7)) + (z >= (1ull << 14)) + (z >= (1ull << 21)) + (z >= (1ull << 28));
#pragma unroll
      for (int q = 0; q < 5; ++q)
        if ((uint32_t)q < len)
          lds[pos + q] = (uint8_t)(((z >> (7 * q)) & 0x7f) | ((uint32_t)q + 1 < len ? 0x80u : 0u));
      pos += len;
    }
  }
  }  // mine
  __syncthreads();
  // MAC operands that depend only on the tile's position: requested here, so that
  // their latency is spent under the keystream computation
  const int row = lane & 15, g = lane >> 4;
  const uint32_t ks0 = 32u + a, ks1 = ks0 + tile_bytes;  // the tile's keystream byte range
  const int kf = (int)(ks0 / kChunkBytes), kl = (int)((ks1 - 1u) / kChunkBytes);
  int last = 0;
  bool any = false;
  v4i wb0[4], wb1[4];
  P130 krow = p130_zero(), rfac = p130_zero();
  if constexpr (MAC) {
    last = last_chunk(pt_len[j]);
    for (int k = kf; k <= kl; ++k) any = any || (k != 0 && k < last);  // block-uniform
    if (any) {
      const uint32_t* pw = pows + (size_t)j * kPowWords;
      // this wave's K-slice of the message's weight digits (columns `row`, 16 + `row`)
      const int8_t* tab = reinterpret_cast<const int8_t*>(pw + kPowTabOff);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int q = 4 * wave + qq;
        wb0[qq] = *reinterpret_cast<const v4i*>(tab + row * kSegBytes + 64 * q + 16 * g);
        wb1[qq] = v4i{0, 0, 0, 0};
        if (row < kPolyDigits - 16)
          wb1[qq] = *reinterpret_cast<const v4i*>(tab + (16 + row) * kSegBytes + 64 * q + 16 * g);
      }
      if (wave == 0) {  // lane (slot g, row): constant and factor of its row value
        const int k = kf + g;
        int T0, T1;  // the row owns the pad bits of its blocks row + 16 t, t in [T0, T1)
        poly_row_owned((int64_t)ks0, (int64_t)ks1, (int64_t)k * kChunkBytes, row, T0, T1);
        krow = poly_row_const(pw + kPowKsegOff, pw + kPowQOff + T0 * 5, pw + kPowQOff + T1 * 5);
        const uint32_t* rf = pw + kPowRowOff + row * 5;
        rfac = P130{{rf[0], rf[1], rf[2], rf[3], rf[4]}};
      }
    }
  }
  // what the message's blocks have in common of their first double round (scalar unit)
  const SalsaPrefix pre = salsa20_prefix(key.subkey, key.nonce[0], key.nonce[1]);
  const uint32_t nblk = work ? (base + tile_bytes + 63) >> 6 : 0u;
  for (uint32_t blk = tid; blk < nblk; blk += un) {
    uint32_t w[16];
    salsa20_block(w, pre, key.subkey, key.nonce[0], key.nonce[1], b0 + blk);
    uint4* q = reinterpret_cast<uint4*>(lds + 64 * blk);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint4 d = q[u];
      d.x ^= w[4 * u]; d.y ^= w[4 * u + 1]; d.z ^= w[4 * u + 2]; d.w ^= w[4 * u + 3];
      q[u] = d;
    }
    if constexpr (MAC) {
      // the MAC reads whole 16-byte blocks: clear what the two edge blocks hold of
      // the neighbouring tiles' positions (same thread as the XOR above, so in order)
      const uint32_t v1 = base + tile_bytes;
      if (blk == 0)
        for (uint32_t x = base & ~15u; x < base; ++x) lds[x] = 0;
      if (blk == (v1 >> 6))
        for (uint32_t x = v1; x < ((v1 + 15u) & ~15u); ++x) lds[x] = 0;
    }
  }
  __syncthreads();
  // From here the block only drains (stores, MAC): ahead of the waves of other blocks
  // that are still in their keystream loop, so that its LDS and wave slots free up
  if constexpr (MAC) __builtin_amdgcn_s_setprio(3);
  uint8_t* gmsg = ct + (size_t)j * stride + 48;
  const uint32_t lo = a & ~15u, hi = work ? (a + tile_bytes + 15u) & ~15u : 0u, end = a + tile_bytes;
  for (uint32_t c = lo + 16u * tid; c < hi; c += 16u * un) {
    if (c >= a && c + 16u <= end) {
      *reinterpret_cast<uint4*>(gmsg + c) = *reinterpret_cast<const uint4*>(lds + (c - a + base));
    } else {
      for (uint32_t q = 0; q < 16; ++q) {
        const uint32_t p = c + q;
        if (p >= a && p < end) gmsg[p] = lds[p - a + base];
      }
    }
  }
  if constexpr (MAC) {
    if (!any) return;  // block-uniform
    {
      const int32_t v0a = (int32_t)(base & ~15u), v1a = (int32_t)((base + tile_bytes + 15u) & ~15u);
      for (int k = kf; k <= kl; ++k) {
        if (k == 0 || k >= last) continue;
        // LDS index of the chunk's first keystream byte (negative: starts before the tile)
        const int32_t xc = (int32_t)((uint32_t)k * kChunkBytes - 64u * b0);
        v4i acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int t = 4 * (4 * wave + qq) + g;  // block row + 16 t of the chunk
          const int32_t x = xc + 16 * row + 256 * t;
          v4i piece = {0, 0, 0, 0};
          if (x >= v0a && x < v1a) piece = *reinterpret_cast<const v4i*>(lds + x);
          piece ^= (int)0x80808080;  // bytes u -> u - 128 (signed)
          acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(piece, wb0[qq], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(piece, wb1[qq], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          atomicAdd(&cacc[k - kf][4 * g + i][row], acc0[i]);
          if (row < kPolyDigits - 16) atomicAdd(&cacc[k - kf][4 * g + i][16 + row], acc1[i]);
        }
      }
    }
    __syncthreads();
    // Row values -> chunk part: lane (slot g, row) of the first wave
    if (wave != 0) return;
    const int k = kf + g;
    const bool mid = g < kSlots && k <= kl && k != 0 && k < last && k < K;
    P130 h = p130_zero();
    if (mid) {
      int32_t c[kPolyDigits];
#pragma unroll
      for (int d = 0; d < kPolyDigits; ++d) c[d] = cacc[g][row][d];
      h = p130_mul(poly_seg_value(c, krow), rfac);
    }
    uint64_t d[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      d[u] = h.v[u];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) d[u] += __shfl_xor(d[u], o, 64);
    }
    if (mid && row == 0) {
      uint64_t cc;
      cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
      cc = d[1] >> 26; d[1] &= kM26; d[2] += cc;
      cc = d[2] >> 26; d[2] &= kM26; d[3] += cc;
      cc = d[3] >> 26; d[3] &= kM26; d[4] += cc;
      cc = d[4] >> 26; d[4] &= kM26; d[0] += cc * 5;
      cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
      // up to three tiles add to one chunk: limbs stay below 2^28
      uint32_t* part = partials + ((size_t)j * K + k) * 8;
#pragma unroll
      for (int u = 0; u < 5; ++u) atomicAdd(&part[u], (uint32_t)d[u]);
    }
  }
  if (pass + 1 < kPasses) __syncthreads();  // the next pass overwrites the tile
  }  // pass
}

// `err` (may be null): a row whose sum is not `expect` raises kErrMalformed there.
__global__ void __launch_bounds__(kBlock) k_segscan(int T, uint32_t* __restrict__ data,
                                                    uint32_t* __restrict__ totals, uint32_t expect,
                                                    uint32_t* err) {
  __shared__ uint32_t scratch[kWaves];
  uint32_t* row = data + (size_t)blockIdx.x * T;
  uint32_t carry = 0;
  for (int b = 0; b < T; b += kBlock) {
    const int i = b + threadIdx.x;
    uint32_t v = i < T ? row[i] : 0u;
    uint32_t tot;
    uint32_t ex = block_excl_scan(v, scratch, &tot);
    if (i < T) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && totals) totals[blockIdx.x] = carry;
  if (threadIdx.x == 0 && err && carry != expect) atomicOr(err, kErrMalformed);
}

// Read 16 ciphertext bytes as a Poly1305 block (block index i of a message of N
// bytes at gmsg; a partial final block reads into the slot padding).
SDA_DEV P130 block_from(const uint4 q, int64_t i, uint32_t N) {
  uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t hibit = 1u << 24;
  const int64_t rem = (int64_t)N - 16 * i;
  if (rem < 16) {
    // partial final block: keep `rem` bytes, append 0x01, zero the rest
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int wi = b >> 2, sh = (b & 3) * 8;
      uint32_t byte = (w[wi] >> sh) & 0xff;
      uint32_t nb = b < rem ? byte : (b == rem ? 1u : 0u);
      w[wi] = (w[wi] & ~(0xffu << sh)) | (nb << sh);
    }
    hibit = 0;
  }
  return p130_block(w[0], w[1], w[2], w[3], hibit);
}
SDA_DEV P130 load_block(const uint8_t* gmsg, int64_t i, uint32_t N) {
  return block_from(*reinterpret_cast<const uint4*>(gmsg + 16 * i), i, N);
}

// r^(4 * (255 - t)) for t = 0..255, per message: the factor that places lane t's
// 4-block Horner sum at its distance from the chunk end. Computed once per
// message (it depends only on the key), so a chunk's combine is one multiply
// per lane plus a sum -- instead of an 8-level multiply tree per chunk.
SDA_DEV uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block sum of P130 values (limbs < 2^28) -> carried P130 on every thread.
SDA_DEV P130 block_sum_p130(const P130& h, uint64_t (*red)[kWaves]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();  // red reuse
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const uint64_t s = wave_sum64((uint64_t)h.v[u]);
    if (lane == 0) red[u][wave] = s;
  }
  __syncthreads();
  uint64_t d[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    d[u] = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) d[u] += red[u][w];
  }
  uint64_t c;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  c = d[1] >> 26; d[1] &= kM26; d[2] += c;
  c = d[2] >> 26; d[2] &= kM26; d[3] += c;
  c = d[3] >> 26; d[3] &= kM26; d[4] += c;
  c = d[4] >> 26; d[4] &= kM26; d[0] += c * 5;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  return P130{{(uint32_t)d[0], (uint32_t)d[1], (uint32_t)d[2], (uint32_t)d[3], (uint32_t)d[4]}};
}

// Per-message Poly1305 tables (layout: kernels.hpp kPow*):
//  * r^(4 (255 - t)) for t = 0..255: the factor that places lane t's 4-block
//    Horner sum at its distance from the chunk end (k_mac_horner);
//  * for the matrix-core rows: the 7-bit digits of the weights W(16 t + a), the
//    row constant, the row factors r^(16 - i) and the pad-bit prefix sums
//    (device_crypto.hpp, poly_seg_value / poly_row_const).
// Depends only on the key: computed once per message on the side stream.
// full == 0: only the Horner factors (messages of at most two chunks have no
// middle chunk, so nothing reads the matrix-core tables: 5 KB instead of 26 KB per
// message, which matters for the many-clerk sets' hundreds of thousands of boxes).
__global__ void __launch_bounds__(kBlock)
    k_poly_powers(const MsgKey* __restrict__ keys, uint32_t* __restrict__ pows, int prio, int full) {
  if (prio) __builtin_amdgcn_s_setprio(3);  // side-stream key work (see k_seal_setup)
  __shared__ P130 rp[64];
  __shared__ uint64_t red[5][kWaves];
  const int j = blockIdx.x, t = threadIdx.x;
  const MsgKey key = keys[j];
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  uint32_t* base = pows + (size_t)j * kPowWords;
  {
    P130 r4 = p130_mul(r, r);
    r4 = p130_mul(r4, r4);
    const P130 f = p130_carry(p130_pow(r4, (uint32_t)(kBlock - 1 - t)));
#pragma unroll
    for (int u = 0; u < 5; ++u) base[t * 5 + u] = f.v[u];
  }
  if (!full) return;  // block-uniform
  // R^(63 - t), R = r^16, for the blocks i + 16 t of a row
  P130 mine = p130_zero();
  if (t < 64) {
    P130 r16 = p130_mul(r, r);
    r16 = p130_mul(r16, r16);
    r16 = p130_mul(r16, r16);
    r16 = p130_mul(r16, r16);
    mine = p130_carry(p130_pow(r16, (uint32_t)(63 - t)));
    rp[t] = mine;
  }
  __syncthreads();
  // weights of positions 4t .. 4t+3 (block t/4, bytes 4(t%4) ..): one u32 of
  // digits per (digit plane, thread)
  const P130 rpow = rp[t >> 2];
  uint32_t dig[kPolyDigits];
#pragma unroll
  for (int d = 0; d < kPolyDigits; ++d) dig[d] = 0;
  P130 wsum = p130_zero();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const P130 w = poly_weight(rpow, 4 * (t & 3) + u);
    wsum = p130_add(wsum, w);
#pragma unroll
    for (int d = 0; d < kPolyDigits; ++d) dig[d] |= p130_digit7(w, d) << (8 * u);
  }
  uint32_t* tab = base + kPowTabOff;
#pragma unroll
  for (int d = 0; d < kPolyDigits; ++d) tab[d * (kSegBytes / 4) + t] = dig[d];
  const P130 sw = block_sum_p130(wsum, red);
  if (t == 0) {
    // the row constant without pad bits: those come from the prefix table below
    const P130 k = poly_kseg(p130_zero(), sw);
#pragma unroll
    for (int u = 0; u < 5; ++u) base[kPowKsegOff + u] = k.v[u];
  }
  if (t < 16) {
    const P130 f = p130_carry(p130_pow(r, (uint32_t)(16 - t)));
#pragma unroll
    for (int u = 0; u < 5; ++u) base[kPowRowOff + t * 5 + u] = f.v[u];
  }
  if (t <= 64) {
    uint64_t d[5] = {0, 0, 0, 0, 0};
    for (int q = 0; q < t; ++q) {
#pragma unroll
      for (int u = 0; u < 5; ++u) d[u] += rp[q].v[u];
    }
    uint64_t c;
    c = d[0] >> 26; d[0] &= kM26; d[1] += c;
    c = d[1] >> 26; d[1] &= kM26; d[2] += c;
    c = d[2] >> 26; d[2] &= kM26; d[3] += c;
    c = d[3] >> 26; d[3] &= kM26; d[4] += c;
    c = d[4] >> 26; d[4] &= kM26; d[0] += c * 5;
    c = d[0] >> 26; d[0] &= kM26; d[1] += c;
    const P130 sum = P130{{(uint32_t)d[0], (uint32_t)d[1], (uint32_t)d[2], (uint32_t)d[3], (uint32_t)d[4]}};
    const P130 q128 = p130_carry(p130_mul(sum, p130_bit(128)));
#pragma unroll
    for (int u = 0; u < 5; ++u) base[kPowQOff + t * 5 + u] = q128.v[u];
  }
}

constexpr int kMacChunksPerBlock = 8;  // k_mac_chunks: chunks of one message per block, at most


// Per-lane Horner Poly1305 partial of chunk k of message j, by the whole block:
// lane t sums the 4 blocks ending 4 (255 - t) blocks before the chunk end eb
// (end-aligned, so blocks before the message start contribute zero) and scales
// by its factor r^(4 (255 - t)). Handles what the matrix-core rows do not: a
// message's first chunk (its first 32 bytes precede the message) and its last
// chunk (partial final block, short tail). Every ciphertext read of the chunk is
// done when the function returns (the caller may then decrypt it in place).
__device__ __forceinline__ void horner_chunk(int j, int k, int K, const MsgKey* __restrict__ keys,
                                             const uint32_t* __restrict__ pows,
                                             const uint8_t* __restrict__ ct, uint64_t stride, uint32_t N,
                                             uint32_t* __restrict__ partials, uint64_t (*lsum)[kWaves]) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t kC = (int64_t)k * kChunkBytes;
  const int64_t start = kC >= 32 ? kC - 32 : 0;
  const int64_t end = min((int64_t)N, kC + kChunkBytes - 32);
  uint32_t* part = partials + ((size_t)j * K + k) * 8;
  if (start >= end) {
    if (tid < 5) part[tid] = 0;
    return;
  }
  const uint8_t* gmsg = ct + (size_t)j * stride + 48;
  const uint32_t* pf = pows + (size_t)j * kPowWords + tid * 5;
  const P130 f = P130{{pf[0], pf[1], pf[2], pf[3], pf[4]}};
  const MsgKey key = keys[j];
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  const int64_t fb = start / 16, eb = (end + 15) / 16;
  P130 c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i = eb - 4 * (int64_t)(kBlock - tid) + q;
    c[q] = i >= fb ? load_block(gmsg, i, N) : p130_zero();
  }
  P130 h = p130_zero();
#pragma unroll
  for (int q = 0; q < 4; ++q) h = p130_mul(p130_add(h, c[q]), r);
  h = p130_mul(h, f);
  uint64_t sv[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) sv[u] = wave_sum64((uint64_t)h.v[u]);
  if (lane == 0) {
#pragma unroll
    for (int u = 0; u < 5; ++u) lsum[u][wave] = sv[u];
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t d[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      d[u] = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) d[u] += lsum[u][w];
    }
    uint64_t cc;
    cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
    cc = d[1] >> 26; d[1] &= kM26; d[2] += cc;
    cc = d[2] >> 26; d[2] &= kM26; d[3] += cc;
    cc = d[3] >> 26; d[3] &= kM26; d[4] += cc;
    cc = d[4] >> 26; d[4] &= kM26; d[0] += cc * 5;
    cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
#pragma unroll
    for (int u = 0; u < 5; ++u) part[u] = (uint32_t)d[u];
  }
  __syncthreads();  // lsum may be written again (the block's next edge chunk)
}

// The edge chunks alone (the encode kernel's own MAC covers the middle ones), or with
// all != 0 every chunk (A/B measurement of the matrix-core path).
__global__ void __launch_bounds__(kBlock)
    k_mac_horner(int K, const MsgKey* __restrict__ keys, const uint32_t* __restrict__ pows,
                 const uint8_t* __restrict__ ct, uint64_t stride, const uint32_t* __restrict__ pt_len,
                 uint32_t* __restrict__ partials, int all) {
  __shared__ uint64_t lsum[5][kWaves];
  const int j = blockIdx.y;
  const uint32_t N = pt_len[j];
  const int last = last_chunk(N);
  int k;
  if (all) {
    k = blockIdx.x;
    if (k > last) return;  // k_mac_chunks zeroes chunks past the message
  } else {
    k = blockIdx.x == 0 ? 0 : last;
    if (blockIdx.x == 1 && last == 0) return;
  }
  horner_chunk(j, k, K, keys, pows, ct, stride, N, partials, lsum);
}

// Middle chunks on the matrix cores (+ in-place decryption and terminator
// counts for every chunk when DECRYPT). A middle chunk (not the message's
// first or last) is 1024 full blocks starting at block fb = kC/16 - 2, taken as
// 16 interleaved rows (row i = blocks fb + i + 16 t, t < 64): the 16 rows of an
// int8 GEMM (device_crypto.hpp, poly_seg_value) with K = the row's 1 KiB of bytes
// (wave w takes t in [16 w, 16 w + 16) of every row) and N = the 19 weight
// digits (two 16-column tiles). Row i is then placed by r^(16 - i). First / last
// chunks go through horner_chunk (by default in a k_mac_horner launch ahead of this
// kernel: it reads the ciphertext this kernel decrypts in place). With this K split
// wave w's operand bytes are exactly the quarter [4096 w, 4096 (w + 1)) of the chunk.
// EDGES: the block also does its message's first / last chunk by Horner instead
// of leaving them to a k_mac_horner launch (measured: the Horner code costs both
// variants registers, 64 -> 92 and 112 -> 117 VGPRs, and the round 0.3 ms for the
// 0.1 ms of launches it saves; selectable with set_mac_mfma(2), not the default).
template <int DECRYPT, bool EDGES>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_mac_chunks(int K, const MsgKey* __restrict__ keys, const uint32_t* __restrict__ pows,
                 uint8_t* __restrict__ ct, uint64_t stride, const uint32_t* __restrict__ pt_len,
                 uint32_t* __restrict__ partials, uint32_t* __restrict__ term_cnt,
                 uint32_t* __restrict__ sub_cnt, int use_mfma, int cpb) {
  // cpb (<= kMacChunksPerBlock): chunks per block; fewer when the launch is small, so
  // that the last, partly filled round of blocks costs less
  // digit sums of every (chunk of the block, segment): the four waves' K-slices
  // meet here through LDS adds, and the 130-bit work on them happens once per
  // block, a lane per segment, instead of per chunk on one wave's 16 lanes
  __shared__ int32_t cacc[kMacChunksPerBlock][16][kPolyDigits + 1];
  __shared__ uint32_t scratch[kWaves];
  __shared__ uint64_t lsum[EDGES ? 5 : 1][kWaves];
  __shared__ __attribute__((aligned(16))) uint32_t kst[DECRYPT ? kWaves * 1024 : 4];  // keystream, per wave
  const int j = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row = lane & 15, g = lane >> 4;
  const uint32_t N = pt_len[j];
  const int last = last_chunk(N);
  uint8_t* gmsg = ct + (size_t)j * stride + 48;
  const uint32_t* pw = pows + (size_t)j * kPowWords;
  const int k0 = blockIdx.x * cpb;
  const int k1 = min(K, k0 + cpb);
  const bool any_middle = use_mfma && k1 > 1 && k0 < last && max(k0, 1) < min(k1, last);
  // the message's weight-digit fragments (this lane's K-slice of its digit
  // columns): loaded once, reused by every chunk of the block
  v4i b0[4], b1[4];
  if (any_middle) {
    const int8_t* tab = reinterpret_cast<const int8_t*>(pw + kPowTabOff);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int q = 4 * wave + qq;
      b0[qq] = *reinterpret_cast<const v4i*>(tab + row * kSegBytes + 64 * q + 16 * g);
      b1[qq] = v4i{0, 0, 0, 0};
      if (row < kPolyDigits - 16)
        b1[qq] = *reinterpret_cast<const v4i*>(tab + (16 + row) * kSegBytes + 64 * q + 16 * g);
    }
    int32_t* flat = &cacc[0][0][0];
    for (int i = tid; i < cpb * 16 * (kPolyDigits + 1); i += kBlock) flat[i] = 0;
    __syncthreads();
  }
  // the message's key, and what its blocks have in common of their first double round
  const MsgKey key = DECRYPT ? keys[j] : MsgKey{};
  const SalsaPrefix pre = DECRYPT ? salsa20_prefix(key.subkey, key.nonce[0], key.nonce[1]) : SalsaPrefix{};
  for (int k = k0; k < k1; ++k) {
    const int64_t kC = (int64_t)k * kChunkBytes;
    const int64_t start = kC >= 32 ? kC - 32 : 0;
    const int64_t end = min((int64_t)N, kC + kChunkBytes - 32);
    uint32_t* part = partials + ((size_t)j * K + k) * 8;
    if (start >= end) {  // chunk beyond the message (or empty message)
      if (tid < 5 && partials != nullptr) part[tid] = 0;
      if (DECRYPT && term_cnt && tid == 0) term_cnt[(size_t)j * K + k] = 0;
      if (DECRYPT && sub_cnt && tid < kSubPerChunk)
        sub_cnt[((size_t)j * K + k) * kSubPerChunk + tid] = 0;
      continue;
    }
    // This lane's four 16-byte pieces of the chunk: piece q = keystream bytes
    // [4096 wave + 1024 q + 16 lane, +16) of the chunk, so that a wave's load (and
    // store) instruction covers 1 KiB contiguously -- a lane reading its own 64
    // contiguous bytes made every instruction touch 64 lines and every store a
    // 16-byte partial line write (350 M write requests per headline round; the
    // memory side alone then took 3.1 ms against 2.4 ms in this layout). The
    // pieces are also exactly this lane's MFMA operand fragments of the
    // interleaved rows (row = lane & 15, t = 16 wave + 4 q + (lane >> 4)): one load
    // serves the MAC and the decryption, and a wave reads only bytes it overwrites
    // itself, so the in-place decryption needs no barrier.
    const bool middle = use_mfma && k != 0 && k != last;
    // EDGES: a message's first and last chunk by Horner here (block-uniform; its
    // reads are done before the decryption below)
    if constexpr (EDGES) {
      if (use_mfma && !middle) horner_chunk(j, k, K, keys, pows, ct, stride, N, partials, lsum);
    }
    uint4 d4[4];
    int64_t pos[4];
    bool in[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pos[q] = kC - 32 + 4096 * wave + 1024 * q + 16 * lane;
      in[q] = pos[q] >= start - 15 && pos[q] >= 0 && pos[q] < end;
      d4[q] = make_uint4(0, 0, 0, 0);
      if ((DECRYPT || middle) && in[q]) d4[q] = *reinterpret_cast<const uint4*>(gmsg + pos[q]);
    }
    // The keystream needs no loaded byte: computed here, its ~1000 instructions
    // run while the chunk's loads (issued above) are in flight. Lane 4 j + i of a
    // wave computes block 16 i + j of the wave's 64: the four lanes of a quad hold
    // the four blocks their pieces lie in (piece q in block 16 q + j, words 4 i ..).
    // A wave whose 4 KiB lie wholly behind the message's end (the last chunk of a short box:
    // 40 KB boxes are two and a half chunks) has no keystream to compute.
    const bool wave_in = __builtin_amdgcn_ballot_w64(in[0] || in[1] || in[2] || in[3]) != 0;
    uint32_t w[16] = {};
    if constexpr (DECRYPT) {
      if (wave_in) {
        const uint32_t blk = (uint32_t)(kC / 64) + 64 * wave + 16 * (lane & 3) + (lane >> 2);
        salsa20_block(w, pre, key.subkey, key.nonce[0], key.nonce[1], blk);
      }
    }
    if (middle) {
      v4i acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const v4i a = {(int)d4[qq].x, (int)d4[qq].y, (int)d4[qq].z, (int)d4[qq].w};
        const v4i x = a ^ (int)0x80808080;  // bytes u -> u - 128 (signed)
        acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, b0[qq], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, b1[qq], acc1, 0, 0, 0);
      }
      // C[row 4 g + i][digit column]: |sum| < 2^23 per wave, 2^25 over the four
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        atomicAdd(&cacc[k - k0][4 * g + i][row], acc0[i]);
        if (row < kPolyDigits - 16) atomicAdd(&cacc[k - k0][4 * g + i][16 + row], acc1[i]);
      }
    }

    if constexpr (DECRYPT) {
      // The keystream to the pieces' layout (ks[q] = words 4 i .. 4 i + 3 of the block
      // that quad lane q computed, i = this lane's place in its quad) through the
      // wave's own 4 KiB of LDS: four 16-byte stores and loads instead of a 64-
      // instruction butterfly on the VALU, which is what bounds this kernel while
      // its LDS port idles. Block b lies at word 16 b; the lane that computed it
      // (place i) rotates its four word groups by i slots, so that 8 consecutive
      // lanes of a store or a load cover all 32 banks. Same wave, LDS keeps program
      // order: no barrier.
      uint32_t ks[4][4] = {};
      if (wave_in) {
        uint32_t* kw = kst + 1024 * wave;
        const int i4 = lane & 3, j4 = lane >> 2;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          *reinterpret_cast<uint4*>(kw + 16 * (16 * i4 + j4) + 4 * ((u + i4) & 3)) =
              make_uint4(w[4 * u], w[4 * u + 1], w[4 * u + 2], w[4 * u + 3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 t = *reinterpret_cast<const uint4*>(kw + 16 * (16 * q + j4) + 4 * ((i4 + q) & 3));
          ks[q][0] = t.x; ks[q][1] = t.y; ks[q][2] = t.z; ks[q][3] = t.w;
        }
      }
      uint32_t cnt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d4[q].x ^= ks[q][0]; d4[q].y ^= ks[q][1]; d4[q].z ^= ks[q][2]; d4[q].w ^= ks[q][3];
        // terminators (MSB clear) among the piece's bytes inside the message
        const int vlo = (int)max((int64_t)0, min((int64_t)16, start - pos[q]));
        const int vhi = (int)max((int64_t)0, min((int64_t)16, end - pos[q]));
        if (vlo == 0 && vhi == 16) {
          cnt[q] = (uint32_t)__popc(~d4[q].x & 0x80808080u) + (uint32_t)__popc(~d4[q].y & 0x80808080u) +
                   (uint32_t)__popc(~d4[q].z & 0x80808080u) + (uint32_t)__popc(~d4[q].w & 0x80808080u);
        } else {
          const uint32_t ws[4] = {d4[q].x, d4[q].y, d4[q].z, d4[q].w};
          uint32_t tmask = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t t = ~ws[u] & 0x80808080u;
            tmask |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * u);
          }
          const uint32_t vmask = vhi > vlo ? ((1u << vhi) - 1u) & ~((1u << vlo) - 1u) : 0u;
          cnt[q] = (uint32_t)__popc(tmask & vmask);
        }
      }
      if (sub_cnt) {  // per 1 KiB sub-chunk 4 wave + q: every lane's piece q
        const uint32_t s01 = wave_read_lane(wave_incl_scan(cnt[0] | (cnt[1] << 16)), 63);
        const uint32_t s23 = wave_read_lane(wave_incl_scan(cnt[2] | (cnt[3] << 16)), 63);
        if (lane < 4) {
          const uint32_t pair = lane < 2 ? s01 : s23;
          sub_cnt[((size_t)j * K + k) * kSubPerChunk + 4 * wave + lane] = (lane & 1) ? pair >> 16 : pair & 0xffffu;
        }
      }
      if (term_cnt) {
        const uint32_t tot = block_sum(cnt[0] + cnt[1] + cnt[2] + cnt[3], scratch);
        if (tid == 0) term_cnt[(size_t)j * K + k] = tot;
      }
      // store plaintext in place (bytes past `end` land in the slot padding)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (in[q]) *reinterpret_cast<uint4*>(gmsg + pos[q]) = d4[q];
    }
  }
  if (!any_middle) return;
  // Segment values -> chunk partials: lane (chunk kk, segment s) turns its 19
  // digit sums into a 130-bit value and places it by r^(64 (15 - s)); the 16
  // lanes of a chunk then add up.
  __syncthreads();
  if (tid < 16 * cpb) {
    const int kk = tid >> 4, s = tid & 15, k = k0 + kk;
    const bool mid = k < k1 && k != 0 && k < last;
    P130 h = p130_zero();
    if (mid) {
      int32_t c[kPolyDigits];
#pragma unroll
      for (int d = 0; d < kPolyDigits; ++d) c[d] = cacc[kk][s][d];
      // every pad bit of the chunk is this block's: prefix table entry 64; placed by r^(16 - s)
      P130 kseg, sfac;
      const uint32_t* pf = pw + kPowRowOff + s * 5;
#pragma unroll
      for (int u = 0; u < 5; ++u) {
        kseg.v[u] = pw[kPowKsegOff + u] + pw[kPowQOff + 64 * 5 + u];
        sfac.v[u] = pf[u];
      }
      h = p130_mul(poly_seg_value(c, p130_carry(kseg)), sfac);
    }
    uint64_t d[5];
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      d[u] = h.v[u];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) d[u] += __shfl_xor(d[u], o, 64);
    }
    if (mid && s == 0) {
      uint64_t cc;
      cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
      cc = d[1] >> 26; d[1] &= kM26; d[2] += cc;
      cc = d[2] >> 26; d[2] &= kM26; d[3] += cc;
      cc = d[3] >> 26; d[3] &= kM26; d[4] += cc;
      cc = d[4] >> 26; d[4] &= kM26; d[0] += cc * 5;
      cc = d[0] >> 26; d[0] &= kM26; d[1] += cc;
      uint32_t* part = partials + ((size_t)j * K + k) * 8;
#pragma unroll
      for (int u = 0; u < 5; ++u) part[u] = (uint32_t)d[u];
    }
  }
}

// Chunk partials -> tag, a wave per message. With n chunks before the last one,
//   H = (sum_{k<n} part_k rC^(n-1-k)) r^(d_last) + part_n,   rC = r^(C/16),
// d_last = the last chunk's length in blocks. Lane l folds the q = ceil(n/64)
// chunks [n - (64-l) q, n - (63-l) q) by Horner (chunks are aligned to the end, so
// every lane's sum sits q chunks before the next lane's), six pairwise steps with
// F = rC^q, F^2, ... bring the sum to lane 63, which finishes the tag. A serial
// chain over all chunks took 70 us however few the messages (113 dependent
// 130-bit multiplies at the headline size).
SDA_DEV P130 p130_shfl_up(const P130& a, int delta) {
  P130 o;
#pragma unroll
  for (int u = 0; u < 5; ++u) o.v[u] = __shfl_up(a.v[u], delta, 64);
  return o;
}

__global__ void __launch_bounds__(kBlock)
    k_mac_final(int M, int K, const MsgKey* __restrict__ keys, const uint32_t* __restrict__ pows,
                uint8_t* __restrict__ ct, uint64_t stride, const uint32_t* __restrict__ pt_len,
                const uint32_t* __restrict__ partials, int verify, uint32_t* __restrict__ ok,
                uint32_t* err) {
  const int j = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= M) return;  // wave-uniform
  const uint32_t N = pt_len[j];
  const MsgKey key = keys[j];
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  const P130 r = p130_r_from_key(rk);
  const uint32_t* pw = pows + (size_t)j * kPowWords;  // chunk factors r^(4 (255 - t))
  auto factor = [&](int t) { return P130{{pw[t * 5], pw[t * 5 + 1], pw[t * 5 + 2], pw[t * 5 + 3], pw[t * 5 + 4]}}; };
  auto part = [&](int k) {
    const uint32_t* pp = partials + ((size_t)j * K + k) * 8;
    return P130{{pp[0], pp[1], pp[2], pp[3], pp[4]}};
  };
  const int Kc = (int)(((int64_t)N + 32 + kChunkBytes - 1) / kChunkBytes);
  // chunks past the partials' capacity cannot be summed: such a box fails its check
  const int n = min(Kc, K) - 1;
  P130 H = part(n);  // the last chunk's (the only one's when n == 0)
  if (n > 0) {
    const P130 rC = p130_mul(factor(0), factor(254));  // r^1020 r^4
    const int q = (n + 63) / 64;
    P130 h = p130_zero();
    for (int i = 0; i < q; ++i) {
      const int k = n - (64 - lane) * q + i;
      if (k >= 0) h = p130_carry(p130_add(p130_mul(h, rC), part(k)));
    }
    P130 F = p130_pow(rC, (uint32_t)q);
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int step = 1 << s;
      const P130 lower = p130_shfl_up(h, step);
      if ((lane & (2 * step - 1)) == 2 * step - 1) h = p130_carry(p130_add(p130_mul(lower, F), h));
      F = p130_mul(F, F);
    }
    // the last chunk's length in blocks (C/16 for a full one)
    const int64_t e_prev = ((int64_t)n * kChunkBytes - 32) / 16;
    const int64_t e_last = Kc <= K ? ((int64_t)N + 15) / 16 : e_prev + kChunkBytes / 16;
    const int d = (int)(e_last - e_prev);
    P130 Rd = rC;
    if (d < kChunkBytes / 16) {
      Rd = (d >> 2) ? factor(255 - (d >> 2)) : P130{{1, 0, 0, 0, 0}};
      for (int b = 0; b < (d & 3); ++b) Rd = p130_mul(Rd, r);
    }
    H = p130_carry(p130_add(p130_mul(h, Rd), H));
  }
  if (lane != 63) return;
  const uint32_t s4[4] = {key.poly_s[0], key.poly_s[1], key.poly_s[2], key.poly_s[3]};
  uint32_t tag[4];
  p130_finish(tag, H, s4);
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ct + (size_t)j * stride + 32);
  if (!verify) {
#pragma unroll
    for (int i = 0; i < 4; ++i) hdr[i] = tag[i];
  } else {
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) diff |= hdr[i] ^ tag[i];
    if (ok) ok[j] = diff == 0 ? 1u : 0u;
    if (diff) atomicOr(err, kErrMac);
  }
}

// ------------------------------------------------ short messages: one pass --
// Boxes of at most kShortMaxChunks chunks (the many-clerk committees seal hundreds
// of thousands of 30-40 KB boxes) take neither the chunk tables nor the partials:
// a wave owns a message and lane t the blocks at distance e = t + 64 i from the
// message's last one, so that one load instruction of the wave reads 1 KiB of
// contiguous ciphertext:
//   tag = sum_e c_e r^(e+1) = sum_t r^(t+1) sum_i c_(t+64i) (r^64)^i,
// a Horner chain in R = r^64 per lane, one multiply by the lane's r^(t+1), a sum
// over the lanes, and the tag -- one multiply per block where the chunked path
// needs 1.25 plus a 256-entry factor table per message (more multiplies than such
// a message's own blocks) and a combining pass. The table here: r^1 .. r^64.
__global__ void __launch_bounds__(kBlock)
    k_poly_powers_short(int M, const MsgKey* __restrict__ keys, uint32_t* __restrict__ pows, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(3);  // side-stream key work (see k_seal_setup)
  const int j = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= M) return;  // wave-uniform
  const MsgKey key = keys[j];
  const uint32_t rk[4] = {key.poly_r[0], key.poly_r[1], key.poly_r[2], key.poly_r[3]};
  // r^(lane + 1) as a running product over the lanes: six multiplies by the value 1, 2, 4, ...
  // lanes below (the lanes without one multiply by 1) instead of a square-and-multiply per
  // lane, which costs the wave all twelve of its steps
  P130 f = p130_r_from_key(rk);
#pragma unroll
  for (int sft = 1; sft < 64; sft <<= 1) {
    P130 y;
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const uint32_t up = (uint32_t)__shfl_up((int)f.v[u], sft, 64);
      y.v[u] = lane >= sft ? up : (u == 0 ? 1u : 0u);
    }
    f = p130_mul(f, y);
  }
  f = p130_carry(f);
  uint32_t* out = pows + (size_t)j * kPowShortWords + lane * 5;
#pragma unroll
  for (int u = 0; u < 5; ++u) out[u] = f.v[u];
}

template <bool VERIFY>
__global__ void __launch_bounds__(kBlock)
    k_mac_short(int M, const MsgKey* __restrict__ keys, const uint32_t* __restrict__ pows,
                uint8_t* __restrict__ ct, uint64_t stride, const uint32_t* __restrict__ pt_len,
                uint32_t* __restrict__ ok, uint32_t* err) {
  const int j = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= M) return;  // wave-uniform
  const uint32_t N = pt_len[j];
  const int nb = (int)(((int64_t)N + 15) / 16);
  const uint8_t* gmsg = ct + (size_t)j * stride + 48;
  const uint32_t* pw = pows + (size_t)j * kPowShortWords;
  const P130 R = P130{{pw[63 * 5], pw[63 * 5 + 1], pw[63 * 5 + 2], pw[63 * 5 + 3], pw[63 * 5 + 4]}};
  const P130 f = P130{{pw[lane * 5], pw[lane * 5 + 1], pw[lane * 5 + 2], pw[lane * 5 + 3], pw[lane * 5 + 4]}};
  // rounds of 64 blocks, in groups of four whose loads are issued together (rounds
  // past the message's first block read as zero and leave h = 0)
  const int I4 = (((nb + 63) / 64) + 3) & ~3;
  auto fetch = [&](int i) -> uint4 {
    const int e = lane + 64 * i;
    return e < nb ? *reinterpret_cast<const uint4*>(gmsg + 16 * (int64_t)(nb - 1 - e)) : make_uint4(0, 0, 0, 0);
  };
  auto block = [&](const uint4& q, int i) -> P130 {
    const int e = lane + 64 * i;
    return e < nb ? block_from(q, nb - 1 - e, N) : p130_zero();
  };
  P130 h = p130_zero();
  for (int i = I4 - 1; i >= 0; i -= 4) {
    const uint4 q0 = fetch(i), q1 = fetch(i - 1), q2 = fetch(i - 2), q3 = fetch(i - 3);
    h = p130_mul(p130_add(h, block(q0, i)), R);
    h = p130_mul(p130_add(h, block(q1, i - 1)), R);
    h = p130_mul(p130_add(h, block(q2, i - 2)), R);
    h = p130_add(h, block(q3, i - 3));
    if (i > 3) h = p130_mul(h, R);  // wave-uniform
  }
  h = p130_carry(p130_mul(h, f));  // limbs <= 2^26
  // over the lanes: rows of 16 on the VALU (16 x 2^26 fits a word), the four rows as
  // 64-bit scalars
  uint64_t d[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const uint32_t rs = row16_incl_scan(h.v[u]);
    d[u] = (uint64_t)wave_read_lane(rs, 15) + wave_read_lane(rs, 31) + wave_read_lane(rs, 47) +
           wave_read_lane(rs, 63);
  }
  if (lane != 0) return;
  uint64_t c;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  c = d[1] >> 26; d[1] &= kM26; d[2] += c;
  c = d[2] >> 26; d[2] &= kM26; d[3] += c;
  c = d[3] >> 26; d[3] &= kM26; d[4] += c;
  c = d[4] >> 26; d[4] &= kM26; d[0] += c * 5;
  c = d[0] >> 26; d[0] &= kM26; d[1] += c;
  const P130 H = P130{{(uint32_t)d[0], (uint32_t)d[1], (uint32_t)d[2], (uint32_t)d[3], (uint32_t)d[4]}};
  const MsgKey key = keys[j];
  const uint32_t s4[4] = {key.poly_s[0], key.poly_s[1], key.poly_s[2], key.poly_s[3]};
  uint32_t tag[4];
  p130_finish(tag, H, s4);
  uint32_t* hdr = reinterpret_cast<uint32_t*>(ct + (size_t)j * stride + 32);
  if constexpr (!VERIFY) {
#pragma unroll
    for (int i = 0; i < 4; ++i) hdr[i] = tag[i];
  } else {
    uint32_t diff = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) diff |= hdr[i] ^ tag[i];
    if (ok) ok[j] = diff == 0 ? 1u : 0u;
    if (diff) atomicOr(err, kErrMac);
  }
}

}  // namespace

// Rows of a few entries (the many-clerk boxes: three byte counts, a handful of terminator
// counts): a thread per row. A 256-thread workgroup per row, scan and two barriers for three
// numbers, was 0.17 ms a call over 728,000 rows.
__global__ void __launch_bounds__(kBlock) k_segscan_rows(int M, int T, uint32_t* __restrict__ data,
                                                         uint32_t* __restrict__ totals, uint32_t expect,
                                                         uint32_t* err) {
  const int j = blockIdx.x * kBlock + threadIdx.x;
  if (j >= M) return;
  uint32_t* row = data + (size_t)j * T;
  uint32_t carry = 0;
  for (int i = 0; i < T; ++i) {
    const uint32_t v = row[i];
    row[i] = carry;
    carry += v;
  }
  if (totals) totals[j] = carry;
  if (err && carry != expect) atomicOr(err, kErrMalformed);
}

void launch_segscan(int M, int T, uint32_t* data, uint32_t* totals, uint32_t expect, uint32_t* err,
                    hipStream_t s) {
  if (M <= 0) return;
  if (T <= 64 && M >= 4096) {
    hipLaunchKernelGGL(k_segscan_rows, dim3((M + kBlock - 1) / kBlock), dim3(kBlock), 0, s, M, T, data, totals,
                       expect, err);
    return;
  }
  hipLaunchKernelGGL(k_segscan, dim3(M), dim3(kBlock), 0, s, T, data, totals, expect, err);
}

// 16-bit values below 2^13 (codes of at most two bytes) in a tile sized for them
static int g_encode_tile2 = 1;
void set_encode_tile2(int on) { g_encode_tile2 = on; }

template <typename VT, int kMaxB>
static void launch_encode_t(int M, int L, const void* vals, const uint32_t* tile_off,
                            const MsgKey* keys, uint8_t* ct, uint64_t stride, const uint32_t* pows,
                            const uint32_t* pt_len, uint32_t* partials, int K, hipStream_t s) {
  if (pows && pt_len && partials)
    hipLaunchKernelGGL((k_encode_encrypt<VT, true, (sizeof(VT) > 2 ? 5 : 3)>), dim3(encode_grid(true, M, L)),
                       dim3(kBlock), 0, s, L, M, (const VT*)vals, tile_off, keys, ct, stride, pows, pt_len, partials, K);
  else
    hipLaunchKernelGGL((k_encode_encrypt<VT, false, kMaxB>), dim3(encode_grid(false, M, L)), dim3(kBlock), 0, s, L,
                       M, (const VT*)vals,
                       tile_off, keys, ct, stride, pows, pt_len, partials, K);
}

void launch_encode_encrypt(int M, int L, int value_bytes, const void* vals,
                           const uint32_t* tile_off, const MsgKey* keys, uint8_t* ct,
                           uint64_t stride, const uint32_t* pows, const uint32_t* pt_len,
                           uint32_t* partials, int K, int max_code_bytes, hipStream_t s) {
  if (M <= 0 || L <= 0) return;
  if (value_bytes == 1)
    launch_encode_t<uint8_t, 3>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
  else if (value_bytes == 2 && max_code_bytes <= 2 && g_encode_tile2 && !(pows && pt_len && partials))
    launch_encode_t<uint16_t, 2>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
  else if (value_bytes == 2)
    launch_encode_t<uint16_t, 3>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
  else if (max_code_bytes <= 3)
    launch_encode_t<uint32_t, 3>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
  else if (max_code_bytes == 4)
    launch_encode_t<uint32_t, 4>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
  else
    launch_encode_t<uint32_t, 5>(M, L, vals, tile_off, keys, ct, stride, pows, pt_len, partials, K, s);
}

extern int g_powers_prio;  // keys.hip (set_key_prio)

void launch_poly_powers(int M, const MsgKey* keys, uint32_t* pows, int full, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_poly_powers, dim3(M), dim3(kBlock), 0, s, keys, pows, g_powers_prio, full);
}

void launch_mac_edges(int M, int K, const MsgKey* keys, const uint32_t* pows, const uint8_t* ct,
                      uint64_t stride, const uint32_t* pt_len, uint32_t* partials, hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  hipLaunchKernelGGL(k_mac_horner, dim3(2, M), dim3(kBlock), 0, s, K, keys, pows, ct, stride, pt_len,
                     partials, 0);
}

void launch_poly_powers_short(int M, const MsgKey* keys, uint32_t* pows, hipStream_t s) {
  if (M <= 0) return;
  hipLaunchKernelGGL(k_poly_powers_short, dim3((M + kWaves - 1) / kWaves), dim3(kBlock), 0, s, M, keys,
                     pows, g_powers_prio);
}

void launch_mac_short(int M, const MsgKey* keys, const uint32_t* pows, uint8_t* ct, uint64_t stride,
                      const uint32_t* pt_len, int verify, uint32_t* ok, uint32_t* err, hipStream_t s) {
  if (M <= 0) return;
  const dim3 grid((M + kWaves - 1) / kWaves);
  if (verify)
    hipLaunchKernelGGL(k_mac_short<true>, grid, dim3(kBlock), 0, s, M, keys, pows, ct, stride, pt_len,
                       ok, err);
  else
    hipLaunchKernelGGL(k_mac_short<false>, grid, dim3(kBlock), 0, s, M, keys, pows, ct, stride, pt_len,
                       ok, err);
}

void launch_decrypt_count(int M, int K, const MsgKey* keys, uint8_t* ct, uint64_t stride,
                          const uint32_t* pt_len, uint32_t* term_cnt, uint32_t* sub_cnt,
                          hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  int cpb = kMacChunksPerBlock;
  while (cpb > 1 && (int64_t)M * ((K + cpb - 1) / cpb) < 16384) cpb /= 2;
  const dim3 grid((K + cpb - 1) / cpb, M);
  hipLaunchKernelGGL((k_mac_chunks<1, false>), grid, dim3(kBlock), 0, s, K, keys, nullptr, ct, stride,
                     pt_len, nullptr, term_cnt, sub_cnt, 0, cpb);
}

static int g_mac_mfma = 1;
void set_mac_mfma(int mode) { g_mac_mfma = mode; }

void launch_mac_chunks(int M, int K, const MsgKey* keys, const uint32_t* pows, uint8_t* ct,
                       uint64_t stride, const uint32_t* pt_len, uint32_t* partials, int decrypt,
                       uint32_t* term_cnt, uint32_t* sub_cnt, hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  // first / last chunks (every chunk when the matrix-core path is off, mode 0) by
  // Horner, ahead of the in-place decryption; mode 2 leaves them to k_mac_chunks
  const bool edges = g_mac_mfma == 2;
  if (!edges)
    hipLaunchKernelGGL(k_mac_horner, dim3(g_mac_mfma ? 2 : K, M), dim3(kBlock), 0, s, K, keys, pows,
                       ct, stride, pt_len, partials, g_mac_mfma ? 0 : 1);
  // 8 chunks per block amortise the weight fragments and the 130-bit tail; a launch of
  // fewer than ~16 rounds of resident blocks (1024 - 2048 at a time) takes 4 per block
  // (measured on the pipelined committee round: 4 waves -0.2 ms; 2 per block is worse)
  int cpb = kMacChunksPerBlock;
  while (cpb > 4 && (int64_t)M * ((K + cpb - 1) / cpb) < 16384) cpb /= 2;
  const dim3 grid_c((K + cpb - 1) / cpb, M);
  auto kern = decrypt ? (edges ? k_mac_chunks<1, true> : k_mac_chunks<1, false>)
                      : (edges ? k_mac_chunks<0, true> : k_mac_chunks<0, false>);
  hipLaunchKernelGGL(kern, grid_c, dim3(kBlock), 0, s, K, keys, pows, ct, stride, pt_len, partials,
                     term_cnt, sub_cnt, g_mac_mfma, cpb);
}

void launch_mac_final(int M, int K, const MsgKey* keys, const uint32_t* pows, uint8_t* ct,
                      uint64_t stride, const uint32_t* pt_len, const uint32_t* partials, int verify,
                      uint32_t* ok, uint32_t* err, hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  hipLaunchKernelGGL(k_mac_final, dim3((M + kWaves - 1) / kWaves), dim3(kBlock), 0, s, M, K, keys,
                     pows, ct, stride, pt_len, partials, verify, ok, err);
}

}  // namespace sdagpu
