// Clerk / recipient kernels after decryption: parallel varint decode, the
// per-clerk modular combine, packed-Shamir (Lagrange) reconstruction, unmask.
//
// Reference: sodium.rs:83-89 (decode until exhausted), sharing/combiner.rs:15-29
// (element-wise sum mod m), sharing/batched.rs:68-99 + tss reconstruct
// (reconstruct per batch, truncate to the dimension), masking/full.rs:54-67.
//
// Parallel decode: every byte with MSB = 0 terminates a varint, so a chunk's
// terminator count gives element ranks by an exclusive scan across chunks
// (launch_segscan over the per-chunk counts from k_mac_chunks<1>); inside a chunk
// the lanes rank their terminators with a block scan and each lane decodes the
// varints ending in its 64 bytes, reading at most 9 bytes back (a 16-byte LDS
// prefix of the previous chunk covers varints straddling the boundary).
#include <type_traits>

#include "block_utils.hpp"
#include "decode_core.hpp"
#include "device_crypto.hpp"
#include "encode_units.hpp"
#include "kernels.hpp"
#include "modarith.hpp"

namespace sdagpu {
namespace {

// Sink of k_decode: the chunk's values staged in LDS at their block-local rank
// (non-terminators into a per-lane dummy slot).
template <typename VT>
struct StageSink {
  static constexpr bool kAdditive = false;
  VT* outb;
  uint32_t dummy;
  SDA_DEV void put(uint32_t local, uint32_t v, uint32_t term) {
    outb[term ? local : dummy] = (VT)v;
  }
  SDA_DEV void put_rank(uint32_t rank, uint32_t v) { outb[rank] = (VT)v; }
};

// One block per (chunk, message). Each lane owns 64 plaintext bytes held in
// registers; terminator positions are a 64-bit mask (popcount -> block scan ->
// ranks); the bytes preceding a lane come from its neighbour by a shuffle (lane
// 0 of a wave loads them); decoded values are staged in LDS so the global store
// of the chunk's contiguous element range is coalesced.
template <typename VT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_decode(int L, ModParams mp, const uint8_t* __restrict__ pt, uint64_t stride,
             const uint32_t* __restrict__ pt_len, const uint32_t* __restrict__ elem_start,
             VT* __restrict__ vals, uint32_t* err) {
  __shared__ VT outb[kChunkBytes + 128];  // + a dummy dword per wave lane
  __shared__ uint32_t scratch[kWaves];
  const int k = blockIdx.x, j = blockIdx.y, K = gridDim.x;
  const int tid = threadIdx.x;
  const uint32_t N = pt_len[j];
  const int64_t kC = (int64_t)k * kChunkBytes;
  const int64_t start = kC >= 32 ? kC - 32 : 0;
  const int64_t end = min((int64_t)N, kC + kChunkBytes - 32);
  if (start >= end) return;
  const uint8_t* gmsg = pt + (size_t)j * stride + 48;
  const int64_t p0 = kC - 32 + 64 * tid;  // message position of this lane's first byte
  uint32_t w[16];
  load_lane_bytes(w, gmsg, p0, end);
  uint32_t wave_prev = 0, wave_prev2 = 0;  // the 8 bytes before a wave's first lane
  if ((tid & 63) == 0 && p0 - 4 >= 0 && p0 - 4 < end) wave_prev = *reinterpret_cast<const uint32_t*>(gmsg + p0 - 4);
  if ((tid & 63) == 0 && p0 - 8 >= 0 && p0 - 8 < end) wave_prev2 = *reinterpret_cast<const uint32_t*>(gmsg + p0 - 8);
  const int lo = (int)max((int64_t)0, start - p0);
  const int hi = (int)min((int64_t)64, end - p0);
  const uint64_t traw = term_mask64(w);
  const uint64_t tmask = traw & byte_range_mask(lo, hi);
  uint32_t total;
  const uint32_t local = block_excl_scan((uint32_t)__popcll(tmask), scratch, &total);  // syncs
  const uint32_t prev_word = wave_shift_up1(w[15], wave_prev);  // lane 0: from global
  const uint32_t prev_word2 = wave_shift_up1(w[14], wave_prev2);
  StageSink<VT> sink{outb, (uint32_t)(kChunkBytes + 2 * (tid & 63))};
  bool bad = decode_lane<sizeof(VT) == 2>(w, prev_word2, prev_word, tmask, traw, local, mp, gmsg, p0, sink);
  // a message must end on a terminator
  if (hi > lo && p0 + hi == (int64_t)N && (gmsg[N - 1] & 0x80)) bad = true;
  __syncthreads();
  const uint32_t base = elem_start[(size_t)j * K + k];
  VT* out = vals + (size_t)j * L;
  for (uint32_t i = tid; i < total; i += kBlock) {
    if (base + i < (uint32_t)L) out[base + i] = outb[i];
    else bad = true;
  }
  if (bad) atomicOr(err, kErrMalformed);
}

// ---------------------------------------------------- clerk decode + combine
// The clerk's combine (sharing/combiner.rs:15-29: element-wise sum over the P
// participants' share vectors) fused with the varint decode, so decoded shares
// never reach HBM. Element tiles are aligned across participants: block (t, r,
// g) owns elements [t*kSumTile, (t+1)*kSumTile) of row r (a clerk) and walks
// participant group g. k_mac_chunks<1> counts terminators per 1 KiB sub-chunk,
// their exclusive scan gives each sub-chunk's first rank, and k_locate_tiles
// records per (message, tile) the sub-chunk holding the tile's first
// terminator, so a block reads only the ~kSumTile * 1.9 bytes of each message
// that hold its tile (plus < 2 KiB of sub-chunk slack). Values are accumulated
// with LDS atomics (ds_add_u32) into a kSumTile-wide u32 accumulator; each
// group writes a slab of raw sums, and k_sum_slabs reduces the slabs mod m.
// The accumulator has kSumMargin slots on both sides of the tile: a pass's
// ranks lie within one 1 KiB sub-chunk (< 1024 terminators) of the tile on
// either side, so every rank lands in [0, kSumTile + 2 * kSumMargin] with no
// bounds check, and a non-terminator adds 0 to the next rank's slot.
constexpr int kSumMargin = kSubBytes;
constexpr int kSumAcc = kSumTile + 2 * kSumMargin + 64;
struct AddSink {
  static constexpr bool kAdditive = true;
  uint32_t* acc;  // acc[kSumMargin] = tile element 0
  uint32_t off;   // accumulator index of block-local rank 0
  SDA_DEV void put(uint32_t local, uint32_t v, uint32_t term) {
    atomicAdd(acc + (local + off), v & (0u - term));
  }
  SDA_DEV void put_masked(uint32_t local, uint32_t v) { atomicAdd(acc + (local + off), v); }
  SDA_DEV void put_rank(uint32_t rank, uint32_t v) { atomicAdd(acc + (rank + off), v); }
};

// The same into 64-bit accumulators (ds_add_u64): moduli above 2^27, whose values a u32
// accumulator can add up only a handful of (two at 2^31 - 1: 500 slabs of a million
// sums each to write and add again for 1000 participants; that was 63 % of such a round).
struct AddSink64 {
  static constexpr bool kAdditive = true;
  unsigned long long* acc;
  uint32_t off;
  SDA_DEV void put(uint32_t local, uint32_t v, uint32_t term) {
    atomicAdd(acc + (local + off), (unsigned long long)(v & (0u - term)));
  }
  SDA_DEV void put_masked(uint32_t local, uint32_t v) { atomicAdd(acc + (local + off), (unsigned long long)v); }
  SDA_DEV void put_rank(uint32_t rank, uint32_t v) { atomicAdd(acc + (rank + off), (unsigned long long)v); }
};

__global__ void __launch_bounds__(kBlock)
    k_locate_tiles(int S, int T, const uint32_t* __restrict__ pre,
                   const uint32_t* __restrict__ totals, uint32_t* __restrict__ tile_sub) {
  const int s = blockIdx.x * kBlock + threadIdx.x, j = blockIdx.y;
  if (s >= S) return;
  const uint32_t tot = totals[j];
  const uint32_t lo = pre[(size_t)j * S + s];
  const uint32_t hi = s + 1 < S ? pre[(size_t)j * S + s + 1] : tot;
  uint32_t* row = tile_sub + (size_t)j * (T + 1);
  // tiles whose first element ends in this sub-chunk (a 1 KiB sub-chunk holds
  // < kSumTile terminators: at most one)
  for (uint32_t t = (lo + kSumTile - 1) / kSumTile; t <= (uint32_t)T && (uint64_t)t * kSumTile < hi; ++t)
    row[t] = (uint32_t)s;
  // tiles past the message's last element (t = T always: the end sentinel)
  if (s == S - 1)
    for (uint64_t t = ((uint64_t)tot + kSumTile - 1) / kSumTile; t <= (uint64_t)T; ++t) row[t] = (uint32_t)S;
}

// Workgroup -> (element tile, row, participant group) of the decode + sum kernels' grid
// (tiles, rows, groups). Workgroups are handed out in grid order, x fastest, round-robin over
// the 8 XCDs: with two tiles a row -- boxes of 10,000 values are a tile of 6,144 and one of
// 3,856 -- every first tile went to the even XCDs and every second one to the odd ones, which
// then waited for the even ones to finish. With fewer than 8 tiles a row the tile index
// therefore runs slowest: all the rows' first tiles, then all their second ones.
SDA_DEV SumTileId sum_tile_id() {
  return sum_tile_of(gridDim.x, gridDim.y, gridDim.z, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Each wave walks its own participants (round-robin over the group) in 4 KiB
// passes -- 64 lanes x 64 bytes, ranks by a wave scan -- so no block barrier
// sits between a pass's loads and the next: 16 independent waves per CU keep
// their loads in flight. The waves share the tile accumulator through ds_add.
template <bool kFast16, typename Sink, typename AccT>
SDA_DEV void decode_sum_body(AccT* acc, uint32_t (*info)[4], int L, int P, int Pg,
                             const ModParams& mp, const uint8_t* __restrict__ pt, uint64_t stride,
                             const uint32_t* __restrict__ pt_len, int S,
                             const uint32_t* __restrict__ pre, const uint32_t* __restrict__ tile_sub,
                             AccT* __restrict__ part, uint32_t* err) {
  constexpr int kWaveBytes = 64 * 64;
  const SumTileId id = sum_tile_id();
  const int t = id.t, r = id.r, g = id.g, R = gridDim.y;
  const int T = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t E0 = (uint32_t)t * kSumTile;
  const uint32_t W = min((uint32_t)kSumTile, (uint32_t)L - E0);
  for (int i = tid; i < kSumAcc; i += kBlock) acc[i] = 0;
  const int pbeg = g * Pg, pend = min(P, pbeg + Pg);
  bool bad = false;
  for (int b0 = pbeg; b0 < pend; b0 += kBlock) {
    const int cnt = min(kBlock, pend - b0);
    __syncthreads();  // previous batch's info reads done (and acc zeroed)
    if (tid < cnt) {
      const size_t j = (size_t)r * P + b0 + tid;
      const uint32_t s0 = tile_sub[j * (T + 1) + t];
      info[tid][0] = s0;
      info[tid][1] = tile_sub[j * (T + 1) + t + 1];
      info[tid][2] = s0 < (uint32_t)S ? pre[j * S + s0] : 0u;
      info[tid][3] = pt_len[j];
    }
    __syncthreads();
    for (int i = wave; i < cnt; i += kWaves) {
      const uint32_t s0 = info[i][0];
      if (s0 >= (uint32_t)S) continue;  // fewer elements than the tile start: malformed, flagged by the totals
      const uint32_t s1 = min(info[i][1], (uint32_t)S - 1);
      const int64_t N = info[i][3];
      const uint8_t* gmsg = pt + ((size_t)r * P + b0 + i) * stride + 48;
      const int64_t qs = max((int64_t)0, (int64_t)s0 * kSubBytes - 32);
      const int64_t qe = min(N, ((int64_t)s1 + 1) * kSubBytes - 32);
      uint32_t rank = info[i][2];
      for (int64_t c0 = (int64_t)s0 * kSubBytes - 32; c0 < qe; c0 += kWaveBytes) {
        const int64_t p0 = c0 + 64 * lane;
        uint32_t w[16];
        load_lane_bytes(w, gmsg, p0, qe);
        uint32_t wave_prev = 0, wave_prev2 = 0;
        if (lane == 0 && p0 - 4 >= 0 && p0 - 4 < N) wave_prev = *reinterpret_cast<const uint32_t*>(gmsg + p0 - 4);
        if (lane == 0 && p0 - 8 >= 0 && p0 - 8 < N) wave_prev2 = *reinterpret_cast<const uint32_t*>(gmsg + p0 - 8);
        const int lo = (int)max((int64_t)0, qs - p0);
        const int hi = (int)min((int64_t)64, qe - p0);
        const uint64_t traw = term_mask64(w);
        const uint64_t tmask = traw & byte_range_mask(lo, hi);
        const uint32_t c = (uint32_t)__popcll(tmask);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = wave_read_lane(incl, 63);
        const uint32_t prev_word = wave_shift_up1(w[15], wave_prev);  // lane 0: from global
        const uint32_t prev_word2 = wave_shift_up1(w[14], wave_prev2);
        Sink sink{acc, rank + kSumMargin - E0};
        bad |= decode_lane<kFast16>(w, prev_word2, prev_word, tmask, traw, incl - c, mp, gmsg, p0, sink);
        if (hi > lo && p0 + hi == N && (gmsg[N - 1] & 0x80)) bad = true;
        rank += total;
      }
    }
  }
  __syncthreads();
  AccT* out = part + ((size_t)g * R + r) * L + E0;
  for (uint32_t i = tid; i < W; i += kBlock) out[i] = acc[kSumMargin + i];
  if (bad) atomicOr(err, kErrMalformed);
}

// No occupancy hint: the unrolled decode paths need ~200 VGPRs (2 waves per
// SIMD); squeezing them into 128 or 168 spilled and measured slower.
template <bool kFast16, bool kWide>
__global__ void __launch_bounds__(kBlock)
    k_decode_sum(int L, int P, int Pg, ModParams mp, const uint8_t* __restrict__ pt,
                 uint64_t stride, const uint32_t* __restrict__ pt_len, int S,
                 const uint32_t* __restrict__ pre, const uint32_t* __restrict__ tile_sub,
                 uint32_t* __restrict__ part, uint32_t* err, const uint32_t* gate) {
  using AccT = std::conditional_t<kWide, unsigned long long, uint32_t>;
  __shared__ AccT acc[kSumAcc];
  __shared__ uint32_t info[kBlock][4];
  // behind the lean kernel: only if it met a stream it does not handle
  if (gate != nullptr && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  decode_sum_body<kFast16, std::conditional_t<kWide, AddSink64, AddSink>, AccT>(
      acc, info, L, P, Pg, mp, pt, stride, pt_len, S, pre, tile_sub, reinterpret_cast<AccT*>(part), err);
}

// ---------------------------------------- clerk decode + combine, lean form
// The common case -- canonical shares below 8192, i.e. every varint one or two
// bytes long and non-negative -- needs no per-element decode at all: the zigzag
// code of an element is the sum of its bytes' contributions
//     (byte & 0x7f) << (7 if the previous byte is a continuation byte else 0)
// so every byte position adds its contribution at the rank of the element it
// belongs to (a continuation byte has the rank of the terminator after it), and
// the accumulator ends up holding sum(z) = 2 * sum(value); k_sum_slabs halves.
// Same tiling, ranks and accumulator window as k_decode_sum; ~1/3 of its VALU
// work. A lane that sees anything else (three-byte varints, an odd = negative
// code) raises `redo`: the generic kernel, launched right after and gated on
// that word, then recomputes every slab (foreign encoders such as the
// reference's Rust-`%` shares, additive.rs:47, take that path).
//
// Ownership at range edges (ranges are cut at 1 KiB sub-chunks, which may split
// a two-byte varint): an element belongs to the range holding its terminator. A
// lane therefore drops a continuation byte in its last valid position and adds
// the continuation byte just before its first valid position (from its own
// words, or from the previous lane's last byte).
// acc[byte_off / 4] += v on an LDS array (32-bit LDS addressing, no return value)
SDA_DEV void lds_add(uint32_t* acc, uint32_t byte_off, uint32_t v) {
  __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(acc) + byte_off), v,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

SDA_DEV uint32_t spread4(uint32_t bits4) {  // 4 bits -> 0xff per set bit, byte k <- bit k
  return ((bits4 * 0x00204081u) & 0x01010101u) * 0xffu;
}

//
// kMaxBytes = 4 widens this to varints of up to four bytes (moduli up to 2^27, the
// large packed-Shamir fields): a byte's shift is 7 x (length of the run of
// continuation bytes right before it), a lane leaves the run of up to three
// continuation bytes at its end to the next lane, which adds them from the four
// bytes before its own; five-byte varints raise `redo`.
//
// kSwz: the accumulator with one pad word after every 32 (or 16) ranks (rank x at
// word x + (x >> 5)). A lane's 64 bytes hold 64 / (code length) elements, so with codes
// that are (nearly) all two, three or four bytes long the lanes' ranks are 32,
// 21.33 or 16 words apart and the same ds_add of every lane falls into one, three
// or two banks; in 33-word rows those strides step through all of them. Costs two
// VALU instructions per add: used for the long codes and for moduli whose codes are
// nearly all two bytes (m > 2048), not for the small moduli with their mix of one-
// and two-byte codes (irregular strides already).
template <int kMaxBytes, bool kSwz>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
    k_decode_sum_z(int L, int P, int Pg, const uint8_t* __restrict__ pt, uint64_t stride,
                   const uint32_t* __restrict__ pt_len, int S, const uint32_t* __restrict__ pre,
                   const uint32_t* __restrict__ tile_sub, uint32_t* __restrict__ part,
                   uint32_t* redo, uint32_t* err) {
  // kMaxBytes = 3: the field's codes have at most three bytes, a fourth raises `redo`
  // (the caller sized the participant groups for 21-bit codes)
  constexpr bool three = kMaxBytes == 3;
  constexpr int kWaveBytes = 64 * 64;
  // pad stride: every 32 words for two-byte codes (ranks 32 apart -> 33), every 16 for
  // the long ones (21.33 / 16 apart -> 22.67 / 17: odd and even banks alike)
  constexpr int kPadShift = kMaxBytes > 2 ? 4 : 5;
  constexpr int kAccWords = kSwz ? kSumAcc + (kSumAcc >> kPadShift) + 1 : kSumAcc;
  __shared__ uint32_t acc[kAccWords];
  __shared__ uint32_t info[kBlock][4];
  // acc[byte offset / 4] += v, through the padded layout when kSwz
  auto add = [&](uint32_t byte_off, uint32_t v) {
    lds_add(acc, kSwz ? byte_off + ((byte_off >> (kPadShift + 2)) << 2) : byte_off, v);
  };
  const SumTileId id = sum_tile_id();
  const int t = id.t, r = id.r, g = id.g, R = gridDim.y;
  const int T = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t E0 = (uint32_t)t * kSumTile;
  const uint32_t W = min((uint32_t)kSumTile, (uint32_t)L - E0);
  for (int i = tid; i < kAccWords; i += kBlock) acc[i] = 0;
  const int pbeg = g * Pg, pend = min(P, pbeg + Pg);
  uint32_t bad = 0;      // bit 7 / bit 0 of any byte: not a canonical short stream
  bool malformed = false;
  for (int b0 = pbeg; b0 < pend; b0 += kBlock) {
    const int cnt = min(kBlock, pend - b0);
    __syncthreads();  // previous batch's info reads done (and acc zeroed)
    if (tid < cnt) {
      const size_t j = (size_t)r * P + b0 + tid;
      const uint32_t s0 = tile_sub[j * (T + 1) + t];
      info[tid][0] = s0;
      info[tid][1] = tile_sub[j * (T + 1) + t + 1];
      info[tid][2] = s0 < (uint32_t)S ? pre[j * S + s0] : 0u;
      info[tid][3] = pt_len[j];
    }
    __syncthreads();
    // This wave's work items of the batch: (message i, 4 KiB pass at c0), walked
    // as one flat sequence so that the next item's bytes are already in flight
    // while the current one is processed (an item's loads are otherwise waited
    // for right after they are issued).
    int ni = wave;  // next message of the batch to open
    const uint8_t* n_gmsg = nullptr;
    int64_t n_c0 = 0, n_qs = 0, n_qe = 0, n_N = 0;
    uint32_t n_rank = 0;
    bool n_first = false, n_valid = false;
    auto open_next = [&]() {  // advance (n_*) to the item after it
      if (n_valid && n_c0 + kWaveBytes < n_qe) {
        n_c0 += kWaveBytes;
        n_first = false;
        return;
      }
      n_valid = false;
      while (ni < cnt) {
        const int i = ni;
        ni += kWaves;
        const uint32_t s0 = info[i][0];
        if (s0 >= (uint32_t)S) continue;  // fewer elements than the tile start: flagged by the totals
        const uint32_t s1 = min(info[i][1], (uint32_t)S - 1);
        n_N = info[i][3];
        n_gmsg = pt + ((size_t)r * P + b0 + i) * stride + 48;
        n_qs = max((int64_t)0, (int64_t)s0 * kSubBytes - 32);
        n_qe = min(n_N, ((int64_t)s1 + 1) * kSubBytes - 32);
        n_c0 = (int64_t)s0 * kSubBytes - 32;
        n_rank = info[i][2];
        n_first = true;
        n_valid = n_c0 < n_qe;
        if (n_valid) return;
      }
    };
    uint32_t wn[16], pn = 0;  // the next item's bytes, and the 4 bytes before lane 0's
    auto fetch_next = [&]() {
      const int64_t p0 = n_c0 + 64 * lane;
      load_lane_bytes(wn, n_gmsg, p0, n_qe);
      pn = 0;
      if (lane == 0 && p0 - 4 >= 0 && p0 - 4 < n_N) pn = *reinterpret_cast<const uint32_t*>(n_gmsg + p0 - 4);
    };
    open_next();
    if (n_valid) fetch_next();
    uint32_t rank = 0;
    while (n_valid) {
      const uint8_t* gmsg = n_gmsg;
      const int64_t c0 = n_c0, qs = n_qs, qe = n_qe, N = n_N;
      if (n_first) rank = n_rank;
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = wn[q];
      const uint32_t wave_prev = pn;
      open_next();
      if (n_valid) fetch_next();
      {
        const int64_t p0 = c0 + 64 * lane;
        // the 4 bytes before this lane's (raw; lane 0's come from global memory)
        uint32_t pm1 = wave_shift_up1(w[15], wave_prev);
        const int lo = (int)max((int64_t)0, qs - p0);
        const int hi = (int)min((int64_t)64, qe - p0);
        // a message must end on a terminator
        if (hi > lo && p0 + hi == N && (gmsg[N - 1] & 0x80)) malformed = true;
        uint32_t tw[16];  // valid terminators, in place (bit 7 of their byte)
        if (lo > 0 || hi < 64) {
          uint64_t K = byte_range_mask(lo, hi);  // bytes that contribute
          const uint64_t V = K;                  // bytes whose terminators count
          if (hi > lo) {
            const uint64_t craw = ~term_mask64(w);
            if (lo > 0) K |= craw & (1ull << (lo - 1));
            uint64_t run = craw & (1ull << (hi - 1));  // continuation bytes at the end: the next lane's
            if constexpr (kMaxBytes > 2) run |= (run >> 1) & craw;
            if constexpr (kMaxBytes > 3) run |= (run >> 1) & craw;
            K &= ~run;
          }
          if (lo > 0 || hi <= lo) pm1 = 0;  // the byte before this lane is not its to add
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t k4 = (uint32_t)(K >> (4 * q)) & 15u, v4 = (uint32_t)(V >> (4 * q)) & 15u;
            tw[q] = ~w[q] & spread4(v4) & 0x80808080u;
            w[q] &= spread4(k4);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q) tw[q] = ~w[q] & 0x80808080u;
          // a continuation byte in the last position belongs to the next lane's element
          if constexpr (kMaxBytes <= 2) {
            w[15] &= ~((uint32_t)((int32_t)w[15] >> 31) & 0xff000000u);
          } else {  // ... the run of up to three (two) of them
            const uint32_t x15 = w[15];
            const uint32_t t3 = (uint32_t)((int32_t)x15 >> 31);
            const uint32_t t2 = t3 & (uint32_t)((int32_t)(x15 << 8) >> 31);
            uint32_t drop = (t3 & 0xff000000u) | (t2 & 0x00ff0000u);
            if constexpr (kMaxBytes > 3) drop |= t2 & (uint32_t)((int32_t)(x15 << 16) >> 31) & 0x0000ff00u;
            w[15] = x15 & ~drop;
          }
        }
        uint32_t c = 0;
        uint32_t lead = 0;  // kMaxBytes > 2: what the continuation run before this lane adds
        if constexpr (kMaxBytes <= 2) {
          uint32_t wp = pm1;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t pcb = __builtin_amdgcn_alignbyte(w[q], wp, 3) & 0x80808080u;
            bad |= w[q] & pcb;                                  // continuation after continuation
            bad |= w[q] & 0x01010101u & ~(pcb >> 7);            // odd first byte: a negative value
            c += (uint32_t)__popc(tw[q]);
            wp = w[q];
          }
          bad |= (pm1 >> 24) & (pm1 >> 31) & 1u;                // ... of the byte before
          bad |= (pm1 >> 16) & (pm1 >> 24) & 0x80u;             // two continuation bytes before it
        } else {
          uint32_t wp = pm1;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t x = w[q];
            const uint32_t c1 = __builtin_amdgcn_alignbyte(x, wp, 3) & 0x80808080u;
            const uint32_t c2 = c1 & __builtin_amdgcn_alignbyte(x, wp, 2);
            if constexpr (three) {
              bad |= x & c2;                                    // one continuation byte too many in a row
            } else {
              bad |= x & c2 & __builtin_amdgcn_alignbyte(x, wp, 1);
            }
            bad |= x & 0x01010101u & ~(c1 >> 7);                // odd first byte: a negative value
            c += (uint32_t)__popc(tw[q]);
            wp = x;
          }
          // the run of continuation bytes right before this lane (the previous lane left
          // it out): b3 is the byte before, then b2, b1; its first byte has shift 0
          const uint32_t b1 = (pm1 >> 8) & 0xffu, b2 = (pm1 >> 16) & 0xffu, b3 = pm1 >> 24;
          const bool t3 = b3 & 0x80u, t2 = t3 && (b2 & 0x80u), t1 = t2 && (b1 & 0x80u);
          // (three continuation bytes before the lane: a four-byte code, flagged below when
          // the field has none; the previous lane then kept the first of them)
          lead = t1 && !three ? ((b1 & 0x7fu) | ((b2 & 0x7fu) << 7) | ((b3 & 0x7fu) << 14))
               : t2 ? ((b2 & 0x7fu) | ((b3 & 0x7fu) << 7))
               : t3 ? (b3 & 0x7fu) : 0u;
          bad |= lead & 1u;                                     // odd first byte of that run
          // too many continuation bytes before it (a code of five / four bytes)
          bad |= three ? (t1 ? 0x80u : 0u) : (pm1 & (pm1 >> 8) & (pm1 >> 16) & (pm1 >> 24) & 0x80u);
        }
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = wave_read_lane(incl, 63);
        // byte offset (within acc) of the rank of this lane's first terminator
        uint32_t a4 = 4u * (rank + kSumMargin - E0 + (incl - c));
        if constexpr (kMaxBytes <= 2) add(a4, ((pm1 >> 24) & 0x7fu) & (0u - (pm1 >> 31)));
        else add(a4, lead);
        uint32_t wp = pm1;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const uint32_t x = w[q];
          // continuation bytes right before each byte: 0 / 1, or the run length 0..3
          uint32_t pc = (__builtin_amdgcn_alignbyte(x, wp, 3) & 0x80808080u) >> 7;
          if constexpr (kMaxBytes > 2) {
            const uint32_t c2 = pc & (__builtin_amdgcn_alignbyte(x, wp, 2) >> 7);
            if constexpr (kMaxBytes > 3) pc += c2 & (__builtin_amdgcn_alignbyte(x, wp, 1) >> 7);
            pc += c2;
          }
          // (opaque steps: left to itself the compiler folds these shift-adds into
          // v_mul_lo_u32, a quarter-rate instruction, and the byte fields below
          // into bit-field extracts instead of free byte selects)
          uint32_t sh4 = pc << 3;
          asm volatile("" : "+v"(sh4));
          sh4 -= pc;                            // 7 per continuation byte before, per byte
          uint32_t w7 = x & 0x7f7f7f7fu;
          // 4 * (terminators before byte u of this word), per byte
          uint32_t pre4 = tw[q] >> 5;           // 4 per terminator
          asm volatile("" : "+v"(pre4));
          pre4 += pre4 << 8;
          asm volatile("" : "+v"(pre4));
          pre4 += pre4 << 16;                   // inclusive
          asm volatile("" : "+v"(pre4));
          uint32_t ex4 = pre4 << 8;             // exclusive
          asm volatile("" : "+v"(ex4), "+v"(w7), "+v"(sh4));
#pragma unroll
          for (int u = 0; u < 4; ++u)
            add(a4 + ((ex4 >> (8 * u)) & 0xffu), ((w7 >> (8 * u)) & 0xffu) << ((sh4 >> (8 * u)) & 0xffu));
          a4 += pre4 >> 24;
          wp = x;
        }
        rank += total;
      }
    }
  }
  __syncthreads();
  uint32_t* out = part + ((size_t)g * R + r) * L + E0;
  for (uint32_t i = tid; i < W; i += kBlock) {
    const uint32_t x = kSumMargin + i;
    out[i] = acc[kSwz ? x + (x >> kPadShift) : x];
  }
  if (bad) atomicOr(redo, 1u);
  if (malformed) atomicOr(err, kErrMalformed);
}

// ------------------------------- clerk decode + combine, lean form for long codes
// Fields whose codes are mostly three or four bytes long (the large packed-Shamir
// primes) spend the byte-wise kernel above badly: three or four LDS adds and ~60 VALU
// instructions per value. Here a wave stages its 4 KiB pass in LDS and every lane walks
// its own terminators: the four bytes ending at a terminator come back as one unaligned
// LDS read whatever lane they started in, the run of continuation bits in front of the
// terminator (0..3) says how many of the four 7-bit groups belong to the code, and the
// code goes to its rank in one add: ~28 VALU instructions and two LDS accesses per
// value. A value belongs to the lane that holds its terminator, so there is no
// hand-over of leading or trailing bytes between lanes. Codes longer than kMaxBytes
// (any run of kMaxBytes continuation bytes, inside a lane or across two) and odd codes
// (negative values) raise `redo` as above.
template <int kMaxBytes, bool kSwz>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
    k_decode_sum_v(int L, int P, int Pg, const uint8_t* __restrict__ pt, uint64_t stride,
                   const uint32_t* __restrict__ pt_len, int S, const uint32_t* __restrict__ pre,
                   const uint32_t* __restrict__ tile_sub, uint32_t* __restrict__ part,
                   uint32_t* redo, uint32_t* err) {
  static_assert(kMaxBytes == 3 || kMaxBytes == 4, "codes of three or four bytes");
  constexpr int kWaveBytes = 64 * 64;
  constexpr int kPadShift = 5;  // one pad word per 32 ranks
  constexpr int kAccWords = kSwz ? kSumAcc + (kSumAcc >> kPadShift) + 1 : kSumAcc;
  // a lane's slot: the 4 bytes before its 64 (its neighbour's last word, or the bytes before
  // the pass) and the 64, 17 words -- an odd stride, so that the lanes' window reads, each
  // inside its own slot, fall into different banks (side by side, 16 words apart, every
  // read was a 32-way conflict); one more word after the last slot for a window's second
  constexpr int kSlotWords = 17;
  constexpr int kStageWords = 64 * kSlotWords + 1;
  __shared__ uint32_t acc[kAccWords];
  constexpr int kBatch = 128;  // messages whose tile descriptors are staged at a time
  __shared__ uint32_t info[kBatch][4];
  __shared__ uint32_t stage[kWaves][kStageWords];
  auto add = [&](uint32_t byte_off, uint32_t v) {
    lds_add(acc, kSwz ? byte_off + ((byte_off >> (kPadShift + 2)) << 2) : byte_off, v);
  };
  const SumTileId id = sum_tile_id();
  const int t = id.t, r = id.r, g = id.g, R = gridDim.y;
  const int T = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t E0 = (uint32_t)t * kSumTile;
  const uint32_t W = min((uint32_t)kSumTile, (uint32_t)L - E0);
  for (int i = tid; i < kAccWords; i += kBlock) acc[i] = 0;
  uint32_t* const slot = &stage[wave][kSlotWords * lane];  // this lane's: [0] history, [1..16] bytes
  const int pbeg = g * Pg, pend = min(P, pbeg + Pg);
  uint32_t bad = 0;
  bool malformed = false;
  for (int b0 = pbeg; b0 < pend; b0 += kBatch) {
    const int cnt = min(kBatch, pend - b0);
    __syncthreads();  // previous batch's info reads done (and acc zeroed)
    if (tid < cnt) {
      const size_t j = (size_t)r * P + b0 + tid;
      const uint32_t s0 = tile_sub[j * (T + 1) + t];
      info[tid][0] = s0;
      info[tid][1] = tile_sub[j * (T + 1) + t + 1];
      info[tid][2] = s0 < (uint32_t)S ? pre[j * S + s0] : 0u;
      info[tid][3] = pt_len[j];
    }
    __syncthreads();
    // work items (message, 4 KiB pass) as in k_decode_sum_z: the next item's bytes are in
    // flight while the current one is processed
    int ni = wave;
    const uint8_t* n_gmsg = nullptr;
    int64_t n_c0 = 0, n_qs = 0, n_qe = 0, n_N = 0;
    uint32_t n_rank = 0;
    bool n_first = false, n_valid = false;
    auto open_next = [&]() {
      if (n_valid && n_c0 + kWaveBytes < n_qe) {
        n_c0 += kWaveBytes;
        n_first = false;
        return;
      }
      n_valid = false;
      while (ni < cnt) {
        const int i = ni;
        ni += kWaves;
        const uint32_t s0 = info[i][0];
        if (s0 >= (uint32_t)S) continue;  // fewer elements than the tile start: flagged by the totals
        const uint32_t s1 = min(info[i][1], (uint32_t)S - 1);
        n_N = info[i][3];
        n_gmsg = pt + ((size_t)r * P + b0 + i) * stride + 48;
        n_qs = max((int64_t)0, (int64_t)s0 * kSubBytes - 32);
        n_qe = min(n_N, ((int64_t)s1 + 1) * kSubBytes - 32);
        n_c0 = (int64_t)s0 * kSubBytes - 32;
        n_rank = info[i][2];
        n_first = true;
        n_valid = n_c0 < n_qe;
        if (n_valid) return;
      }
    };
    uint32_t wn[16], pn = 0;  // the next item's bytes, and the 4 bytes before lane 0's
    auto fetch_next = [&]() {
      const int64_t p0 = n_c0 + 64 * lane;
      load_lane_bytes(wn, n_gmsg, p0, n_qe);
      pn = 0;
      if (lane == 0 && p0 - 4 >= 0 && p0 - 4 < n_N) pn = *reinterpret_cast<const uint32_t*>(n_gmsg + p0 - 4);
    };
    open_next();
    if (n_valid) fetch_next();
    uint32_t rank = 0;
    while (n_valid) {
      const uint8_t* gmsg = n_gmsg;
      const int64_t c0 = n_c0, qs = n_qs, qe = n_qe, N = n_N;
      if (n_first) rank = n_rank;
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = wn[q];
      const uint32_t wave_prev = pn;
      open_next();
      if (n_valid) fetch_next();
      const int64_t p0 = c0 + 64 * lane;
      const int lo = (int)max((int64_t)0, qs - p0);
      const int hi = (int)min((int64_t)64, qe - p0);
      if (hi > lo && p0 + hi == N && (gmsg[N - 1] & 0x80)) malformed = true;  // must end on a terminator
      // the pass into LDS (the previous item's reads were issued before these writes)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < 16; ++q) slot[1 + q] = w[q];
      if (lane < 63) slot[kSlotWords] = w[15];  // the next lane's history
      if (lane == 0) slot[0] = wave_prev;
      const uint64_t traw = term_mask64(w);
      const uint64_t tmask = traw & byte_range_mask(lo, hi);
      // too long a code: kMaxBytes continuation bytes in a row, within the lane ...
      {
        // (bytes from `hi` on are the next range's or past the message: taken as terminators)
        const uint64_t tv = traw | ~byte_range_mask(0, hi);
        const uint64_t craw = ~tv;
        uint64_t runs = craw & (craw >> 1) & (craw >> 2);
        if constexpr (kMaxBytes > 3) runs &= craw >> 3;
        // ... or across the lane's start: those at the end of the lane before + those here
        const uint32_t head = tv ? (uint32_t)__builtin_ctzll(tv) : 64u;
        const uint32_t tail = tv ? (uint32_t)__builtin_clzll(tv) : 64u;
        const uint32_t hist = ~wave_prev & 0x80808080u;  // lane 0: the four bytes before the pass
        const uint32_t tail0 = hist ? (uint32_t)__builtin_clz(hist) >> 3 : 4u;
        const uint32_t before = wave_shift_up1(tail, tail0);
        bad |= (runs != 0 ? 0x80u : 0u) | (before + head >= (uint32_t)kMaxBytes ? 0x40u : 0u);
      }
      const uint32_t c = (uint32_t)__popcll(tmask);
      const uint32_t incl = wave_incl_scan(c);
      const uint32_t total = wave_read_lane(incl, 63);
      uint32_t a4 = 4u * (rank + kSumMargin - E0 + (incl - c));  // byte offset of the lane's first rank
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // the lane's terminators, low half of its bytes then high half; the window of the
      // next terminator is requested before the current one is worked on
      // A value's window -- bytes p - 3 .. p of the lane, the terminator on top -- is two
      // aligned words and a byte shift (an unaligned LDS access costs several aligned ones),
      // requested one turn ahead and put together only when used.
      struct Window {
        uint32_t lo, hi, sh;
      };
      auto request = [&](int p) {
        const uint32_t off = (uint32_t)p + 1u;  // byte offset in the slot of byte p - 3
        const uint32_t* q = slot + (off >> 2);
        return Window{q[0], q[1], off & 3u};
      };
      auto emit = [&](const Window& wd, uint32_t at) {
        const uint32_t win = __builtin_amdgcn_alignbyte(wd.hi, wd.lo, wd.sh);
        const uint32_t m7 = win >> 7;
        const uint32_t c2 = (m7 >> 16) & 1u;   // byte p - 1 continues
        const uint32_t c1 = (m7 >> 8) & c2;    // ... and p - 2
        const uint32_t c0 = m7 & c1;           // ... and p - 3
        const uint32_t rl = c2 + c1 + c0;
        const uint32_t g7 = win & 0x7f7f7f7fu;
        const uint32_t x = (g7 & 0x007f007fu) | ((g7 & 0x7f007f00u) >> 1);
        const uint32_t full = (x & 0x3fffu) | ((x >> 2) & 0x0fffc000u);
        const uint32_t z = full >> (21u - 7u * rl);
        bad |= z & 1u;  // odd: a negative value
        add(at, z);
      };
      // both halves of the lane's bytes side by side: one terminator of each per turn (two
      // independent chains, half the loop turns)
      uint32_t t0 = (uint32_t)tmask, t1 = (uint32_t)(tmask >> 32);
      uint32_t a40 = a4, a41 = a4 + 4u * (uint32_t)__popc(t0);
      Window n0 = {0, 0, 0}, n1 = {0, 0, 0};
      if (t0 != 0) n0 = request(__builtin_ctz(t0));
      if (t1 != 0) n1 = request(__builtin_ctz(t1) + 32);
      // one turn: the windows in (c0, c1) are worked on, the next ones requested into (x0, x1).
      // Two turns a loop pass with the roles of the two window pairs swapped, so that no
      // window is copied from "next" to "current" (8 moves a turn otherwise: 11.5 -> 11.1 ms).
      // The branches stay: with requests and adds unconditional (idle lanes reading a window
      // they do not use and adding zero) the kernel took 12.0 ms -- a half of the lanes' bytes
      // that has run out in every lane is skipped whole by the branch.
      auto turn = [&](const Window& c0, const Window& c1, Window& x0, Window& x1) {
        const bool h0 = t0 != 0, h1 = t1 != 0;
        t0 &= t0 - 1;
        t1 &= t1 - 1;
        if (t0 != 0) x0 = request(__builtin_ctz(t0));
        if (t1 != 0) x1 = request(__builtin_ctz(t1) + 32);
        if (h0) {
          emit(c0, a40);
          a40 += 4u;
        }
        if (h1) {
          emit(c1, a41);
          a41 += 4u;
        }
      };
      Window m0 = {0, 0, 0}, m1 = {0, 0, 0};
      while (__builtin_amdgcn_ballot_w64((t0 | t1) != 0) != 0) {
        turn(n0, n1, m0, m1);
        if (__builtin_amdgcn_ballot_w64((t0 | t1) != 0) == 0) break;
        turn(m0, m1, n0, n1);
      }
      rank += total;
    }
  }
  __syncthreads();
  uint32_t* out = part + ((size_t)g * R + r) * L + E0;
  for (uint32_t i = tid; i < W; i += kBlock) {
    const uint32_t x = kSumMargin + i;
    out[i] = acc[kSwz ? x + (x >> kPadShift) : x];
  }
  if (bad) atomicOr(redo, bad);  // 0x80 / 0x40: a code too long (inside a lane / across two), 1: an odd code
  if (malformed) atomicOr(err, kErrMalformed);
}

// out[x] = sum_g part[g][x] mod m   (x < X = rows * L); with `acc` the result is added
// to acc[x] instead (the running sums of a round done in participant waves).
// `zform` (may be null): *zform == 0 means the slabs hold sums of zigzag codes
// (2 * value, from k_decode_sum_z) and are halved first.
__global__ void __launch_bounds__(kBlock)
    k_sum_slabs(int G, int64_t X, ModParams mp, const uint32_t* __restrict__ part,
                uint32_t* __restrict__ out, const uint32_t* zform, int64_t* __restrict__ acc) {
  const int64_t x = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
  if (x >= X) return;
  const int sh = (zform != nullptr && *zform == 0u) ? 1 : 0;
  if (x + 4 <= X) {
    // 16-byte loads at 4-byte alignment: slab g starts at g * X words, X any length
    // (333,334 batches in the packed-Shamir rounds)
    struct __attribute__((packed, aligned(4))) Q {
      uint32_t w[4];
    };
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int g = 0;
    for (; g + 8 <= G; g += 8) {  // eight slabs' loads in flight at once (the slabs are far apart)
      Q q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = *reinterpret_cast<const Q*>(part + (int64_t)(g + u) * X + x);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a0 += q[u].w[0]; a1 += q[u].w[1]; a2 += q[u].w[2]; a3 += q[u].w[3];
      }
    }
    for (; g < G; ++g) {
      const Q q = *reinterpret_cast<const Q*>(part + (int64_t)g * X + x);
      a0 += q.w[0]; a1 += q.w[1]; a2 += q.w[2]; a3 += q.w[3];
    }
    const uint4 r = make_uint4(mod64(a0 >> sh, mp), mod64(a1 >> sh, mp), mod64(a2 >> sh, mp),
                               mod64(a3 >> sh, mp));
    if (acc != nullptr) {
      acc[x] += r.x; acc[x + 1] += r.y; acc[x + 2] += r.z; acc[x + 3] += r.w;
    } else {
      *reinterpret_cast<Q*>(out + x) = Q{{r.x, r.y, r.z, r.w}};  // `out` may be a row of a wider tensor
    }
  } else {
    for (int64_t y = x; y < min(X, x + 4); ++y) {
      uint64_t a = 0;
      for (int g = 0; g < G; ++g) a += part[g * X + y];
      const uint32_t r = mod64(a >> sh, mp);
      if (acc != nullptr) acc[y] += r;
      else out[y] = r;
    }
  }
}

// The same over 64-bit slabs (k_decode_sum<.., true>: sums of canonical values).
__global__ void __launch_bounds__(kBlock)
    k_sum_slabs64(int G, int64_t X, ModParams mp, const unsigned long long* __restrict__ part,
                  uint32_t* __restrict__ out, int64_t* __restrict__ acc) {
  const int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (x >= X) return;
  // every slab's sum is below P 2^32; reduced one by one, the total of residues below G 2^32
  uint64_t a = 0;
  for (int g = 0; g < G; ++g) a += mod64(part[(int64_t)g * X + x], mp);
  const uint32_t r = mod64(a, mp);
  if (acc != nullptr) acc[x] += r;
  else out[x] = r;
}

template <typename VT, typename ACC>
__global__ void __launch_bounds__(kBlock)
    k_colsum(int R, int L, ModParams mp, const VT* __restrict__ vals, uint32_t* __restrict__ out) {
  const int g = blockIdx.y;
  const int l0 = (blockIdx.x * kBlock + threadIdx.x) * 8;
  if (l0 >= L) return;
  const VT* src = vals + (size_t)g * R * L;
  ACC acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool vec = (L % 8) == 0;
  if (vec) {
    for (int r = 0; r < R; ++r) {
      const VT* row = src + (size_t)r * L + l0;
      if constexpr (sizeof(VT) == 2) {
        uint4 q = *reinterpret_cast<const uint4*>(row);
        acc[0] += q.x & 0xffff; acc[1] += q.x >> 16; acc[2] += q.y & 0xffff; acc[3] += q.y >> 16;
        acc[4] += q.z & 0xffff; acc[5] += q.z >> 16; acc[6] += q.w & 0xffff; acc[7] += q.w >> 16;
      } else {
        uint4 a = reinterpret_cast<const uint4*>(row)[0];
        uint4 b = reinterpret_cast<const uint4*>(row)[1];
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
    }
  } else {
    for (int r = 0; r < R; ++r) {
      const VT* row = src + (size_t)r * L;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (l0 + i < L) acc[i] += row[l0 + i];
    }
  }
  uint32_t* o = out + (size_t)g * L;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (l0 + i < L) o[l0 + i] = mod64((uint64_t)acc[i], mp);
}

__global__ void __launch_bounds__(kBlock)
    k_pss_reconstruct(int B, int k, int nI, int D, ModParams mp, const uint32_t* __restrict__ lag,
                      const uint32_t* __restrict__ ys, uint32_t* __restrict__ out) {
  extern __shared__ uint32_t sL[];
  for (int i = threadIdx.x; i < k * nI; i += kBlock) sL[i] = lag[i];
  __syncthreads();
  const int b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= B) return;
  for (int s = 0; s < k; ++s) {
    const int e = b * k + s;
    if (e >= D) break;
    uint32_t acc = 0;
    for (int i = 0; i < nI; ++i)
      acc = add_mod(acc, mod64((uint64_t)sL[s * nI + i] * ys[(size_t)i * B + b], mp), mp.m);
    out[e] = acc;
  }
}

__global__ void k_sub_mod(int D, uint32_t m, const uint32_t* __restrict__ a,
                          const uint32_t* __restrict__ b, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D) out[i] = sub_mod(a[i], b[i], m);
}

}  // namespace

static int g_decode_lean = 1;
void set_decode_lean(int mode) { g_decode_lean = mode; }
static int g_decode_long = -1;  // long-code lean decode: -1 by field, 1 value-wise (k_decode_sum_v), 0 byte-wise
void set_decode_long(int mode) { g_decode_long = mode; }
static int g_decode_swz = -1;  // padded accumulator rows: -1 by modulus, 0 never, 1 always
void set_decode_swz(int mode) { g_decode_swz = mode; }

void launch_decode(int M, int K, int L, uint32_t m, int value_bytes, const uint8_t* pt,
                   uint64_t stride, const uint32_t* pt_len, const uint32_t* elem_start,
                   void* vals, uint32_t* err, hipStream_t s) {
  if (M <= 0 || K <= 0) return;
  ModParams mp = make_mod_params(m);
  dim3 grid(K, M);
  if (value_bytes == 2)
    hipLaunchKernelGGL(k_decode<uint16_t>, grid, dim3(kBlock), 0, s, L, mp, pt, stride, pt_len,
                       elem_start, (uint16_t*)vals, err);
  else
    hipLaunchKernelGGL(k_decode<uint32_t>, grid, dim3(kBlock), 0, s, L, mp, pt, stride, pt_len,
                       elem_start, (uint32_t*)vals, err);
}

void launch_locate_tiles(int M, int S, int L, const uint32_t* pre, const uint32_t* totals,
                         uint32_t* tile_sub, hipStream_t s) {
  if (M <= 0 || S <= 0 || L <= 0) return;
  const int T = (L + kSumTile - 1) / kSumTile;
  hipLaunchKernelGGL(k_locate_tiles, dim3((S + kBlock - 1) / kBlock, M), dim3(kBlock), 0, s, S, T,
                     pre, totals, tile_sub);
}

void launch_decode_sum(int R, int P, int Pg, int L, uint32_t m, const uint8_t* pt, uint64_t stride,
                       const uint32_t* pt_len, int S, const uint32_t* pre, const uint32_t* tile_sub,
                       uint32_t* part, uint32_t* out, int64_t* acc, uint32_t* err, uint32_t* redo,
                       hipStream_t s) {
  if (R <= 0 || P <= 0 || L <= 0 || Pg <= 0 || m == 0) return;
  const ModParams mp = make_mod_params(m);
  const int T = (L + kSumTile - 1) / kSumTile;
  const int G = (P + Pg - 1) / Pg;
  dim3 grid(T, R, G);
  // lean kernel first where every canonical value is a 1- or 2-byte varint; the
  // generic one then runs only if `redo` was raised (it rewrites every slab)
  // (codes of 2 bytes below 2^14, of 4 bytes below 2^28: moduli up to 2^13 / 2^27)
  const bool lean = g_decode_lean && redo != nullptr && m <= (1u << 27);
  // padded accumulator rows where they measured faster: fields of (nearly) all
  // two-byte codes (ranks 32 words apart) and of three-byte codes (21.33 apart: 728
  // clerks x 1000 participants, 24.9 -> 22.9 ms); with mostly four-byte codes the two
  // extra instructions per add cost more than the conflicts (5.8 -> 6.7 ms)
  const bool three = 2ull * (m - 1) < (1ull << 21);
  const bool swz = g_decode_swz < 0 ? (m > 2048u && (m <= 8192u || three)) : g_decode_swz != 0;
  if (lean && m <= 8192u) {
    auto kern = swz ? k_decode_sum_z<2, true> : k_decode_sum_z<2, false>;
    hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, s, L, P, Pg, pt, stride, pt_len, S, pre,
                       tile_sub, part, redo, err);
  } else if (lean) {  // canonical codes 2 (m - 1) below 2^21 have at most three bytes
    // value-wise kernel or byte-wise one. Measured: three-byte codes, 1000 participants a
    // row: 18.0 against 22.3 ms (728 rows); four-byte codes, 16 participants a row: 8.2
    // against 5.6 ms (19,682 rows: the value-wise kernel's larger LDS footprint -- three
    // workgroups a CU instead of four -- and per-workgroup set-up weigh more than its
    // fewer LDS adds). g_decode_long: -1 by that rule (default), 0 byte-wise, 1 value-wise.
    const bool by_value = g_decode_long < 0 ? three : g_decode_long != 0;
    auto kern = by_value
                    ? (three ? (swz ? k_decode_sum_v<3, true> : k_decode_sum_v<3, false>)
                             : (swz ? k_decode_sum_v<4, true> : k_decode_sum_v<4, false>))
                    : (three ? (swz ? k_decode_sum_z<3, true> : k_decode_sum_z<3, false>)
                             : (swz ? k_decode_sum_z<4, true> : k_decode_sum_z<4, false>));
    hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, s, L, P, Pg, pt, stride, pt_len, S, pre,
                       tile_sub, part, redo, err);
  }
  const uint32_t* gate = lean ? redo : nullptr;
  const int64_t X = (int64_t)R * L;
  if (decode_sum_wide(m)) {
    // values a u32 accumulator could add up only a few of: 64-bit accumulators and slabs
    hipLaunchKernelGGL((k_decode_sum<false, true>), grid, dim3(kBlock), 0, s, L, P, Pg, mp, pt, stride,
                       pt_len, S, pre, tile_sub, part, err, gate);
    hipLaunchKernelGGL(k_sum_slabs64, dim3((unsigned)((X + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, G, X, mp,
                       reinterpret_cast<const unsigned long long*>(part), out, acc);
    return;
  }
  if (m < 65536u)
    hipLaunchKernelGGL((k_decode_sum<true, false>), grid, dim3(kBlock), 0, s, L, P, Pg, mp, pt, stride,
                       pt_len, S, pre, tile_sub, part, err, gate);
  else
    hipLaunchKernelGGL((k_decode_sum<false, false>), grid, dim3(kBlock), 0, s, L, P, Pg, mp, pt, stride,
                       pt_len, S, pre, tile_sub, part, err, gate);
  const int64_t threads = (X + 3) / 4;
  hipLaunchKernelGGL(k_sum_slabs, dim3((unsigned)((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     G, X, mp, part, out, gate, acc);
}

void launch_colsum(int G, int R, int L, uint32_t m, int value_bytes, const void* vals,
                   uint32_t* out, hipStream_t s) {
  if (G <= 0 || L <= 0) return;
  ModParams mp = make_mod_params(m);
  const int threads = (L + 7) / 8;
  dim3 grid((threads + kBlock - 1) / kBlock, G);
  if (value_bytes == 2 && (uint64_t)R * 65535ull < 0xffffffffull)
    hipLaunchKernelGGL((k_colsum<uint16_t, uint32_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint16_t*)vals, out);
  else if (value_bytes == 2)
    hipLaunchKernelGGL((k_colsum<uint16_t, uint64_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint16_t*)vals, out);
  else
    hipLaunchKernelGGL((k_colsum<uint32_t, uint64_t>), grid, dim3(kBlock), 0, s, R, L, mp,
                       (const uint32_t*)vals, out);
}

void launch_pss_reconstruct(int B, int k, int nI, int D, uint32_t p, const uint32_t* lag,
                            const uint32_t* ys, uint32_t* out, hipStream_t s) {
  if (B <= 0) return;
  ModParams mp = make_mod_params(p);
  hipLaunchKernelGGL(k_pss_reconstruct, dim3((B + kBlock - 1) / kBlock), dim3(kBlock),
                     (size_t)k * nI * sizeof(uint32_t), s, B, k, nI, D, mp, lag, ys, out);
}

void launch_sub_mod(int D, uint32_t m, const uint32_t* a, const uint32_t* b, uint32_t* out,
                    hipStream_t s) {
  if (D <= 0) return;
  hipLaunchKernelGGL(k_sub_mod, dim3((D + 255) / 256), dim3(256), 0, s, D, m, a, b, out);
}

}  // namespace sdagpu
