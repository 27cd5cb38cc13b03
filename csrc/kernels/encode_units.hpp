// Which (tile, message) a workgroup -- or, for short message ends, each of its waves -- of the
// encode + encrypt kernel works on, and which (tile, row, group) a workgroup of the decode + sum
// kernels. Shared by the kernels, the launcher and the host-side check (host_emul.cpp) that
// every piece of work is taken exactly once.
#pragma once

#include <hip/hip_runtime.h>

#include "block_utils.hpp"
#include "kernels.hpp"

namespace sdagpu {

struct EncodeUnit {
  int tile;   // tile index within the message (kEncodeValues values a tile)
  int msg;    // message index (clamped to a valid one for an idle wave)
  bool ends;  // the workgroup holds the short ends of kWaves messages, a wave each
  bool idle;  // this wave has no message (the last workgroup of the ends)
};

// Whether the messages' ends (the values behind their last whole tile) go kWaves to a
// workgroup: when an end has no more than a wave's share of a tile. (Not in the kernel
// variant that also computes the MAC: its tables are laid out per workgroup.)
__host__ __device__ inline bool encode_short_ends(bool mac, int L) {
  const int r = L % kEncodeValues;
  return !mac && r > 0 && r <= kEncodeValues / kWaves;
}

// Workgroups of a launch: the whole tiles of all messages first, then the ends.
__host__ __device__ inline unsigned encode_grid(bool mac, int M, int L) {
  const unsigned whole = (unsigned)(L / kEncodeValues) * (unsigned)M;
  if (L % kEncodeValues == 0) return whole;
  return whole + (encode_short_ends(mac, L) ? (unsigned)(M + kWaves - 1) / kWaves : (unsigned)M);
}

// Workgroups are handed to the 8 XCDs round-robin in grid order. Messages of fewer than 8 whole
// tiles take the message index fastest (with the tile index fastest, messages of a whole tile
// and a short end sent all whole tiles to the even XCDs and all ends to the odd ones), long
// messages the tile index (neighbours in time are then neighbours in memory: 4 % faster).
__host__ __device__ inline EncodeUnit encode_unit(bool mac, int M, int L, int b, int wave) {
  const int whole = L / kEncodeValues;
  EncodeUnit u;
  u.ends = b >= whole * M && encode_short_ends(mac, L);
  int j;
  if (b < whole * M) {
    if (whole < 8) {
      u.tile = b / M;
      j = b - u.tile * M;
    } else {
      j = b / whole;
      u.tile = b - j * whole;
    }
  } else {
    u.tile = whole;
    j = u.ends ? kWaves * (b - whole * M) + wave : b - whole * M;
  }
  u.idle = j >= M;
  u.msg = u.idle ? M - 1 : j;
  return u;
}

// The decode + sum kernels' grid is (element tiles, rows, participant groups). With fewer
// than 8 tiles a row the tile index runs slowest instead of fastest (the same XCD round-robin:
// rows of a long tile and a short one would park the short ones on half the chip).
struct SumTileId {
  int t, r, g;
};
__host__ __device__ inline SumTileId sum_tile_of(unsigned T, unsigned R, unsigned G, unsigned x, unsigned y,
                                                 unsigned z) {
  if (T >= 8u || (uint64_t)T * R * G >= (1ull << 31)) return {(int)x, (int)y, (int)z};
  const unsigned n = x + T * (y + R * z), RG = R * G;
  const unsigned t = n / RG, rest = n - t * RG, g = rest / R;
  return {(int)t, (int)(rest - g * R), (int)g};
}

}  // namespace sdagpu
