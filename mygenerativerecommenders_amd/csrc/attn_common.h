// Shared pieces of the jagged HSTU attention kernels (forward and backward).
#pragma once

#include "common.h"

namespace gr {

__host__ __device__ inline int attn_tiles_per_seq(int N) {
  const int T = (N + 63) / 64;
  return T * (T + 1) / 2;
}
__host__ __device__ inline int attn_tile_id(int qt, int kt) { return qt * (qt + 1) / 2 + kt; }

// Index (in dwords) of the bucket-map word a lane reads for the 16 x 16 block
// whose first query is q and first key is k (both multiples of 16, k <= q + 15):
// map tiles are 64 x 64, row-major in the first index of the orientation; `lane_off`
// is (row-in-tile) * 16 + lg for the lane's row.
__device__ __forceinline__ int64_t map_block_word(int64_t map_seq, int q, int k, int lane_off,
                                                  bool query_major) {
  const int t = attn_tile_id(q >> 6, k >> 6);
  const int sub = query_major ? ((k & 63) >> 4) : ((q & 63) >> 4);
  return map_seq + (int64_t)t * 1024 + lane_off + sub * 4;
}

// Register-staged ROWS-row tile of a jagged column block: rows [r0, r0 + ROWS) of a
// (rows, ld) matrix, columns [c0, c0 + ncols) zero-padded to CP, rows >= L zero.
// Loads are unconditional (clamped) and issued together; store() writes LDS.
template <int CP, int ROWS = 64>
struct TileStage {
  static constexpr int PER = (ROWS * CP + 255) / 256;
  float v[PER];
  __device__ __forceinline__ void load(const float* base, int64_t ld, int64_t s0, int r0, int L,
                                       int c0, int ncols) {
    gptr<float> g = as_global(base);
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + 256 * i;
      const int r = e / CP, c = e - (e / CP) * CP;
      const int row = r0 + r;
      const bool ok = e < ROWS * CP && row < L && c < ncols;
      const int rc = row < L ? row : L - 1;
      const int cc = c < ncols ? c : ncols - 1;
      const float x = g[(s0 + rc) * ld + c0 + cc];
      v[i] = ok ? x : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* lds, int ldl) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = tid + 256 * i;
      if (e < ROWS * CP) {
        const int r = e / CP, c = e - (e / CP) * CP;
        lds[r * ldl + c] = v[i];
      }
    }
  }
};

}  // namespace gr
