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

// Wave-uniform buffer descriptor over one sequence's rows of a column block:
// element (r, c) of the block sits at byte ((r * ld) + c) * 4 from `base + s0*ld + c0`.
// The record count ends exactly after column ncols-1 of row L-1, so every load of a row
// >= L (and of the padding columns of the last row) returns 0 in hardware — no clamping.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seq_rsrc(const float* base, int64_t ld,
                                                          int64_t s0, int c0, int L, int ncols) {
  const float* p = base + s0 * ld + c0;
  const int64_t bytes = L > 0 ? ((int64_t)(L - 1) * ld + ncols) * 4 : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff),
                                           0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ uint32_t buf_ld_u32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}

// Register-staged ROWS x CP tile of a jagged column block, loaded through a seq_rsrc
// descriptor; rows past the sequence come back as 0 from the range check.
//   dword path: thread t owns column t % CPR (CPR = CP rounded up to a power of two) of
//               rows t / CPR + RPP i;
//   pair path (vec2: 8-byte aligned rows, even ncols): thread t owns columns 2(t % CPH),
//               +1 (CPH = CPR / 2) of rows t / CPH + RPP2 i — half the load / LDS-store
//               instructions (vector-memory issue is the limiter when a CU's waves
//               stage tiles together).
// One voffset VGPR per thread, the row step is an SGPR soffset.
template <int CP, int ROWS>
struct BufTile {
  static constexpr int CPR = CP <= 16 ? 16 : CP <= 32 ? 32 : CP <= 64 ? 64 : CP <= 128 ? 128 : 256;
  static constexpr int RPP = 256 / CPR;  // rows per pass (dwords)
  static constexpr int PER = (ROWS + RPP - 1) / RPP;
  static constexpr int CPH = CPR / 2;
  static constexpr int RPP2 = 256 / CPH;  // rows per pass (pairs)
  static constexpr int PER2 = (ROWS + RPP2 - 1) / RPP2;
  static constexpr int NV = PER > 2 * PER2 ? PER : 2 * PER2;
  float v[NV];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int64_t ld, int r0, int ncols,
                                       bool vec2) {
    const int tid = threadIdx.x;
    if (vec2) {
      const int c = 2 * (tid % CPH), rr = tid / CPH;
      const int voff = c < ncols ? ((r0 + rr) * (int)ld + c) * 4 : OOB_OFF;
      const int step = RPP2 * (int)ld * 4;
#pragma unroll
      for (int i = 0; i < PER2; ++i) {
        typedef unsigned int u2_ __attribute__((ext_vector_type(2)));
        const u2_ x = __builtin_amdgcn_raw_buffer_load_b64(r, voff, i * step, 0);
        v[2 * i] = __uint_as_float(x.x);
        v[2 * i + 1] = __uint_as_float(x.y);
      }
    } else {
      // columns past ncols read out of range (0 from the range check): no select after
      // the load, so all PER loads stay in flight
      const int c = tid % CPR, rr = tid / CPR;
      const int voff = c < ncols ? ((r0 + rr) * (int)ld + c) * 4 : OOB_OFF;
      const int step = RPP * (int)ld * 4;
#pragma unroll
      for (int i = 0; i < PER; ++i) v[i] = buf_ld(r, voff, i * step);
    }
  }
  __device__ __forceinline__ void store(float* lds, int ldl, bool vec2) const {
    const int tid = threadIdx.x;
    if (vec2) {
      const int c = 2 * (tid % CPH), rr = tid / CPH;
      if (c < CP) {
#pragma unroll
        for (int i = 0; i < PER2; ++i)
          if (RPP2 * PER2 == ROWS || rr + RPP2 * i < ROWS)
            *reinterpret_cast<float2*>(lds + (rr + RPP2 * i) * ldl + c) =
                make_float2(v[2 * i], v[2 * i + 1]);
      }
    } else {
      const int c = tid % CPR, rr = tid / CPR;
      if (c < CP) {
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (RPP * PER == ROWS || rr + RPP * i < ROWS) lds[(rr + RPP * i) * ldl + c] = v[i];
      }
    }
  }
};

// Work rank of workgroup `id` (rank 0 = heaviest).  Workgroups id and id + C (C = number
// of CUs) land on the same CU when the grid is resident in a few rounds, so odd rounds
// are reversed ("snake"): each CU pairs a heavy tile with a light one instead of two
// heavy or two light ones (C2: 6 vs 4 tile-units per CU becomes 5 and 5).
__device__ __forceinline__ int snake_rank(int id, int C) {
  const int r = id / C, p = id - r * C;
  return r * C + ((r & 1) ? C - 1 - p : p);
}

// Host: true when every pointer is 8-byte aligned and every stride / width is even.
inline int pair_aligned(std::initializer_list<const void*> ptrs, std::initializer_list<int64_t> vals) {
  for (const void* p : ptrs)
    if ((uintptr_t)p % 8 != 0) return 0;
  for (int64_t v : vals)
    if (v % 2 != 0) return 0;
  return 1;
}

// Bucket-map descriptor for sequence b (tiles of 4096 bytes; records = 0 when there is
// no map, so every map load returns bucket 0).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t map_rsrc(const uint8_t* map, int b, int tpb) {
  const uint8_t* p = map ? map + (int64_t)b * tpb * 4096 : nullptr;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, map ? tpb * 4096 : 0, 0x00020000);
}
// soffset (bytes) of the map word for the 16 x 16 block (q, k) (multiples of 16) in the
// query-major (or key-major) orientation; the lane part is lane_off * 4.
__device__ __forceinline__ int map_soff(int q, int k, bool query_major) {
  const int t = attn_tile_id(q >> 6, k >> 6);
  const int sub = query_major ? ((k & 63) >> 4) : ((q & 63) >> 4);
  return (t * 1024 + sub * 4) * 4;
}

// Epilogue store of NR x NT accumulator values (row i, column tile t) as
// out[row][c] = v * silu'(hp[row][c]) (plain v when hp is null), rows past L and columns
// >= width skipped.  The silu'(h) loads are issued branch-free (clamped addresses) for all
// NR x NT values before any is used: with a per-element `if (valid) load; use; store` the
// compiler waited for each load in turn (vmcnt(0) per element: ~50 us of serial latency
// per workgroup at d = 256).
//   row_of(i): the element row (sequence-relative), col_of(t): the column
//   OutT / HT: float, or __bf16 for the bf16-activation layout (hstu_attn_bwd_a16)
template <int NR, int NT, typename V, typename RowF, typename ColF, typename OutT, typename HT>
__device__ __forceinline__ void store_scaled(const V& val, int L, int width, int64_t s0,
                                             OutT* out, int64_t ld_out, const HT* hp,
                                             int64_t ld_h, int c0, RowF row_of, ColF col_of) {
  float hv[NR][NT];
  if (hp) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = row_of(i);
      const int64_t row = s0 + (r < L ? r : 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = col_of(t);
        hv[i][t] = (float)as_global(hp)[row * ld_h + c0 + (c < width ? c : 0)];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = row_of(i);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = col_of(t);
      float g = val(i, t);
      if (hp) g *= silu_grad_(hv[i][t]);
      if (r < L && c < width) out[(s0 + r) * ld_out + c0 + c] = (OutT)g;
    }
  }
}

}  // namespace gr
