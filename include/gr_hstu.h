/*
 * gr_hstu.h — C-ABI of the MI355X (gfx950) HSTU-encoder + MIPS-retrieval hot path.
 *
 * One shared library, libgr_hstu.so, built by hipcc for gfx950.  Every entry point:
 *   - takes plain device pointers, sizes and strides (no framework types);
 *   - is stream-ordered on the caller's `stream` (a hipStream_t passed as void*);
 *     no host synchronisation, no allocation: the caller owns every buffer,
 *     including workspaces (size queries below);
 *   - returns 0 on success, non-zero on error, with a thread-local message in
 *     gr_last_error().
 * Pointers to jagged tensors index rows by `offsets` (int64, B + 1 entries, device),
 * the exclusive prefix sum of the per-sequence lengths (reference
 * src/generative_recommenders_pl/models/utils/ops.py:18-38).  `max_rows` is a host
 * upper bound on offsets[B] (e.g. B*N) used only to size grids; kernels read the
 * true total from offsets[B] on the device, so no host sync is needed.
 *
 * All reference citations are relative to src/generative_recommenders_pl/models/.
 */
#ifndef GR_HSTU_H_
#define GR_HSTU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_HSTU_ABI_VERSION 1

#ifndef GR_API
#define GR_API __attribute__((visibility("default")))
#endif

/* Thread-local message describing the last non-zero status. */
GR_API const char* gr_last_error(void);
/* Returns GR_HSTU_ABI_VERSION. */
GR_API int gr_version(void);

/* ---------------------------------------------------------------- jagged layout
 * Replaces utils/ops.py:18-38 asynchronous_complete_cumsum:
 *   offsets[0] = 0, offsets[b+1] = offsets[b] + lengths[b].
 */
GR_API int gr_complete_cumsum(const int64_t* lengths, int B, int64_t* offsets, void* stream);

/* Replaces utils/ops.py:41-64 dense_to_jagged: dense (B, N, D) row-major f32 ->
 * jagged (offsets[B], D). */
GR_API int gr_dense_to_jagged(const float* dense, const int64_t* offsets, int B, int N, int D,
                       int64_t max_rows, float* jagged, void* stream);

/* Replaces utils/ops.py:67-114 jagged_to_padded_dense (padding_value 0):
 * jagged (offsets[B], D) -> dense (B, N, D); rows >= length are zero. */
GR_API int gr_jagged_to_padded(const float* jagged, const int64_t* offsets, int B, int N, int D,
                        float* dense, void* stream);

/* ---------------------------------------------------------------- HSTU attention
 * Replaces sequential_encoders/hstu.py:134-205 (_hstu_attention_maybe_from_cache,
 * non-cache branch) fused with the relative bias of hstu.py:96-128
 * (RelativeBucketedTimeAndPositionBasedBias.forward):
 *   out[i, h, :] = sum_{j <= i < L_b} silu(q_i,h . k_j,h + pos_w[N-1+j-i]
 *                                          + ts_w[bucket(ts_next(i) - ts(j))]) / N * v_j,h
 * q/k rows: (total, H*dqk) with row stride ld_qk; v rows: (total, H*dv), stride ld_v;
 * out: (total, H*dv), stride ld_out.  ts: (B, N) int64 timestamps or NULL (then NO
 * bias at all, hstu.py:191).  bucket_thr: (num_buckets + 1) int64 thresholds,
 * bucket(dt) = max{b : bucket_thr[b] <= |dt|}.  max_len: host upper bound on the
 * sequence lengths (<= N), sizes the grid.  fp32 in / fp32 out, f32 MFMA.
 * Supports dqk, dv <= 128.
 */
GR_API int hstu_attn_fwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                  int64_t ld_v, const int64_t* offsets, int B, int N, int max_len, int H,
                  int dqk, int dv, const int64_t* ts, const float* pos_w,
                  const float* ts_w, const int64_t* bucket_thr, int num_buckets,
                  float* out, int64_t ld_out, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* GR_HSTU_H_ */
