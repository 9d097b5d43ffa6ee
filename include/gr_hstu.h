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

#define GR_HSTU_ABI_VERSION 18

#ifndef GR_API
#define GR_API __attribute__((visibility("default")))
#endif

/* Thread-local message describing the last non-zero status. */
GR_API const char* gr_last_error(void);
/* Returns GR_HSTU_ABI_VERSION. */
GR_API int gr_version(void);

/* Live per-kernel timing (measurement only; off by default).  When enabled, every
 * launch records a HIP event pair on its stream; gr_timing_query(kernel, ...) waits
 * for and drains that kernel's pairs, returning the summed device time and launch
 * count.  Kernel names: bucket_map, attn_fwd, attn_bwd_dkv, attn_bwd_dq, attn_fwd_bnd
 * (attention + layer boundary), attn_fwd_bnd1 (+ gate_o of the last layer), attn_bwd_dq_bnd
 * (dQ + layer boundary), attn_bwd_dq_bnd1 (+ ln_uvqk_bwd of the first layer),
 * attn_bias_reduce, ln_uvqk_fwd, gate_o_fwd, gate_o_bwd, ln_uvqk_bwd, wgrad_partial,
 * wgrad_reduce, mips_pack, mips_select, mips_merge, cumsum, dense_to_jagged, encoder_prologue, bf16_scale_add, adamw,
 * jagged_to_padded, l2_normalize, current_embeddings, sampled_softmax_fwd,
 * sampled_softmax_bwd, sampled_softmax_csr, sampled_softmax_table_grad, preproc, rows_copy,
 * decode_scatter, decode_attn, softmax_attn_fwd, softmax_attn_bwd, rel_bias_fwd, rel_bias_bwd.  Not for use inside a captured graph.
 */
GR_API int gr_timing_enable(int on);
GR_API int gr_timing_query(const char* kernel, double* total_ms, int* launches);
GR_API int gr_timing_reset(void);

/* Launch options (the library reads no environment variables).  gr_set_option sets the
 * process-wide value; gr_set_thread_option overrides it for the calling thread only
 * (gr_clear_thread_option(opt) drops one override, opt = 0 all of them), so threads or
 * streams driven from different threads can use different options without racing
 * (ABI 15; tests/test_capi.py::test_thread_options_are_per_thread).  Every launch and
 * workspace query reads the calling thread's value.  Set options before the launches they
 * should affect; not while a graph that used them is being captured.  gr_get_option
 * returns the calling thread's current value (or -1 for an unknown option).
 * Workspace sizes: a *_workspace_size query answers for the options in force when it
 * is called, and every launch re-derives its need under the options in force at launch.
 * A workspace sized under other options is therefore never overrun: the launch returns
 * non-zero with "workspace N B < M B" (gr_wgrad*, mips_topk, sampled softmax, rel bias),
 * or, for hstu_attn_bwd's optional dS tiles, runs the recomputing form that needs only
 * the bias slabs (tests/test_capi.py::test_option_changed_between_sizing_and_launch...).
 *   GR_OPT_MIPS_FILTER_FP32  0|1  bf16 items table off: the filter pass scores on the
 *                                  f32 table (slower, exact scores; results identical)
 *   GR_OPT_MIPS_FILTER_WGS    >=0  filter workgroups per CU per round (0 = default: 3 at
 *                                  D <= 64, whose kernels fit 3 per CU: 10M x 50 filter
 *                                  221 -> 202 us; 2 above)
 *   GR_OPT_MIPS_FILTER_ROUNDS >=0  filter rounds (0 = chosen from the catalog size)
 *   GR_OPT_MIPS_FORCE_FALLBACK 0|1 thresholds forced to +inf: every query takes the
 *                                  exact fallback scan (tests / profiling)
 *   GR_OPT_ATTN_BWD_SPLIT     0|1  f32 attention backward as separate dK/dV and dQ
 *                                  launches instead of the fused launch
 *   GR_OPT_ROWWAVE            0|1  row-wave GEMM kernels (default 1) or the row-panel ones
 *   GR_OPT_ATTN_BWD_PAIRS   0|1|2  f32 attention backward: workgroups take causal tile pairs
 *                                  (p, T-1-p): 1 = when that grid fits one round (default),
 *                                  2 = always (64-row tiles), 0 = never
 *   GR_OPT_ATTN_BWD_DS      0|1|2  f32 attention backward at N <= 512: the dK/dV pass stores dS
 *                                  tiles and dQ = dS K runs without recompute, 1 = in a second
 *                                  launch, 2 = in the same launch (the dQ workgroups take each
 *                                  key tile's dS once its producer publishes it), 0 = the
 *                                  recomputing one-launch form.  Default 1 (C2: 37.8 + 13.0 us
 *                                  against 57.1 us for the recomputing launch).  The workspace
 *                                  size (hstu_attn_bwd_workspace_size) depends on this option.
 *   GR_OPT_DETERMINISTIC      0|1  reductions that default to fp32 atomics run in a fixed
 *                                  order instead (gr_item_embedding_bwd: owner-computes)
 *   GR_OPT_WGRAD_ROWS         >=0  f32 / bf16 weight gradients (64-wide panels): rows per
 *                                  split (0 = chosen from the row count; rounded up to 64).
 *                                  The workspace size (gr_wgrad*_workspace_size) depends on it.
 *   GR_OPT_PANEL_VEC        0|1|2  bf16 backward projection GEMMs at K % 32 == 0 with
 *                                  16-byte aligned rows and 256-column panels: float4
 *                                  operand staging (default 1) or the scalar-staged row panel;
 *                                  2 also routes hstu_ln_uvqk_fwd_a16 to the float4-staged
 *                                  panel (A/B only: C3 1.090 vs 1.093 ms per step)
 *   GR_OPT_ATTN_BWD_WIDE_DS   0|1  f32 attention backward at wide heads (dqk or dv > 128): the
 *                                  dK/dV pass stores dS tiles and dQ = dS K runs in a second
 *                                  launch without recomputing S / dP (default 1), or 0 = the
 *                                  recomputing dQ pass.  Needs the workspace of
 *                                  hstu_attn_bwd_workspace_size_d (which depends on it).
 *   GR_OPT_ATTN_BWD_WIDE_SPLIT 0|1|2 f32 attention backward at wide heads with stored dS:
 *                                  dV and dK in one workgroup (0, default: C3 dK/dV 1.88 ms
 *                                  per layer), as separate workgroups of one launch (1:
 *                                  2.62 ms), or as two launches (2: 2 x 1.08 ms)
 *   GR_OPT_MIPS_FILTER_PAIRED 0|1  filter pass with several 128-query chunks (B > 128; a
 *                                  workgroup holds 128 queries at every D <= 256):
 *                                  the chunks of one item range run on one XCD back to back
 *                                  (default 1: the range streams from HBM once) or as the
 *                                  2-D grid (0: every chunk streams the table)
 *   GR_OPT_MIPS_SAMPLE_STRIDE >=0  filter path: item blocks between the blocks the sample
 *                                  pass scores (0 = 32); the threshold is the (1024 /
 *                                  stride)-th largest group maximum (~1024 candidates)
 *   GR_OPT_WGRAD_STREAM       0|1  f32 weight gradients at Ka <= 64, Nb <= 256: the streaming
 *                                  form (default 1: operands loaded straight into MFMA
 *                                  fragments, one workgroup per (problem, row split), splits
 *                                  per problem by MFMA work) or the LDS-staged panels (0).
 *                                  Workspace queries cover both forms.
 *   GR_OPT_BOUNDARY_FUSE      0|1  hstu_attn_bwd_bnd: the layer boundary as the epilogue of
 *                                  the dQ launch where the shapes allow (default 1), or the
 *                                  attention backward and the boundary as separate calls (0).
 *                                  The epilogue exists on the two-pass dS path only
 *                                  (GR_OPT_ATTN_BWD_DS = 1 with a bucket map); other forms
 *                                  run the separate calls whatever this option says
 */
enum {
  GR_OPT_MIPS_FILTER_FP32 = 1,
  GR_OPT_MIPS_FILTER_WGS = 2,
  GR_OPT_MIPS_FILTER_ROUNDS = 3,
  GR_OPT_MIPS_FORCE_FALLBACK = 4,
  GR_OPT_ATTN_BWD_SPLIT = 5,
  GR_OPT_ROWWAVE = 6,
  GR_OPT_ATTN_BWD_PAIRS = 7,
  GR_OPT_ATTN_BWD_DS = 8,
  GR_OPT_DETERMINISTIC = 9,
  GR_OPT_WGRAD_ROWS = 10,
  GR_OPT_PANEL_VEC = 11,
  GR_OPT_ATTN_BWD_WIDE_DS = 12,
  GR_OPT_ATTN_BWD_WIDE_SPLIT = 13,
  GR_OPT_MIPS_FILTER_PAIRED = 14,
  GR_OPT_MIPS_SAMPLE_STRIDE = 15,
  GR_OPT_WGRAD_STREAM = 16,
  GR_OPT_BOUNDARY_FUSE = 17,
  GR_OPT_COUNT_ = 18
};
GR_API int gr_set_option(int option, int64_t value);
GR_API int gr_set_thread_option(int option, int64_t value);
GR_API int gr_clear_thread_option(int option);
GR_API int64_t gr_get_option(int option);

/* ---------------------------------------------------------------- jagged layout
 * Replaces utils/ops.py:18-38 asynchronous_complete_cumsum:
 *   offsets[0] = 0, offsets[b+1] = offsets[b] + lengths[b].
 */
GR_API int gr_complete_cumsum(const int64_t* lengths, int B, int64_t* offsets, void* stream);

/* Replaces utils/ops.py:41-64 dense_to_jagged: dense (B, N, D) row-major f32 ->
 * jagged rows, sequence b at rows offsets[b] .. offsets[b] + min(len_b, N).  Nothing is
 * written at or past row max_rows (the jagged buffer's size).  zero_fill != 0 also
 * zeroes the rows a sequence owns past N (lengths above N are truncated, as fbgemm's
 * gradient of jagged_to_padded_dense) and the rows [offsets[B], max_rows). */
GR_API int gr_dense_to_jagged(const float* dense, const int64_t* offsets, int B, int N, int D,
                              int64_t max_rows, int zero_fill, float* jagged, void* stream);

/* Replaces utils/ops.py:67-114 jagged_to_padded_dense (padding_value 0):
 * jagged (offsets[B], D) -> dense (B, N, D); rows >= length are zero. */
GR_API int gr_jagged_to_padded(const float* jagged, const int64_t* offsets, int B, int N, int D,
                        float* dense, void* stream);

/* Replaces postprocessors.py:47-56 (L2NormEmbeddingPostprocessor.forward) and
 * negative_sampler.py:31-37: out[r] = x[r] / max(||x[r]||_2, eps), rows of width D. */
GR_API int gr_l2_normalize(const float* x, int64_t ld_x, int64_t rows, int D, float eps, float* out,
                           int64_t ld_out, void* stream);
/* Autograd backward of gr_l2_normalize (recomputes ||x||). */
GR_API int gr_l2_normalize_bwd(const float* x, int64_t ld_x, const float* dy, int64_t ld_dy,
                               int64_t rows, int D, float eps, float* dx, int64_t ld_dx,
                               void* stream);
/* Replaces utils/ops.py:171-187 get_current_embeddings: out[b] = encoded[b, lengths[b]-1]
 * of a (B, N, D) tensor, optionally L2-normalised (the retrieval query path). */
GR_API int gr_current_embeddings(const float* encoded, const int64_t* lengths, int B, int N, int D,
                                 int normalize, float eps, float* out, void* stream);

/* ---------------------------------------------------------------- input preprocessor
 * Replaces LearnablePositionalEmbeddingInputFeaturesPreprocessor.forward
 * (preprocessors/learnable_positional_embedding.py:42-58) on (B, N, D) contiguous rows:
 *   y = dropout(x * scale + pos_w[n]) * (past_ids != 0),   scale = sqrt(D) in the reference
 * dropout keeps an element iff hash(seed + *seed_offset, element index) >= p * 2^32 (kept
 * values scaled by 1/(1-p)); seed_offset is a device counter (NULL = 0) so a captured graph
 * draws a new mask per replay.  The backward regenerates the mask:
 *   dx = dy * mask * scale,  dpos_w[n] = sum_b dy[b, n] * mask (fixed order over b);
 * either output may be NULL. */
GR_API int gr_preproc_fwd(const float* x, const int64_t* past_ids, const float* pos_w, int B, int N,
                          int D, float scale, float dropout_p, uint64_t seed,
                          const int64_t* seed_offset, float* y, void* stream);
GR_API int gr_preproc_bwd(const float* dy, const int64_t* past_ids, int B, int N, int D, float scale,
                          float dropout_p, uint64_t seed, const int64_t* seed_offset, float* dx,
                          float* dpos_w, void* stream);

/* ---------------------------------------------------------------- item embeddings
 * Replaces LocalEmbeddingModule.get_item_embeddings (embeddings/embeddings.py:94-97):
 *   out[i] = cat(w0[ids[i]], w1[map1[clamp(ids[i], 0, map_len - 1)]])     (n, d0 + d1)
 * w0 (rows0, d0) is the item table, w1 (rows1, d1) the year table and map1 the item ->
 * year lookup (map1 NULL: w1 is indexed by the id itself; w1 NULL: a plain gather, as
 * CategoricalEmbeddingModule uses with its mapped ids).  Ids outside a table read 0.
 * Backward: dw0 / dw1 (either may be NULL) are zeroed, then dW[row] += dout[i] for every
 * gathering i, except row padding_idx (nn.Embedding padding_idx; < 0 = none); fp32
 * atomics, unordered like index_add_.  GR_OPT_DETERMINISTIC: owner-computes in id order,
 * limited to ceil(max(rows0, rows1) / 8) * n <= 2^33. */
GR_API int gr_item_embedding_fwd(const int64_t* ids, int64_t n, const float* w0, int64_t rows0,
                                 int d0, const float* w1, int64_t rows1, int d1,
                                 const int64_t* map1, int64_t map_len, float* out, void* stream);
GR_API int gr_item_embedding_bwd(const int64_t* ids, int64_t n, const float* dout, int64_t rows0,
                                 int d0, int64_t rows1, int d1, const int64_t* map1,
                                 int64_t map_len, int64_t padding_idx, float* dw0, float* dw1,
                                 void* stream);

/* ---------------------------------------------------------------- sampled-softmax loss
 * Fused LocalNegativesSampler.forward (negative_sampler.py:105-131, after its randint) +
 * DotProductSimilarity.forward (dot_product.py:31-64) + SampledSoftmaxLoss.jagged_forward
 * (autoregressive_losses.py:259-306), per jagged token t of M, R sampled negatives:
 *   pos_logit = <out[t], pos[t]> / T
 *   neg_r     = id(off[t,r]) == sup_ids[t] ? -5e4 : <out[t], table[off[t,r]]> / T
 *   loss[t]   = logsumexp(pos_logit, neg_0..neg_{R-1}) - pos_logit,  lse[t] saved.
 * `pos` is the (normalised) positive embedding, `table` the (normalised) embedding of
 * every catalog row, indexed by the sampled offset (0 <= off < V; clamped);
 * id(off) = all_ids[off], or off when all_ids is NULL.  D <= 256.  The weighted mean
 * (autoregressive_losses.py:306) is left to the caller. */
GR_API int gr_sampled_softmax_fwd(const float* out, int64_t ld_out, const float* pos, int64_t ld_pos,
                                  const int64_t* sup_ids, const float* table, int64_t ld_table,
                                  int64_t V, const int64_t* all_ids, const int64_t* offsets,
                                  int64_t M, int R, int D, float temperature, float* loss,
                                  float* lse, void* stream);
/* Backward of gr_sampled_softmax_fwd given dloss[t] (the per-token upstream gradient):
 * writes d_out and d_pos (M x D) and d_table (V x D, every row; rows never sampled get 0).
 * The table gradient is accumulated per catalog row after a counting sort of the
 * offsets; its summation order within a row is not fixed (integer atomics).  M*R and V must fit int32; tables
 * and row arrays must be < 2 GiB.  workspace: gr_sampled_softmax_workspace_size bytes. */
GR_API size_t gr_sampled_softmax_workspace_size(int64_t M, int R, int64_t V, int D);
/* Byte offset of the backward's status word inside its workspace (valid after a backward
 * with M * R > 0): 0 = clean; bit 0 = a sample row outside [0, V); bit 1 = a counting-sort
 * slot outside its row's range.  Flagged samples are dropped, never written out of bounds. */
GR_API size_t gr_sampled_softmax_status_offset(int64_t M, int R, int64_t V, int D);
GR_API int gr_sampled_softmax_bwd(const float* out, int64_t ld_out, const float* pos, int64_t ld_pos,
                                  const int64_t* sup_ids, const float* table, int64_t ld_table,
                                  int64_t V, const int64_t* all_ids, const int64_t* offsets,
                                  int64_t M, int R, int D, float temperature, const float* lse,
                                  const float* dloss, float* d_out, int64_t ld_dout, float* d_pos,
                                  int64_t ld_dpos, float* d_table, int64_t ld_dtable,
                                  void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- Muon step (ABI 17)
 * out[i] = bf16(bf16(s * x[i]) + y[i]) over n bf16 values (bit patterns): the two
 * combines of the Newton-Schulz chain of optimizers/muon.py:3-29 (B = b*A + (c*A)@A,
 * X = a*X + B@X) with the reference's two roundings, in one launch.  out may alias x or y. */
GR_API int gr_bf16_scale_add(const uint16_t* x, float s, const uint16_t* y, uint16_t* out,
                             int64_t n, void* stream);

/* gr_adamw_step (ABI 17): torch.optim.AdamW's update (fused=True, capturable=True: the
 * reference's optimizer) over n_tensors fp32 tensors in ONE launch per 48 tensors, the
 * step counter advanced inside the last one (torch: the step-count _foreach_add_ launch +
 * the fused kernel).  params / grads / offs / numel: host arrays; tensor i is
 * params[i][0 .. numel[i]) with its gradient grads[i] and its moments at exp_avg /
 * exp_avg_sq + offs[i] (flat fp32 buffers); numel[i] == 0 skips it.  The pointers go into
 * the kernel arguments, so a captured graph replays the ones it was captured with.  step:
 * one fp32 counter (read as t - 1, written t); done: one uint32 completion counter, zero
 * before the first call (the kernel re-arms it).
 *   p -= lr wd p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;
 *   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 * with ATen's promotion of the double hyper-parameters against the fp32 tensors. */
GR_API int gr_adamw_step(float* const* params, const float* const* grads, const int64_t* offs,
                         const int64_t* numel, int n_tensors, float* exp_avg, float* exp_avg_sq,
                         float* step, uint32_t* done, double lr, double beta1, double beta2,
                         double eps, double weight_decay, void* stream);

/* ---------------------------------------------------------------- HSTU attention
 * hstu_bucket_map: the relative-time bucket of every causal (query i, key j) pair of
 * every sequence, computed ONCE per batch and shared by all layers' attention forward
 * and backward (reference hstu.py:111-123 rebuilds an int64 (B, N, N) tensor per
 * layer).  bucket(i, j) = max{b : bucket_thr[b] <= |ts_next(i) - ts(j)|},
 * ts_next(i) = ts[b, i + 1] (ts[b, N - 1] for i = N - 1), hstu.py:113-119;
 * bucket_thr: (num_buckets + 1) int64 thresholds of the reference bucket function
 * (hstu.py:579-581), num_buckets < 256.  ts: (B, N) int64.  `map` needs
 * hstu_bucket_map_bytes(B, N) bytes (uint8, two tile orientations).
 */
GR_API size_t hstu_bucket_map_bytes(int B, int N);
GR_API int hstu_bucket_map(const int64_t* ts, const int64_t* offsets, int B, int N,
                    const int64_t* bucket_thr, int num_buckets, uint8_t* map, void* stream);

/* hstu_encoder_prologue (ABI 17): the batch setup of an encoder forward in one launch
 * (HSTU.forward, hstu.py:502 + utils/ops.py:18-64, and the bucket map above):
 *   offsets = gr_complete_cumsum(lengths)                       (B + 1 entries)
 *   x_jagged = gr_dense_to_jagged(x, offsets, B, N, D, max_rows, zero_fill = 0)
 *   map = hstu_bucket_map(ts, offsets, B, N, ...)               (skipped when map is NULL)
 *   *step += 1                                                  (skipped when step is NULL)
 * with results identical to those calls (tests/test_gpu_jagged.py).  x (B, N, D) f32,
 * ts (B, N) int64; lengths are not bounded by N (rows past N are not copied, as
 * gr_dense_to_jagged).  No workgroup waits on another: each copy workgroup sums the
 * lengths before its sequence itself. */
GR_API int hstu_encoder_prologue(const int64_t* lengths, int B, int N, const float* x, int D,
                                 int64_t max_rows, const int64_t* ts, const int64_t* bucket_thr,
                                 int num_buckets, int64_t* offsets, float* x_jagged,
                                 uint8_t* map, int64_t* step, void* stream);

/* ---------------------------------------------------------------- cached decoding (ABI 18)
 * The delta_x_offsets / cache branch of SequentialTransductionUnitJagged.forward
 * (sequential_encoders/hstu.py:151-177, 293-298, 321-322, 393-423): a step re-encodes one
 * jagged row per sequence against per-layer caches (v jagged, q / k padded (B, n, .),
 * outputs jagged) that a full pass with return_cache_states produced.
 *
 * gr_rows_copy (replaces the index_select / index_copy_ row moves of that branch):
 *   dst[row_d(e)][0:width] = src[row_s(e)][0:width] for e < n,
 *   row_s(e) = src_index ? src_index[e] + e * src_step : e   (row_d likewise),
 * rows outside [0, src_rows) / [0, dst_rows) are skipped.  src_step = n gives the
 * reference's flattened padded index delta[1][e] + e * n (hstu.py:153-159).
 */
GR_API int gr_rows_copy(const float* src, int64_t ld_src, const int64_t* src_index,
                        int64_t src_step, int64_t src_rows, float* dst, int64_t ld_dst,
                        const int64_t* dst_index, int64_t dst_step, int64_t dst_rows, int n,
                        int width, void* stream);
/* hstu_decode_scatter (replaces the cache updates of hstu.py:321-322 and :160-177, three
 * index_copy_ in one launch): for e < n, with v | q | k the columns hv .. of row e of uvqk
 * (u | v | q | k, widths hv, hv, hq, hq):
 *   v_cache[rows[e]] = v_e  (v_cache (v_rows, hv)),
 *   q_cache[pos[e] + e N] = q_e, k_cache[pos[e] + e N] = k_e  (q / k caches (qk_rows, hq)).
 * Out-of-range rows are skipped. */
GR_API int hstu_decode_scatter(const float* uvqk, int64_t ld_u, int hv, int hq,
                               const int64_t* rows, const int64_t* pos, int n, int N,
                               float* v_cache, int64_t v_rows, float* q_cache, float* k_cache,
                               int64_t qk_rows, void* stream);
/* hstu_decode_attn (replaces hstu.py:186-205 + 393-397 of the cached branch: the full
 * (B, h, n, n) attention over the caches of which only the delta rows are kept): for
 * e < n_rows, h < H, with r = rows[e] in sequence b (offsets[b] <= r < offsets[b + 1])
 * at position p = r - offsets[b]:
 *   out[e][h dv + c] = sum_{j <= p} silu(q_cache[b][p] . k_cache[b][j] + bias(b, p, j)) / N
 *                      * v_cache[offsets[b] + j][h dv + c]
 * (head h's columns h dqk .. of q / k; bias as hstu_rel_bias_fwd, none when ts is NULL).
 * q_cache / k_cache (B, N, ld_qk) f32, v_cache (v_rows, ld_v) f32 jagged, out (n_rows,
 * ld_out).  Rows outside [0, offsets[B]) give zeros.  Two launches: 64-key chunks of each
 * row into workspace partials, then their sum in chunk order (deterministic);
 * n_rows <= 65535.
 */
GR_API size_t hstu_decode_attn_workspace_size(int n_rows, int N, int H, int dv);
GR_API int hstu_decode_attn(const float* q_cache, const float* k_cache, int64_t ld_qk,
                            const float* v_cache, int64_t ld_v, int64_t v_rows,
                            const int64_t* offsets, int B, const int64_t* rows, int n_rows,
                            int N, int H, int dqk, int dv, const int64_t* ts,
                            const int64_t* bucket_thr, int num_buckets, const float* pos_w,
                            const float* ts_w, float* out, int64_t ld_out, void* workspace,
                            size_t ws_bytes, void* stream);

/* hstu_decode_ln_uvqk / hstu_decode_gate_o: the cached step's two projections at one row
 * per sequence (n rows, inference: no statistics, pre-activations or dropout), tiled for
 * small n (16 rows x 16 output columns per workgroup):
 *   uvqk[r] = act(LN(x[r]) @ w_uvqk)                       (hstu_ln_uvqk_fwd; D <= 512)
 *   y[r]    = (u[r] * LN(attn[r])) @ w_o^T + b_o + x_res[r]  (hstu_gate_o_fwd at dropout 0;
 *                                                           hdv <= 256; b_o, x_res may be NULL)
 * timed as ln_uvqk_fwd / gate_o_fwd. */
GR_API int hstu_decode_ln_uvqk(const float* x, int64_t ld_x, int n, int D, const float* w_uvqk,
                               int n_out, float eps, int activation, float* uvqk,
                               int64_t ld_out, void* stream);
GR_API int hstu_decode_gate_o(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                              int n, int hdv, int D, const float* w_o, const float* b_o,
                              const float* x_res, int64_t ld_x, float eps, float* y,
                              int64_t ld_y, void* stream);

/* ---------------------------------------------------------------- softmax attention (ABI 18)
 * hstu_softmax_attn_fwd replaces the normalization="softmax_rel_bias" branch of
 * SequentialTransductionUnitJagged.forward (sequential_encoders/hstu.py:341-389, no
 * cache): for every sequence b and query row i < L_b (= offsets[b+1] - offsets[b], at most
 * N), over ALL N keys j (k_j = 0 for j >= L_b, as the padded tensor):
 *   s_j = (q_i . k_j + bias[b][i][j]) / sqrt_d      (q / k: the hdq = h dqk columns at once;
 *                                                   bias (B, N, N) or NULL = no bias)
 *   out_i = sum_{j <= i} softmax(s)_j v_j           (softmax over all N, then the causal mask)
 *   stats[row] = (max_j s_j, sum_j exp(s_j - max))  (row = offsets[b] + i, kept for the bwd)
 * hstu_softmax_attn_bwd: the gradients of q, k, v (times silu'(h) when the pre-activations
 * hq / hk / hv are given, as hstu_attn_bwd) and, when dbias is not NULL, of the bias
 * (B, N, N; rows i >= L_b zero); workspace hstu_softmax_attn_bwd_workspace_size(B, N,
 * dbias != NULL) bytes.  LDS bounds hdq + hdv + N <= 4096.
 */
GR_API size_t hstu_softmax_attn_bwd_workspace_size(int B, int N, int with_dbias);
GR_API int hstu_softmax_attn_fwd(const float* q, const float* k, int64_t ld_qk, const float* v,
                                 int64_t ld_v, const int64_t* offsets, int B, int N, int hdq,
                                 int hdv, float sqrt_d, const float* bias, float* out,
                                 int64_t ld_out, float* stats, void* stream);
GR_API int hstu_softmax_attn_bwd(const float* q, const float* k, int64_t ld_qk, const float* v,
                                 int64_t ld_v, const int64_t* offsets, int B, int N, int hdq,
                                 int hdv, float sqrt_d, const float* bias, const float* out,
                                 int64_t ld_out, const float* stats, const float* dout,
                                 int64_t ld_do, const float* hq, const float* hk,
                                 const float* hv, int64_t ld_h, float* dq, float* dk,
                                 float* dv, int64_t ld_d, float* dbias, void* workspace,
                                 size_t ws_bytes, void* stream);

/* hstu_rel_bias_fwd / _bwd (ABI 13) — replaces RelativeBucketedTimeAndPositionBasedBias
 * .forward (sequential_encoders/hstu.py:96-128) for callers that materialise the bias
 * (the module called on its own); the attention kernels never need it.
 *   out[b, i, j] = pos_w[N - 1 + j - i] + ts_w[bucket(ts_next(b, i) - ts(b, j))]
 * for ALL 0 <= i, j < N (causal or not, as the reference), out (B, N, N) fp32.
 * Backward: d_pos_w (2N - 1), d_ts_w (num_buckets + 1), both overwritten, summed in a
 * fixed order (deterministic); workspace hstu_rel_bias_bwd_workspace_size bytes.
 */
GR_API int hstu_rel_bias_fwd(const int64_t* ts, int B, int N, const int64_t* bucket_thr,
                    int num_buckets, const float* pos_w, const float* ts_w, float* out,
                    void* stream);
GR_API size_t hstu_rel_bias_bwd_workspace_size(int B, int N, int num_buckets);
GR_API int hstu_rel_bias_bwd(const int64_t* ts, int B, int N, const int64_t* bucket_thr,
                    int num_buckets, const float* dout, float* d_pos_w, float* d_ts_w,
                    void* workspace, size_t ws_bytes, void* stream);

/* hstu_attn_fwd — replaces sequential_encoders/hstu.py:134-205
 * (_hstu_attention_maybe_from_cache, non-cache branch) fused with the relative bias of
 * hstu.py:96-128 (RelativeBucketedTimeAndPositionBasedBias.forward):
 *   out[i, h, :] = sum_{j <= i < L_b} silu(q_i,h . k_j,h + pos_w[N-1+j-i]
 *                                          + ts_w[bucket(i, j)]) / N * v_j,h
 * q/k rows: (total, H*dqk) with row stride ld_qk; v rows: (total, H*dv), stride ld_v;
 * out: (total, H*dv), stride ld_out.  bucket_map: from hstu_bucket_map, or NULL for
 * NO bias at all (no timestamps, hstu.py:191).  max_len: host upper bound on the
 * sequence lengths (<= N), sizes the grid.  fp32 in / out, f32 MFMA.  dqk, dv <= 256.
 */
GR_API int hstu_attn_fwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                  int64_t ld_v, const int64_t* offsets, int B, int N, int max_len, int H,
                  int dqk, int dv, const uint8_t* bucket_map, const float* pos_w,
                  const float* ts_w, int num_buckets, float* out, int64_t ld_out,
                  void* stream);

/* hstu_attn_fwd_bf16: hstu_attn_fwd with bf16 MFMA operands and fp32 accumulation (the
 * opt-in bf16 compute mode): Q, K, V are rounded to bf16 as they are staged and
 * P = silu(S + bias) / N is rounded to bf16 before P.V; S, the bias, silu and the
 * output are fp32.  Same arguments and layout as hstu_attn_fwd, plus `copies`:
 * NULL, or (wide heads only: dqk == dv in (128, 256], even strides) the bf16 copies of
 * Q, K, V made by hstu_attn_bf16_copies, which the wide kernels stage into LDS by DMA.
 * The same copies can be passed to hstu_attn_bwd_bf16 (saved with the activations). */
GR_API size_t hstu_attn_bf16_copies_bytes(int B, int N, int H, int dqk, int dv);
GR_API int hstu_attn_bf16_copies(const float* q, const float* k, const float* v, int64_t ld_qk,
                                 int64_t ld_v, const int64_t* offsets, int B, int N, int H,
                                 int dqk, int dv, void* copies, void* stream);
GR_API int hstu_attn_fwd_bf16(const float* q, const float* k, const float* v, int64_t ld_qk,
                              int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                              int H, int dqk, int dv, const uint8_t* bucket_map,
                              const float* pos_w, const float* ts_w, int num_buckets, float* out,
                              int64_t ld_out, const void* copies, void* stream);

/* Backward of hstu_attn_fwd (replaces the autograd backward of hstu.py:134-205 and of
 * the bias module hstu.py:96-128, including the index_add_ into _ts_w and the
 * slice/pad backward into _pos_w).  dout: (total, H*dv), stride ld_dout.
 * Writes dq, dk (total, H*dqk) and dv (total, H*dv), all with row stride ld_d.
 * hq/hk/hv: optional UVQK pre-activation columns (stride ld_h); when given the
 * outputs are multiplied by silu'(h) (hstu.py:303-305), i.e. they are gradients of
 * the pre-activation.  dpos_w (2N-1) and dts_w (num_buckets+1) are OVERWRITTEN
 * with this call's bias gradients (summed over heads) when bucket_map != NULL.
 * Deterministic: no global atomics; the workspace (size below, only needed with a
 * bucket map) holds one partial slab per workgroup, reduced in a fixed order.
 */
GR_API size_t hstu_attn_bwd_workspace_size(int B, int N, int max_len, int H, int num_buckets);
/* ABI 13: the same with the head dims, needed with or without a bucket map: at wide heads
 * (dqk or dv > 128, GR_OPT_ATTN_BWD_WIDE_DS) it also holds the dS tiles of the dQ pass
 * (B H ceil(N/16) (ceil(N/16) + 1) / 2 tiles of 1 KiB: 275 MB at C3).  A smaller
 * workspace (the size above) still works: dQ is then recomputed. */
GR_API size_t hstu_attn_bwd_workspace_size_d(int B, int N, int max_len, int H, int dqk, int dv,
                                             int num_buckets);
GR_API int hstu_attn_bwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                  int64_t ld_v, const float* dout, int64_t ld_dout, const int64_t* offsets,
                  int B, int N, int max_len, int H, int dqk, int dv,
                  const uint8_t* bucket_map, const float* pos_w, const float* ts_w,
                  int num_buckets, const float* hq, const float* hk, const float* hv,
                  int64_t ld_h, float* dq, float* dk, float* dv_out, int64_t ld_d,
                  float* dpos_w, float* dts_w, void* workspace, size_t ws_bytes,
                  void* stream);

/* hstu_attn_bwd_bf16: hstu_attn_bwd with bf16 MFMA operands (Q, K, V, dO, P, dS) and
 * fp32 accumulation / elementwise (the opt-in bf16 compute mode); the bias gradients
 * sum fp32 dS in a fixed order.  Same arguments as hstu_attn_bwd plus `copies` (NULL or
 * the forward's hstu_attn_bf16_copies, wide heads); the workspace size also depends on
 * the head dims and is needed at wide heads with or without a bucket map. */
GR_API size_t hstu_attn_bwd_bf16_workspace_size(int B, int N, int max_len, int H, int dqk,
                                                int dv, int num_buckets);
/* ABI 13: the workspace when `copies` (the forward's hstu_attn_bf16_copies) is passed:
 * the wide form then needs no Q/K/V copies of its own (~100 MB per layer at C3). */
GR_API size_t hstu_attn_bwd_bf16_workspace_size_copies(int B, int N, int max_len, int H, int dqk,
                    int dv, int num_buckets);
GR_API int hstu_attn_bwd_bf16(const float* q, const float* k, const float* v, int64_t ld_qk,
                              int64_t ld_v, const float* dout, int64_t ld_dout,
                              const int64_t* offsets, int B, int N, int max_len, int H, int dqk,
                              int dv, const uint8_t* bucket_map, const float* pos_w,
                              const float* ts_w, int num_buckets, const float* hq,
                              const float* hk, const float* hv, int64_t ld_h, float* dq,
                              float* dk, float* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                              const void* copies, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- STU projections
 * All take jagged rows (total = offsets[B] <= max_rows), fp32, f32 MFMA.
 * Row statistics are stored as float2 (mean, rstd) per row, biased variance, as
 * F.layer_norm without affine (hstu.py:258-264).
 *
 * hstu_ln_uvqk_fwd  (replaces hstu.py:300-305: layer_norm -> mm(_uvqk) -> silu):
 *   x_stats[m] = (mean, rstd) of x[m, :D];  h = LN(x) @ w_uvqk (w: (D, n_out) row-major)
 *   uvqk = activation ? silu(h) : h  (activation 1 = "silu", 0 = "none");
 *   h_pre (optional, same stride ld_out) receives h for the backward.
 */
GR_API int hstu_ln_uvqk_fwd(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                     int64_t max_rows, int D, const float* w_uvqk, int n_out, float eps,
                     int activation, float* x_stats, float* h_pre, float* uvqk,
                     int64_t ld_out, void* stream);
/* hstu_ln_uvqk_fwd with bf16 MFMA operands (autocast_dtype = bfloat16): the transformed A
 * values and the weights rounded to bf16, fp32 accumulation and epilogue; same
 * arguments and outputs. */
GR_API int hstu_ln_uvqk_fwd_bf16(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                          int64_t max_rows, int D, const float* w_uvqk, int n_out, float eps,
                          int activation, float* x_stats, float* h_pre, float* uvqk,
                          int64_t ld_out, void* stream);

/* hstu_gate_o_fwd  (replaces hstu.py:393-413 with concat_ua = False):
 *   attn_stats[m] = (mean, rstd) of attn[m, :hdv]
 *   o_in = dropout_p(u * LN(attn))  (mask = counter hash of (seed', m*hdv + k), with
 *   seed' = seed + *seed_offset when seed_offset (a device int64) is given: a graph
 *   replay then draws a fresh mask by bumping the device counter)
 *   y = o_in @ w_o^T + b_o + x_res   (w_o: (D, hdv) row-major = nn.Linear.weight)
 *   o_in (optional, contiguous (rows, hdv)) is stored for the weight gradient.
 *   b_o and x_res may be NULL.
 */
GR_API int hstu_gate_o_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                    const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                    const float* w_o, const float* b_o, const float* x_res, int64_t ld_x,
                    float eps, float dropout_p, uint64_t seed, const int64_t* seed_offset,
                    float* attn_stats, float* o_in, float* y, int64_t ld_y, void* stream);
/* hstu_gate_o_fwd with bf16 MFMA operands (autocast_dtype = bfloat16): the transformed A
 * values and the weights rounded to bf16, fp32 accumulation and epilogue; same
 * arguments and outputs. */
GR_API int hstu_gate_o_fwd_bf16(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                         const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                         const float* w_o, const float* b_o, const float* x_res, int64_t ld_x,
                         float eps, float dropout_p, uint64_t seed, const int64_t* seed_offset,
                         float* attn_stats, float* o_in, float* y, int64_t ld_y, void* stream);

/* hstu_gate_o_bwd  (backward of hstu_gate_o_fwd w.r.t. u and attn; hdv <= 256):
 *   g = (dy @ w_o) * dropout mask;  du = g * LN(attn) [* silu'(h_u) if h_u];
 *   d_attn = LayerNorm_backward(attn; g * u).
 */
GR_API int hstu_gate_o_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                    int64_t max_rows, int hdv, int D, const float* w_o, const float* u,
                    int64_t ld_u, const float* attn, int64_t ld_attn,
                    const float* attn_stats, const float* h_u, int64_t ld_h,
                    float dropout_p, uint64_t seed, const int64_t* seed_offset, float* du,
                    int64_t ld_du, float* d_attn, int64_t ld_da, void* stream);
/* hstu_gate_o_bwd with bf16 MFMA operands (autocast_dtype = bfloat16): the transformed A
 * values and the weights rounded to bf16, fp32 accumulation and epilogue; same
 * arguments and outputs. */
GR_API int hstu_gate_o_bwd_bf16(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                         int64_t max_rows, int hdv, int D, const float* w_o, const float* u,
                         int64_t ld_u, const float* attn, int64_t ld_attn,
                         const float* attn_stats, const float* h_u, int64_t ld_h,
                         float dropout_p, uint64_t seed, const int64_t* seed_offset, float* du,
                         int64_t ld_du, float* d_attn, int64_t ld_da, void* stream);

/* hstu_gate_o_cat_fwd / _bwd: the concat_ua = True form of hstu_gate_o_fwd / _bwd
 * (hstu.py:398-400): o_in = dropout_p([u, LN(attn), u * LN(attn)]) (rows, 3 hdv; the mask
 * hashes (row, column of o_in)), y = o_in @ w_o^T + b_o + x_res.  w_pad is the (D, 3 hvp)
 * row-major weight with w_o's three hdv-wide column blocks at column offsets 0, hvp,
 * 2 hvp and zeros elsewhere; hvp = 16 ceil(hdv / 16) rounded up to 16, 32 or 64
 * (hdv <= 64, D <= 128, even widths and 8-byte aligned rows).  The backward returns
 * du (* silu'(h_u) when h_u) and d_attn = LayerNorm_backward(attn; g2 + g3 * u). */
GR_API int hstu_gate_o_cat_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const int64_t* offsets, int B, int64_t max_rows, int hdv, int hvp,
                               int D, const float* w_pad, const float* b_o, const float* x_res,
                               int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                               const int64_t* seed_offset, float* attn_stats, float* o_in,
                               float* y, int64_t ld_y, void* stream);
GR_API int hstu_gate_o_cat_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                               int64_t max_rows, int hdv, int hvp, int D, const float* w_pad,
                               const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const float* attn_stats, const float* h_u, int64_t ld_h,
                               float dropout_p, uint64_t seed, const int64_t* seed_offset,
                               float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                               void* stream);

/* hstu_gate_o_cat_wide_fwd / _bwd: concat_ua at any width (the forms above need
 * hdv <= 64, D <= 128): o_in (REQUIRED, (rows, 3 hdv), the GEMM operand) is built by an
 * elementwise pass and y = o_in @ w_o^T + b_o + x_res streams the unpadded w_o (D, 3 hdv)
 * through the row-panel GEMM.  Same dropout mask (hash of the o_in row and column).  The
 * backward takes g: a (max_rows, 3 hdv) fp32 scratch for dy @ w_o. */
GR_API int hstu_gate_o_cat_wide_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                    const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                                    const float* w_o, const float* b_o, const float* x_res,
                                    int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                    const int64_t* seed_offset, float* attn_stats, float* o_in,
                                    float* y, int64_t ld_y, void* stream);
GR_API int hstu_gate_o_cat_wide_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                                    int64_t max_rows, int hdv, int D, const float* w_o,
                                    const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                    const float* attn_stats, const float* h_u, int64_t ld_h,
                                    float dropout_p, uint64_t seed, const int64_t* seed_offset,
                                    float* g, float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                                    void* stream);

/* hstu_ln_uvqk_bwd  (backward of hstu_ln_uvqk_fwd w.r.t. x, plus the residual; D <= 256):
 *   dn = dh @ w_uvqk^T;  dx = dy_res + LayerNorm_backward(x; dn)   (dy_res may be NULL;
 *   dx may alias dy_res).  dh is the gradient of the pre-activation h.
 */
GR_API int hstu_ln_uvqk_bwd(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                     int64_t max_rows, int D, int n_out, const float* w_uvqk,
                     const float* x, int64_t ld_x, const float* x_stats,
                     const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                     void* stream);
/* hstu_ln_uvqk_bwd with bf16 MFMA operands (autocast_dtype = bfloat16): the transformed A
 * values and the weights rounded to bf16, fp32 accumulation and epilogue; same
 * arguments and outputs. */
GR_API int hstu_ln_uvqk_bwd_bf16(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                          int64_t max_rows, int D, int n_out, const float* w_uvqk,
                          const float* x, int64_t ld_x, const float* x_stats,
                          const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                          void* stream);

/* hstu_boundary_fwd / _bwd (ABI 13) — one encoder layer boundary as ONE launch (the
 * encoder's autograd node, ops.STUStackFunction, calls them between layers):
 *   fwd: hstu_gate_o_fwd of layer l (y = x_res + dropout(u * LN(attn)) W_o^T + b_o) then
 *        hstu_ln_uvqk_fwd of layer l + 1 on y (x_stats, h_pre, uvqk of layer l + 1);
 *   bwd: hstu_ln_uvqk_bwd of layer l (dx = dy_res + LN_bwd(dh W_uvqk^T)) then
 *        hstu_gate_o_bwd of layer l - 1 with dy = dx (du, d_attn of layer l - 1).
 * Arguments: those of the two calls it replaces (the second call's row input is the
 * first one's output, y / dx, which is still stored).  Results agree with the two calls to
 * fp32 summation order (the fused UVQK product is a row-wave MFMA chain where the separate
 * launch may take the row panel); shapes the fused form does not cover (D or h dv > 64,
 * n_out > 256, unaligned rows) run exactly those two calls, bit-identical.  fp32 only. */
GR_API int hstu_boundary_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                    const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                    const float* w_o, const float* b_o, const float* x_res, int64_t ld_x,
                    float eps, float dropout_p, uint64_t seed, const int64_t* seed_offset,
                    float* attn_stats, float* o_in, float* y, int64_t ld_y,
                    const float* w_uvqk, int n_out, int activation, float* x_stats,
                    float* h_pre, float* uvqk, int64_t ld_out, void* stream);
GR_API int hstu_boundary_bwd(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                    int64_t max_rows, int D, int n_out, const float* w_uvqk, const float* x,
                    int64_t ld_x, const float* x_stats, const float* dy_res, int64_t ld_dy,
                    float* dx, int64_t ld_dx, int hdv, const float* w_o, const float* u,
                    int64_t ld_u, const float* attn, int64_t ld_attn, const float* attn_stats,
                    const float* h_u, int64_t ld_h, float dropout_p, uint64_t seed,
                    const int64_t* seed_offset, float* du, int64_t ld_du, float* d_attn,
                    int64_t ld_da, void* stream);

/* ABI 14: the attention forward of layer l followed by its layer boundary, i.e.
 * hstu_attn_fwd(... out ...) then hstu_boundary_fwd(bnd..., attn = out) -- or, with
 * bnd->w_uvqk == NULL for the last layer, hstu_gate_o_fwd(bnd...) -- in one call.  At
 * narrow single-head shapes (H == 1, dqk, dv <= 64; D, h dv in (32, 64], n_out <= 256)
 * the boundary runs as the epilogue of the attention launch: a workgroup's 64 query rows
 * are complete once stored, so its waves re-stage the K / V tile area with the weight
 * panels and run the row-wave boundary unit of their 16 rows (one launch and one re-read
 * of u / attn fewer); otherwise the two calls run as they are.  Results agree with the two
 * calls' to fp32 rounding (the epilogue is hstu_boundary_fwd's row-wave unit, the last
 * layer's gate_o alone the row-wave form of hstu_gate_o_fwd; hipcc may contract their
 * multiply-adds differently inside the attention kernel: a few ulp). */
typedef struct GrBoundaryFwd {
  const float* u;
  int64_t ld_u;
  int64_t max_rows;
  int hdv;
  int D;
  const float* w_o;
  const float* b_o;
  const float* x_res;
  int64_t ld_x;
  float eps;
  float dropout_p;
  uint64_t seed;
  const int64_t* seed_offset;
  float* attn_stats;
  float* o_in;
  float* y;
  int64_t ld_y;
  const float* w_uvqk;  /* NULL: no next layer (the last layer: gate_o alone) */
  int n_out;
  int activation;
  float* x_stats;
  float* h_pre;
  float* uvqk;
  int64_t ld_out;
} GrBoundaryFwd;
GR_API int hstu_attn_fwd_bnd(const float* q, const float* k, const float* v, int64_t ld_qk,
                    int64_t ld_v, const int64_t* offsets, int B, int N, int max_len, int H,
                    int dqk, int dv, const uint8_t* bucket_map, const float* pos_w,
                    const float* ts_w, int num_buckets, float* out, int64_t ld_out,
                    const GrBoundaryFwd* bnd, void* stream);

/* ABI 14: the attention backward of layer l followed by its layer boundary, i.e.
 * hstu_attn_bwd(...) then hstu_boundary_bwd(bnd...) (or, with bnd->hdv == 0 for the first
 * layer, hstu_ln_uvqk_bwd(bnd...)) in one call.  At narrow single-head shapes (H == 1,
 * dqk, dv <= 64, N <= 512 with a bucket map and the dS workspace; D, h dv <= 64,
 * n_out <= 256) the boundary runs as the epilogue of the dQ launch: each 16-query block's
 * wave, once its dq rows are stored, runs the row-wave boundary unit of those 16 rows
 * (d_uvqk of the rows is then complete: du from the previous boundary, dk / dv from the
 * dK/dV launch, dq just stored) -- one launch and one re-read of the rows fewer.
 * The epilogue form needs the two-pass stored-dS backward (option GR_OPT_ATTN_BWD_DS at 1,
 * the default; at 0 or 2 the attention runs without it and the boundary is the second call)
 * and dq / dk / dv_out as column slices of bnd->dh (ld_d == ld_dh, each pointer within
 * dh's first row), since the epilogue reads the rows' d_uvqk back from dh.
 * Otherwise the two calls run as they are.  `bnd` holds the boundary call's arguments
 * (dh = the d_uvqk the attention writes into, stride ld_dh = n_out); results agree with
 * the two calls' to fp32 summation order (the fused epilogue is the row-wave unit of
 * hstu_boundary_bwd; the first layer's hstu_ln_uvqk_bwd alone may take the row panel). */
typedef struct GrBoundaryBwd {
  const float* dh;
  int64_t ld_dh;
  int64_t max_rows;
  int D;
  int n_out;
  const float* w_uvqk;
  const float* x;
  int64_t ld_x;
  const float* x_stats;
  const float* dy_res;
  int64_t ld_dy;
  float* dx;
  int64_t ld_dx;
  int hdv;              /* 0: no gate_o backward of a previous layer (the first layer) */
  const float* w_o;
  const float* u;
  int64_t ld_u;
  const float* attn;
  int64_t ld_attn;
  const float* attn_stats;
  const float* h_u;
  int64_t ld_h;
  float dropout_p;
  uint64_t seed;
  const int64_t* seed_offset;
  float* du;
  int64_t ld_du;
  float* d_attn;
  int64_t ld_da;
} GrBoundaryBwd;
GR_API int hstu_attn_bwd_bnd(const float* q, const float* k, const float* v, int64_t ld_qk,
                    int64_t ld_v, const float* dout, int64_t ld_dout, const int64_t* offsets,
                    int B, int N, int max_len, int H, int dqk, int dv,
                    const uint8_t* bucket_map, const float* pos_w, const float* ts_w,
                    int num_buckets, const float* hq, const float* hk, const float* hv,
                    int64_t ld_h, float* dq, float* dk, float* dv_out, int64_t ld_d,
                    float* dpos_w, float* dts_w, void* workspace, size_t ws_bytes,
                    const GrBoundaryBwd* bnd, void* stream);

/* gr_wgrad: weight gradient C = A'^T B over all jagged rows (replaces the mm-backward
 * of hstu.py:303 and of the _o Linear at hstu.py:404-411):
 *   C[ka, nb] = sum_m A'[m, ka] * Bm[m, nb],  A' = A or (A - mean_m) * rstd_m when
 *   a_stats != NULL;  a_colsum (optional) = sum_m A[m, :] (the Linear bias gradient).
 *   C (Ka, Nb) and a_colsum are overwritten.  Deterministic split-M slabs.
 */
GR_API size_t gr_wgrad_workspace_size(int64_t max_rows, int Ka, int Nb);
GR_API int gr_wgrad(const float* a, int64_t lda, const float* a_stats, const float* bm,
             int64_t ldb, const int64_t* offsets, int B, int64_t max_rows, int Ka, int Nb,
             float* c, float* a_colsum, void* workspace, size_t ws_bytes, void* stream);

/* gr_wgrad2: the two weight gradients of one STU layer in ONE launch (two independent
 * gr_wgrad problems over the same jagged rows: problem 0 = LN(x)^T dh -> d_uvqk,
 * problem 1 = dy^T o_in -> d_o.weight with colsum d_o.bias) and one slab reduce.
 * Each problem as gr_wgrad; workspace: gr_wgrad2_workspace_size bytes. */
GR_API size_t gr_wgrad2_workspace_size(int64_t max_rows, int Ka0, int Nb0, int Ka1, int Nb1);
GR_API int gr_wgrad2(const float* a0, int64_t lda0, const float* a_stats0, const float* b0,
                     int64_t ldb0, int Ka0, int Nb0, float* c0, float* colsum0,
                     const float* a1, int64_t lda1, const float* a_stats1, const float* b1,
                     int64_t ldb1, int Ka1, int Nb1, float* c1, float* colsum1,
                     const int64_t* offsets, int B, int64_t max_rows, void* workspace,
                     size_t ws_bytes, void* stream);
/* gr_wgrad2 with bf16 MFMA operands (LayerNorm applied in fp32 before rounding; fp32
 * accumulation and slab reduce); same arguments, workspace and outputs. */
GR_API int gr_wgrad2_bf16(const float* a0, int64_t lda0, const float* a_stats0, const float* b0,
                          int64_t ldb0, int Ka0, int Nb0, float* c0, float* colsum0,
                          const float* a1, int64_t lda1, const float* a_stats1, const float* b1,
                          int64_t ldb1, int Ka1, int Nb1, float* c1, float* colsum1,
                          const int64_t* offsets, int B, int64_t max_rows, void* workspace,
                          size_t ws_bytes, void* stream);

/* gr_wgrad_multi (ABI 13) — the weight gradients of several problems in ONE partial
 * launch and ONE fixed-order reduce (the encoder's backward defers every layer's _uvqk
 * and _o gradients to one call: 2 launches per step instead of 2 per layer).
 * desc: n_problems (1..16) x 9 int64 {a, lda, a_stats, b, ldb, Ka, Nb, c, colsum} with
 * the meaning of gr_wgrad's arguments (pointers as integers; a_stats, colsum may be 0).
 * All problems share the jagged rows (offsets, B, max_rows); at most two distinct panel
 * widths (the narrow kernels' classes).  bf16: bf16 operands as gr_wgrad2_bf16.
 * Deterministic (fixed-order slab reduce, no atomics). */
GR_API size_t gr_wgrad_multi_workspace_size(const int64_t* desc, int n_problems, int64_t max_rows);
GR_API int gr_wgrad_multi(const int64_t* desc, int n_problems, const int64_t* offsets, int B,
                    int64_t max_rows, int bf16, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- bf16 activations
 * ABI 16.  HSTU(autocast_dtype=torch.bfloat16) at wide heads (dqk == dv = d, d % 32 == 0,
 * 128 < d <= 256: the ml-20m width) keeps the layer's activations in HBM as bf16, as the
 * reference's autocast region does (hstu.py:439-480: the mm outputs h, silu(h) and their
 * gradients are bf16 there; LayerNorm statistics, accumulation, parameters, the residual
 * stream x / y and d_attn stay fp32).  bf16 buffers are uint16_t* (raw bf16 bits).
 * Every entry runs the same kernels as its *_bf16 counterpart on the same bf16 operands,
 * so results equal that entry's on the bf16-rounded inputs, rounded to bf16 where the
 * output is bf16 (tests/test_gpu_a16.py).  What the layout removes: the Q/K/V conversion
 * pass (the attention DMAs its tiles straight from the bf16 uvqk rows), half of every
 * projection's activation bytes, and the weight gradients' fp32 operand reads.
 *
 * Weights enter the a16 projections as bf16 [N][K] images (autocast casts each mm's
 * weight to bf16 the same way), made once per step by gr_weight_images_bf16: desc = n
 * (<= 32) x 5 int64 {src (fp32, rows x cols row-major), rows, cols, transpose, dst (bf16:
 * rows x cols, or cols x rows when transpose = 1)}.  Images: wt_uvqk = W_uvqk^T (n_out, D),
 * w_o16 = W_o (D, hdv), wt_o16 = W_o^T (hdv, D), w_uvqk16 = W_uvqk (D, n_out); K (the
 * image's row length) % 8 == 0, 16-byte aligned.
 * hstu_ln_uvqk_fwd_a16: hstu_ln_uvqk_fwd with bf16 h_pre (optional) and uvqk (n_out,
 *   ld_out even), plus optional xn (rows, D) = bf16 LN(x), the weight gradient's A operand
 *   (replaces hstu.py:258-305 under autocast).  stats_given = 1: x_stats already holds the
 *   rows' LayerNorm (mean, rstd) -- the previous layer's hstu_gate_o_fwd_a16 y_stats --
 *   and the statistics pass over x is skipped (the same values: same sums, same order).
 * hstu_gate_o_fwd_a16: y_stats (optional, 240 < D <= 256): the LayerNorm statistics of
 *   each y row with `eps`, i.e. the next layer's x_stats.
 * hstu_attn_fwd_a16: hstu_attn_fwd_bf16 on bf16 q / k / v rows (16-byte aligned, ld_qkv a
 *   multiple of 8); zrow = d zero bf16 values (caller-owned, 16-byte aligned).
 * hstu_gate_o_fwd_a16 / _bwd_a16: u, h_u, o_in, du and d_attn in bf16 (hstu.py:393-413).
 * hstu_attn_bwd_a16: dq / dk / dv (bf16, written with silu'(h) from bf16 h applied) of
 *   hstu_attn_bwd_bf16; dout = gate_o_bwd_a16's bf16 d_attn (ld_dout = H d), staged by
 *   DMA as is (no conversion pass); zrow as in the forward; workspace from
 *   hstu_attn_bwd_a16_workspace_size.
 * hstu_ln_uvqk_bwd_a16: dh (d_uvqk) in bf16.
 * gr_wgrad_multi_a16: gr_wgrad_multi with bf16 MFMA operands and a 10th descriptor word of
 *   flags per problem (bit 0: A rows bf16, bit 1: B rows bf16); Ka <= 256, Ka, Nb, lda,
 *   ldb multiples of 4, bf16 rows 8-byte aligned, a bf16 A takes no row stats. */
GR_API int gr_weight_images_bf16(const int64_t* desc, int n, void* stream);
GR_API int hstu_ln_uvqk_fwd_a16(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                    int64_t max_rows, int D, const uint16_t* wt_uvqk, int n_out, float eps,
                    int activation, float* x_stats, int stats_given, uint16_t* h_pre,
                    uint16_t* uvqk, int64_t ld_out, uint16_t* xn, void* stream);
GR_API int hstu_attn_fwd_a16(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                    int64_t ld_qkv, const int64_t* offsets, int B, int N, int max_len, int H,
                    int d, const uint8_t* bucket_map, const float* pos_w, const float* ts_w,
                    int num_buckets, const uint16_t* zrow, float* out, int64_t ld_out,
                    void* stream);
GR_API int hstu_gate_o_fwd_a16(const uint16_t* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                    const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                    const uint16_t* w_o16, const float* b_o, const float* x_res, int64_t ld_x,
                    float eps, float dropout_p, uint64_t seed, const int64_t* seed_offset,
                    float* attn_stats, uint16_t* o_in, float* y, int64_t ld_y, float* y_stats,
                    void* stream);
GR_API int hstu_gate_o_bwd_a16(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                    int64_t max_rows, int hdv, int D, const uint16_t* wt_o16, const uint16_t* u,
                    int64_t ld_u, const float* attn, int64_t ld_attn, const float* attn_stats,
                    const uint16_t* h_u, int64_t ld_h, float dropout_p, uint64_t seed,
                    const int64_t* seed_offset, uint16_t* du, int64_t ld_du, uint16_t* d_attn,
                    int64_t ld_da, void* stream);
GR_API size_t hstu_attn_bwd_a16_workspace_size(int B, int N, int max_len, int H, int d,
                    int num_buckets);
GR_API int hstu_attn_bwd_a16(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                    int64_t ld_qkv, const uint16_t* dout, int64_t ld_dout, const int64_t* offsets,
                    int B, int N, int max_len, int H, int d, const uint8_t* bucket_map,
                    const float* pos_w, const float* ts_w, int num_buckets, const uint16_t* hq,
                    const uint16_t* hk, const uint16_t* hv, int64_t ld_h, uint16_t* dq,
                    uint16_t* dk, uint16_t* dv_out, int64_t ld_d, float* dpos_w, float* dts_w,
                    const uint16_t* zrow, void* workspace, size_t ws_bytes, void* stream);
GR_API int hstu_ln_uvqk_bwd_a16(const uint16_t* dh, int64_t ld_dh, const int64_t* offsets, int B,
                    int64_t max_rows, int D, int n_out, const uint16_t* w_uvqk16, const float* x,
                    int64_t ld_x, const float* x_stats, const float* dy_res, int64_t ld_dy,
                    float* dx, int64_t ld_dx, void* stream);
GR_API size_t gr_wgrad_multi_a16_workspace_size(const int64_t* desc, int n_problems,
                    int64_t max_rows);
GR_API int gr_wgrad_multi_a16(const int64_t* desc, int n_problems, const int64_t* offsets, int B,
                    int64_t max_rows, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- MIPS retrieval
 * Replaces indexing/top_k.py:44-70 (MIPSBruteForceTopK: mm + torch.topk) and
 * indexing/candidate_index.py:107-164 (get_top_k_outputs: top-(k+N0), drop the row's
 * invalid ids, keep the first k) with one fused pass: scores are never materialised
 * and invalid ids are excluded during selection (equivalent).
 *
 * mips_pack_items: re-lays the (X, D) row-major fp32 item table into the
 * MFMA-native blocked layout the scorer streams (done once per
 * CandidateIndex.update_embeddings); `packed` needs mips_packed_items_bytes(X, D).
 * For filter-path catalogs (below) the packed buffer also holds a bf16 copy of the
 * table and its largest row norm (ABI 5).
 *
 * mips_topk: queries (B, D) fp32; scores are the k-ordered fp32 fmaf chain over d.
 * Output rows are sorted by score desc, then catalog index asc (torch.topk leaves
 * ties unspecified).  Candidate item i (local row) has global index index_base + i
 * and id item_ids[i] (or index_base + i when item_ids is NULL).  Items whose id is in
 * the query's row of invalid_ids (B, N0) are excluded (padding zeros included, as in
 * the reference).  Rows with fewer than k valid items are padded with
 * (-inf, id -1, index -1).  out_index (B, k) is optional.  Limits: D <= 256,
 * k <= 4096, N0 <= 8192, X < 2^31.  N0 > 256 (ml-20m validation passes past_ids of
 * width 2059) sorts each query's list into the workspace first.  k > 256 (the
 * reference CandidateIndex asks its top-k module for k + N0) takes a chunked exact
 * path: all scores of a chunk of items, then a per-query radix select merged with the
 * running top-k; same scores, ids and order, no fused fast path.
 * Catalogs of X >= 262,144 items with D <= 256 take a threshold-filter path (sampled
 * per-query threshold, one all-query scoring pass over the bf16 copy that reads it
 * once, exact f32 rescoring of the candidates in the merge, which trusts only scores
 * above the bf16 error bound); inputs that defeat the threshold raise a device flag
 * and an exact path, gated on that flag, recomputes (no host sync).  The first int32
 * of the workspace is that flag after the call (1 = the exact fallback ran).
 */
GR_API size_t mips_packed_items_bytes(int64_t X, int D);
GR_API int mips_pack_items(const float* items, int64_t X, int D, float* packed, void* stream);
GR_API size_t mips_topk_workspace_size(int B, int64_t X, int D, int k, int N0);
GR_API int mips_topk(const float* queries, const float* packed_items, int64_t X, int D,
              const int64_t* item_ids, int64_t index_base, const int64_t* invalid_ids,
              int N0, int B, int k, float* out_scores, int64_t* out_ids, int64_t* out_index,
              void* workspace, size_t ws_bytes, void* stream);

/* mips_merge_topk: merges n_lists candidate lists per query (e.g. the all-gathered
 * per-shard results of a row-sharded catalog) into the global top-k with the same
 * canonical order.  cand_* are (n_lists, B, k_in); cand_index -1 marks an empty slot.
 * n_lists * k_in <= 8192, k <= 256.
 */
GR_API int mips_merge_topk(const float* cand_scores, const int64_t* cand_index,
                    const int64_t* cand_ids, int n_lists, int B, int k_in, int k,
                    float* out_scores, int64_t* out_ids, int64_t* out_index, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* GR_HSTU_H_ */
