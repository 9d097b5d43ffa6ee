// Item-embedding gather, forward and backward.
//
// Replaces LocalEmbeddingModule.get_item_embeddings (embeddings/embeddings.py:94-97):
//   out[i] = cat(item_w[id_i], year_w[year_table[clamp(id_i, 0, len - 1)]])
// which PyTorch runs as clamp + index + two embedding gathers + cat (and as two sorted
// embedding backwards).  One pass here: a 16-lane group per output row, each lane
// copying columns of both halves.  With year_w NULL it is a plain embedding gather
// (CategoricalEmbeddingModule passes its mapped ids).
//
// Backward: dW[row] += dout[i] for every i gathering that row, skipping the tables'
// padding row (nn.Embedding padding_idx=0: its gradient is always zero).  Default: fp32
// atomics (unordered, like index_add_; the ml-1m batch gathers each item ~7 times),
// after a zeroing kernel (graph-capture safe, see common.h).  GR_OPT_DETERMINISTIC:
// owner-computes instead -- a workgroup owns EMB_OWN rows of one table, scans every id
// in order, compacts its matches in id order through LDS and each thread sums its
// (row, column) in that order, so the result does not depend on scheduling.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

struct EmbArgs {
  const int64_t* ids;
  int64_t n;
  const float* w0;
  int64_t rows0;
  int d0;
  const float* w1;  // optional second table (year)
  int64_t rows1;
  int d1;
  const int64_t* map1;  // row of w1 = map1[clamp(id, 0, map_len - 1)]
  int64_t map_len;
  float* out;  // (n, d0 + d1)
  const float* dout;
  float* dw0;
  float* dw1;
  int64_t padding_idx;  // < 0: none
};

__device__ __forceinline__ int64_t emb_row1(const EmbArgs& a, int64_t id) {
  if (!a.map1) return id;
  const int64_t c = id < 0 ? 0 : (id >= a.map_len ? a.map_len - 1 : id);
  return a.map1[c];
}

__global__ __launch_bounds__(256) void item_embedding_fwd_kernel(EmbArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (i >= a.n) return;
  const int sub = threadIdx.x & 15, dd = a.d0 + a.d1;
  const int64_t id = a.ids[i];
  float* o = a.out + i * dd;
  // out-of-range rows read as 0 (nn.Embedding would raise; never fault here)
  const bool ok0 = id >= 0 && id < a.rows0;
  gptr<float> r0 = as_global(a.w0) + (ok0 ? id : 0) * a.d0;
  for (int c = sub; c < a.d0; c += 16) o[c] = ok0 ? r0[c] : 0.f;
  if (a.w1) {
    const int64_t y = emb_row1(a, id);
    const bool ok1 = y >= 0 && y < a.rows1;
    gptr<float> r1 = as_global(a.w1) + (ok1 ? y : 0) * a.d1;
    for (int c = sub; c < a.d1; c += 16) o[a.d0 + c] = ok1 ? r1[c] : 0.f;
  }
}

__global__ __launch_bounds__(256) void item_embedding_bwd_kernel(EmbArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (i >= a.n) return;
  const int sub = threadIdx.x & 15, dd = a.d0 + a.d1;
  const int64_t id = a.ids[i];
  gptr<float> g = as_global(a.dout) + i * dd;
  if (a.dw0 && id >= 0 && id < a.rows0 && id != a.padding_idx)
    for (int c = sub; c < a.d0; c += 16) atomicAdd(a.dw0 + id * a.d0 + c, g[c]);
  if (a.w1 && a.dw1) {
    const int64_t y = emb_row1(a, id);
    if (y >= 0 && y < a.rows1 && y != a.padding_idx)
      for (int c = sub; c < a.d1; c += 16) atomicAdd(a.dw1 + y * a.d1 + c, g[a.d0 + c]);
  }
}

// Deterministic backward: blockIdx.y = table (0 item, 1 year), blockIdx.x = row group.
constexpr int EMB_OWN = 8;  // table rows per workgroup (thread t: row t / 32, column t % 32)
__global__ __launch_bounds__(256) void item_embedding_bwd_owner_kernel(EmbArgs a) {
  __shared__ int s_i[256];
  __shared__ int s_r[256];
  __shared__ int s_cnt[4];
  const int tab = blockIdx.y;
  const int d = tab ? a.d1 : a.d0, coff = tab ? a.d0 : 0, dd = a.d0 + a.d1;
  const int64_t rows = tab ? a.rows1 : a.rows0;
  float* dw = tab ? a.dw1 : a.dw0;
  if (!dw || d == 0) return;
  const int64_t r0 = (int64_t)blockIdx.x * EMB_OWN;
  if (r0 >= rows) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int my_r = tid >> 5, my_c0 = tid & 31;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // columns my_c0 + 32 j (d <= 128)
  for (int64_t i0 = 0; i0 < a.n; i0 += 256) {
    const int64_t i = i0 + tid;
    int64_t row = -1;
    if (i < a.n) {
      const int64_t id = a.ids[i];
      row = tab ? emb_row1(a, id) : id;
      if (!(row >= 0 && row < rows && row != a.padding_idx && row >= r0 && row < r0 + EMB_OWN)) row = -1;
    }
    // in-order compaction: wave prefix by ballot, waves in id order
    const unsigned long long m = __ballot(row >= 0);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_cnt[wv] = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += s_cnt[w];
    const int tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    if (row >= 0) {
      s_i[base + before] = (int)(i - i0);
      s_r[base + before] = (int)(row - r0);
    }
    __syncthreads();
    for (int e = 0; e < tot; ++e) {  // every thread walks the matches in id order
      if (s_r[e] != my_r) continue;
      gptr<float> g = as_global(a.dout) + (i0 + s_i[e]) * dd + coff;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = my_c0 + 32 * j;
        if (c < d) acc[j] += g[c];
      }
    }
    __syncthreads();
  }
  const int64_t row = r0 + my_r;
  if (row < rows) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = my_c0 + 32 * j;
      if (c < d) dw[row * d + c] = acc[j];
    }
  }
}

}  // namespace gr

extern "C" {

int gr_item_embedding_fwd(const int64_t* ids, int64_t n, const float* w0, int64_t rows0, int d0,
                          const float* w1, int64_t rows1, int d1, const int64_t* map1,
                          int64_t map_len, float* out, void* stream) {
  GR_REQUIRE(n >= 0 && rows0 > 0 && d0 > 0 && (w1 == nullptr || (rows1 > 0 && d1 > 0)),
             "gr_item_embedding_fwd: bad sizes (n=%lld rows0=%lld d0=%d)", (long long)n,
             (long long)rows0, d0);
  GR_REQUIRE(map1 == nullptr || map_len > 0, "gr_item_embedding_fwd: empty year table");
  if (n == 0) return 0;
  GR_REQUIRE(ids && w0 && out, "gr_item_embedding_fwd: null pointer");
  gr::EmbArgs a{};
  a.ids = ids; a.n = n; a.w0 = w0; a.rows0 = rows0; a.d0 = d0;
  a.w1 = w1; a.rows1 = w1 ? rows1 : 0; a.d1 = w1 ? d1 : 0; a.map1 = map1; a.map_len = map_len;
  a.out = out;
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("item_embedding", st,
           hipLaunchKernelGGL(gr::item_embedding_fwd_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256),
                              0, st, a));
  GR_LAUNCH_CHECK("gr_item_embedding_fwd");
  return 0;
}

int gr_item_embedding_bwd(const int64_t* ids, int64_t n, const float* dout, int64_t rows0, int d0,
                          int64_t rows1, int d1, const int64_t* map1, int64_t map_len,
                          int64_t padding_idx, float* dw0, float* dw1, void* stream) {
  GR_REQUIRE(n >= 0 && rows0 > 0 && d0 > 0 && d1 >= 0 && (d1 == 0 || rows1 > 0),
             "gr_item_embedding_bwd: bad sizes");
  GR_REQUIRE(map1 == nullptr || map_len > 0, "gr_item_embedding_bwd: empty year table");
  GR_REQUIRE(dw0 || dw1, "gr_item_embedding_bwd: no gradient requested");
  const hipStream_t st = (hipStream_t)stream;
  if (gr::option(GR_OPT_DETERMINISTIC) != 0) {
    GR_REQUIRE(d0 <= 128 && d1 <= 128, "gr_item_embedding_bwd: deterministic mode needs d <= 128");
    GR_REQUIRE(n <= 0x7fffffffLL, "gr_item_embedding_bwd: n too large");
    GR_REQUIRE(n == 0 || (ids && dout), "gr_item_embedding_bwd: null pointer");
    {
      // every owner workgroup scans all n ids: bound the scan work (the mode is a
      // reproducibility check, not a production path; 2^33 id reads is ~C5 size)
      const int64_t rm = rows0 > rows1 ? rows0 : rows1;
      GR_REQUIRE((rm + gr::EMB_OWN - 1) / gr::EMB_OWN * (double)n <= 8589934592.0,
                 "gr_item_embedding_bwd: deterministic mode limited to ceil(rows/8) * n <= 2^33 "
                 "(rows=%lld n=%lld)", (long long)rm, (long long)n);
    }
    gr::EmbArgs a{};
    a.ids = ids; a.n = n; a.rows0 = rows0; a.d0 = d0;
    a.rows1 = rows1; a.d1 = d1; a.map1 = map1; a.map_len = map_len;
    a.dout = dout; a.dw0 = dw0; a.dw1 = d1 > 0 ? dw1 : nullptr; a.padding_idx = padding_idx;
    const int64_t rmax = rows0 > rows1 ? rows0 : rows1;
    GR_TIMED("item_embedding", st,
             hipLaunchKernelGGL(gr::item_embedding_bwd_owner_kernel,
                                dim3((unsigned)((rmax + gr::EMB_OWN - 1) / gr::EMB_OWN), 2),
                                dim3(256), 0, st, a));
    GR_LAUNCH_CHECK("gr_item_embedding_bwd(deterministic)");
    return 0;
  }
  if (dw0) gr::zero_words_async(dw0, rows0 * d0, st);
  if (dw1 && d1 > 0) gr::zero_words_async(dw1, rows1 * d1, st);
  if (n > 0) {
    GR_REQUIRE(ids && dout, "gr_item_embedding_bwd: null pointer");
    gr::EmbArgs a{};
    a.ids = ids; a.n = n; a.rows0 = rows0; a.d0 = d0;
    // w1 only flags that a second table exists (its values are not read)
    a.w1 = d1 > 0 ? reinterpret_cast<const float*>(dout) : nullptr;
    a.rows1 = rows1; a.d1 = d1; a.map1 = map1; a.map_len = map_len;
    a.dout = dout; a.dw0 = dw0; a.dw1 = dw1; a.padding_idx = padding_idx;
    GR_TIMED("item_embedding", st,
             hipLaunchKernelGGL(gr::item_embedding_bwd_kernel, dim3((unsigned)((n + 15) / 16)),
                                dim3(256), 0, st, a));
  }
  GR_LAUNCH_CHECK("gr_item_embedding_bwd");
  return 0;
}

}  // extern "C"
