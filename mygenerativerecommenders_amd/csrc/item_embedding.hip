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
// padding row (nn.Embedding padding_idx=0: its gradient is always zero).  fp32 atomics
// (unordered, like index_add_; the ml-1m batch gathers each item ~7 times).  The
// gradients are zeroed by a kernel first (graph-capture safe, see common.h).
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
