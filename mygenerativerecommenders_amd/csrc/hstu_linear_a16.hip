// Projection GEMMs of the STU layer in the bf16-activation layout (ABI 16, the *_a16
// entries): the row-panel kernels and the Op templates of hstu_linear.hip instantiated
// with A16 = true, in a translation unit of their own so the two compile in parallel.
#define GR_LINEAR_LIB_ONLY
#include "hstu_linear.hip"

namespace gr {

// ---------------------------------------------------------------- weight images
// out (bf16) = w (fp32, rows x cols row-major) or its transpose: the [N][K] images the
// a16 row panels stage 16 bytes at a time.  One launch for up to 32 images (grid.y);
// 32 x 32 tiles through LDS so both the reads and the writes are row-contiguous.
constexpr int WI_MAX = 32;
struct WImg {
  const float* src[WI_MAX];
  __bf16* dst[WI_MAX];
  int rows[WI_MAX], cols[WI_MAX], tr[WI_MAX];
  int n;
};
__global__ __launch_bounds__(256) void weight_image_kernel(WImg a) {
  __shared__ float tile[32][33];
  const int i = blockIdx.y;
  const int R = a.rows[i], C = a.cols[i];
  const int tc = (C + 31) / 32;
  const int r0 = (blockIdx.x / tc) * 32, c0 = (blockIdx.x % tc) * 32;
  if (r0 >= R) return;
  const float* src = a.src[i];
  __bf16* dst = a.dst[i];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  if (!a.tr[i]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = r0 + ty + 8 * p, c = c0 + tx;
      if (r < R && c < C) dst[(int64_t)r * C + c] = (__bf16)src[(int64_t)r * C + c];
    }
    return;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + ty + 8 * p, c = c0 + tx;
    tile[ty + 8 * p][tx] = (r < R && c < C) ? src[(int64_t)r * C + c] : 0.f;
  }
  __syncthreads();
  // out (C x R): row c0 + ty + 8 p, column r0 + tx
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int c = c0 + ty + 8 * p, r = r0 + tx;
    if (r < R && c < C) dst[(int64_t)c * R + r] = (__bf16)tile[tx][ty + 8 * p];
  }
}

}  // namespace gr

using namespace gr;

extern "C" int gr_weight_images_bf16(const int64_t* desc, int n, void* stream) {
  GR_REQUIRE(desc && n >= 1 && n <= WI_MAX, "gr_weight_images_bf16: %d images (1..%d)", n, WI_MAX);
  WImg a{};
  a.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const int64_t* d = desc + 5 * i;
    a.src[i] = (const float*)d[0];
    a.rows[i] = (int)d[1];
    a.cols[i] = (int)d[2];
    a.tr[i] = (int)d[3];
    a.dst[i] = (__bf16*)d[4];
    GR_REQUIRE(a.src[i] && a.dst[i] && a.rows[i] > 0 && a.cols[i] > 0 && (d[3] == 0 || d[3] == 1),
               "gr_weight_images_bf16: image %d has a null pointer or a bad shape", i);
    tiles = std::max(tiles, ceil_div(a.rows[i], 32) * ceil_div(a.cols[i], 32));
  }
  GR_TIMED("weight_images", stream, hipLaunchKernelGGL(weight_image_kernel, dim3(tiles, n), dim3(256), 0,
                                                       (hipStream_t)stream, a));
  GR_LAUNCH_CHECK("gr_weight_images_bf16");
  return 0;
}

// ---------------------------------------------------------------- bf16 activations (ABI 16)
// autocast_dtype = bfloat16 at wide heads: uvqk / h_pre / o_in / d_uvqk in bf16 and the
// weights as bf16 [N][K] images (gr_weight_images_bf16; autocast casts them per mm the
// same way).  Same bf16 row panels; results equal the *_bf16 entries' on the same
// (bf16-rounded) inputs, rounded to bf16 where the output is bf16.
static bool img_ok(const void* w16, int N, int K) {
  return w16 && (uintptr_t)w16 % 16 == 0 && K % 8 == 0 && (int64_t)N * K * 2 < 0x7fffffffLL;
}

extern "C" int hstu_ln_uvqk_fwd_a16(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                                    int64_t max_rows, int D, const uint16_t* wt_uvqk, int n_out,
                                    float eps, int activation, float* x_stats, int stats_given,
                                    uint16_t* h_pre, uint16_t* uvqk, int64_t ld_out, uint16_t* xn,
                                    void* stream) {
  GR_REQUIRE(x && offsets && uvqk && x_stats, "hstu_ln_uvqk_fwd_a16: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0 && max_rows >= 0, "hstu_ln_uvqk_fwd_a16: bad sizes");
  GR_REQUIRE(activation == 0 || activation == 1, "hstu_ln_uvqk_fwd_a16: activation must be 0|1");
  GR_REQUIRE(n_out % 2 == 0 && ld_out % 2 == 0 && (uintptr_t)uvqk % 4 == 0 && (uintptr_t)h_pre % 4 == 0,
             "hstu_ln_uvqk_fwd_a16: n_out and ld_out must be even, outputs 4-byte aligned");
  GR_REQUIRE(img_ok(wt_uvqk, n_out, D),
             "hstu_ln_uvqk_fwd_a16: wt_uvqk must be the 16-byte aligned (n_out, D) bf16 image, D %% 8 == 0");
  OpLnUvqkT<true> op{offsets, B, D, n_out, x, ld_x, nullptr, eps, activation, (float2*)x_stats,
                     (__bf16*)h_pre, (__bf16*)uvqk, ld_out, (__bf16*)xn, stats_given != 0,
                     (const __bf16*)wt_uvqk};
  // GR_OPT_PANEL_VEC = 2: the float4-staged panel for this forward too (A/B)
  return launch_rowpanel_bf16(op, max_rows, false, "hstu_ln_uvqk_fwd", (hipStream_t)stream,
                              option(GR_OPT_PANEL_VEC) == 2 && (uintptr_t)x % 16 == 0 && ld_x % 4 == 0);
}

extern "C" int hstu_gate_o_fwd_a16(const uint16_t* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                                   const uint16_t* w_o16, const float* b_o, const float* x_res,
                                   int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                   const int64_t* seed_offset, float* attn_stats, uint16_t* o_in,
                                   float* y, int64_t ld_y, float* y_stats, void* stream) {
  GR_REQUIRE(u && attn && offsets && y && attn_stats, "hstu_gate_o_fwd_a16: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_fwd_a16: bad sizes");
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_gate_o_fwd_a16: dropout_p %f", dropout_p);
  GR_REQUIRE(img_ok(w_o16, D, hdv),
             "hstu_gate_o_fwd_a16: w_o16 must be the 16-byte aligned (D, hdv) bf16 image, hdv %% 8 == 0");
  // y_stats: the whole row in one 256-column panel (launch_rowpanel_bf16 picks NT = 16 only
  // when D > 240; narrower D takes the general epilogue, which cannot reduce a row)
  GR_REQUIRE(!y_stats || (D > 240 && D <= 256), "hstu_gate_o_fwd_a16: y_stats needs 240 < D <= 256, D %d", D);
  OpGateOT<true> op{offsets, B, hdv, D, (const __bf16*)u, ld_u, attn, ld_attn, nullptr, b_o, x_res,
                    ld_x, eps, dropout_p, seed, seed_offset, (float2*)attn_stats, (__bf16*)o_in, y,
                    ld_y, (float2*)y_stats, (const __bf16*)w_o16};
  return launch_rowpanel_bf16(op, max_rows, false, "hstu_gate_o_fwd", (hipStream_t)stream);
}

extern "C" int hstu_gate_o_bwd_a16(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                                   int64_t max_rows, int hdv, int D, const uint16_t* wt_o16,
                                   const uint16_t* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const float* attn_stats, const uint16_t* h_u, int64_t ld_h,
                                   float dropout_p, uint64_t seed, const int64_t* seed_offset,
                                   uint16_t* du, int64_t ld_du, uint16_t* d_attn, int64_t ld_da,
                                   void* stream) {
  GR_REQUIRE(dy && offsets && u && attn && attn_stats && du && d_attn,
             "hstu_gate_o_bwd_a16: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_bwd_a16: bad sizes");
  GR_REQUIRE(hdv % 2 == 0 && ld_u % 2 == 0 && ld_h % 2 == 0 && ld_du % 2 == 0 && ld_da % 2 == 0 &&
                 (uintptr_t)u % 4 == 0 && (uintptr_t)h_u % 4 == 0 && (uintptr_t)du % 4 == 0 &&
                 (uintptr_t)d_attn % 4 == 0,
             "hstu_gate_o_bwd_a16: bf16 rows must be 4-byte aligned with even widths and strides");
  GR_REQUIRE(img_ok(wt_o16, hdv, D),
             "hstu_gate_o_bwd_a16: wt_o16 must be the 16-byte aligned (hdv, D) bf16 image, D %% 8 == 0");
  OpGateOBwdT<true> op;
  op.offsets = offsets; op.B = B; op.K = D; op.N = hdv; op.dy = dy; op.lddy = ld_dy;
  op.w = nullptr; op.w16 = (const __bf16*)wt_o16;
  op.u = (const __bf16*)u; op.ldu = ld_u; op.attn = attn; op.lda = ld_attn;
  op.a_stats = (const float2*)attn_stats; op.h_u = (const __bf16*)h_u; op.ldh = ld_h;
  op.p = dropout_p; op.seed = seed; op.seed_off = seed_offset; op.du = (__bf16*)du; op.lddu = ld_du;
  op.da = (__bf16*)d_attn; op.ldda = ld_da;
  const bool vec = (uintptr_t)dy % 16 == 0 && ld_dy % 4 == 0;
  return launch_rowpanel_bf16(op, max_rows, true, "hstu_gate_o_bwd", (hipStream_t)stream, vec);
}

extern "C" int hstu_ln_uvqk_bwd_a16(const uint16_t* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                    int64_t max_rows, int D, int n_out, const uint16_t* w_uvqk16,
                                    const float* x, int64_t ld_x, const float* x_stats,
                                    const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                    void* stream) {
  GR_REQUIRE(dh && offsets && x && x_stats && dx, "hstu_ln_uvqk_bwd_a16: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0, "hstu_ln_uvqk_bwd_a16: bad sizes");
  GR_REQUIRE(img_ok(w_uvqk16, D, n_out),
             "hstu_ln_uvqk_bwd_a16: w_uvqk16 must be the 16-byte aligned (D, n_out) bf16 image");
  OpLnUvqkBwdT<true> op;
  op.offsets = offsets; op.B = B; op.K = n_out; op.N = D; op.dh = (const __bf16*)dh; op.lddh = ld_dh;
  op.w = nullptr; op.w16 = (const __bf16*)w_uvqk16;
  op.x = x; op.ldx = ld_x; op.x_stats = (const float2*)x_stats;
  op.dy = dy_res; op.lddy = ld_dy; op.dx = dx; op.lddx = ld_dx;
  // the float4 panel takes dh as 8-byte pieces of 4 bf16
  const bool vec = (uintptr_t)dh % 8 == 0 && ld_dh % 4 == 0;
  return launch_rowpanel_bf16(op, max_rows, true, "hstu_ln_uvqk_bwd", (hipStream_t)stream, vec);
}
