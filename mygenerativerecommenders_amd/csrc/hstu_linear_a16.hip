// Projection GEMMs of the STU layer in the bf16-activation layout (ABI 16, the *_a16
// entries): the row-panel kernels and the Op templates of hstu_linear.hip instantiated
// with A16 = true, in a translation unit of their own so the two compile in parallel.
#define GR_LINEAR_LIB_ONLY
#include "hstu_linear.hip"

using namespace gr;

// ---------------------------------------------------------------- bf16 activations (ABI 16)
// autocast_dtype = bfloat16 at wide heads: uvqk / h_pre / o_in / d_uvqk in bf16 (see the
// Op templates).  Same bf16 row panels; results equal the *_bf16 entries' on the same
// (bf16-rounded) inputs, rounded to bf16 where the output is bf16.
extern "C" int hstu_ln_uvqk_fwd_a16(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                                    int64_t max_rows, int D, const float* w_uvqk, int n_out,
                                    float eps, int activation, float* x_stats, int stats_given,
                                    uint16_t* h_pre, uint16_t* uvqk, int64_t ld_out, uint16_t* xn,
                                    void* stream) {
  GR_REQUIRE(x && offsets && w_uvqk && uvqk && x_stats, "hstu_ln_uvqk_fwd_a16: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0 && max_rows >= 0, "hstu_ln_uvqk_fwd_a16: bad sizes");
  GR_REQUIRE(activation == 0 || activation == 1, "hstu_ln_uvqk_fwd_a16: activation must be 0|1");
  GR_REQUIRE(n_out % 2 == 0 && ld_out % 2 == 0 && (uintptr_t)uvqk % 4 == 0 && (uintptr_t)h_pre % 4 == 0,
             "hstu_ln_uvqk_fwd_a16: n_out and ld_out must be even, outputs 4-byte aligned");
  OpLnUvqkT<true> op{offsets, B, D, n_out, x, ld_x, w_uvqk, eps, activation, (float2*)x_stats,
                     (__bf16*)h_pre, (__bf16*)uvqk, ld_out, (__bf16*)xn, stats_given != 0};
  return launch_rowpanel_bf16(op, max_rows, false, "hstu_ln_uvqk_fwd", (hipStream_t)stream);
}

extern "C" int hstu_gate_o_fwd_a16(const uint16_t* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                                   const float* w_o, const float* b_o, const float* x_res,
                                   int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                   const int64_t* seed_offset, float* attn_stats, uint16_t* o_in,
                                   float* y, int64_t ld_y, float* y_stats, void* stream) {
  GR_REQUIRE(u && attn && offsets && w_o && y && attn_stats, "hstu_gate_o_fwd_a16: null pointer");
  GR_REQUIRE(!y_stats || D <= 256, "hstu_gate_o_fwd_a16: y_stats needs D <= 256 (one panel), D %d", D);
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_fwd_a16: bad sizes");
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_gate_o_fwd_a16: dropout_p %f", dropout_p);
  OpGateOT<true> op{offsets, B, hdv, D, (const __bf16*)u, ld_u, attn, ld_attn, w_o, b_o, x_res, ld_x,
                    eps, dropout_p, seed, seed_offset, (float2*)attn_stats, (__bf16*)o_in, y, ld_y,
                    (float2*)y_stats};
  // y_stats: the whole row in one 256-column panel (launch_rowpanel_bf16 picks NT = 16 only
  // when D > 240; narrower D takes the general epilogue, which cannot reduce a row)
  GR_REQUIRE(!y_stats || D > 240, "hstu_gate_o_fwd_a16: y_stats needs 240 < D <= 256, D %d", D);
  return launch_rowpanel_bf16(op, max_rows, false, "hstu_gate_o_fwd", (hipStream_t)stream);
}

extern "C" int hstu_gate_o_bwd_a16(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                                   int64_t max_rows, int hdv, int D, const float* w_o,
                                   const uint16_t* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const float* attn_stats, const uint16_t* h_u, int64_t ld_h,
                                   float dropout_p, uint64_t seed, const int64_t* seed_offset,
                                   uint16_t* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                                   void* stream) {
  GR_REQUIRE(dy && offsets && w_o && u && attn && attn_stats && du && d_attn,
             "hstu_gate_o_bwd_a16: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_bwd_a16: bad sizes");
  GR_REQUIRE(hdv % 2 == 0 && ld_u % 2 == 0 && ld_h % 2 == 0 && ld_du % 2 == 0 &&
                 (uintptr_t)u % 4 == 0 && (uintptr_t)h_u % 4 == 0 && (uintptr_t)du % 4 == 0,
             "hstu_gate_o_bwd_a16: bf16 rows must be 4-byte aligned with even widths and strides");
  OpGateOBwdT<true> op;
  op.offsets = offsets; op.B = B; op.K = D; op.N = hdv; op.dy = dy; op.lddy = ld_dy;
  op.w = w_o; op.u = (const __bf16*)u; op.ldu = ld_u; op.attn = attn; op.lda = ld_attn;
  op.a_stats = (const float2*)attn_stats; op.h_u = (const __bf16*)h_u; op.ldh = ld_h;
  op.p = dropout_p; op.seed = seed; op.seed_off = seed_offset; op.du = (__bf16*)du; op.lddu = ld_du;
  op.da = d_attn; op.ldda = ld_da;
  return launch_rowpanel_bf16(op, max_rows, true, "hstu_gate_o_bwd", (hipStream_t)stream,
                              rw_vec({dy, w_o}, {ld_dy, hdv}) == 4);
}

extern "C" int hstu_ln_uvqk_bwd_a16(const uint16_t* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                    int64_t max_rows, int D, int n_out, const float* w_uvqk,
                                    const float* x, int64_t ld_x, const float* x_stats,
                                    const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                    void* stream) {
  GR_REQUIRE(dh && offsets && w_uvqk && x && x_stats && dx, "hstu_ln_uvqk_bwd_a16: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0, "hstu_ln_uvqk_bwd_a16: bad sizes");
  OpLnUvqkBwdT<true> op;
  op.offsets = offsets; op.B = B; op.K = n_out; op.N = D; op.dh = (const __bf16*)dh; op.lddh = ld_dh;
  op.w = w_uvqk; op.x = x; op.ldx = ld_x; op.x_stats = (const float2*)x_stats;
  op.dy = dy_res; op.lddy = ld_dy; op.dx = dx; op.lddx = ld_dx;
  // the float4 panel takes dh as 8-byte pieces of 4 bf16
  const bool vec = (uintptr_t)dh % 8 == 0 && ld_dh % 4 == 0 && rw_vec({w_uvqk}, {D}) == 4;
  return launch_rowpanel_bf16(op, max_rows, true, "hstu_ln_uvqk_bwd", (hipStream_t)stream, vec);
}

