// Elementwise step of the Muon optimizer's bf16 Newton-Schulz chain (SURVEY §8 N4,
// reference optimizers/muon.py:3-29):  out = bf16(bf16(s * x) + y)  over bf16 tensors.
// The chain's two combines per iteration, B = b*A + (c*A)@A and X = a*X + B@X, each cost
// the reference two elementwise launches (the scaled operand, then the sum) with a
// rounding to bf16 after each; this kernel is one launch with the same two roundings,
// so the chain's result is bit-identical (tests/test_gpu_next_rows.py).  Any other
// rounding (a GEMM epilogue with beta, a single-rounding axpy) moves the orthogonalised
// update by ~5 % of its largest entry: the bf16 chain amplifies it.
#include <algorithm>
#include <vector>

#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

__device__ __forceinline__ float bf16_bits_to_float(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t float_to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// 8 elements (one 16-byte load per operand) per thread, grid-stride
__global__ __launch_bounds__(256) void bf16_scale_add_kernel(const uint4* x, float s, const uint4* y,
                                                             uint4* out, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const uint4 xv = x[i], yv = y[i];
    const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w}, ys[4] = {yv.x, yv.y, yv.z, yv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t w = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float sx = bf16_bits_to_float(float_to_bf16_bits(s * bf16_bits_to_float((uint16_t)(xs[j] >> (16 * h)))));
        const float r = sx + bf16_bits_to_float((uint16_t)(ys[j] >> (16 * h)));
        w |= (uint32_t)float_to_bf16_bits(r) << (16 * h);
      }
      o[j] = w;
    }
    out[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(256) void bf16_scale_add_tail_kernel(const uint16_t* x, float s, const uint16_t* y,
                                                                  uint16_t* out, int64_t i0, int64_t n) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const float sx = bf16_bits_to_float(float_to_bf16_bits(s * bf16_bits_to_float(x[i])));
    out[i] = float_to_bf16_bits(sx + bf16_bits_to_float(y[i]));
  }
}

}  // namespace gr

extern "C" int gr_bf16_scale_add(const uint16_t* x, float s, const uint16_t* y, uint16_t* out,
                                 int64_t n, void* stream) {
  GR_REQUIRE(n >= 0 && (n == 0 || (x && y && out)), "gr_bf16_scale_add: bad args");
  if (n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                     reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  const int64_t n8 = vec ? n / 8 : 0;
  if (n8 > 0) {
    const int64_t want = (n8 + 255) / 256;
    const unsigned grid = (unsigned)(want < 8 * 256 ? want : 8 * 256);
    GR_TIMED("bf16_scale_add", st, hipLaunchKernelGGL(gr::bf16_scale_add_kernel, dim3(grid), dim3(256), 0, st,
                                                      (const uint4*)x, s, (const uint4*)y, (uint4*)out, n8));
  }
  const int64_t rest = n - n8 * 8;  // unaligned operands, or the last n % 8 elements
  if (rest > 0)
    GR_TIMED("bf16_scale_add", st, hipLaunchKernelGGL(gr::bf16_scale_add_tail_kernel, dim3((unsigned)((rest + 255) / 256)),
                                                      dim3(256), 0, st, x, s, y, out, n8 * 8, n));
  GR_LAUNCH_CHECK("gr_bf16_scale_add");
  return 0;
}

// ------------------------------------------------------------------ AdamW, one launch
// torch.optim.AdamW(fused=True, capturable=True)'s update (the reference's optimizer,
// configs/model/*.yaml) over a parameter list in ONE launch, with the step counter
// advanced inside it.  torch runs it as two launches per step (the step-count
// _foreach_add_ and the fused multi-tensor kernel).  The tensors travel in the kernel
// arguments (so a captured graph replays the pointers it was captured with, as torch's
// tensor lists do), up to ADAMW_MAX per launch; workgroup w takes chunk w of the
// concatenated list (`chunk` elements, never crossing a tensor; chosen per call so that
// small lists get many workgroups and large tables few enough passes).  Scalar
// hyper-parameters are doubles and tensors fp32, with the arithmetic promoted as in
// ATen's FusedAdamMathFunctor (ADAMW mode).  In the launch that advances the counter,
// the last workgroup to finish (a completion counter the caller zeroes once; the kernel
// re-arms it) writes step + 1, so every workgroup reads the same step.
namespace gr {
constexpr int ADAMW_MAX = 48;
constexpr int ADAMW_SUB = 1024;  // elements per workgroup pass (4 per thread)
struct AdamWArgs {
  float* param[ADAMW_MAX];
  const float* grad[ADAMW_MAX];
  int64_t off[ADAMW_MAX];   // into exp_avg / exp_avg_sq
  int64_t n[ADAMW_MAX];
  int first_chunk[ADAMW_MAX + 1];
  int64_t chunk;            // elements per workgroup: a multiple of ADAMW_SUB
  int n_tensors;
  int advance;              // this launch writes step + 1
  float* exp_avg;
  float* exp_avg_sq;
  float* step;
  uint32_t* done;
  double lr, beta1, beta2, eps, wd;
};

__device__ __forceinline__ void adamw_elem(const AdamWArgs& a, float step_size, float bc2_sqrt,
                                           float& p, float g, float& m, float& v) {
  if (a.wd != 0.0) p = (float)((double)p - a.lr * a.wd * (double)p);
  m = (float)(a.beta1 * (double)m + (1.0 - a.beta1) * (double)g);
  v = (float)(a.beta2 * (double)v + (1.0 - a.beta2) * (double)g * (double)g);
  const float denom = (float)((double)(sqrtf(v) / bc2_sqrt) + a.eps);
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(256) void adamw_kernel(AdamWArgs a) {
  __shared__ int last;
  __shared__ float sc[4];  // t, step size, sqrt(1 - b2^t): the double pow()s once per workgroup
  const int w = blockIdx.x;
  int t = 0;
  while (t + 1 < a.n_tensors && a.first_chunk[t + 1] <= w) ++t;  // wave-uniform
  const int64_t c0 = (int64_t)(w - a.first_chunk[t]) * a.chunk;
  const int64_t cend = a.n[t] < c0 + a.chunk ? a.n[t] : c0 + a.chunk;
  float* param = a.param[t];
  const float* grad = a.grad[t];
  float* ma = a.exp_avg + a.off[t];
  float* va = a.exp_avg_sq + a.off[t];
  // sub-chunks of ADAMW_SUB elements, 4 per thread: one float4 per operand where the tensor
  // allows (16-byte aligned, a multiple of 4 long), scalars otherwise.  The first
  // sub-chunk's loads are issued before the step counter is read, so a workgroup starts
  // after one round trip, not two.
  const bool vec = (a.n[t] & 3) == 0 && ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                                          reinterpret_cast<uintptr_t>(ma) | reinterpret_cast<uintptr_t>(va)) & 15) == 0;
  float p[4], g[4], m[4], v[4];
  auto elem = [&](int64_t s0, int e) -> int64_t {
    return vec ? s0 + 4 * (int64_t)threadIdx.x + e : s0 + (int64_t)threadIdx.x + 256 * e;
  };
  auto load = [&](int64_t s0) {
    if (vec) {
      const int64_t i = s0 + 4 * (int64_t)threadIdx.x;
      const bool in = i < cend;
      const float4 pv = in ? *reinterpret_cast<const float4*>(param + i) : float4{};
      const float4 gv = in ? *reinterpret_cast<const float4*>(grad + i) : float4{};
      const float4 mv = in ? *reinterpret_cast<const float4*>(ma + i) : float4{};
      const float4 vv = in ? *reinterpret_cast<const float4*>(va + i) : float4{};
      p[0] = pv.x; p[1] = pv.y; p[2] = pv.z; p[3] = pv.w;
      g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
      m[0] = mv.x; m[1] = mv.y; m[2] = mv.z; m[3] = mv.w;
      v[0] = vv.x; v[1] = vv.y; v[2] = vv.z; v[3] = vv.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = elem(s0, e);
        const bool in = i < cend;
        p[e] = in ? param[i] : 0.f;
        g[e] = in ? grad[i] : 0.f;
        m[e] = in ? ma[i] : 0.f;
        v[e] = in ? va[i] : 0.f;
      }
    }
  };
  auto store = [&](int64_t s0) {
    if (vec) {
      const int64_t i = s0 + 4 * (int64_t)threadIdx.x;
      if (i < cend) {
        *reinterpret_cast<float4*>(param + i) = float4{p[0], p[1], p[2], p[3]};
        *reinterpret_cast<float4*>(ma + i) = float4{m[0], m[1], m[2], m[3]};
        *reinterpret_cast<float4*>(va + i) = float4{v[0], v[1], v[2], v[3]};
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = elem(s0, e);
        if (i < cend) {
          param[i] = p[e];
          ma[i] = m[e];
          va[i] = v[e];
        }
      }
    }
  };
  load(c0);
  if (threadIdx.x == 0) {
    const float ts = a.step[0] + 1.f;
    const float bc1 = (float)(1.0 - pow(a.beta1, (double)ts));
    const float bc2 = (float)(1.0 - pow(a.beta2, (double)ts));
    sc[0] = ts;
    sc[1] = (float)(a.lr / (double)bc1);
    sc[2] = sqrtf(bc2);
  }
  __syncthreads();
  const float ts = sc[0], step_size = sc[1], bc2_sqrt = sc[2];
  for (int64_t s0 = c0; s0 < cend; s0 += ADAMW_SUB) {
    if (s0 != c0) load(s0);
#pragma unroll
    for (int e = 0; e < 4; ++e) adamw_elem(a, step_size, bc2_sqrt, p[e], g[e], m[e], v[e]);
    store(s0);
  }
  if (!a.advance) return;
  // completion: the last workgroup advances the step and re-arms the counter.  Relaxed:
  // the increment only has to follow this workgroup's read of the step (thread 0 consumed
  // it before the barrier above); the parameter and moment stores need no ordering inside
  // the launch (an agent-scope release per workgroup: 0.60 against 0.19 ms for a 33.6 M
  // element table, scripts/adamw_micro.py)
  if (threadIdx.x == 0) {
    last = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    if (last) {
      a.step[0] = ts;
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
}  // namespace gr

extern "C" int gr_adamw_step(float* const* params, const float* const* grads, const int64_t* offs,
                             const int64_t* numel, int n_tensors, float* exp_avg, float* exp_avg_sq,
                             float* step, uint32_t* done, double lr, double beta1, double beta2,
                             double eps, double weight_decay, void* stream) {
  GR_REQUIRE(n_tensors >= 0 && (n_tensors == 0 || (params && grads && offs && numel && exp_avg &&
                                                   exp_avg_sq && step && done)),
             "gr_adamw_step: bad args");
  const hipStream_t st = (hipStream_t)stream;
  // launches of up to ADAMW_MAX tensors; the last one advances the counter
  std::vector<int> idx;
  for (int i = 0; i < n_tensors; ++i) {
    GR_REQUIRE(numel[i] >= 0 && offs[i] >= 0 && (numel[i] == 0 || (params[i] && grads[i])),
               "gr_adamw_step: tensor %d: bad pointer / size", i);
    if (numel[i] > 0) idx.push_back(i);
  }
  if (idx.empty()) return 0;
  int64_t total = 0;
  for (int i : idx) total += numel[i];
  // >= ~4096 workgroups' worth of passes before a workgroup takes more than one
  int64_t subs = total / ((int64_t)gr::ADAMW_SUB * 4096) + 1;
  subs = subs > 8 ? 8 : subs;
  const int64_t chunk = gr::ADAMW_SUB * subs;
  for (size_t b = 0; b < idx.size(); b += gr::ADAMW_MAX) {
    gr::AdamWArgs a{};
    a.chunk = chunk;
    int chunks = 0;
    a.n_tensors = (int)std::min(idx.size() - b, (size_t)gr::ADAMW_MAX);
    for (int j = 0; j < a.n_tensors; ++j) {
      const int i = idx[b + j];
      a.param[j] = params[i];
      a.grad[j] = grads[i];
      a.off[j] = offs[i];
      a.n[j] = numel[i];
      a.first_chunk[j] = chunks;
      const int64_t c = (numel[i] + chunk - 1) / chunk;
      GR_REQUIRE(chunks + c < 0x7fffffff, "gr_adamw_step: too many chunks");
      chunks += (int)c;
    }
    a.first_chunk[a.n_tensors] = chunks;
    a.advance = b + gr::ADAMW_MAX >= idx.size();
    a.exp_avg = exp_avg;
    a.exp_avg_sq = exp_avg_sq;
    a.step = step;
    a.done = done;
    a.lr = lr;
    a.beta1 = beta1;
    a.beta2 = beta2;
    a.eps = eps;
    a.wd = weight_decay;
    GR_TIMED("adamw", st, hipLaunchKernelGGL(gr::adamw_kernel, dim3((unsigned)chunks), dim3(256), 0, st, a));
  }
  GR_LAUNCH_CHECK("gr_adamw_step");
  return 0;
}
