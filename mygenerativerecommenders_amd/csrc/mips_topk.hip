// Brute-force MIPS top-k with fused invalid-id exclusion — gfx950, f32 MFMA.
//
// Replaces reference indexing/top_k.py:44-70 (mm -> (B, X) logits in HBM -> torch.topk)
// and indexing/candidate_index.py:107-164 (top-(k+N0), (B, k', N0) compare, cumsum,
// nonzero host sync, gather).  Nothing (B, X) is ever materialised.
//
// Item table layout (mips_pack_items): MFMA-native blocks of 16 items.  For item i,
// dim d: block ib = i/16, lane l = 16*(d%4) + i%16, k-step st = d/4, stored at
//   packed[((ib * KS2 + st/2) * 64 + l) * 2 + st%2]        (KS2 = ceil(ceil(D/4)/2))
// so the A operand of v_mfma_f32_16x16x4_f32 for a whole block is read with fully
// coalesced 512-B float2 loads (no LDS staging): the table is re-laid out once per
// CandidateIndex.update_embeddings, not per query batch.
//
// Scores are the k-ordered fp32 fmaf chain over d = 0..D-1 (an f32 MFMA IS that chain),
// bit-identical to oracle/topk_oracle.c.  Order: score desc, then catalog index asc.
//
// Phase 1 (mips_select_kernel): a workgroup = 4 waves = 16 queries x a contiguous item
// range; every lane keeps its query's running threshold tau (the k-th best VALID score
// seen so far).  Scores > tau are appended (LDS atomics) to a per-query LDS buffer;
// when a buffer may overflow, the 4 waves compact it (invalid ids dropped by binary
// search in the query's sorted invalid list, exact k-th by 8-bit radix select, ties
// by index) and raise tau.  Each workgroup emits its range's exact top-k per query.
// Phase 2 (mips_merge_kernel): one workgroup per query merges the per-range lists
// (also used for the cross-GPU merge of a row-sharded catalog), radix-selects the
// global top-k and bitonic-sorts it.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

constexpr int QG = 16;       // queries per workgroup (MFMA column block)
constexpr int SW = 8;        // waves per select workgroup (2 per SIMD, one LDS buffer set)
constexpr int ST = SW * 64;  // select threads
constexpr int CAP = 512;     // per-query candidate buffer: k (<= 256) + one step (SW * STEP <= 256)
constexpr int INV_MAX = 256; // invalid ids per query the select kernel keeps in LDS
constexpr int INV_BIG = 8192; // max invalid ids per query (ml-20m validation: N0 = 2059)
constexpr uint32_t VERIFIED = 0x80000000u;

// Sorted invalid lists are padded with INT64_MAX to n0p = a power of two >= 64.
__host__ __device__ inline int inv_pad(int N0) {
  if (N0 <= 0) return 0;
  int p = 64;
  while (p < N0) p <<= 1;
  return p;
}

// Ascending bitonic sort of v[0 .. n) in LDS (n a power of two), all threads of the
// block (any size) joining; the caller has stored v and synchronised.
__device__ void block_bitonic_i64(int64_t* v, int n) {
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = threadIdx.x; p < n / 2; p += blockDim.x) {
        const int i = 2 * p - (p & (stride - 1)), j = i + stride;
        const bool up = (i & size) == 0;
        const int64_t x = v[i], y = v[j];
        if ((x > y) == up) {
          v[i] = y;
          v[j] = x;
        }
      }
      __syncthreads();
    }
}

// N0 > INV_MAX: each query's invalid row, sorted ascending and padded to n0p, into
// the workspace (the select kernel binary-searches it there; 16 queries' lists do not
// fit its LDS).  One workgroup per query, n0p * 8 B of dynamic LDS.
__global__ __launch_bounds__(1024) void mips_sort_invalid_kernel(const int64_t* invalid, int N0,
                                                                 int n0p, int64_t* out,
                                                                 const int* gate) {
  if (gate && *gate == 0) return;
  extern __shared__ int64_t vs[];
  const int64_t* src = invalid + (int64_t)blockIdx.x * N0;
  for (int j = threadIdx.x; j < n0p; j += blockDim.x) vs[j] = j < N0 ? src[j] : INT64_MAX;
  __syncthreads();
  block_bitonic_i64(vs, n0p);
  int64_t* dst = out + (int64_t)blockIdx.x * n0p;
  for (int j = threadIdx.x; j < n0p; j += blockDim.x) dst[j] = vs[j];
}

__device__ __forceinline__ uint32_t ord_key(float s) {
  // monotone map float -> uint32 with -0 == +0; 0 is reserved for "dropped"
  if (s == 0.f) s = 0.f;
  uint32_t b = __float_as_uint(s);
  uint32_t k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  return k == 0u ? 1u : k;
}
__device__ __forceinline__ float key_to_float(uint32_t k) {
  uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(b);
}

__device__ __forceinline__ bool sorted_contains(const int64_t* v, int n, int64_t key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (v[m] < key) lo = m + 1; else hi = m;
  }
  return lo < n && v[lo] == key;
}

// ----------------------------------------------------------------- bf16 filter copy
// bf16 with round-to-nearest-even: |bf16(x) - x| <= 2^-8 |x| (NaN stays NaN).
__device__ __forceinline__ uint32_t bf16_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f4 mfma16x16x32bf16(u32x4 a, u32x4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Large catalogs carry a second, bf16 copy of the table for the filter pass (half the
// bytes, 16x the MFMA rate of the f32 path), in the A-operand order of
// v_mfma_f32_16x16x32_bf16: for block ib, k-chunk c (KC = ceil(D/32)) and lane l, one
// 16-byte word (element j in bits 16j .. 16j+15) = bf16(item ib*16 + l%16, dims
// 32c + 8(l/16) + 0..7).  The last chunk stores only its first LG = ceil((D - 32(KC-1))/8)
// lane groups (dims past D would be zero): a block is BB = 1024 (KC-1) + 256 LG bytes
// (D = 50: 1,792 B instead of 2,048), word (ib, c, l) at byte ib BB + 1024 c + 16 l.  The
// filter's lanes of the unstored groups re-read group 0's word (same address: no extra
// bytes) against zero query dims.  When the last chunk ends 1 or 2 dims past a whole lane
// group (D = 50: dims 48, 49), that group is a 64-byte tail after the chunks instead (one
// u32 of <= 2 bf16 per item): its lanes build their A operand {tail, 0, 0, 0} -- the same
// operand the full word held, so the scores are unchanged -- and D = 50 stores 1,600 B
// per block instead of 1,792.  The largest item L2 norm (fp32 bits, for
// the filter's error bound) follows the copy.
__host__ __device__ inline int bf16_tail_dims(int D, int KC) {  // (KC <= 2 only)
  const int rem = D - 32 * (KC - 1), t = rem % 8;
  return KC <= 2 && rem > 8 && (t == 1 || t == 2) ? t : 0;
}
__host__ __device__ inline int bf16_last_groups(int D, int KC) {
  return bf16_tail_dims(D, KC) ? (D - 32 * (KC - 1)) / 8 : (D - 32 * (KC - 1) + 7) / 8;
}
__host__ __device__ inline int bf16_block_bytes(int D, int KC) {
  return 1024 * (KC - 1) + 256 * bf16_last_groups(D, KC) + (bf16_tail_dims(D, KC) ? 64 : 0);
}
__global__ void pack_bf16_kernel(const float* items, int64_t X, int D, int KC, u32x4* packed16) {
  const int words = bf16_block_bytes(D, KC) / 16;  // 16-byte words per block
  const int chunk_words = 64 * (KC - 1) + 16 * bf16_last_groups(D, KC);
  const int dt = D - bf16_tail_dims(D, KC);  // first tail dim (D without a tail)
  // (tail word j: items 4j .. 4j + 3)
  const int64_t total = (X + 15) / 16 * words;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ib = e / words;
    const int u = (int)(e - ib * words);
    uint32_t w[4];
    if (u < chunk_words) {
      const int c = u >> 6, l = u & 63;
      const int64_t i = ib * 16 + (l & 15);
      const int d0 = 32 * c + 8 * (l >> 4);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int d = d0 + 2 * h;
        const float v0 = (i < X && d < dt) ? items[i * D + d] : 0.f;
        const float v1 = (i < X && d + 1 < dt) ? items[i * D + d + 1] : 0.f;
        w[h] = bf16_bits(v0) | (bf16_bits(v1) << 16);
      }
    } else {  // tail word j = u - chunk_words: items 4j .. 4j + 3, dims dt, dt + 1
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int64_t i = ib * 16 + 4 * (u - chunk_words) + h;
        const float v0 = (i < X && dt < D) ? items[i * D + dt] : 0.f;
        const float v1 = (i < X && dt + 1 < D) ? items[i * D + dt + 1] : 0.f;
        w[h] = bf16_bits(v0) | (bf16_bits(v1) << 16);
      }
    }
    packed16[e] = u32x4{w[0], w[1], w[2], w[3]};
  }
}

// rows[i][0 .. DP) = items[i][0 .. D), zero padded
__global__ void pack_rows_kernel(const float* items, int64_t X, int D, int DP, float* rows) {
  const int64_t total = X * DP;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / DP;
    const int d = (int)(e - i * DP);
    rows[e] = d < D ? items[i * D + d] : 0.f;
  }
}

__device__ __forceinline__ float bf16_round(float f) { return __uint_as_float(bf16_bits(f) << 16); }

// The filter's error-bound inputs, as fp32 bits (non-negative floats order like their bit
// patterns; both words zeroed beforehand):
//   maxbits[0] = max_i ||bf16(x_i)||_2,   maxbits[1] = max_i ||bf16(x_i) - x_i||_2.
// NaN / inf rows push them to NaN-like bits, which disables the filter (its thresholds
// compare false) and routes the batch to the exact path.
__global__ __launch_bounds__(256) void item_norm_max_kernel(const float* items, int64_t X, int D,
                                                            uint32_t* maxbits) {
  uint32_t m = 0, me = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < X; i += (int64_t)gridDim.x * 256) {
    float ss = 0.f, se = 0.f;
    for (int d = 0; d < D; ++d) {
      const float v = items[i * D + d], r = bf16_round(v), e = r - v;
      ss = fmaf(r, r, ss);
      se = fmaf(e, e, se);
    }
    const uint32_t b = __float_as_uint(sqrtf(ss)), be = __float_as_uint(sqrtf(se));
    m = b > m ? b : m;
    me = be > me ? be : me;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t v = __shfl_xor(m, o, 64), ve = __shfl_xor(me, o, 64);
    m = v > m ? v : m;
    me = ve > me ? ve : me;
  }
  if ((threadIdx.x & 63) == 0) {
    if (m) atomicMax(maxbits, m);
    if (me) atomicMax(maxbits + 1, me);
  }
}

// ----------------------------------------------------------------- packing
__global__ void pack_items_kernel(const float* items, int64_t X, int D, int KS2, float* packed) {
  const int64_t nblk = (X + 15) / 16;
  const int64_t total = nblk * KS2 * 128;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int h = (int)(e & 1);
    const int l = (int)((e >> 1) & 63);
    const int64_t t = e >> 7;  // ib * KS2 + j
    const int j = (int)(t % KS2);
    const int64_t ib = t / KS2;
    const int st = 2 * j + h;
    const int d = 4 * st + (l >> 4);
    const int64_t i = ib * 16 + (l & 15);
    packed[e] = (i < X && d < D) ? items[i * D + d] : 0.f;
  }
}

// ----------------------------------------------------------------- wave radix select
// Finds K* = the k-th largest of the nonzero keys held by the wave (EPL per lane) and
// how many entries equal to K* are needed (k_rem).  hist: 256 ints of LDS per wave.
template <int EPL>
__device__ void wave_radix_select(const uint32_t (&key)[EPL], int k, int* hist, uint32_t& kstar,
                                  int& k_rem) {
  const int lane = threadIdx.x & 63;
  uint32_t prefix = 0, mask = 0;
  int need = k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = lane; i < 256; i += 64) hist[i] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int t = 0; t < EPL; ++t)
      if (key[t] != 0u && (key[t] & mask) == prefix) atomicAdd(&hist[(key[t] >> shift) & 255], 1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // lane l owns digits 255-4l .. 252-4l (descending)
    int c[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = hist[255 - 4 * lane - j];
      s += c[j];
    }
    int incl = s;  // inclusive scan over lanes (descending digits)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int excl = incl - s;
    // the lane whose range crosses `need`
    const bool mine = excl < need && incl >= need;
    const unsigned long long bal = __ballot(mine);
    const int owner = __ffsll((long long)bal) - 1;
    int digit = 0, above = 0;
    if (mine) {
      int run = excl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (run + c[j] >= need) {
          digit = 255 - 4 * lane - j;
          above = run;
          break;
        }
        run += c[j];
      }
    }
    digit = __shfl(digit, owner, 64);
    above = __shfl(above, owner, 64);
    prefix |= (uint32_t)digit << shift;
    mask |= 0xFFu << shift;
    need -= above;
  }
  kstar = prefix;
  k_rem = need;
}

// ----------------------------------------------------------------- phase 1
struct SelectArgs {
  const float* q;
  const float* packed;
  int64_t X;
  int D, B, k, N0, n_ranges;
  int k_part;           // entries per (range, query) partial list (>= k)
  int64_t range_items;  // multiple of 4*64
  const int64_t* item_ids;
  int64_t index_base;
  const int64_t* invalid;
  float* part_score;   // [n_ranges][B][k_part]
  int64_t* part_index; // [n_ranges][B][k_part]  (global index, -1 = empty)
  const int* gate;      // non-null: run only when *gate != 0 (fallback of the filter path)
  const int64_t* inv_sorted;  // N0 > INV_MAX: [B][n0p] sorted lists (mips_sort_invalid_kernel)
};

// One (item range, query group) unit of the select kernel.
template <int KS, int BLOCKS>
__device__ __forceinline__ void mips_select_unit(const SelectArgs& a, const int bid) {
  constexpr int KS2 = (KS + 1) / 2;
  constexpr int STEP = BLOCKS * 16;  // items per wave per step
  __shared__ float cs[QG * CAP];
  __shared__ uint32_t ci[QG * CAP];
  __shared__ int64_t inv[QG * INV_MAX];
  __shared__ int hist[SW * 256];
  __shared__ int cnt[QG];
  __shared__ float tau_s[QG];
  __shared__ int need_compact;

  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  // XCD-aware decode: the query groups of one item range share blockIdx % 8
  const int n_qg = (a.B + QG - 1) / QG;
  const int xcd = bid & 7, rest = bid >> 3;
  const int g = rest % n_qg;
  const int range = (rest / n_qg) * 8 + xcd;
  if (range >= a.n_ranges) return;
  const int q0 = g * QG;
  const int64_t x_begin = (int64_t)range * a.range_items;
  const int64_t x_end = min(a.X, x_begin + a.range_items);

  // ---- prologue: sorted invalid lists (LDS, or the pre-sorted workspace rows), counters
  const bool big = a.inv_sorted != nullptr;
  const int n0p = inv_pad(a.N0);
  for (int e = tid; e < (big ? 0 : QG * n0p); e += ST) {
    const int qq = e / n0p, j = e - qq * n0p;
    int64_t v = INT64_MAX;
    if (q0 + qq < a.B && j < a.N0) v = a.invalid[(int64_t)(q0 + qq) * a.N0 + j];
    inv[qq * INV_MAX + j] = v;
  }
  if (tid < QG) {
    cnt[tid] = 0;
    tau_s[tid] = q0 + tid < a.B ? -INFINITY : INFINITY;  // padded queries collect nothing
  }
  __syncthreads();
  for (int size = 2; size <= (big ? 0 : n0p); size <<= 1) {  // bitonic sort, QG independent rows
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = tid; e < QG * (n0p / 2); e += ST) {
        const int qq = e / (n0p / 2), p = e - qq * (n0p / 2);
        const int i = 2 * p - (p & (stride - 1));
        const int j = i + stride;
        const bool up = (i & size) == 0;
        int64_t* row = inv + qq * INV_MAX;
        const int64_t x = row[i], y = row[j];
        if ((x > y) == up) {
          row[i] = y;
          row[j] = x;
        }
      }
      __syncthreads();
    }
  }

  // ---- query fragments (B operand): Q[q0 + lr][4 st + lg]
  float qreg[KS];
  {
    const int qq = q0 + lr;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int d = 4 * st + lg;
      qreg[st] = (qq < a.B && d < a.D) ? a.q[(int64_t)qq * a.D + d] : 0.f;
    }
  }

  const int64_t n_items = x_end > x_begin ? x_end - x_begin : 0;
  const int n_steps = (int)((n_items + SW * STEP - 1) / (SW * STEP));
  typedef float fv2 __attribute__((ext_vector_type(2)));
  gptr<fv2> pk = as_global(reinterpret_cast<const fv2*>(a.packed));
  int* whist = hist + w * 256;

  auto compact = [&](int qq, int kk) {
    // one wave compacts query qq's buffer to its exact top-kk valid entries
    uint32_t key[CAP / 64];
    float sc[CAP / 64];
    uint32_t ix[CAP / 64];
    const int n = cnt[qq];
    const int64_t* qinv =
        big ? a.inv_sorted + (int64_t)min(q0 + qq, a.B - 1) * n0p : inv + qq * INV_MAX;
    int nvalid = 0;
    // all LDS/global loads unconditional (clamped) so they are in flight together
    int64_t id[CAP / 64];
    bool need[CAP / 64];
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) {
      const int j = lane + 64 * t;
      const int jc = j < n ? j : 0;
      sc[t] = cs[qq * CAP + jc];
      ix[t] = ci[qq * CAP + jc];
      need[t] = j < n && !(ix[t] & VERIFIED);
      const int64_t li = (int64_t)(ix[t] & ~VERIFIED);
      id[t] = a.item_ids ? as_global(a.item_ids)[li < a.X ? li : 0] : a.index_base + li;
    }
    const int nbits = a.N0 > 0 ? 32 - __clz(n0p - 1) : 0;  // log2(n0p)
    // branchless lower_bounds over the sorted (INT64_MAX padded) n0p-entry list, the
    // lane's CAP/64 searches stepped together (independent probes in flight: the
    // big-list rows are read from L2)
    int pos[CAP / 64];
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) pos[t] = 0;
    for (int bit = nbits - 1; bit >= 0; --bit) {
      int64_t pv[CAP / 64];
#pragma unroll
      for (int t = 0; t < CAP / 64; ++t) pv[t] = qinv[pos[t] + (1 << bit) - 1];
#pragma unroll
      for (int t = 0; t < CAP / 64; ++t) pos[t] += (pv[t] < id[t]) ? (1 << bit) : 0;
    }
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) {
      const bool hit = a.N0 > 0 && qinv[pos[t] < n0p ? pos[t] : n0p - 1] == id[t];
      const int j = lane + 64 * t;
      const bool ok = j < n && !(need[t] && hit);
      ix[t] |= VERIFIED;
      key[t] = ok ? ord_key(sc[t]) : 0u;
      nvalid += ok;
    }
    // total valid count
    int tot = nvalid;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tot += __shfl_xor(tot, o, 64);
    uint32_t kstar = 0u;
    int k_rem = 0;
    bool all = tot <= kk;
    int eq_cnt = 0;
    if (!all) {
      wave_radix_select<CAP / 64>(key, kk, whist, kstar, k_rem);
#pragma unroll
      for (int t = 0; t < CAP / 64; ++t) eq_cnt += key[t] == kstar;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) eq_cnt += __shfl_xor(eq_cnt, o, 64);
    }
    // keep flags; ties at kstar: keep the k_rem smallest indices (O(T^2), rare)
    bool keep[CAP / 64];
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) {
      keep[t] = key[t] != 0u && (all || key[t] > kstar);
      if (!all && key[t] == kstar) {
        if (eq_cnt == k_rem) {
          keep[t] = true;
        } else {
          // rank among equal keys by index: count equal entries with smaller index
          const uint32_t my = ix[t] & ~VERIFIED;
          int smaller = 0;
          for (int j = 0; j < n; ++j) {
            const uint32_t oj = ci[qq * CAP + j];
            // equal keys only; already-dropped invalid ones never equal a valid key
            // because they may carry the same score: re-check via the key array is
            // not possible across lanes, so compare scores + verified-valid status
            if (ord_key(cs[qq * CAP + j]) == kstar && (oj & ~VERIFIED) < my) {
              const int64_t li = (int64_t)(oj & ~VERIFIED);
              const int64_t id = a.item_ids ? a.item_ids[li] : a.index_base + li;
              if (!(a.N0 > 0 && sorted_contains(qinv, a.N0, id))) ++smaller;
            }
          }
          keep[t] = smaller < k_rem;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    // write back compacted (wave-ordered), all reads above are done
    int base = 0;
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) {
      const unsigned long long bal = __ballot(keep[t]);
      const int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
      if (keep[t]) {
        cs[qq * CAP + pos] = sc[t];
        ci[qq * CAP + pos] = ix[t];
      }
      base += __popcll(bal);
    }
    if (lane == 0) {
      cnt[qq] = base;
      tau_s[qq] = all ? -INFINITY : key_to_float(kstar);
    }
  };

  // Double-buffered register prefetch (two named buffers: static indexing only).
  // Loads are unconditional (block index clamped into the table): a guarded load
  // would make hipcc branch around it and wait vmcnt(0) per element.
  const int64_t last_blk = (a.X + 15) / 16 - 1;
  fv2 fa[BLOCKS][KS2], fb[BLOCKS][KS2];
  auto load_step = [&](fv2 (&f)[BLOCKS][KS2], int step) {
    const int64_t xb = x_begin + ((int64_t)step * SW + w) * STEP;
#pragma unroll
    for (int bb = 0; bb < BLOCKS; ++bb) {
      int64_t ib = (xb >> 4) + bb;
      ib = ib > last_blk ? last_blk : ib;
      gptr<fv2> src = pk + ib * KS2 * 64 + lane;
#pragma unroll
      for (int j = 0; j < KS2; ++j) f[bb][j] = src[j * 64];
    }
  };
  auto process = [&](const fv2 (&f)[BLOCKS][KS2], int step) {
    const float tau = tau_s[lr];
    const int64_t xb = x_begin + ((int64_t)step * SW + w) * STEP;
    f4 s[BLOCKS];
#pragma unroll
    for (int bb = 0; bb < BLOCKS; ++bb) s[bb] = f4_zero();
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int bb = 0; bb < BLOCKS; ++bb)
        s[bb] = mfma16x16x4((st & 1) ? f[bb][st >> 1].y : f[bb][st >> 1].x, qreg[st], s[bb]);
#pragma unroll
    for (int bb = 0; bb < BLOCKS; ++bb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t item = xb + bb * 16 + 4 * lg + r;
        if (item < x_end && s[bb][r] > tau) {
          const int slot = atomicAdd(&cnt[lr], 1);
          cs[lr * CAP + slot] = s[bb][r];
          ci[lr * CAP + slot] = (uint32_t)item;  // local index
        }
      }
    }
    lds_barrier();
    if (w == 0) {
      const bool fl = lane < QG && cnt[lane] > CAP - SW * STEP;
      const unsigned long long bal = __ballot(fl);
      if (lane == 0) need_compact = bal != 0ull;
    }
    lds_barrier();
    if (need_compact) {
      for (int qq = w; qq < QG; qq += SW)
        if (cnt[qq] > a.k) compact(qq, a.k);
      lds_barrier();
    }
  };

  // prefetches past the last step re-load the last step (harmless; keeps the loads
  // unconditional so the waitcnt pass can count them)
  const int last_step = n_steps > 0 ? n_steps - 1 : 0;
  load_step(fa, 0);
  for (int step = 0; step < n_steps; step += 2) {
    load_step(fb, min(step + 1, last_step));
    process(fa, step);
    if (step + 1 >= n_steps) break;
    load_step(fa, min(step + 2, last_step));
    process(fb, step + 1);
  }
  // ---- final: this range's candidates per query (exact top-k_part, invalid removed;
  // when at most k_part remain this is only the invalid-id filter: the merge selects)
  __syncthreads();
  for (int qq = w; qq < QG; qq += SW) {
    if (q0 + qq >= a.B) continue;
    compact(qq, a.k_part);
  }
  __syncthreads();
  for (int e = tid; e < QG * a.k_part; e += ST) {
    const int qq = e / a.k_part, j = e - qq * a.k_part;
    if (q0 + qq >= a.B) continue;
    const int64_t o = ((int64_t)range * a.B + q0 + qq) * a.k_part + j;
    if (j < cnt[qq]) {
      a.part_score[o] = cs[qq * CAP + j];
      a.part_index[o] = a.index_base + (int64_t)(ci[qq * CAP + j] & ~VERIFIED);
    } else {
      a.part_score[o] = -INFINITY;
      a.part_index[o] = -1;
    }
  }
}

// Units blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8: a workgroup's units stay
// on its XCD).  The gated fallback launches at most two workgroups per CU, so the common
// case (flag clear) costs one small grid that exits at once instead of every unit's
// workgroup being dispatched to read the flag.
template <int KS, int BLOCKS>
__global__ __launch_bounds__(ST) void mips_select_kernel(SelectArgs a, int n_units) {
  if (a.gate && *a.gate == 0) return;
  for (int bid = blockIdx.x; bid < n_units; bid += gridDim.x) {
    mips_select_unit<KS, BLOCKS>(a, bid);
    __syncthreads();  // the next unit rewrites the LDS lists
  }
}

// ----------------------------------------------------------------- phase 2: merge
struct MergeArgs {
  const float* cand_score;    // [n_lists][B][k_in]
  const int64_t* cand_index;  // [n_lists][B][k_in], -1 = empty
  const int64_t* cand_ids;    // same shape or null
  int n_lists, B, k_in, k;
  const int64_t* item_ids;    // resolve ids when cand_ids == null
  int64_t index_base;
  float* out_score;
  int64_t* out_ids;
  int64_t* out_index;
  const int* gate;            // non-null: run only when *gate != 0
};

constexpr int MERGE_MAX = 8192;

// Block-level digit search over a 256-bin histogram (wave 0): the digit d such that
// count(digit > d) < need <= count(digit >= d); returns (d, count above d).
__device__ __forceinline__ void hist_find_digit(const int* hist, int need, int* out_digit,
                                                int* out_above) {
  const int lane = threadIdx.x & 63;
  int c[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = hist[255 - 4 * lane - j];
    s += c[j];
  }
  int incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  const int excl = incl - s;
  if (excl < need && incl >= need) {
    int run = excl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (run + c[j] >= need) {
        *out_digit = 255 - 4 * lane - j;
        *out_above = run;
        break;
      }
      run += c[j];
    }
  }
}

// Shared LDS state of the block-level exact selection (merge kernels).
struct SelLDS {
  int hist[256];
  int digit, above, cnt;
  int red[4];
  uint32_t s_key[256];
  int64_t s_idx[256];
  int s_src[256];
  uint32_t part[2][4][2];  // ballot counts per wave, two phases
};

// k-th largest nonzero key of key[0..M) (256 threads): a threshold search over the keys,
// 2 bits per step -- three candidate thresholds, each counted by wave ballots (SALU
// popcounts, no atomics), one barrier per step.  (An 8-bit radix histogram put every key
// of a query into the few bins its scores share: LDS atomics serialised on them.)
template <int PER>
__device__ void ballot_kth(const uint32_t* key, int M, int kk, SelLDS& L, uint32_t& kstar,
                           int& k_rem) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t kr[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int e = tid + 256 * t;
    kr[t] = e < M ? key[e] : 0u;
  }
  int ph = 0;
  uint32_t T = 0u;
  for (int b = 30; b >= 0; b -= 2) {
    const uint32_t c1 = T | (1u << b), c2 = T | (2u << b), c3 = T | (3u << b);
    uint32_t n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      n1 += __popcll(__ballot(kr[t] >= c1));
      n2 += __popcll(__ballot(kr[t] >= c2));
      n3 += __popcll(__ballot(kr[t] >= c3));
    }
    if (lane == 0) {
      L.part[ph][wv][0] = n1 | (n2 << 16);
      L.part[ph][wv][1] = n3;
    }
    __syncthreads();
    uint32_t t12 = 0, t3 = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      t12 += L.part[ph][w][0];
      t3 += L.part[ph][w][1];
    }
    ph ^= 1;
    T = (int)t3 >= kk ? c3 : (int)(t12 >> 16) >= kk ? c2 : (int)(t12 & 0xFFFF) >= kk ? c1 : T;
  }
  uint32_t gt = 0;
#pragma unroll
  for (int t = 0; t < PER; ++t) gt += __popcll(__ballot(kr[t] > T));
  if (lane == 0) L.part[ph][wv][0] = gt;
  __syncthreads();
  uint32_t g = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) g += L.part[ph][w][0];
  __syncthreads();  // L.part is free again for the caller's next selection
  kstar = T;
  k_rem = kk - (int)g;
}

// k-th largest nonzero key of key[0..M), M <= MERGE_MAX (= 32 keys per thread), k <= 8192
__device__ void block_kth(const uint32_t* key, int M, int kk, SelLDS& L, uint32_t& kstar,
                                int& k_rem) {
  if (M <= 1024) ballot_kth<4>(key, M, kk, L, kstar, k_rem);
  else if (M <= 2048) ballot_kth<8>(key, M, kk, L, kstar, k_rem);
  else if (M <= 4096) ballot_kth<16>(key, M, kk, L, kstar, k_rem);
  else ballot_kth<32>(key, M, kk, L, kstar, k_rem);
}

__device__ __forceinline__ int block_sum(int v, SelLDS& L) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) L.red[threadIdx.x >> 6] = v;
  __syncthreads();
  return L.red[0] + L.red[1] + L.red[2] + L.red[3];
}

// The kk (<= 256) largest nonzero keys of key[0..M) (tot = their count), ties at the
// k-th key broken by the smaller idx, sorted (key desc, idx asc) into L.s_key / s_idx /
// s_src (source position); returns how many were taken.
__device__ int block_topk_sorted(const uint32_t* key, const int64_t* idx, int M, int kk, int tot,
                                 SelLDS& L) {
  const int tid = threadIdx.x;
  uint32_t kstar = 0u;
  int k_rem = 0;
  const bool all = tot <= kk;
  if (!all) block_kth(key, M, kk, L, kstar, k_rem);
  // ties at kstar: count them; if more than k_rem, keep the smallest indices
  int eq = 0;
  if (!all)
    for (int e = tid; e < M; e += 256) eq += key[e] == kstar;
  const int eq_tot = block_sum(eq, L);
  if (tid == 0) L.cnt = 0;
  __syncthreads();
  for (int e = tid; e < M; e += 256) {
    const uint32_t x = key[e];
    if (x == 0u) continue;
    bool take = all || x > kstar;
    if (!all && x == kstar) {
      if (eq_tot == k_rem) {
        take = true;
      } else {
        const int64_t my = idx[e];
        int smaller = 0;
        for (int f = 0; f < M; ++f) smaller += (key[f] == kstar && idx[f] < my);
        take = smaller < k_rem;
      }
    }
    if (take) {
      const int p = atomicAdd(&L.cnt, 1);
      L.s_key[p] = x;
      L.s_idx[p] = idx[e];
      L.s_src[p] = e;
    }
  }
  __syncthreads();
  const int n = L.cnt;
  for (int p = n + tid; p < 256; p += 256) {
    L.s_key[p] = 0u;
    L.s_idx[p] = INT64_MAX;
    L.s_src[p] = -1;
  }
  __syncthreads();
  // bitonic sort of the 256 entries, one per thread: key desc, then catalog index asc.
  // Strides < 64 exchange inside the wave by lane shuffles (no barrier: 33 of the 36
  // stages); strides 64 and 128 go through LDS.
  uint32_t k = L.s_key[tid];
  int64_t ix = L.s_idx[tid];
  int sr = L.s_src[tid];
  __syncthreads();
  for (int size = 2; size <= 256; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      uint32_t ko;
      int64_t io;
      int so;
      if (stride >= 64) {
        L.s_key[tid] = k;
        L.s_idx[tid] = ix;
        L.s_src[tid] = sr;
        __syncthreads();
        ko = L.s_key[tid ^ stride];
        io = L.s_idx[tid ^ stride];
        so = L.s_src[tid ^ stride];
        __syncthreads();
      } else {
        ko = (uint32_t)__shfl_xor((int)k, stride, 64);
        io = (int64_t)__shfl_xor((long long)ix, stride, 64);
        so = __shfl_xor(sr, stride, 64);
      }
      // the pair's lower position keeps the first element when the run ascends
      const bool me_first = (k > ko) || (k == ko && ix < io);
      const bool want_first = ((tid & stride) == 0) == ((tid & size) == 0);
      if (me_first != want_first) {
        k = ko;
        ix = io;
        sr = so;
      }
    }
  }
  L.s_key[tid] = k;
  L.s_idx[tid] = ix;
  L.s_src[tid] = sr;
  __syncthreads();
  return n;
}

// Ascending sort of v[0 .. n) in LDS, n in {64, 128, 256}, by the 256 threads of the
// block (thread t < n holds v[t]; the others only join the barriers): strides < 64 by
// lane shuffles, 64 and 128 through v.
__device__ void block_sort_i64_asc(int64_t* v, int n) {
  const int tid = threadIdx.x;
  int64_t x = tid < n ? v[tid] : INT64_MAX;
  __syncthreads();
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      int64_t o;
      if (stride >= 64) {
        if (tid < n) v[tid] = x;
        __syncthreads();
        o = tid < n ? v[tid ^ stride] : INT64_MAX;
        __syncthreads();
      } else {
        o = (int64_t)__shfl_xor((long long)x, stride, 64);
      }
      const bool want_small = ((tid & stride) == 0) == ((tid & size) == 0);
      x = want_small ? (x < o ? x : o) : (x < o ? o : x);
    }
  }
  if (tid < n) v[tid] = x;
  __syncthreads();
}

__global__ __launch_bounds__(256) void mips_merge_kernel(MergeArgs a) {
  if (a.gate && *a.gate == 0) return;  // fallback merge: only when the filter path failed
  __shared__ uint32_t key[MERGE_MAX];
  __shared__ int64_t idx[MERGE_MAX];
  __shared__ SelLDS L;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int M = a.n_lists * a.k_in;
  auto src_of = [&](int e) -> int64_t {
    const int l = e / a.k_in, j = e - l * a.k_in;
    return ((int64_t)l * a.B + q) * a.k_in + j;
  };
  int nvalid = 0;
  // batches of 8 elements per thread with all loads issued first (a plain strided loop
  // waited for each element's loads in turn)
  constexpr int PB = 8;
  for (int e0 = tid; e0 < M; e0 += 256 * PB) {
    int64_t gv[PB];
    float sv[PB];
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      const int e = e0 + 256 * t;
      const int64_t s = src_of(e < M ? e : M - 1);
      gv[t] = a.cand_index[s];
      sv[t] = a.cand_score[s];
    }
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      const int e = e0 + 256 * t;
      if (e < M) {
        const bool ok = gv[t] >= 0;
        key[e] = ok ? ord_key(sv[t]) : 0u;
        idx[e] = ok ? gv[t] : INT64_MAX;
        nvalid += ok;
      }
    }
  }
  const int tot = block_sum(nvalid, L);
  const int kk = a.k;
  const int n = block_topk_sorted(key, idx, M, kk, tot, L);
  for (int r = tid; r < kk; r += 256) {
    const int64_t o = (int64_t)q * kk + r;
    if (r < n) {
      const int64_t s = src_of(L.s_src[r]);
      const int64_t gi = L.s_idx[r];
      a.out_score[o] = a.cand_score[s];
      if (a.out_index) a.out_index[o] = gi;
      int64_t id;
      if (a.cand_ids) id = a.cand_ids[s];
      else id = a.item_ids ? a.item_ids[gi - a.index_base] : gi;
      a.out_ids[o] = id;
    } else {
      a.out_score[o] = -INFINITY;
      if (a.out_index) a.out_index[o] = -1;
      a.out_ids[o] = -1;
    }
  }
}

// ----------------------------------------------------------------- small catalogs
// X <= MERGE_MAX: workgroup (query, chunk) scores one chunk of the items (the same
// k-ordered fmaf chain, read from the packed layout), excludes its invalid ids (arange
// ids: direct index scatter after the scores are written; explicit ids: binary search in
// the sorted list) and writes the scores into the query's one candidate list for the
// merge kernel.  Replaces the range/threshold machinery, whose fixed per-workgroup costs
// dominate at ml-1m sizes.  Chunks (blockIdx.y) spread a query over several CUs: with
// one workgroup per query the 128 queries of a batch left half the chip idle and each
// thread walked 16 items serially (22 us at ml-1m).
struct ScoreAllArgs {
  const float* q;
  const float* packed;
  int64_t X;
  int D, B, N0;
  const int64_t* item_ids;
  int64_t index_base;
  const int64_t* invalid;
  float* out_score;    // [B][X]
  int64_t* out_index;  // [B][X], -1 = excluded
  int64_t chunk;       // items per workgroup (blockIdx.y = chunk index)
};

// Explicit ids with N0 > 0: the query's sorted invalid list in n0p * 8 B of dynamic LDS.
template <int KS2>
__global__ __launch_bounds__(256) void mips_scoreall_kernel(ScoreAllArgs a) {
  __shared__ float qv[8 * KS2];
  extern __shared__ int64_t inv[];
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int d = tid; d < 8 * KS2; d += 256) qv[d] = d < a.D ? a.q[(int64_t)q * a.D + d] : 0.f;
  const bool search = a.item_ids && a.N0 > 0;
  const int n0p = inv_pad(a.N0);
  if (search) {
    for (int j = tid; j < n0p; j += 256) inv[j] = j < a.N0 ? a.invalid[(int64_t)q * a.N0 + j] : INT64_MAX;
    __syncthreads();
    block_bitonic_i64(inv, n0p);
  }
  __syncthreads();
  typedef float fv2 __attribute__((ext_vector_type(2)));
  gptr<fv2> pk = as_global(reinterpret_cast<const fv2*>(a.packed));
  float* os = a.out_score + (int64_t)q * a.X;
  int64_t* oi = a.out_index + (int64_t)q * a.X;
  const int64_t lo = (int64_t)blockIdx.y * a.chunk;
  const int64_t hi = lo + a.chunk < a.X ? lo + a.chunk : a.X;
  for (int64_t i = lo + tid; i < hi; i += 256) {
    const int64_t ib = i >> 4;
    const int il = (int)(i & 15);
    float e[8 * KS2];
#pragma unroll
    for (int j = 0; j < KS2; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const fv2 v = pk[(ib * KS2 + j) * 64 + 16 * c + il];
        e[8 * j + c] = v.x;      // d = 8j + c      (k-step 2j)
        e[8 * j + 4 + c] = v.y;  // d = 8j + 4 + c  (k-step 2j + 1)
      }
    float sc = 0.f;
#pragma unroll
    for (int d = 0; d < 8 * KS2; ++d) sc = fmaf(qv[d], e[d], sc);  // padding adds +0 exactly
    bool ok = true;
    if (search) ok = !sorted_contains(inv, n0p, a.item_ids[i]);
    os[i] = ok ? sc : -INFINITY;
    oi[i] = ok ? a.index_base + i : -1;
  }
  if (!a.item_ids && a.N0 > 0) {  // arange ids: exclude by direct index
    __syncthreads();
    for (int j = tid; j < a.N0; j += 256) {
      const int64_t li = a.invalid[(int64_t)q * a.N0 + j] - a.index_base;
      if (li >= lo && li < hi) {
        os[li] = -INFINITY;
        oi[li] = -1;
      }
    }
  }
}

// ----------------------------------------------------------------- small-catalog selection
// The merge of the score-all lists (X <= MERGE_MAX, k <= 256): one workgroup of 1024
// threads per query, a thread holding 8 consecutive items' keys in registers:
//   1. the k-th largest key T by a threshold search, 2 bits per step: three candidate
//      thresholds per step, their counts packed into one 64-bit block sum -- no
//      histogram atomics (the radix merge's first digit passes put a query's scores into
//      a few bins and serialised on them: 31 us per batch at ml-1m);
//   2. winners = keys > T plus the first k - count(> T) keys == T in index order (one
//      block scan), compacted in index order, then each written at its rank in
//      (score desc, index asc) order by counting (<= 256 entries, LDS broadcast reads).
// Same order and outputs as mips_merge_kernel over the one list (bit-identical).
struct SmallArgs {
  const float* score;    // [B][X] (score-all output)
  const int64_t* index;  // [B][X], -1 = excluded
  int X, k;
  const int64_t* item_ids;
  int64_t index_base;
  float* out_score;
  int64_t* out_ids;
  int64_t* out_index;
};
constexpr int SM_T = 1024;                // threads
constexpr int SM_PER = MERGE_MAX / SM_T;  // consecutive items per thread
static_assert(SM_PER == 8, "two 16-byte score loads per thread");

// Block totals of per-lane predicates by wave ballots (no lane shuffles): each wave's
// counts land in one LDS slot, one barrier, every thread sums the 16 slots.  Two phase
// buffers, so a buffer is rewritten only after the barrier that follows every read of it.
__device__ __forceinline__ int wave_count(bool p) { return __popcll(__ballot(p)); }

__global__ __launch_bounds__(1024) void mips_small_select_kernel(SmallArgs a) {
  __shared__ float sc[MERGE_MAX];
  __shared__ __attribute__((aligned(16))) uint32_t part[2][SM_T / 64][2];
  __shared__ uint32_t wgt[SM_T / 64], weq[SM_T / 64];
  __shared__ __attribute__((aligned(16))) uint32_t s_key[256];
  __shared__ __attribute__((aligned(16))) int s_idx[256];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int X = a.X, i0 = SM_PER * tid;
  typedef float fv4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef int i4 __attribute__((ext_vector_type(4)));
  uint32_t kr[SM_PER];
  {
    const float* srow = a.score + (int64_t)q * X;
    const int64_t* irow = a.index + (int64_t)q * X;
    float v[SM_PER];
    int64_t ix[SM_PER];
    if (i0 + SM_PER <= X && (X & 3) == 0) {  // rows 16-byte aligned
      const fv4 v0 = *reinterpret_cast<const fv4*>(srow + i0);
      const fv4 v1 = *reinterpret_cast<const fv4*>(srow + i0 + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
      v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
#pragma unroll
      for (int e = 0; e < SM_PER; ++e) ix[e] = irow[i0 + e];
    } else {
#pragma unroll
      for (int e = 0; e < SM_PER; ++e) {
        const bool in = i0 + e < X;
        v[e] = in ? srow[i0 + e] : 0.f;
        ix[e] = in ? irow[i0 + e] : -1;
      }
    }
#pragma unroll
    for (int e = 0; e < SM_PER; ++e) {
      kr[e] = ix[e] >= 0 ? ord_key(v[e]) : 0u;
      if (i0 + e < X) sc[i0 + e] = v[e];
    }
  }
  int ph = 0;
  // block totals of two wave-uniform counts (each <= 8192: 16 bits)
  auto block_sum2 = [&](uint32_t c0, uint32_t c1, uint32_t& t0, uint32_t& t1) {
    if (lane == 0) {
      part[ph][wv][0] = c0;
      part[ph][wv][1] = c1;
    }
    __syncthreads();
    t0 = t1 = 0u;
#pragma unroll
    for (int w = 0; w < SM_T / 64; w += 2) {
      const u4 x = *reinterpret_cast<const u4*>(&part[ph][w][0]);
      t0 += x.x + x.z;
      t1 += x.y + x.w;
    }
    ph ^= 1;
  };
  uint32_t nz = 0;
#pragma unroll
  for (int e = 0; e < SM_PER; ++e) nz += wave_count(kr[e] != 0u);
  uint32_t tot_u, unused;
  block_sum2(nz, 0u, tot_u, unused);
  const int tot = (int)tot_u;
  const int kk = a.k;
  uint32_t T = 1u;  // every nonzero key when tot <= k
  int k_rem = SM_T * SM_PER;
  if (tot > kk) {
    T = 0u;
    for (int b = 30; b >= 0; b -= 2) {
      const uint32_t c1 = T | (1u << b), c2 = T | (2u << b), c3 = T | (3u << b);
      uint32_t n1 = 0, n2 = 0, n3 = 0;
#pragma unroll
      for (int e = 0; e < SM_PER; ++e) {
        n1 += wave_count(kr[e] >= c1);
        n2 += wave_count(kr[e] >= c2);
        n3 += wave_count(kr[e] >= c3);
      }
      uint32_t t12, t3;
      block_sum2(n1 | (n2 << 16), n3, t12, t3);
      T = (int)t3 >= kk ? c3 : (int)(t12 >> 16) >= kk ? c2 : (int)(t12 & 0xFFFF) >= kk ? c1 : T;
    }
    uint32_t gt = 0;
#pragma unroll
    for (int e = 0; e < SM_PER; ++e) gt += wave_count(kr[e] > T);
    uint32_t gt_tot;
    block_sum2(gt, 0u, gt_tot, unused);
    k_rem = kk - (int)gt_tot;
  }
  // winners in index order: the (count > T, count == T) of the items before a thread's
  // own, from the ballots (lanes below in the wave) plus the waves below
  uint32_t gt_l = 0, eq_l = 0, gt_w = 0, eq_w = 0;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (int e = 0; e < SM_PER; ++e) {
    const uint64_t mg = __ballot(kr[e] > T), me = __ballot(kr[e] == T);
    gt_l += __popcll(mg & below);
    eq_l += __popcll(me & below);
    gt_w += __popcll(mg);
    eq_w += __popcll(me);
  }
  if (lane == 0) {
    wgt[wv] = gt_w;
    weq[wv] = eq_w;
  }
  __syncthreads();
  for (int w = 0; w < wv; ++w) {
    gt_l += wgt[w];
    eq_l += weq[w];
  }
  int gt_b = (int)gt_l, eq_b = (int)eq_l;
#pragma unroll
  for (int e = 0; e < SM_PER; ++e) {
    const uint32_t x = kr[e];
    if (x == 0u) continue;
    int pos = -1;
    if (x > T) {
      pos = gt_b + (eq_b < k_rem ? eq_b : k_rem);
      ++gt_b;
    } else if (x == T) {
      if (eq_b < k_rem) pos = gt_b + eq_b;
      ++eq_b;
    }
    if (pos >= 0) {
      s_key[pos] = x;
      s_idx[pos] = i0 + e;
    }
  }
  const int n_sel = tot < kk ? tot : kk;
  for (int p = n_sel + tid; p < 256; p += SM_T) {  // padding: sorts after every winner
    s_key[p] = 0u;
    s_idx[p] = 0x7fffffff;
  }
  __syncthreads();
  // rank of each winner in (key desc, index asc) order: 16-byte broadcast reads
  if (tid < n_sel) {
    const uint32_t x = s_key[tid];
    const int ix = s_idx[tid];
    int r = 0;
    const int nq = (n_sel + 3) >> 2;
#pragma unroll 4
    for (int f = 0; f < nq; ++f) {
      const u4 y = *reinterpret_cast<const u4*>(&s_key[4 * f]);
      const i4 z = *reinterpret_cast<const i4*>(&s_idx[4 * f]);
      r += (y.x > x) | ((y.x == x) & (z.x < ix));
      r += (y.y > x) | ((y.y == x) & (z.y < ix));
      r += (y.z > x) | ((y.z == x) & (z.z < ix));
      r += (y.w > x) | ((y.w == x) & (z.w < ix));
    }
    const int64_t o = (int64_t)q * kk + r;
    const int64_t gi = a.index_base + ix;
    a.out_score[o] = sc[ix];
    if (a.out_index) a.out_index[o] = gi;
    a.out_ids[o] = a.item_ids ? a.item_ids[ix] : gi;
  } else if (tid < kk) {
    const int64_t o = (int64_t)q * kk + tid;
    a.out_score[o] = -INFINITY;
    if (a.out_index) a.out_index[o] = -1;
    a.out_ids[o] = -1;
  }
}

// ----------------------------------------------------------------- large catalogs
// Threshold-filter path (D <= 64, X >= FILTER_MIN_X).  The 16-query-per-workgroup
// select above re-reads the table once per query group (8x at B = 128) and keeps
// per-query candidate buffers in LDS; here every workgroup scores ALL queries of its
// chunk (up to 128, fragments held in VGPRs) against each item block it loads, so the
// table streams from HBM once and the MFMA pipe is the bound.  The per-query selection
// state becomes one threshold tau_q, fixed before the pass:
//   1. sample:  score every SR-th item block; each workgroup reduces its group of
//      sample blocks (a few per wave) to one max per query -> smax[q][g] (G groups =
//      the sample workgroups; a group per wave made the tau kernel's selection 4x wider).
//   2. tau:     tau_q = the M-th largest of the G group maxima (M = 1024 / SR).  Those
//      maxima are real catalog items, so >= M items score >= tau_q, and (1/SR
//      sampled) about M * SR = 1024 do.
//   3. filter:  full pass; scores >= tau_q are appended (global atomics; ~1e-4 of
//      scores) to a per-query list of FILTER_CAP.
//   4. merge:   per query, drop invalid ids, exact top-k (threshold select + sort).  Every
//      uncollected item scores < tau_q <= every collected one, so the result is exact
//      whenever the list did not overflow and kept >= k valid items.  Otherwise the
//      merge raises a device flag and the exact select + merge kernels above (gated on
//      that flag, no host sync) recompute every query.
constexpr int SAMPLE_STRIDE = 32;       // sample every 32nd item block (10M items: sample
                                        // 26.0 us at 16, 14.0 at 32, 10.7 at 64 but merge +4.5)
constexpr int SAMPLE_WAVES = 4096;      // target number of sample waves (4 per group)
constexpr int SAMPLE_CAND = 1024;       // M = SAMPLE_CAND / stride: ~1024 candidates per query
constexpr int SAMPLE_GB = 10;           // sample blocks per wave (when G stays >= 4 M)
constexpr int FILTER_CAP = 4096;        // candidate list per query
constexpr int NSUB = 16;                // ... split into sub-lists by workgroup (blockIdx % 16)
constexpr int SUBCAP = FILTER_CAP / NSUB;  // so each counter sees 1/16 of the atomics
constexpr int64_t FILTER_MIN_X = (int64_t)16 * 16 * 1024;  // >= 1024 blocks at a 16-block stride

struct FilterArgs {
  const float* q;
  const float* packed;
  const u32x4* packed16;  // bf16 copy (KC > 0 instantiations)
  int BB, LG;             // its block bytes and stored lane groups of the last chunk
  int TD;                 // tail dims (0, 1, 2): lane group LG of the last chunk reads the tail
  int64_t X;
  int D, B;
  int64_t n_blocks;
  // sample pass
  int GB, G;          // sample blocks per wave, groups (= sample workgroups)
  int sr;             // sample stride (item blocks)
  float* smax;        // [B][G]
  // filter pass
  int64_t RB;         // item blocks per wave
  const float* tau;   // [B]
  int* cnt;           // [B][NSUB]
  float* cand_s;      // [B][NSUB][SUBCAP]
  int* cand_i;        // [B][NSUB][SUBCAP]  local item index
  int* flag;          // set when a workgroup's staging buffer overflows
  int nohit;          // GR_OPT_MIPS_FORCE_FALLBACK: thresholds +inf
  // bf16 filter: hits are rescored exactly at flush time from row-major f32 copies
  const float* rows;    // items, DP floats per row
  const float* q_rows;  // queries, DP floats per row (workspace)
  int DP;
  // filter pass with several query chunks: a 1-D grid whose workgroups 8 apart (one XCD
  // under the round-robin placement) take the chunks of one item range in turn, so the
  // range streams from HBM once and the other chunks read it from that XCD's L2
  int nch;   // query chunks (0: the 2-D grid, blockIdx.y = chunk)
  int gx;    // workgroups per chunk
};

constexpr int WG_CAP = 2048;  // per-workgroup LDS staging of filter hits (~450 expected at 10M)
constexpr int WV_CAP = WG_CAP / 4;  // per-wave segment

// KC == 0: f32 table (KS k-steps of 16x16x4); KC > 0: the bf16 copy (KC k-chunks of
// 16x16x32), scores approximate to within the bound the tau kernel folds into tau.
template <int KS, int KC, int NQG, bool SAMPLE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KC >= 1 && KC <= 2 ? 3 : 1)))
void mips_filter_kernel(FilterArgs a) {
  constexpr int KS2 = (KS + 1) / 2;
  constexpr bool BF = KC > 0;
  typedef float fv2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  int bx = blockIdx.x, by = blockIdx.y;
  if (!SAMPLE && a.nch > 1) {
    const int xcd = bx & 7, slot = bx >> 3;
    by = slot % a.nch;
    bx = (slot / a.nch) * 8 + xcd;
    if (bx >= a.gx) return;
  }
  const int64_t wv = (int64_t)bx * 4 + wave_id();
  const int qb = by * (NQG * 16);

  int64_t b0 = 0, b1 = 0, bstride;
  if (SAMPLE) {
    const int64_t n_sb = (a.n_blocks + a.sr - 1) / a.sr;
    const int64_t s0 = wv * a.GB, s1 = min(n_sb, s0 + a.GB);
    if (s0 < n_sb) {
      b0 = s0 * a.sr;
      b1 = s1 * a.sr;
    }
    bstride = a.sr;
  } else {
    b0 = wv * a.RB;
    b1 = min(a.n_blocks, b0 + a.RB);
    bstride = 1;
  }
  __shared__ float l_s[SAMPLE ? 1 : WG_CAP];
  __shared__ int l_i[SAMPLE ? 1 : WG_CAP];
  __shared__ uint8_t l_q[SAMPLE ? 1 : WG_CAP];
  __shared__ int l_wn[4];
  const int w_base = wave_id() * WV_CAP;
  int w_n = 0;  // wave-uniform hit count of this wave's segment
  // The chunk's query fragments, staged once per workgroup with coalesced row reads
  // (every wave of the grid loading its own fragments hammers the L2 lines of the
  // same 25 KB query block: ~90 us of contention at launch), in MFMA B-operand order
  // so each wave's reads are conflict-free: frag[(g KS + st) 64 + lr + 16 lg] =
  // Q[qb + 16 g + lr][4 st + lg].
  // (bf16: frag16[(g KC + c) 64 + lr + 16 lg] = bf16(Q[qb + 16 g + lr][32 c + 8 lg + 0..7]))
  // Wide bf16 rows (KC > 2) with 8 query groups: groups 0..3 live in VGPRs, 4..7 are read
  // from LDS per block (all 128 queries of a batch in one pass over the table; 8 groups in
  // VGPRs would not fit beside the block prefetch)
  constexpr int NQR = (BF && NQG == 8 && KC > 2) ? (SAMPLE ? 2 : 3) : NQG;  // query groups in VGPRs
  constexpr int NQL = NQG - NQR;                             // query groups read from LDS
  constexpr int NQS = NQR > NQL ? NQR : NQL;                 // groups staged at a time
  __shared__ float q_lds[BF ? 1 : NQG * KS * 64];
  __shared__ u32x4 q16_lds[BF ? NQS * KC * 64 : 1];
  __shared__ float tau_lds[NQG * 16];
  u32x4 qreg16[NQR][BF ? KC : 1];
  float qreg[NQG][BF ? 1 : KS];
  {
    const int rows = NQG * 16;
    if constexpr (BF) {
      auto stage = [&](int g0, int ng) {
        for (int e = threadIdx.x; e < ng * 16 * KC * 4; e += 256) {
          const int r = e / (KC * 4), u = e - r * (KC * 4);
          const int qq = qb + 16 * g0 + r, d0 = 32 * (u >> 2) + 8 * (u & 3);
          uint32_t w[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int d = d0 + 2 * h;
            const float v0 = (qq < a.B && d < a.D) ? a.q[(int64_t)qq * a.D + d] : 0.f;
            const float v1 = (qq < a.B && d + 1 < a.D) ? a.q[(int64_t)qq * a.D + d + 1] : 0.f;
            w[h] = bf16_bits(v0) | (bf16_bits(v1) << 16);
          }
          q16_lds[((r >> 4) * KC + (u >> 2)) * 64 + (r & 15) + 16 * (u & 3)] = u32x4{w[0], w[1], w[2], w[3]};
        }
      };
      stage(0, NQR);
      __syncthreads();
#pragma unroll
      for (int g = 0; g < NQR; ++g)
#pragma unroll
        for (int c = 0; c < KC; ++c) qreg16[g][c] = q16_lds[(g * KC + c) * 64 + lane];
      if constexpr (NQL > 0) {
        __syncthreads();
        stage(NQR, NQL);
      }
    } else {
      const int cols = 4 * KS;
      for (int e = threadIdx.x; e < rows * cols; e += 256) {
        const int r = e / cols, d = e - r * cols;
        const int qq = qb + r;
        const float v = (qq < a.B && d < a.D) ? a.q[(int64_t)qq * a.D + d] : 0.f;
        q_lds[((r >> 4) * KS + (d >> 2)) * 64 + (r & 15) + 16 * (d & 3)] = v;
      }
    }
    for (int r = threadIdx.x; r < rows; r += 256) {
      const int qq = qb + r;
      tau_lds[r] = SAMPLE ? -INFINITY : (qq < a.B && !a.nohit ? a.tau[qq] : INFINITY);
    }
    __syncthreads();
  }
  if constexpr (!BF) {
#pragma unroll
    for (int g = 0; g < NQG; ++g)
#pragma unroll
      for (int st = 0; st < KS; ++st) qreg[g][st] = q_lds[(g * KS + st) * 64 + lane];
  }
  float thr[NQG];  // filter: tau of query 16 g + lr (+inf for padded queries); sample: running max
#pragma unroll
  for (int g = 0; g < NQG; ++g) thr[g] = tau_lds[16 * g + lr];

  gptr<fv2> pk = as_global(reinterpret_cast<const fv2*>(a.packed));
  gptr<float> pk1 = as_global(a.packed);
  // An odd KS leaves the .y half of the last pair unused (zero padding): load only the
  // .x half, so no in-flight load targets a register the compiler considers dead (it
  // would reuse it as a temporary and wait vmcnt(0) on the prefetch).
  constexpr int NP = BF ? 0 : KS / 2;  // full pairs
  // bf16 copy: lanes of the last chunk's unstored lane groups read group 0's word
  const int last_lane = lg < a.LG ? lane : lr;
  struct Frag {
    fv2 p[NP > 0 ? NP : 1];
    float t;
    u32x4 h[BF ? KC : 1];
    uint32_t tw;  // bf16 tail: item lr's last dims (lane group LG of the last chunk)
  };
  // byte offset of item lr's tail u32 in a block (word 0 of the block without a tail)
  const int tail_off = a.TD ? (64 * (KC - 1) + 16 * a.LG) * 16 + 4 * lr : 0;
  const bool tail_lane = a.TD && lg == a.LG;
  Frag fa, fb;
  auto load = [&](Frag& f, int64_t ib) {
    ib = ib < b1 ? ib : b1 - bstride;  // clamped: loads stay unconditional
    if constexpr (BF) {
      gptr<u32x4> src = as_global(reinterpret_cast<const u32x4*>(
          reinterpret_cast<const char*>(a.packed16) + ib * a.BB));
      // the table streams once: non-temporal loads (10M items: filter 259 -> 233 us;
      // no-hit streaming 227 -> 202 us = 6.3 TB/s)
#pragma unroll
      for (int c = 0; c < KC; ++c)
        f.h[c] = __builtin_nontemporal_load(&src[c * 64 + (c == KC - 1 ? last_lane : lane)]);
      f.tw = __builtin_nontemporal_load(as_global(reinterpret_cast<const uint32_t*>(
          reinterpret_cast<const char*>(a.packed16) + ib * a.BB + tail_off)));
    } else {
      gptr<fv2> src = pk + ib * KS2 * 64 + lane;
#pragma unroll
      for (int j = 0; j < NP; ++j) f.p[j] = src[j * 64];
      if (KS & 1) f.t = pk1[((ib * KS2 + NP) * 64 + lane) * 2];
    }
  };
  auto process = [&](const Frag& f, int64_t ib) {
    f4 s[NQG];
#pragma unroll
    for (int g = 0; g < NQG; ++g) s[g] = f4_zero();
    // the last chunk's tail lanes: {tail, 0, 0, 0} (built here, at the use, so the select
    // does not wait on the prefetch)
    u32x4 hlast = f.h[KC > 0 ? KC - 1 : 0];
    if constexpr (BF) hlast = tail_lane ? u32x4{f.tw, 0u, 0u, 0u} : hlast;
    if constexpr (!BF) {
    } else if constexpr (NQL == 0) {
#pragma unroll
      for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int g = 0; g < NQG; ++g) s[g] = mfma16x16x32bf16(c == KC - 1 ? hlast : f.h[c], qreg16[g][c], s[g]);
    } else {
      // the LDS groups' fragments of chunk c + 1 are read while chunk c's MFMAs run (a
      // barrier per chunk keeps hipcc from hoisting every chunk's reads: 4x the registers)
      u32x4 ql[2][NQL > 0 ? NQL : 1];
#pragma unroll
      for (int g = 0; g < NQL; ++g) ql[0][g] = q16_lds[(g * KC) * 64 + lane];
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        if (c + 1 < KC) {
#pragma unroll
          for (int g = 0; g < NQL; ++g) ql[(c + 1) & 1][g] = q16_lds[(g * KC + c + 1) * 64 + lane];
        }
#pragma unroll
        for (int g = 0; g < NQR; ++g) s[g] = mfma16x16x32bf16(c == KC - 1 ? hlast : f.h[c], qreg16[g][c], s[g]);
#pragma unroll
        for (int g = 0; g < NQL; ++g)
          s[NQR + g] = mfma16x16x32bf16(c == KC - 1 ? hlast : f.h[c], ql[c & 1][g], s[NQR + g]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (!BF) {
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const float av = (st >> 1) < NP ? ((st & 1) ? f.p[st >> 1].y : f.p[st >> 1].x) : f.t;
#pragma unroll
        for (int g = 0; g < NQG; ++g) s[g] = mfma16x16x4(av, qreg[g][st], s[g]);
      }
    }
    const int64_t item0 = ib * 16 + 4 * lg;  // rows 4 lg + r of the block
    const bool full = ib * 16 + 16 <= a.X;   // wave-uniform
    if (SAMPLE) {
#pragma unroll
      for (int g = 0; g < NQG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          thr[g] = fmaxf(thr[g], (full || item0 + r < a.X) ? s[g][r] : -INFINITY);
    } else {
      // hits are rare (~1e-4 of scores): one wave-wide OR per block; a block with any
      // hit appends them to this wave's private LDS segment at positions from
      // ballots and a wave-uniform (scalar) counter: no atomics, no waits
      // screen: max over the 4 rows, minus the query's threshold, max over the query
      // groups, one compare (~30 VALU and one ballot per block instead of a compare and a
      // mask OR per score).  m - t >= 0 holds whenever m >= t (a flushed denormal
      // difference reads +-0: at worst a false positive, which the exact per-score test
      // below drops); +inf - +inf (a padded query's threshold) is NaN and never a hit
      float dmax = -INFINITY;
#pragma unroll
      for (int g = 0; g < NQG; ++g) {
        const float m = fmaxf(fmaxf(s[g][0], s[g][1]), fmaxf(s[g][2], s[g][3]));
        dmax = fmaxf(dmax, m - thr[g]);
      }
      const bool hit = dmax >= 0.f;
      if (__builtin_expect(__ballot(hit) != 0ull, 0) && ib < b1) {
#pragma unroll
        for (int g = 0; g < NQG; ++g) {
          bool hg = false;
#pragma unroll
          for (int r = 0; r < 4; ++r) hg |= s[g][r] >= thr[g];
          if (__ballot(hg) == 0ull) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool h = s[g][r] >= thr[g] && (full || item0 + r < a.X);
            const uint64_t bl = __ballot(h);
            if (bl) {
              const int p = w_n + __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0));
              if (h && p < WV_CAP) {
                l_s[w_base + p] = s[g][r];
                l_i[w_base + p] = (int)(item0 + r);
                l_q[w_base + p] = (uint8_t)(16 * g + lr);
              }
              w_n += __popcll(bl);
            }
          }
        }
      }
    }
  };

  if (SAMPLE && b0 < b1) {
    // a few sample blocks per wave at a 16-block stride: issue a chunk's loads
    // together, then score them (duplicated clamped blocks leave the max unchanged)
    constexpr int CH = KC <= 2 ? 4 : 2;
    for (int64_t ib = b0; ib < b1; ib += CH * bstride) {
      Frag f[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) load(f[c], ib + c * bstride);
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int64_t jb = ib + c * bstride;
        process(f[c], jb < b1 ? jb : b1 - bstride);
      }
    }
  } else if (!SAMPLE && b0 < b1 && BF) {
    // bf16 blocks are 1-2 KB of HBM per ~16 MFMAs: keep PD blocks in flight per wave
    // (a slot is refilled PD blocks ahead as soon as it is consumed)
    constexpr int PD = KC <= 2 ? 4 : 2;
    Frag f[PD];
    // issue order f[0], f[1], ... pinned (sched_barrier): the loop's waits count loads in
    // that order, and a reordered prologue made hipcc drain vmcnt(0) every iteration
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      load(f[u], b0 + u);
      __builtin_amdgcn_sched_barrier(0);
    }
    // whole rounds of PD blocks, no early exit inside (a branch there let the prologue's
    // and the loop's pending loads disagree, and hipcc drained vmcnt(0) per round);
    // blocks past b1 are clamped re-reads that process() ignores
    for (int64_t ib = b0; ib < b1; ib += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        process(f[u], ib + u);
        load(f[u], ib + u + PD);  // into the registers just consumed: no copies
      }
    }
  } else if (!SAMPLE && b0 < b1) {
    load(fa, b0);
    for (int64_t ib = b0; ib < b1; ib += 2 * bstride) {
      load(fb, ib + bstride);
      process(fa, ib);
      if (ib + bstride >= b1) break;
      load(fa, ib + 2 * bstride);
      process(fb, ib + bstride);
    }
  }
  if (!SAMPLE) {  // flush the workgroup's hits to the per-query lists
    if (lane == 0) l_wn[wave_id()] = w_n;
    __syncthreads();
    if (threadIdx.x == 0 && (l_wn[0] > WV_CAP || l_wn[1] > WV_CAP || l_wn[2] > WV_CAP ||
                             l_wn[3] > WV_CAP))
      atomicExch(a.flag, 1);  // a segment overflowed: the exact fallback recomputes
    for (int w = 0; w < 4; ++w) {
      const int n = l_wn[w] < WV_CAP ? l_wn[w] : WV_CAP;
      for (int e = threadIdx.x; e < n; e += 256) {
        const int src = w * WV_CAP + e;
        const int qq = qb + l_q[src];
        float sc = l_s[src];
        if constexpr (BF) {
          // exact f32 score of the hit: the k-ordered fmaf chain over d < D (the f32
          // MFMA's and the oracle's) from the row-major copy; the row's and the query's
          // float4 loads are issued together
          typedef float fv4 __attribute__((ext_vector_type(4)));
          gptr<fv4> xr = as_global(reinterpret_cast<const fv4*>(a.rows)) +
                         (int64_t)l_i[src] * (a.DP >> 2);
          gptr<fv4> qr = as_global(reinterpret_cast<const fv4*>(a.q_rows)) +
                         (int64_t)qq * (a.DP >> 2);
          sc = 0.f;
          for (int j0 = 0; j0 < a.DP; j0 += 64) {  // 64 dims per round (D <= 256: <= 4)
            fv4 xv[16], qv[16];
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if (j0 + 4 * j < a.DP) {
                xv[j] = xr[(j0 >> 2) + j];
                qv[j] = qr[(j0 >> 2) + j];
              }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const int d = j0 + 4 * j;
              if (d < a.D) sc = fmaf(xv[j].x, qv[j].x, sc);
              if (d + 1 < a.D) sc = fmaf(xv[j].y, qv[j].y, sc);
              if (d + 2 < a.D) sc = fmaf(xv[j].z, qv[j].z, sc);
              if (d + 3 < a.D) sc = fmaf(xv[j].w, qv[j].w, sc);
            }
          }
        }
        const int64_t sub = (int64_t)qq * NSUB + (bx & (NSUB - 1));
        const int pos = atomicAdd(&a.cnt[sub], 1);
        if (pos < SUBCAP) {
          a.cand_s[sub * SUBCAP + pos] = sc;
          a.cand_i[sub * SUBCAP + pos] = l_i[src];
        }
      }
    }
  }
  if constexpr (SAMPLE) {  // the group max of each query: its 4 waves' maxima
    __shared__ float smx[4][NQG * 16];
#pragma unroll
    for (int g = 0; g < NQG; ++g) {
      float m = thr[g];  // -inf for a wave without sample blocks
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      if (lg == 0) smx[wave_id()][16 * g + lr] = m;
    }
    __syncthreads();
    for (int r = threadIdx.x; r < NQG * 16; r += 256) {
      const int qq = qb + r;
      if (qq < a.B)
        a.smax[(int64_t)qq * a.G + bx] = fmaxf(fmaxf(smx[0][r], smx[1][r]), fmaxf(smx[2][r], smx[3][r]));
    }
  }
}

// Error bound of a bf16 filter score s~ against the exact f32 score s of the same pair,
// with q~ = bf16(q), x~ = bf16(x) (round to nearest even, as the filter converts them):
//   s~ - s = sum (q~_d x~_d - q_d x_d) + (f32 accumulation error)
//          = (q~ - q).x~ + q.(x~ - x) + acc,
//   |(q~ - q).x~| <= ||q~ - q|| max_i ||x~_i||,   |q.(x~ - x)| <= ||q|| max_i ||x~_i - x_i||
// (Cauchy-Schwarz), and |acc| <= gamma_D sum|q~_d x~_d| <= 2^-15 ||q~|| max_i ||x~_i||
// (bf16 products are exact in f32; D <= 256 additions).  So
//   |s~ - s| <= delta_q = ||q~ - q|| XN + ||q|| EX + 2^-15 ||q~|| XN  (+ a denormal-flush
// allowance), XN / EX from item_norm_max_kernel, the query terms measured here.  The
// rounding error norms are what bf16 actually did (about 2^-9.2 of the norm for random
// data) rather than the worst case 2^-8 per factor, so delta_q is about 2.2x smaller
// than ||q|| max ||x|| (2^-7 + 2^-16): fewer candidates, and none of the sub-list
// overflows at D = 256 that the worst-case bound caused.
struct TauArgs {
  const float* smax;
  int G;
  const float* q;          // bf16 filter: the f32 queries (for ||q||)
  int D;
  const uint32_t* maxnorm; // bf16 filter: {XN, EX} bits (item_norm_max_kernel); null = exact f32 scores
  float* tau;              // filter threshold
  float* tau_e;            // exactness threshold of the rescored candidates
  int* cnt;
  int* flag;
  float* q_rows;           // bf16 filter: the queries padded to DP floats (for the rescoring)
  int DP;
  int m;                   // tau~ = the m-th largest group maximum
};

// tau~ = m-th largest group max (one workgroup per query).  f32 filter:
// tau = tau_e = tau~.  bf16 filter, with d = delta_q (1 + 2^-10):
//   tau = tau~ - 2 d  (collect s~ >= tau),   tau_e = tau + d.
// Any item with exact s >= tau_e has s~ >= s - delta_q >= tau, so it was collected;
// the m sampled maxima (s~ >= tau~) all have s >= tau~ - delta_q >= tau_e.
// (The 2^-10 inflation covers the fp32 rounding of tau + d.)  Also resets the query's
// candidate counters and (query 0) the fallback flag.
__global__ __launch_bounds__(256) void mips_tau_kernel(TauArgs a) {
  __shared__ uint32_t key[SAMPLE_WAVES / 4];
  __shared__ SelLDS L;
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < a.G; e += 256) key[e] = ord_key(a.smax[(int64_t)q * a.G + e]);
  __syncthreads();
  const int m = a.G < a.m ? a.G : a.m;
  uint32_t kstar;
  int k_rem;
  block_kth(key, a.G, m, L, kstar, k_rem);
  if (tid < NSUB) a.cnt[q * NSUB + tid] = 0;
  if (a.q_rows && tid < a.DP) a.q_rows[(int64_t)q * a.DP + tid] = tid < a.D ? a.q[(int64_t)q * a.D + tid] : 0.f;
  // ||q||^2, ||q~||^2, ||q~ - q||^2 by wave 0 (lane-strided partial sums, fixed-order
  // butterfly)
  float ss = 0.f, sr = 0.f, se = 0.f;
  if (tid < 64) {
    for (int d = tid; d < a.D; d += 64) {
      const float v = a.q[(int64_t)q * a.D + d], r = bf16_round(v), e = r - v;
      ss = fmaf(v, v, ss);
      sr = fmaf(r, r, sr);
      se = fmaf(e, e, se);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      ss += __shfl_xor(ss, o, 64);
      sr += __shfl_xor(sr, o, 64);
      se += __shfl_xor(se, o, 64);
    }
  }
  if (tid == 0) {
    const float t = key_to_float(kstar);
    if (a.maxnorm) {
      const float qn = sqrtf(ss), qrn = sqrtf(sr), qen = sqrtf(se);
      const float xn = __uint_as_float(a.maxnorm[0]), xen = __uint_as_float(a.maxnorm[1]);
      // (1 + 2^-10) covers the f32 evaluation of the norms and of this sum
      const float dl = (qen * xn + qn * xen + 0.000030517578125f * qrn * xn +
                        1e-35f * (qn + xn + 1.f)) * (1.f + 0.0009765625f);
      a.tau[q] = t - 2.f * dl;
      a.tau_e[q] = a.tau[q] + dl;
    } else {
      a.tau[q] = t;
      a.tau_e[q] = t;
    }
    if (q == 0) *a.flag = 0;
  }
}

struct FilterMergeArgs {
  const float* cand_s;
  const int* cand_i;
  const int* cnt;
  int B, k, N0;
  const int64_t* item_ids;
  int64_t index_base;
  const int64_t* invalid;
  float* out_score;
  int64_t* out_ids;
  int64_t* out_index;
  int* flag;
  // bf16 filter: candidates are rescored exactly from the f32 table and only those with
  // s >= tau_e count (see mips_tau_kernel)
  int rescore;
  const float* tau_e;
};

__global__ __launch_bounds__(256) void mips_filter_merge_kernel(FilterMergeArgs a) {
  __shared__ uint32_t key[FILTER_CAP];
  __shared__ int64_t idx[FILTER_CAP];
  extern __shared__ int64_t inv[];  // inv_pad(N0) entries (dynamic LDS)
  __shared__ SelLDS L;
  __shared__ int sub_off[NSUB + 1];
  __shared__ float cs[FILTER_CAP];
  const int q = blockIdx.x, tid = threadIdx.x;
  // the invalid row's loads go out first, beside the counter loads (independent of them)
  const int n0p = inv_pad(a.N0);
  for (int j = tid; j < n0p; j += 256)
    inv[j] = j < a.N0 ? a.invalid[(int64_t)q * a.N0 + j] : INT64_MAX;
  if (tid == 0) {
    int o = 0;
    bool over = false;
    for (int u = 0; u < NSUB; ++u) {
      const int c = a.cnt[q * NSUB + u];
      over |= c > SUBCAP;
      sub_off[u] = o;
      o += c < SUBCAP ? c : SUBCAP;
    }
    sub_off[NSUB] = over ? -1 : o;
  }
  __syncthreads();
  const int n_raw = sub_off[NSUB];
  if (n_raw < 0) {  // a sub-list overflowed: the exact fallback recomputes
    if (tid == 0) atomicExch(a.flag, 1);
    return;
  }
  // Compaction and the validity test run on registers: thread t holds list positions
  // t + 256 j.  Every score / index load is issued before any use, then every id gather
  // (a loop over the positions gathered each id in turn: a dependent round trip per
  // element), and the ids are tested after the invalid row is sorted.
  constexpr int PER = FILTER_CAP / 256;
  float vs[PER];
  int vi[PER];
  int64_t vid[PER];
  {
    int off[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) off[u] = __builtin_amdgcn_readfirstlane(sub_off[u]);
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int p = tid + 256 * t;
      vs[t] = -INFINITY;
      vi[t] = 0;
      if (p < n_raw) {
        int u = 0;
#pragma unroll
        for (int w = 1; w < NSUB; ++w) u = off[w] <= p ? w : u;
        int base = off[0];
#pragma unroll
        for (int w = 1; w < NSUB; ++w) base = w == u ? off[w] : base;
        const int64_t src = ((int64_t)q * NSUB + u) * SUBCAP + (p - base);
        vs[t] = a.cand_s[src];
        vi[t] = a.cand_i[src];
      }
    }
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int p = tid + 256 * t;
      vid[t] = a.index_base + vi[t];
      if (a.item_ids && p < n_raw) vid[t] = a.item_ids[vi[t]];
    }
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int p = tid + 256 * t;
      if (p < n_raw) cs[p] = vs[t];
    }
  }
  if (n0p > 256) block_bitonic_i64(inv, n0p);
  else if (n0p > 0) block_sort_i64_asc(inv, n0p);
  // bf16 filter: cs holds the exact scores (rescored at the filter's flush); only candidates at
  // or above tau_e are provably complete
  const float te = a.rescore ? a.tau_e[q] : -INFINITY;
  // invalid-id tests: branch-free binary searches over the sorted row (n0p a power of
  // two; pos = the last entry <= the id), the searches of 4 candidates interleaved (one
  // search per candidate in turn waited log2(n0p) dependent LDS reads each)
  bool bad[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) bad[t] = false;
  if (n0p > 0) {
#pragma unroll
    for (int c = 0; c < PER / 4; ++c) {
      if (1024 * c < n_raw) {
        const int64_t k0 = vid[4 * c], k1 = vid[4 * c + 1], k2 = vid[4 * c + 2], k3 = vid[4 * c + 3];
        int p0 = 0, p1 = 0, p2 = 0, p3 = 0;
        for (int step = n0p >> 1; step > 0; step >>= 1) {
          const int64_t v0 = inv[p0 + step], v1 = inv[p1 + step], v2 = inv[p2 + step], v3 = inv[p3 + step];
          p0 += v0 <= k0 ? step : 0;
          p1 += v1 <= k1 ? step : 0;
          p2 += v2 <= k2 ? step : 0;
          p3 += v3 <= k3 ? step : 0;
        }
        bad[4 * c] = inv[p0] == k0;
        bad[4 * c + 1] = inv[p1] == k1;
        bad[4 * c + 2] = inv[p2] == k2;
        bad[4 * c + 3] = inv[p3] == k3;
      }
    }
  }
  int nvalid = 0;
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int p = tid + 256 * t;
    if (p < n_raw) {
      const bool ok = !bad[t] && vs[t] >= te;
      key[p] = ok ? ord_key(vs[t]) : 0u;
      idx[p] = a.index_base + vi[t];
      nvalid += ok;
    }
  }
  const int tot = block_sum(nvalid, L);
  if (tot < a.k) {  // fewer than k valid items at or above tau: not provably exact
    if (tid == 0) atomicExch(a.flag, 1);
    return;
  }
  const int n = block_topk_sorted(key, idx, n_raw, a.k, tot, L);
  for (int r = tid; r < a.k; r += 256) {
    const int64_t o = (int64_t)q * a.k + r;
    const int e = L.s_src[r];  // r < n == k
    const int64_t gi = L.s_idx[r];
    a.out_score[o] = cs[e];
    if (a.out_index) a.out_index[o] = gi;
    a.out_ids[o] = a.item_ids ? a.item_ids[gi - a.index_base] : gi;
  }
  (void)n;
}

// ----------------------------------------------------------------- wide k (k > 256)
// torch.topk takes any k; the reference's CandidateIndex asks its top-k module for
// k' = k + N0 (candidate_index.py:132), 2,259 at ml-20m.  The fused paths above keep
// per-query selections of <= 256 in LDS, so k > 256 runs this chunked exact path:
//   W1 (mips_wide_score_kernel): keys of a chunk of <= Xc items for all queries
//      (the same k-ordered fmaf chain read from the packed layout; explicit ids are
//      excluded here by binary search in the pre-sorted invalid rows);
//   W2 (mips_wide_select_kernel): per query, the exact top-k of (running list ++
//      chunk) by 8-bit radix select, ties at the k-th key by position (= catalog index:
//      the running list holds earlier chunks, ties inside it sorted by index), then a
//      bitonic sort (key desc, index asc) into the running list or the outputs.
constexpr int KW_MAX = 4096;

struct WideArgs {
  const float* q;
  const float* packed;
  int64_t X;
  int D, B, N0, k;
  const int64_t* item_ids;
  int64_t index_base;
  const int64_t* invalid;
  const int64_t* inv_sorted;  // explicit ids, N0 > 0: [B][n0p]
  int n0p;
  int64_t xc;                 // chunk row stride of ckey
  int64_t c0, n;              // this chunk: local items [c0, c0 + n)
  uint32_t* ckey;             // [B][xc], 0 = excluded
  uint32_t* rkey;             // [B][k] running list (sorted), 0 = empty
  int64_t* ridx;              // [B][k]
  int first, last;
  float* out_score;
  int64_t* out_ids;
  int64_t* out_index;
};

__global__ __launch_bounds__(256) void mips_wide_score_kernel(WideArgs a) {
  __shared__ float qv[256];
  const int q = blockIdx.y, tid = threadIdx.x;
  const int KS2 = (ceil_div(a.D, 4) + 1) / 2;
  for (int d = tid; d < 8 * KS2; d += 256) qv[d] = d < a.D ? a.q[(int64_t)q * a.D + d] : 0.f;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + tid;
  if (i >= a.n) return;
  const int64_t li = a.c0 + i;
  typedef float fv2 __attribute__((ext_vector_type(2)));
  gptr<fv2> pk = as_global(reinterpret_cast<const fv2*>(a.packed));
  const int64_t ib = li >> 4;
  const int il = (int)(li & 15);
  float sc = 0.f;
  for (int j = 0; j < KS2; ++j) {
    fv2 v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = pk[(ib * KS2 + j) * 64 + 16 * c + il];
#pragma unroll
    for (int c = 0; c < 4; ++c) sc = fmaf(qv[8 * j + c], v[c].x, sc);      // d = 8j + c
#pragma unroll
    for (int c = 0; c < 4; ++c) sc = fmaf(qv[8 * j + 4 + c], v[c].y, sc);  // d = 8j + 4 + c
  }
  bool ok = true;
  if (a.item_ids && a.N0 > 0)
    ok = !sorted_contains(a.inv_sorted + (int64_t)q * a.n0p, a.n0p, a.item_ids[li]);
  a.ckey[(int64_t)q * a.xc + i] = ok ? ord_key(sc) : 0u;
}

// k-th largest nonzero key of the virtual array key_at(0 .. M) (any block size).
template <class KeyAt>
__device__ void block_radix_kth_any(KeyAt key_at, int64_t M, int kk, int* hist, int* sh,
                                    uint32_t& kstar, int& k_rem) {
  uint32_t prefix = 0, mask = 0;
  int need = kk;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int64_t e = threadIdx.x; e < M; e += blockDim.x) {
      const uint32_t x = key_at(e);
      if (x != 0u && (x & mask) == prefix) atomicAdd(&hist[(x >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) hist_find_digit(hist, need, &sh[0], &sh[1]);
    __syncthreads();
    prefix |= (uint32_t)sh[0] << shift;
    mask |= 0xFFu << shift;
    need -= sh[1];
    __syncthreads();
  }
  kstar = prefix;
  k_rem = need;
}

__global__ __launch_bounds__(1024) void mips_wide_select_kernel(WideArgs a) {
  __shared__ uint32_t skey[KW_MAX];
  __shared__ int64_t sidx[KW_MAX];
  __shared__ int hist[256];
  __shared__ int sh[4];
  __shared__ int wsum[16];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t* ck = a.ckey + (int64_t)q * a.xc;
  uint32_t* rk = a.rkey + (int64_t)q * a.k;
  int64_t* rx = a.ridx + (int64_t)q * a.k;
  if (!a.item_ids && a.N0 > 0) {  // arange ids: drop the query's invalid items by index
    for (int j = tid; j < a.N0; j += 1024) {
      const int64_t li = a.invalid[(int64_t)q * a.N0 + j] - a.index_base - a.c0;
      if (li >= 0 && li < a.n) ck[li] = 0u;
    }
    __syncthreads();
  }
  const int rc = a.first ? 0 : a.k;  // running list: k slots, empty ones keyed 0
  const int64_t M = rc + a.n;
  auto key_at = [&](int64_t e) -> uint32_t { return e < rc ? rk[e] : ck[e - rc]; };
  auto idx_at = [&](int64_t e) -> int64_t {
    return e < rc ? rx[e] : a.index_base + a.c0 + (e - rc);
  };
  int nz = 0;
  for (int64_t e = tid; e < M; e += 1024) nz += key_at(e) != 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) nz += __shfl_xor(nz, o, 64);
  if (lane == 0) wsum[w] = nz;
  if (tid == 0) sh[2] = 0;
  __syncthreads();
  int tot = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) tot += wsum[u];
  __syncthreads();
  const bool all = tot <= a.k;
  uint32_t kstar = 0u;
  int k_rem = 0;
  if (!all) block_radix_kth_any(key_at, M, a.k, hist, sh, kstar, k_rem);
  // entries above kstar (any order: sorted below)
  for (int64_t e = tid; e < M; e += 1024) {
    const uint32_t x = key_at(e);
    if (x != 0u && (all || x > kstar)) {
      const int p = atomicAdd(&sh[2], 1);
      skey[p] = x;
      sidx[p] = idx_at(e);
    }
  }
  // ties at kstar: the first k_rem in position order, tile by tile
  int taken = 0;
  for (int64_t t0 = 0; !all && t0 < M && taken < k_rem; t0 += 1024) {
    const int64_t e = t0 + tid;
    const bool eq = e < M && key_at(e) == kstar;
    const unsigned long long bal = __ballot(eq);
    __syncthreads();
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int before = 0, tile = 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      before += u < w ? wsum[u] : 0;
      tile += wsum[u];
    }
    const int r = taken + before + __popcll(bal & ((1ull << lane) - 1ull));
    if (eq && r < k_rem) {
      const int p = atomicAdd(&sh[2], 1);
      skey[p] = kstar;
      sidx[p] = idx_at(e);
    }
    taken += tile;
  }
  __syncthreads();
  const int nsel = sh[2];
  int P = 2;
  while (P < nsel) P <<= 1;
  for (int p = nsel + tid; p < P; p += 1024) {
    skey[p] = 0u;
    sidx[p] = INT64_MAX;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1)  // key desc, index asc
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = tid; p < P / 2; p += 1024) {
        const int i = 2 * p - (p & (stride - 1)), j = i + stride;
        const bool desc = (i & size) == 0;
        const uint32_t ki = skey[i], kj = skey[j];
        const int64_t xi = sidx[i], xj = sidx[j];
        const bool i_first = ki > kj || (ki == kj && xi < xj);
        if (i_first != desc) {
          skey[i] = kj; skey[j] = ki;
          sidx[i] = xj; sidx[j] = xi;
        }
      }
      __syncthreads();
    }
  if (!a.last) {
    for (int r = tid; r < a.k; r += 1024) {
      rk[r] = r < nsel ? skey[r] : 0u;
      rx[r] = r < nsel ? sidx[r] : INT64_MAX;
    }
    return;
  }
  for (int r = tid; r < a.k; r += 1024) {
    const int64_t o = (int64_t)q * a.k + r;
    if (r < nsel) {
      const int64_t gi = sidx[r];
      a.out_score[o] = key_to_float(skey[r]);
      if (a.out_index) a.out_index[o] = gi;
      a.out_ids[o] = a.item_ids ? a.item_ids[gi - a.index_base] : gi;
    } else {
      a.out_score[o] = -INFINITY;
      if (a.out_index) a.out_index[o] = -1;
      a.out_ids[o] = -1;
    }
  }
}

struct TopkPlan {
  bool small, filter;
  int KS, n_ranges, k_part;
  int64_t range_items;
  size_t part_bytes;   // legacy select partial lists (also the filter path's fallback)
  // filter path
  int64_t n_blocks, RB;
  int GB, G, NQG, n_chunks, filter_waves, sr, m;
  int KC;              // > 0: the filter scores the bf16 copy (KC k-chunks of 32 dims)
  size_t off_tau, off_tau_e, off_qrows, off_cnt, off_smax, off_cs, off_ci, off_part, total_bytes;
  int n0p;             // inv_pad(N0)
  size_t off_inv;      // N0 > INV_MAX on the select path: [B][n0p] sorted invalid lists
  bool wide;           // k > 256: the chunked exact path
  int64_t xc;          // its chunk (items)
  size_t off_rkey, off_ridx;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Packed-table layout: the f32 blocks, then (filter-sized catalogs: X >= FILTER_MIN_X,
// D <= 64) the bf16 copy, the max item norm and a row-major f32 copy with rows padded
// to DP = 4 ceil(D/4) floats (16-byte aligned: the merge's exact rescoring gathers a
// candidate row with DP/4 float4 loads, ~4 sectors, instead of 2 D scattered floats).
struct PackLayout {
  bool bf16;
  int KC, DP;
  size_t off16, off_norm, off_rows, total;
};

static PackLayout pack_layout(int64_t X, int D) {
  PackLayout L{};
  const int64_t nblk = (X + 15) / 16;
  const size_t f32 = sizeof(float) * (size_t)nblk * ((ceil_div(D, 4) + 1) / 2) * 128;
  L.total = f32;
  L.bf16 = X >= FILTER_MIN_X && ceil_div(D, 4) <= 64;  // D <= 256: KC <= 8 k-chunks
  if (L.bf16) {
    L.KC = ceil_div(D, 32);
    L.off16 = align256(f32);
    L.off_norm = L.off16 + align256((size_t)nblk * bf16_block_bytes(D, L.KC));
    L.DP = 4 * ceil_div(D, 4);
    L.off_rows = L.off_norm + 256;
    L.total = L.off_rows + align256(sizeof(float) * (size_t)X * L.DP);
  }
  return L;
}

static TopkPlan plan_topk(int B, int64_t X, int D, int k, int N0) {
  TopkPlan p{};
  p.KS = ceil_div(D, 4);
  const int n_qg = ceil_div(B, QG);
  int target = ceil_div(256, n_qg);  // ~one workgroup per CU
  int64_t step4 = SW * 64;
  int64_t ri = (X + target - 1) / target;
  ri = ((ri + step4 - 1) / step4) * step4;
  if (ri < step4) ri = step4;
  p.range_items = ri;
  p.n_ranges = (int)((X + ri - 1) / ri);
  if (p.n_ranges < 1) p.n_ranges = 1;
  while ((int64_t)p.n_ranges * k > MERGE_MAX) {  // merge capacity
    p.range_items *= 2;
    p.n_ranges = (int)((X + p.range_items - 1) / p.range_items);
  }
  // hand the merge up to CAP/2 candidates per range when it has room: a range that
  // saw <= k_part valid items then needs no selection in phase 1
  int kp = MERGE_MAX / p.n_ranges;
  kp = kp > CAP / 2 ? CAP / 2 : kp;
  p.k_part = kp > k ? kp : k;
  p.part_bytes = (size_t)p.n_ranges * B * p.k_part * (sizeof(float) + sizeof(int64_t));
  p.small = X > 0 && X <= MERGE_MAX && (p.KS + 1) / 2 <= 8;  // D <= 64
  if (p.small) {
    const size_t sb = (size_t)B * X * (sizeof(float) + sizeof(int64_t));
    if (sb > p.part_bytes) p.part_bytes = sb;
  }
  // the f32 filter holds every query fragment in registers (D <= 64); the bf16 filter runs
  // to D = 256 with fewer queries per workgroup beyond D = 64
  const int kc_bf = option(GR_OPT_MIPS_FILTER_FP32) ? 0 : pack_layout(X, D).KC;
  p.filter = !p.small && X >= FILTER_MIN_X && (p.KS <= 16 || kc_bf > 0);
  p.total_bytes = p.part_bytes;
  p.off_part = 0;
  if (p.filter) {
    p.n_blocks = (X + 15) / 16;
    // sample stride sr and rank m = 1024 / sr keep ~1024 candidates per query at any stride
    // (a 32-block stride with m fixed at 64 doubled them: merge +9 us, filter +34 us)
    p.sr = option(GR_OPT_MIPS_SAMPLE_STRIDE) > 0 ? (int)option(GR_OPT_MIPS_SAMPLE_STRIDE) : SAMPLE_STRIDE;
    p.m = std::max(8, SAMPLE_CAND / p.sr);
    const int64_t n_sb = (p.n_blocks + p.sr - 1) / p.sr;
    // ~SAMPLE_GB blocks per wave while the groups (4 waves each) stay >= 4 m, and at most
    // SAMPLE_WAVES waves: fewer workgroups each staging the queries
    int64_t gb = std::min<int64_t>(SAMPLE_GB, n_sb / (16 * (int64_t)p.m));
    gb = std::max<int64_t>({gb, 1, (n_sb + SAMPLE_WAVES - 1) / SAMPLE_WAVES});
    p.GB = (int)gb;
    p.G = ceil_div((int)((n_sb + p.GB - 1) / p.GB), 4);  // sample workgroups
    p.NQG = B <= 32 ? 2 : 8;  // KC > 2: 3 groups in VGPRs and 5 read from LDS (filter), 2 and 6 (sample)
    p.n_chunks = ceil_div(B, p.NQG * 16);
    // whole rounds of 2 four-wave workgroups per CU, >= ~48 blocks per wave
    // (GR_OPT_MIPS_FILTER_WGS = 0: 3 per CU at KC <= 2, whose kernels hold 168 VGPRs)
    const int64_t wgs = option(GR_OPT_MIPS_FILTER_WGS) > 0 ? option(GR_OPT_MIPS_FILTER_WGS)
                                                           : (kc_bf > 0 && kc_bf <= 2 ? 3 : 2);
    const int64_t per_round = (int64_t)device_cus() * 4 * wgs;
    // GR_OPT_MIPS_FILTER_FP32: filter on the f32 table (exact scores, 16x fewer flop/s)
    p.KC = kc_bf;
    // f32: >= ~48 blocks per wave.  bf16 (streaming-bound): one round (10M items: 7
    // rounds 302 us, 2 rounds 253 us, 1 round 251 us)
    const int64_t min_rb = p.KC ? 4096 : 48;
    int64_t rounds = (p.n_blocks + per_round * min_rb - 1) / (per_round * min_rb);
    if (option(GR_OPT_MIPS_FILTER_ROUNDS) > 0) rounds = option(GR_OPT_MIPS_FILTER_ROUNDS);
    if (rounds < 1) rounds = 1;
    p.RB = (p.n_blocks + per_round * rounds - 1) / (per_round * rounds);
    p.filter_waves = (int)((p.n_blocks + p.RB - 1) / p.RB);
    size_t o = 256;  // [0, 4): fallback flag
    p.off_tau = o;  o = align256(o + sizeof(float) * B);
    p.off_tau_e = o; o = align256(o + sizeof(float) * B);
    p.off_qrows = o; o = align256(o + sizeof(float) * B * 4 * p.KS);  // bf16 filter: padded f32 queries
    p.off_cnt = o;  o = align256(o + sizeof(int) * B * NSUB);
    p.off_smax = o; o = align256(o + sizeof(float) * (size_t)B * p.G);
    p.off_cs = o;   o = align256(o + sizeof(float) * (size_t)B * FILTER_CAP);
    p.off_ci = o;   o = align256(o + sizeof(int) * (size_t)B * FILTER_CAP);
    p.off_part = o;
    p.total_bytes = o + p.part_bytes;
  }
  p.n0p = inv_pad(N0);
  p.off_inv = 0;
  p.wide = k > 256;
  if (p.wide) {  // [B][xc] chunk keys (<= 256 MiB), [B][k] running list, sorted invalid rows
    const int64_t cap = ((int64_t)1 << 26) / B;
    p.xc = X < cap ? X : (cap < 4096 ? 4096 : cap);
    p.small = p.filter = false;
    size_t o = align256(sizeof(uint32_t) * (size_t)B * p.xc);
    p.off_rkey = o; o = align256(o + sizeof(uint32_t) * (size_t)B * k);
    p.off_ridx = o; o = align256(o + sizeof(int64_t) * (size_t)B * k);
    p.off_inv = o;  o += sizeof(int64_t) * (size_t)B * p.n0p;
    p.total_bytes = o;
    return p;
  }
  if (!p.small && N0 > INV_MAX) {
    p.off_inv = align256(p.total_bytes);
    p.total_bytes = p.off_inv + sizeof(int64_t) * (size_t)B * p.n0p;
  }
  return p;
}

template <int KS, int KC, int NQG>
static int launch_filter_pair(const FilterArgs& f, const TopkPlan& p, bool sample, hipStream_t st) {
  if (sample) {
    const dim3 g(p.G, p.n_chunks);
    GR_TIMED("mips_sample", st, hipLaunchKernelGGL((mips_filter_kernel<KS, KC, NQG, true>), g, dim3(256), 0, st, f));
    GR_LAUNCH_CHECK("mips_topk(sample)");
  } else {
    const int gx = ceil_div(p.filter_waves, 4);
    FilterArgs fx = f;
    dim3 g(gx, p.n_chunks);
    if (p.n_chunks > 1 && option(GR_OPT_MIPS_FILTER_PAIRED) != 0) {
      fx.nch = p.n_chunks;
      fx.gx = gx;
      g = dim3(ceil_div(gx, 8) * 8 * p.n_chunks, 1);
    }
    GR_TIMED("mips_filter", st, hipLaunchKernelGGL((mips_filter_kernel<KS, KC, NQG, false>), g, dim3(256), 0, st, fx));
    GR_LAUNCH_CHECK("mips_topk(filter)");
  }
  return 0;
}

template <int KS, int KC>
static int launch_filter_ks(const FilterArgs& f, const TopkPlan& p, bool sample, hipStream_t st) {
  return p.NQG == 2 ? launch_filter_pair<KS, KC, 2>(f, p, sample, st)
                    : launch_filter_pair<KS, KC, 8>(f, p, sample, st);
}

static int launch_filter(const FilterArgs& f, const TopkPlan& p, bool sample, hipStream_t st) {
  switch (p.KC) {
    case 1: return launch_filter_ks<1, 1>(f, p, sample, st);
    case 2: return launch_filter_ks<1, 2>(f, p, sample, st);
    case 3: return launch_filter_ks<1, 3>(f, p, sample, st);
    case 4: return launch_filter_ks<1, 4>(f, p, sample, st);
    case 5: return launch_filter_ks<1, 5>(f, p, sample, st);
    case 6: return launch_filter_ks<1, 6>(f, p, sample, st);
    case 7: return launch_filter_ks<1, 7>(f, p, sample, st);
    case 8: return launch_filter_ks<1, 8>(f, p, sample, st);
    default: break;
  }
  switch (p.KS) {
    case 1: case 2: return launch_filter_ks<2, 0>(f, p, sample, st);
    case 3: case 4: return launch_filter_ks<4, 0>(f, p, sample, st);
    case 5: case 6: case 7: case 8: return launch_filter_ks<8, 0>(f, p, sample, st);
    case 9: case 10: case 11: case 12: case 13: return launch_filter_ks<13, 0>(f, p, sample, st);
    default: return launch_filter_ks<16, 0>(f, p, sample, st);
  }
}

template <int KS>
static int launch_select(const SelectArgs& a, hipStream_t st) {
  constexpr int BLOCKS = KS <= 16 ? 2 : 1;  // SW * 16 * BLOCKS <= CAP - 256
  const int n_qg = ceil_div(a.B, QG);
  const int n_r8 = ceil_div(a.n_ranges, 8) * 8;
  const int units = n_r8 * n_qg;
  const int cap = 2 * ceil_div(device_cus(), 8) * 8;
  const int grid = a.gate && units > cap ? cap : units;
  GR_TIMED(a.gate ? "mips_select_fallback" : "mips_select", st, hipLaunchKernelGGL((mips_select_kernel<KS, BLOCKS>), dim3(grid), dim3(ST), 0, st, a, units));
  GR_LAUNCH_CHECK("mips_topk(select)");
  return 0;
}

}  // namespace gr

using namespace gr;

extern "C" size_t mips_packed_items_bytes(int64_t X, int D) {
  if (X < 0 || D <= 0) return 0;
  return pack_layout(X, D).total;
}

extern "C" int mips_pack_items(const float* items, int64_t X, int D, float* packed, void* stream) {
  GR_REQUIRE(items && packed && X >= 0 && D > 0, "mips_pack_items: bad args");
  if (X == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const int KS2 = (ceil_div(D, 4) + 1) / 2;
  const PackLayout L = pack_layout(X, D);
  GR_TIMED("mips_pack", st, {
    hipLaunchKernelGGL(pack_items_kernel, dim3(2048), dim3(256), 0, st, items, X, D, KS2, packed);
    if (L.bf16) {
      char* base = (char*)packed;
      uint32_t* maxbits = (uint32_t*)(base + L.off_norm);
      hipLaunchKernelGGL(pack_bf16_kernel, dim3(2048), dim3(256), 0, st, items, X, D, L.KC,
                         (u32x4*)(base + L.off16));
      zero_words_async(maxbits, 2, st);
      hipLaunchKernelGGL(item_norm_max_kernel, dim3(2048), dim3(256), 0, st, items, X, D, maxbits);
      hipLaunchKernelGGL(pack_rows_kernel, dim3(2048), dim3(256), 0, st, items, X, D, L.DP,
                         (float*)(base + L.off_rows));
    }
  });
  GR_LAUNCH_CHECK("mips_pack_items");
  return 0;
}

extern "C" size_t mips_topk_workspace_size(int B, int64_t X, int D, int k, int N0) {
  if (B <= 0 || X <= 0 || D <= 0 || k <= 0 || N0 < 0) return 0;
  return plan_topk(B, X, D, k, N0).total_bytes;
}

extern "C" int mips_topk(const float* queries, const float* packed_items, int64_t X, int D,
                         const int64_t* item_ids, int64_t index_base, const int64_t* invalid_ids,
                         int N0, int B, int k, float* out_scores, int64_t* out_ids,
                         int64_t* out_index, void* workspace, size_t ws_bytes, void* stream) {
  GR_REQUIRE(queries && packed_items && out_scores && out_ids, "mips_topk: null pointer");
  GR_REQUIRE(B >= 0 && X >= 0 && D > 0 && D <= 256, "mips_topk: D=%d not in [1, 256]", D);
  GR_REQUIRE(k > 0 && k <= KW_MAX, "mips_topk: k=%d not in [1, %d]", k, KW_MAX);
  GR_REQUIRE(N0 >= 0 && N0 <= INV_BIG && (N0 == 0 || invalid_ids),
             "mips_topk: N0=%d not in [0, %d] (or invalid_ids null)", N0, INV_BIG);
  GR_REQUIRE(X < 0x7FFFFFFF, "mips_topk: X must be < 2^31 per shard");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0) return 0;
  TopkPlan p = plan_topk(B, X > 0 ? X : 1, D, k, N0);
  GR_REQUIRE(workspace && ws_bytes >= p.total_bytes, "mips_topk: workspace %zu B < %zu B", ws_bytes,
             p.total_bytes);
  if (p.wide) {
    char* ws = (char*)workspace;
    WideArgs w{queries, packed_items, X, D, B, N0, k, item_ids, index_base, invalid_ids, nullptr,
               p.n0p, p.xc, 0, 0, (uint32_t*)ws, (uint32_t*)(ws + p.off_rkey),
               (int64_t*)(ws + p.off_ridx), 1, 0, out_scores, out_ids, out_index};
    if (item_ids && N0 > 0) {
      int64_t* sorted_rows = (int64_t*)(ws + p.off_inv);
      w.inv_sorted = sorted_rows;
      GR_TIMED("mips_sort_invalid", st, hipLaunchKernelGGL(mips_sort_invalid_kernel, dim3(B), dim3(1024),
                                                           sizeof(int64_t) * p.n0p, st, invalid_ids, N0,
                                                           p.n0p, sorted_rows, nullptr));
      GR_LAUNCH_CHECK("mips_topk(sort invalid)");
    }
    for (int64_t c0 = 0; c0 < X || c0 == 0; c0 += p.xc) {
      w.c0 = c0;
      w.n = X - c0 < p.xc ? X - c0 : p.xc;
      w.last = c0 + p.xc >= X;
      if (w.n > 0) {
        GR_TIMED("mips_wide_score", st, hipLaunchKernelGGL(mips_wide_score_kernel,
                 dim3((unsigned)((w.n + 255) / 256), B), dim3(256), 0, st, w));
        GR_LAUNCH_CHECK("mips_topk(wide score)");
      }
      GR_TIMED("mips_wide_select", st, hipLaunchKernelGGL(mips_wide_select_kernel, dim3(B), dim3(1024), 0, st, w));
      GR_LAUNCH_CHECK("mips_topk(wide select)");
      w.first = 0;
      if (w.last) break;
    }
    return 0;
  }
  if (p.small) {
    float* sc = (float*)workspace;
    int64_t* ix = (int64_t*)(sc + (size_t)B * X);
    // ~4 workgroups per CU over the launch, chunks of whole 256-item sweeps
    const int64_t want = std::max<int64_t>(1, (int64_t)4 * device_cus() / std::max(B, 1));
    int64_t chunk = (X + want - 1) / want;
    chunk = std::max<int64_t>(256, (chunk + 255) / 256 * 256);
    const unsigned n_chunks = (unsigned)((X + chunk - 1) / chunk);
    ScoreAllArgs s{queries, packed_items, X, D, B, N0, item_ids, index_base, invalid_ids, sc, ix,
                   chunk};
    const size_t inv_lds = item_ids ? sizeof(int64_t) * p.n0p : 0;
    const int KS2 = (p.KS + 1) / 2;
#define GR_SA(K2)                                                                           \
  case K2:                                                                                  \
    GR_TIMED("mips_select", st, hipLaunchKernelGGL(mips_scoreall_kernel<K2>, dim3(B, n_chunks), dim3(256), inv_lds, st, s)); \
    break;
    switch (KS2) {
      GR_SA(1) GR_SA(2) GR_SA(3) GR_SA(4) GR_SA(5) GR_SA(6) GR_SA(7) GR_SA(8)
      default: GR_REQUIRE(false, "mips_topk: score-all path needs D <= 64");
    }
#undef GR_SA
    GR_LAUNCH_CHECK("mips_topk(score-all)");
    SmallArgs m{sc, ix, (int)X, k, item_ids, index_base, out_scores, out_ids, out_index};
    GR_TIMED("mips_small", st, hipLaunchKernelGGL(mips_small_select_kernel, dim3(B), dim3(SM_T), 0, st, m));
    GR_LAUNCH_CHECK("mips_topk(small select)");
    return 0;
  }
  char* ws = (char*)workspace;
  int* flag = nullptr;
  if (p.filter) {
    flag = (int*)ws;
    float* tau = (float*)(ws + p.off_tau);
    int* cnt = (int*)(ws + p.off_cnt);
    float* tau_e = (float*)(ws + p.off_tau_e);
    const PackLayout L = pack_layout(X, D);
    const char* pbase = (const char*)packed_items;
    FilterArgs f{queries, packed_items, p.KC ? (const u32x4*)(pbase + L.off16) : nullptr,
                 p.KC ? bf16_block_bytes(D, p.KC) : 0, p.KC ? bf16_last_groups(D, p.KC) : 0,
                 p.KC ? bf16_tail_dims(D, p.KC) : 0, X, D, B,
                 p.n_blocks, p.GB, p.G, p.sr, (float*)(ws + p.off_smax),
                 p.RB, tau, cnt, (float*)(ws + p.off_cs), (int*)(ws + p.off_ci), (int*)ws,
                 option(GR_OPT_MIPS_FORCE_FALLBACK) != 0,
                 p.KC ? (const float*)(pbase + L.off_rows) : nullptr, (float*)(ws + p.off_qrows),
                 L.DP};
    int rc = launch_filter(f, p, true, st);
    if (rc) return rc;
    TauArgs ta{f.smax, p.G, queries, D, p.KC ? (const uint32_t*)(pbase + L.off_norm) : nullptr,
               tau, tau_e, cnt, flag, p.KC ? (float*)(ws + p.off_qrows) : nullptr, L.DP, p.m};
    GR_TIMED("mips_tau", st, hipLaunchKernelGGL(mips_tau_kernel, dim3(B), dim3(256), 0, st, ta));
    GR_LAUNCH_CHECK("mips_topk(tau)");
    rc = launch_filter(f, p, false, st);
    if (rc) return rc;
    FilterMergeArgs fm{f.cand_s, f.cand_i, cnt, B, k, N0, item_ids, index_base, invalid_ids,
                       out_scores, out_ids, out_index, flag, p.KC > 0, tau_e};
    GR_TIMED("mips_merge", st, hipLaunchKernelGGL(mips_filter_merge_kernel, dim3(B), dim3(256),
                                                  sizeof(int64_t) * p.n0p, st, fm));
    GR_LAUNCH_CHECK("mips_topk(filter merge)");
  }
  // exact range-select path (the filter path's fallback, gated on its flag)
  float* part_score = (float*)(ws + p.off_part);
  int64_t* part_index = (int64_t*)(part_score + (size_t)p.n_ranges * B * p.k_part);
  int64_t* inv_sorted = nullptr;
  if (p.off_inv) {  // N0 > INV_MAX: sorted lists for the select kernel's binary searches
    inv_sorted = (int64_t*)(ws + p.off_inv);
    GR_TIMED("mips_sort_invalid", st, hipLaunchKernelGGL(mips_sort_invalid_kernel, dim3(B), dim3(1024),
                                                         sizeof(int64_t) * p.n0p, st, invalid_ids, N0,
                                                         p.n0p, inv_sorted, flag));
    GR_LAUNCH_CHECK("mips_topk(sort invalid)");
  }
  SelectArgs a{queries, packed_items, X, D, B, k, N0, p.n_ranges, p.k_part, p.range_items,
               item_ids, index_base, invalid_ids, part_score, part_index, flag, inv_sorted};
  int rc;
  switch (p.KS) {
    case 1: case 2: rc = launch_select<2>(a, st); break;
    case 3: case 4: rc = launch_select<4>(a, st); break;
    case 5: case 6: case 7: case 8: rc = launch_select<8>(a, st); break;
    case 9: case 10: case 11: case 12: case 13: rc = launch_select<13>(a, st); break;
    case 14: case 15: case 16: rc = launch_select<16>(a, st); break;
    default:
      if (p.KS <= 32) rc = launch_select<32>(a, st);
      else rc = launch_select<64>(a, st);
  }
  if (rc) return rc;
  MergeArgs m{part_score, part_index, nullptr, p.n_ranges, B, p.k_part, k, item_ids, index_base,
              out_scores, out_ids, out_index, flag};
  GR_TIMED(flag ? "mips_merge_fallback" : "mips_merge", st, hipLaunchKernelGGL(mips_merge_kernel, dim3(B), dim3(256), 0, st, m));
  GR_LAUNCH_CHECK("mips_topk(merge)");
  return 0;
}

extern "C" int mips_merge_topk(const float* cand_scores, const int64_t* cand_index,
                               const int64_t* cand_ids, int n_lists, int B, int k_in, int k,
                               float* out_scores, int64_t* out_ids, int64_t* out_index,
                               void* stream) {
  GR_REQUIRE(cand_scores && cand_index && cand_ids && out_scores && out_ids,
             "mips_merge_topk: null pointer");
  GR_REQUIRE(k > 0 && k <= 256 && k_in > 0 && n_lists > 0 && (int64_t)n_lists * k_in <= MERGE_MAX,
             "mips_merge_topk: need 0 < k <= 256 and n_lists*k_in <= %d", MERGE_MAX);
  if (B == 0) return 0;
  MergeArgs m{cand_scores, cand_index, cand_ids, n_lists, B, k_in, k, nullptr, 0,
              out_scores, out_ids, out_index, nullptr};
  GR_TIMED("mips_merge", (hipStream_t)stream, hipLaunchKernelGGL(mips_merge_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, m));
  GR_LAUNCH_CHECK("mips_merge_topk");
  return 0;
}
