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
constexpr int INV_MAX = 256; // max invalid ids per query
constexpr uint32_t VERIFIED = 0x80000000u;

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
};

template <int KS, int BLOCKS>
__global__ __launch_bounds__(ST) void mips_select_kernel(SelectArgs a) {
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
  const int bid = blockIdx.x;
  const int xcd = bid & 7, rest = bid >> 3;
  const int g = rest % n_qg;
  const int range = (rest / n_qg) * 8 + xcd;
  if (range >= a.n_ranges) return;
  const int q0 = g * QG;
  const int64_t x_begin = (int64_t)range * a.range_items;
  const int64_t x_end = min(a.X, x_begin + a.range_items);

  // ---- prologue: sorted invalid lists, counters
  const int n0p = a.N0 > 0 ? (a.N0 <= 64 ? 64 : (a.N0 <= 128 ? 128 : 256)) : 0;
  for (int e = tid; e < QG * n0p; e += ST) {
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
  for (int size = 2; size <= n0p; size <<= 1) {  // bitonic sort, QG independent rows
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
    const int64_t* qinv = inv + qq * INV_MAX;
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
#pragma unroll
    for (int t = 0; t < CAP / 64; ++t) {
      // branchless lower_bound over the sorted (INT64_MAX padded) n0p-entry list
      int pos = 0;
      for (int bit = nbits - 1; bit >= 0; --bit) {
        const int probe = pos + (1 << bit) - 1;
        pos += (qinv[probe] < id[t]) ? (1 << bit) : 0;
      }
      const bool hit = a.N0 > 0 && qinv[pos < n0p ? pos : n0p - 1] == id[t];
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

__global__ __launch_bounds__(256) void mips_merge_kernel(MergeArgs a) {
  __shared__ uint32_t key[MERGE_MAX];
  __shared__ int64_t idx[MERGE_MAX];
  __shared__ int hist[256];
  __shared__ int sh_digit, sh_above;
  __shared__ uint32_t s_key[256];
  __shared__ int64_t s_idx[256];
  __shared__ int s_src[256];
  __shared__ int s_cnt;
  __shared__ int red[4];
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int M = a.n_lists * a.k_in;
  auto src_of = [&](int e) -> int64_t {
    const int l = e / a.k_in, j = e - l * a.k_in;
    return ((int64_t)l * a.B + q) * a.k_in + j;
  };
  int nvalid = 0;
  for (int e = tid; e < M; e += 256) {
    const int64_t s = src_of(e);
    const int64_t gi = a.cand_index[s];
    const bool ok = gi >= 0;
    key[e] = ok ? ord_key(a.cand_score[s]) : 0u;
    idx[e] = ok ? gi : INT64_MAX;
    nvalid += ok;
  }
  int v = nvalid;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  const int tot = red[0] + red[1] + red[2] + red[3];
  const int kk = a.k;
  uint32_t kstar = 0u;
  int k_rem = 0;
  const bool all = tot <= kk;
  if (!all) {
    uint32_t prefix = 0, mask = 0;
    int need = kk;
    for (int shift = 24; shift >= 0; shift -= 8) {
      hist[tid] = 0;
      __syncthreads();
      for (int e = tid; e < M; e += 256) {
        const uint32_t x = key[e];
        if (x != 0u && (x & mask) == prefix) atomicAdd(&hist[(x >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid < 64) hist_find_digit(hist, need, &sh_digit, &sh_above);
      __syncthreads();
      prefix |= (uint32_t)sh_digit << shift;
      mask |= 0xFFu << shift;
      need -= sh_above;
    }
    kstar = prefix;
    k_rem = need;
  }
  // ties at kstar: count them; if more than k_rem, keep the smallest indices
  int eq = 0;
  if (!all)
    for (int e = tid; e < M; e += 256) eq += key[e] == kstar;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) eq += __shfl_xor(eq, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = eq;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const int eq_tot = red[0] + red[1] + red[2] + red[3];
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
      const int p = atomicAdd(&s_cnt, 1);
      s_key[p] = x;
      s_idx[p] = idx[e];
      s_src[p] = e;
    }
  }
  __syncthreads();
  const int n = s_cnt;
  for (int p = n + tid; p < 256; p += 256) {
    s_key[p] = 0u;
    s_idx[p] = INT64_MAX;
    s_src[p] = -1;
  }
  __syncthreads();
  // bitonic sort 256 entries: key desc, then catalog index asc
  for (int size = 2; size <= 256; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int i = tid;
      const int j = i ^ stride;
      if (j > i) {
        const uint32_t ki = s_key[i], kj = s_key[j];
        const int64_t ii = s_idx[i], ij = s_idx[j];
        const bool i_first = (ki > kj) || (ki == kj && ii < ij);
        const bool asc = (i & size) == 0;
        if (i_first != asc) {
          s_key[i] = kj;
          s_key[j] = ki;
          s_idx[i] = ij;
          s_idx[j] = ii;
          const int t = s_src[i];
          s_src[i] = s_src[j];
          s_src[j] = t;
        }
      }
      __syncthreads();
    }
  }
  for (int r = tid; r < kk; r += 256) {
    const int64_t o = (int64_t)q * kk + r;
    if (r < n) {
      const int64_t s = src_of(s_src[r]);
      const int64_t gi = s_idx[r];
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
// X <= MERGE_MAX: a workgroup per query scores every item (the same k-ordered fmaf chain,
// read from the packed layout), excludes its invalid ids (arange ids: direct index
// scatter after the scores are written; explicit ids: binary search in the sorted list)
// and hands all X scores to the merge kernel as one candidate list.  Replaces the
// range/threshold machinery, whose fixed per-workgroup costs dominate at ml-1m sizes.
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
};

template <int KS2>
__global__ __launch_bounds__(256) void mips_scoreall_kernel(ScoreAllArgs a) {
  __shared__ float qv[8 * KS2];
  __shared__ int64_t inv[INV_MAX];
  const int q = blockIdx.x, tid = threadIdx.x;
  for (int d = tid; d < 8 * KS2; d += 256) qv[d] = d < a.D ? a.q[(int64_t)q * a.D + d] : 0.f;
  const bool search = a.item_ids && a.N0 > 0;
  const int n0p = a.N0 <= 64 ? 64 : (a.N0 <= 128 ? 128 : 256);
  if (search) {
    for (int j = tid; j < n0p; j += 256) inv[j] = j < a.N0 ? a.invalid[(int64_t)q * a.N0 + j] : INT64_MAX;
    __syncthreads();
    for (int size = 2; size <= n0p; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int p = tid; p < n0p / 2; p += 256) {
          const int i = 2 * p - (p & (stride - 1)), j = i + stride;
          const bool up = (i & size) == 0;
          const int64_t x = inv[i], y = inv[j];
          if ((x > y) == up) {
            inv[i] = y;
            inv[j] = x;
          }
        }
        __syncthreads();
      }
  }
  __syncthreads();
  typedef float fv2 __attribute__((ext_vector_type(2)));
  gptr<fv2> pk = as_global(reinterpret_cast<const fv2*>(a.packed));
  float* os = a.out_score + (int64_t)q * a.X;
  int64_t* oi = a.out_index + (int64_t)q * a.X;
  for (int64_t i = tid; i < a.X; i += 256) {
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
    if (search) ok = !sorted_contains(inv, a.N0 > 0 ? n0p : 0, a.item_ids[i]);
    os[i] = ok ? sc : -INFINITY;
    oi[i] = ok ? a.index_base + i : -1;
  }
  if (!a.item_ids && a.N0 > 0) {  // arange ids: exclude by direct index
    __syncthreads();
    for (int j = tid; j < a.N0; j += 256) {
      const int64_t li = a.invalid[(int64_t)q * a.N0 + j] - a.index_base;
      if (li >= 0 && li < a.X) {
        os[li] = -INFINITY;
        oi[li] = -1;
      }
    }
  }
}

struct TopkPlan {
  bool small;
  int KS, n_ranges, k_part;
  int64_t range_items;
  size_t part_bytes;
};

static TopkPlan plan_topk(int B, int64_t X, int D, int k) {
  TopkPlan p;
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
  return p;
}

template <int KS>
static int launch_select(const SelectArgs& a, hipStream_t st) {
  constexpr int BLOCKS = KS <= 16 ? 2 : 1;  // SW * 16 * BLOCKS <= CAP - 256
  const int n_qg = ceil_div(a.B, QG);
  const int n_r8 = ceil_div(a.n_ranges, 8) * 8;
  const int grid = n_r8 * n_qg;
  GR_TIMED("mips_select", st, hipLaunchKernelGGL((mips_select_kernel<KS, BLOCKS>), dim3(grid), dim3(ST), 0, st, a));
  GR_LAUNCH_CHECK("mips_topk(select)");
  return 0;
}

}  // namespace gr

using namespace gr;

extern "C" size_t mips_packed_items_bytes(int64_t X, int D) {
  const int KS2 = (ceil_div(D, 4) + 1) / 2;
  return sizeof(float) * (size_t)((X + 15) / 16) * KS2 * 128;
}

extern "C" int mips_pack_items(const float* items, int64_t X, int D, float* packed, void* stream) {
  GR_REQUIRE(items && packed && X >= 0 && D > 0, "mips_pack_items: bad args");
  if (X == 0) return 0;
  const int KS2 = (ceil_div(D, 4) + 1) / 2;
  GR_TIMED("mips_pack", (hipStream_t)stream, hipLaunchKernelGGL(pack_items_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, items, X,
                     D, KS2, packed));
  GR_LAUNCH_CHECK("mips_pack_items");
  return 0;
}

extern "C" size_t mips_topk_workspace_size(int B, int64_t X, int D, int k) {
  if (B <= 0 || X <= 0 || D <= 0 || k <= 0) return 0;
  return plan_topk(B, X, D, k).part_bytes;
}

extern "C" int mips_topk(const float* queries, const float* packed_items, int64_t X, int D,
                         const int64_t* item_ids, int64_t index_base, const int64_t* invalid_ids,
                         int N0, int B, int k, float* out_scores, int64_t* out_ids,
                         int64_t* out_index, void* workspace, size_t ws_bytes, void* stream) {
  GR_REQUIRE(queries && packed_items && out_scores && out_ids, "mips_topk: null pointer");
  GR_REQUIRE(B >= 0 && X >= 0 && D > 0 && D <= 256, "mips_topk: D=%d not in [1, 256]", D);
  GR_REQUIRE(k > 0 && k <= 256, "mips_topk: k=%d not in [1, 256]", k);
  GR_REQUIRE(N0 >= 0 && N0 <= INV_MAX && (N0 == 0 || invalid_ids),
             "mips_topk: N0=%d not in [0, %d] (or invalid_ids null)", N0, INV_MAX);
  GR_REQUIRE(X < 0x7FFFFFFF, "mips_topk: X must be < 2^31 per shard");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0) return 0;
  TopkPlan p = plan_topk(B, X > 0 ? X : 1, D, k);
  GR_REQUIRE(workspace && ws_bytes >= p.part_bytes, "mips_topk: workspace %zu B < %zu B", ws_bytes,
             p.part_bytes);
  if (p.small) {
    float* sc = (float*)workspace;
    int64_t* ix = (int64_t*)(sc + (size_t)B * X);
    ScoreAllArgs s{queries, packed_items, X, D, B, N0, item_ids, index_base, invalid_ids, sc, ix};
    const int KS2 = (p.KS + 1) / 2;
#define GR_SA(K2)                                                                           \
  case K2:                                                                                  \
    GR_TIMED("mips_select", st, hipLaunchKernelGGL(mips_scoreall_kernel<K2>, dim3(B), dim3(256), 0, st, s)); \
    break;
    switch (KS2) {
      GR_SA(1) GR_SA(2) GR_SA(3) GR_SA(4) GR_SA(5) GR_SA(6) GR_SA(7) GR_SA(8)
      default: GR_REQUIRE(false, "mips_topk: score-all path needs D <= 64");
    }
#undef GR_SA
    GR_LAUNCH_CHECK("mips_topk(score-all)");
    MergeArgs m{sc, ix, nullptr, 1, B, (int)X, k, item_ids, index_base,
                out_scores, out_ids, out_index};
    GR_TIMED("mips_merge", st, hipLaunchKernelGGL(mips_merge_kernel, dim3(B), dim3(256), 0, st, m));
    GR_LAUNCH_CHECK("mips_topk(merge)");
    return 0;
  }
  float* part_score = (float*)workspace;
  int64_t* part_index = (int64_t*)(part_score + (size_t)p.n_ranges * B * p.k_part);
  SelectArgs a{queries, packed_items, X, D, B, k, N0, p.n_ranges, p.k_part, p.range_items,
               item_ids, index_base, invalid_ids, part_score, part_index};
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
              out_scores, out_ids, out_index};
  GR_TIMED("mips_merge", st, hipLaunchKernelGGL(mips_merge_kernel, dim3(B), dim3(256), 0, st, m));
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
              out_scores, out_ids, out_index};
  GR_TIMED("mips_merge", (hipStream_t)stream, hipLaunchKernelGGL(mips_merge_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, m));
  GR_LAUNCH_CHECK("mips_merge_topk");
  return 0;
}
