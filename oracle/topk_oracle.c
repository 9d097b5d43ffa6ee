/*
 * CPU oracle for brute-force MIPS top-k with invalid-id exclusion.
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product path.
 *
 * Restates, in plain C:
 *   reference src/generative_recommenders_pl/models/indexing/top_k.py:44-70
 *     logits = q @ E^T ; topk(k', sorted, largest) ; ids = item_ids[idx]
 *   reference src/generative_recommenders_pl/models/indexing/candidate_index.py:107-164
 *     k' = min(k + N0, X); drop ids present in the row's invalid_ids; keep first k.
 * Fused form (probe-verified equivalent): exclude invalid ids,
 * then take the top-k.  Canonical order: score descending, then catalog index
 * ascending (torch.topk leaves tie order unspecified).
 *
 * Scores are the k-ordered fp32 fmaf chain  acc = fmaf(q[d], e[d], acc), d = 0..D-1,
 * starting from +0.0f — bit-identical to the gfx950 f32 MFMA accumulation used by
 * the HIP kernel (an MFMA 16x16x4 f32 is a k-ordered fmaf chain), so GPU and oracle
 * agree bit-for-bit on scores and hence on the whole ordered top-k.
 *
 * Rows with fewer than k valid candidates (only possible when k + N0 > X, where the
 * reference raises in .view(-1, k)) are padded with score -inf, id -1, index -1.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float s;
    int64_t i;
} cand_t;

/* a ranks better than b */
static inline int better(float as, int64_t ai, float bs, int64_t bi) {
    return (as > bs) || (as == bs && ai < bi);
}

/* min-heap on "better" (root = worst kept) */
static void sift_down(cand_t *h, int n, int p) {
    for (;;) {
        int l = 2 * p + 1, r = l + 1, w = p;
        if (l < n && better(h[w].s, h[w].i, h[l].s, h[l].i)) w = l;
        if (r < n && better(h[w].s, h[w].i, h[r].s, h[r].i)) w = r;
        if (w == p) return;
        cand_t t = h[p]; h[p] = h[w]; h[w] = t; p = w;
    }
}

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

static int cmp_cand(const void *a, const void *b) {
    const cand_t *x = (const cand_t *)a, *y = (const cand_t *)b;
    if (better(x->s, x->i, y->s, y->i)) return -1;
    if (better(y->s, y->i, x->s, x->i)) return 1;
    return 0;
}

static int in_sorted(const int64_t *v, int n, int64_t key) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (v[m] < key) lo = m + 1; else hi = m;
    }
    return lo < n && v[lo] == key;
}

float gr_oracle_dot(const float *q, const float *e, int D) {
    float acc = 0.0f;
    for (int d = 0; d < D; ++d) acc = fmaf(q[d], e[d], acc);
    return acc;
}

/* scores for a (B, X) block, row-major; used by tests on small cases */
void gr_oracle_scores(const float *Q, const float *E, int B, int64_t X, int D, float *out) {
    #pragma omp parallel for schedule(static)
    for (int b = 0; b < B; ++b)
        for (int64_t x = 0; x < X; ++x)
            out[(int64_t)b * X + x] = gr_oracle_dot(Q + (int64_t)b * D, E + x * D, D);
}

/* returns 0 on success */
int gr_oracle_mips_topk(const float *Q, const float *E, const int64_t *item_ids,
                        const int64_t *invalid, int B, int64_t X, int D, int N0, int k,
                        float *scores_out, int64_t *ids_out, int64_t *idx_out) {
    if (k <= 0 || B < 0 || X < 0 || D <= 0) return 1;
    int err = 0;
    #pragma omp parallel
    {
        cand_t *heap = (cand_t *)malloc(sizeof(cand_t) * (size_t)k);
        int64_t *inv = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N0 > 0 ? N0 : 1));
        if (!heap || !inv) err = 2;
        #pragma omp for schedule(dynamic, 1)
        for (int b = 0; b < B; ++b) {
            if (!heap || !inv) continue;
            int n_inv = 0;
            if (invalid && N0 > 0) {
                memcpy(inv, invalid + (int64_t)b * N0, sizeof(int64_t) * (size_t)N0);
                qsort(inv, (size_t)N0, sizeof(int64_t), cmp_i64);
                n_inv = N0;
            }
            const float *q = Q + (int64_t)b * D;
            int n = 0;
            for (int64_t x = 0; x < X; ++x) {
                float s = gr_oracle_dot(q, E + x * D, D);
                if (n == k && !better(s, x, heap[0].s, heap[0].i)) continue;
                int64_t id = item_ids ? item_ids[x] : x;
                if (n_inv && in_sorted(inv, n_inv, id)) continue;
                if (n < k) {
                    heap[n].s = s; heap[n].i = x; ++n;
                    if (n == k)
                        for (int p = k / 2 - 1; p >= 0; --p) sift_down(heap, k, p);
                } else {
                    heap[0].s = s; heap[0].i = x;
                    sift_down(heap, k, 0);
                }
            }
            qsort(heap, (size_t)n, sizeof(cand_t), cmp_cand);
            for (int r = 0; r < k; ++r) {
                int64_t o = (int64_t)b * k + r;
                if (r < n) {
                    scores_out[o] = heap[r].s;
                    idx_out[o] = heap[r].i;
                    ids_out[o] = item_ids ? item_ids[heap[r].i] : heap[r].i;
                } else {
                    scores_out[o] = -INFINITY; idx_out[o] = -1; ids_out[o] = -1;
                }
            }
        }
        free(heap);
        free(inv);
    }
    return err;
}
