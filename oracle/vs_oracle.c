/*
 * vs_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Nothing in the product path (photo_search_engine_amd/) may link, load or call this file.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the reported CPU number.
 *
 * What it restates (see DESIGN.md "Oracle"):
 *
 *   1. faiss IndexFlatIP / IndexFlatL2 search semantics as the reference drives them
 *      (/root/reference/utils/vector_store.py:79-81 builds the index, :164 adds, :191 searches).
 *      faiss itself (faiss-cpu>=1.7.0, /root/reference/requirements.txt:5) is a third-party
 *      dependency that is NOT vendored under /root/reference and NOT installed here, so its
 *      published algorithm is restated:
 *        - knn_inner_product / knn_L2sqr: nq < 20 -> per query, rows scanned j = 0..N-1 with
 *          fvec_inner_product / fvec_L2sqr (AVX2: 8 fp32 lanes, mul+add, horizontal hadd) and a
 *          size-k heap (min-heap for IP, max-heap for L2) that replaces its top only on a
 *          STRICT improvement; nq >= 20 -> blocked sgemm (4096 queries x 1024 rows) + the same
 *          heap update; heap_reorder sorts the result. Effective order: score desc (IP) / asc
 *          (L2), ties -> lower id. Unfilled slots: id -1, score -FLT_MAX (IP) / +FLT_MAX (L2).
 *        -> orc_knn_faiss_fp32()  (also the CPU baseline, kind "port").
 *   2. The CANONICAL EXACT score used for bit-exact parity of the HIP path:
 *        IP:  S = sum_i (double)x_i * (double)q_i
 *        L2:  S = sum_i ((double)x_i - (double)q_i)^2   (difference rounded, square rounded)
 *      accumulated in fp64 in a fixed order: element i goes to lane (i >> 3) & 63, each lane sums
 *      its elements in increasing i, then an xor-butterfly over lanes with strides 32,16,8,4,2,1.
 *      The HIP refine kernel evaluates exactly this expression tree, so scores agree bit for bit
 *      and the top-k ids (score desc / asc, ties -> lower id) agree exactly.
 *        -> orc_knn_exact()
 *   3. The synthetic corpus/query generator (counter-based splitmix64 hash, 4 x 22-bit uniforms,
 *      canonical fp32 row normalisation, RNE cast to bf16/f16) that the HIP generator reproduces
 *      bit for bit.   -> orc_synth_rows()
 *
 * Build: oracle/Makefile (gcc -O3 -fopenmp -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_METRIC_IP 0
#define ORC_METRIC_L2 1
#define ORC_DTYPE_F32 0
#define ORC_DTYPE_BF16 1
#define ORC_DTYPE_F16 2

int orc_version(void) { return 3; }

/* ------------------------------------------------------------------------------------------ */
/* bit helpers                                                                                 */
/* ------------------------------------------------------------------------------------------ */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = f2u(f);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x40u); /* quiet NaN */
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static inline float bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

static inline uint16_t f32_to_f16_rne(float f) {
    uint32_t x = f2u(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return (uint16_t)(sign | (ax > 0x7F800000u ? 0x7E00u : 0x7C00u));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u); /* >= 65520 -> inf */
    if (ax < 0x38800000u) {                                    /* below 2^-14: subnormal/zero */
        float v = u2f(ax) * 16777216.0f;                       /* exact: scale by 2^24 */
        return (uint16_t)(sign | (uint32_t)rintf(v));          /* RNE (default rounding mode) */
    }
    uint32_t e = (ax >> 23) - 127u + 15u;
    uint32_t mant = ax & 0x7FFFFFu;
    uint32_t r = (e << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) r++;
    return (uint16_t)(sign | r);
}
static inline float f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0) {
        float v = (float)m * (1.0f / 16777216.0f); /* m * 2^-24, exact */
        return sign ? -v : v;
    }
    if (e == 31) return u2f(sign | 0x7F800000u | (m << 13));
    return u2f(sign | ((e - 15u + 127u) << 23) | (m << 13));
}

static inline float round_to_dtype(float f, int dtype) {
    if (dtype == ORC_DTYPE_BF16) return bf16_to_f32(f32_to_bf16_rne(f));
    if (dtype == ORC_DTYPE_F16) return f16_to_f32(f32_to_f16_rne(f));
    return f;
}

/* Round an fp32 array to the storage dtype and back (the values the GPU index holds). */
void orc_round_dtype(const float* in, int64_t n, int dtype, float* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) out[i] = round_to_dtype(in[i], dtype);
}
void orc_to_bf16_bits(const float* in, int64_t n, uint16_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = f32_to_bf16_rne(in[i]);
}
void orc_to_f16_bits(const float* in, int64_t n, uint16_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = f32_to_f16_rne(in[i]);
}

/* ------------------------------------------------------------------------------------------ */
/* synthetic data                                                                              */
/* ------------------------------------------------------------------------------------------ */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
#define SYNTH_SCALE ((float)(1.7320508075688772 / 4194304.0)) /* sqrt(3) / 2^22 -> unit variance */

/* raw ~N(0,1) value of element (row, col): sum of four 22-bit uniforms, exact in fp32 */
static inline float synth_raw(uint64_t base, uint64_t ctr) {
    uint64_t h1 = splitmix64(base + 2u * ctr);
    uint64_t h2 = splitmix64(base + 2u * ctr + 1u);
    uint32_t a = (uint32_t)(h1 & 0x3FFFFFu), b = (uint32_t)((h1 >> 22) & 0x3FFFFFu);
    uint32_t c = (uint32_t)(h2 & 0x3FFFFFu), d = (uint32_t)((h2 >> 22) & 0x3FFFFFu);
    int32_t s = (int32_t)(a + b + c + d) - (1 << 23);
    return (float)s * SYNTH_SCALE;
}

/* Rows [row0, row0+n) of the synthetic matrix with d columns, optionally L2-normalised with the
 * canonical fp32 order (lane = i & 63, fmaf per lane, xor-butterfly 32..1, sqrtf, divide), then
 * rounded to `dtype` and returned as fp32 (out is n x d, row-major). */
void orc_synth_rows(uint64_t seed, int64_t row0, int64_t n, int d, int normalize, int dtype, float* out) {
    const uint64_t base = splitmix64(seed);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        float* v = out + r * (int64_t)d;
        const uint64_t rowctr = (uint64_t)(row0 + r) * (uint64_t)d;
        for (int i = 0; i < d; ++i) v[i] = synth_raw(base, rowctr + (uint64_t)i);
        if (normalize) {
            float part[64];
            for (int j = 0; j < 64; ++j) part[j] = 0.0f;
            for (int i = 0; i < d; ++i) part[i & 63] = fmaf(v[i], v[i], part[i & 63]);
            for (int s = 32; s >= 1; s >>= 1) {
                float t[64];
                for (int j = 0; j < 64; ++j) t[j] = part[j] + part[j ^ s];
                memcpy(part, t, sizeof(t));
            }
            float nrm = sqrtf(part[0]);
            if (nrm != 0.0f)
                for (int i = 0; i < d; ++i) v[i] = v[i] / nrm;
        }
        if (dtype != ORC_DTYPE_F32)
            for (int i = 0; i < d; ++i) v[i] = round_to_dtype(v[i], dtype);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* canonical exact scores (fp64, fixed expression tree shared with the HIP refine kernel)       */
/* ------------------------------------------------------------------------------------------ */
static inline double butterfly64(double* part) {
    for (int s = 32; s >= 1; s >>= 1) {
        double t[64];
        for (int j = 0; j < 64; ++j) t[j] = part[j] + part[j ^ s];
        memcpy(part, t, sizeof(t));
    }
    return part[0];
}
static inline double canon_score(const float* x, const float* q, int d, int metric) {
    double part[64];
    for (int j = 0; j < 64; ++j) part[j] = 0.0;
    if (metric == ORC_METRIC_IP) {
        for (int i = 0; i < d; ++i) {
            double p = (double)x[i] * (double)q[i]; /* exact (24b x 24b < 53b) */
            part[(i >> 3) & 63] = part[(i >> 3) & 63] + p;
        }
    } else {
        for (int i = 0; i < d; ++i) {
            double dl = (double)x[i] - (double)q[i];
            double p = dl * dl;
            part[(i >> 3) & 63] = part[(i >> 3) & 63] + p;
        }
    }
    return butterfly64(part);
}

void orc_canon_scores(const float* x, int64_t N, int d, const float* q, int64_t nq, int metric, double* S) {
#pragma omp parallel for schedule(static) collapse(2)
    for (int64_t a = 0; a < nq; ++a)
        for (int64_t j = 0; j < N; ++j) S[a * N + j] = canon_score(x + j * (int64_t)d, q + a * (int64_t)d, d, metric);
}

/* "a is better than b": IP larger first, L2 smaller first, ties -> lower id. */
static inline int better(double sa, int64_t ia, double sb, int64_t ib, int metric) {
    if (sa != sb) return metric == ORC_METRIC_IP ? (sa > sb) : (sa < sb);
    return ia < ib;
}

/* size-k heap whose root is the WORST kept element under `better` */
typedef struct { double* s; int64_t* id; int n, k, metric; } xheap;
static void xheap_sift_down(xheap* h, int i) {
    for (;;) {
        int l = 2 * i + 1, r = l + 1, w = i;
        if (l < h->n && better(h->s[w], h->id[w], h->s[l], h->id[l], h->metric)) w = l;
        if (r < h->n && better(h->s[w], h->id[w], h->s[r], h->id[r], h->metric)) w = r;
        if (w == i) return;
        double ts = h->s[i]; h->s[i] = h->s[w]; h->s[w] = ts;
        int64_t ti = h->id[i]; h->id[i] = h->id[w]; h->id[w] = ti;
        i = w;
    }
}
static void xheap_push(xheap* h, double s, int64_t id) {
    if (h->n < h->k) {
        int i = h->n++;
        h->s[i] = s; h->id[i] = id;
        while (i > 0) {
            int p = (i - 1) / 2;
            if (better(h->s[p], h->id[p], h->s[i], h->id[i], h->metric)) {
                double ts = h->s[i]; h->s[i] = h->s[p]; h->s[p] = ts;
                int64_t ti = h->id[i]; h->id[i] = h->id[p]; h->id[p] = ti;
                i = p;
            } else break;
        }
    } else if (better(s, id, h->s[0], h->id[0], h->metric)) {
        h->s[0] = s; h->id[0] = id;
        xheap_sift_down(h, 0);
    }
}
/* pop everything: writes best-first into outS/outI (length n) */
static void xheap_drain(xheap* h, double* outS, int64_t* outI) {
    int n = h->n;
    for (int pos = n - 1; pos >= 0; --pos) {
        outS[pos] = h->s[0]; outI[pos] = h->id[0];
        h->n--;
        h->s[0] = h->s[h->n]; h->id[0] = h->id[h->n];
        xheap_sift_down(h, 0);
    }
}

/* Exact top-k under the canonical fp64 score. S/I are nq x k; unfilled: I = -1,
 * S = -DBL_MAX (IP) / +DBL_MAX (L2). Parallel over row blocks, merged deterministically. */
void orc_knn_exact(const float* x, int64_t N, int d, const float* q, int64_t nq, int k, int metric,
                   double* S, int64_t* I) {
    int nthr = 1;
#ifdef _OPENMP
    nthr = omp_get_max_threads();
#endif
    double* hs = (double*)malloc(sizeof(double) * (size_t)k * (size_t)nthr);
    int64_t* hi = (int64_t*)malloc(sizeof(int64_t) * (size_t)k * (size_t)nthr);
    int* hn = (int*)malloc(sizeof(int) * (size_t)nthr);
    for (int64_t a = 0; a < nq; ++a) {
        const float* qa = q + a * (int64_t)d;
#pragma omp parallel
        {
            int t = 0, nt = 1;
#ifdef _OPENMP
            t = omp_get_thread_num(); nt = omp_get_num_threads();
#endif
            xheap h = {hs + (size_t)t * k, hi + (size_t)t * k, 0, k, metric};
            int64_t lo = N * t / nt, hi_ = N * (t + 1) / nt;
            for (int64_t j = lo; j < hi_; ++j) xheap_push(&h, canon_score(x + j * (int64_t)d, qa, d, metric), j);
            hn[t] = h.n;
        }
        xheap m = {S + a * k, I + a * k, 0, k, metric};
        double* tmpS = (double*)malloc(sizeof(double) * (size_t)k);
        int64_t* tmpI = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
        for (int t = 0; t < nthr; ++t)
            for (int e = 0; e < hn[t]; ++e) xheap_push(&m, hs[(size_t)t * k + e], hi[(size_t)t * k + e]);
        int got = m.n;
        xheap_drain(&m, tmpS, tmpI);
        for (int e = 0; e < k; ++e) {
            if (e < got) { S[a * k + e] = tmpS[e]; I[a * k + e] = tmpI[e]; }
            else { S[a * k + e] = metric == ORC_METRIC_IP ? -DBL_MAX : DBL_MAX; I[a * k + e] = -1; }
        }
        free(tmpS); free(tmpI);
    }
    free(hs); free(hi); free(hn);
}

/* Merge G sorted per-shard lists (each nq x k, ids already global) into the global top-k:
 * the K3 / all-gather merge restated. */
void orc_merge_topk(const double* S_in, const int64_t* I_in, int G, int64_t nq, int k, int metric,
                    double* S, int64_t* I) {
    double* tmpS = (double*)malloc(sizeof(double) * (size_t)k);
    int64_t* tmpI = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
    for (int64_t a = 0; a < nq; ++a) {
        xheap m = {S + a * k, I + a * k, 0, k, metric};
        for (int g = 0; g < G; ++g)
            for (int e = 0; e < k; ++e) {
                int64_t id = I_in[((int64_t)g * nq + a) * k + e];
                if (id >= 0) xheap_push(&m, S_in[((int64_t)g * nq + a) * k + e], id);
            }
        int got = m.n;
        xheap_drain(&m, tmpS, tmpI);
        for (int e = 0; e < k; ++e) {
            if (e < got) { S[a * k + e] = tmpS[e]; I[a * k + e] = tmpI[e]; }
            else { S[a * k + e] = metric == ORC_METRIC_IP ? -DBL_MAX : DBL_MAX; I[a * k + e] = -1; }
        }
    }
    free(tmpS); free(tmpI);
}

/* ------------------------------------------------------------------------------------------ */
/* faiss fp32 restatement (also the CPU baseline, kind "port")                                 */
/* ------------------------------------------------------------------------------------------ */
typedef float v8f __attribute__((vector_size(32)));

/* faiss fvec_inner_product (AVX2 form): 8 fp32 lanes, mul then add, hadd reduction */
static inline float fvec_ip(const float* x, const float* y, int d) {
    v8f acc = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 8 <= d; i += 8) {
        v8f a, b;
        memcpy(&a, x + i, 32); memcpy(&b, y + i, 32);
        acc = acc + a * b;
    }
    float m0 = acc[0] + acc[4], m1 = acc[1] + acc[5], m2 = acc[2] + acc[6], m3 = acc[3] + acc[7];
    float s = (m0 + m1) + (m2 + m3);
    for (; i < d; ++i) s += x[i] * y[i];
    return s;
}
static inline float fvec_l2(const float* x, const float* y, int d) {
    v8f acc = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 8 <= d; i += 8) {
        v8f a, b;
        memcpy(&a, x + i, 32); memcpy(&b, y + i, 32);
        v8f t = a - b;
        acc = acc + t * t;
    }
    float m0 = acc[0] + acc[4], m1 = acc[1] + acc[5], m2 = acc[2] + acc[6], m3 = acc[3] + acc[7];
    float s = (m0 + m1) + (m2 + m3);
    for (; i < d; ++i) { float t = x[i] - y[i]; s += t * t; }
    return s;
}

/* faiss float heap: root = worst kept; replace only on a STRICT improvement; ties of equal
 * score resolve to the lower id because rows arrive in increasing id order per (thread) range
 * and the final merge breaks ties by id (faiss CMin/CMax cmp2). */
typedef struct { float* s; int64_t* id; int n, k, metric; } fheap;
static inline int fbetter(float sa, int64_t ia, float sb, int64_t ib, int metric) {
    if (sa != sb) return metric == ORC_METRIC_IP ? (sa > sb) : (sa < sb);
    return ia < ib;
}
static void fheap_sift_down(fheap* h, int i) {
    for (;;) {
        int l = 2 * i + 1, r = l + 1, w = i;
        if (l < h->n && fbetter(h->s[w], h->id[w], h->s[l], h->id[l], h->metric)) w = l;
        if (r < h->n && fbetter(h->s[w], h->id[w], h->s[r], h->id[r], h->metric)) w = r;
        if (w == i) return;
        float ts = h->s[i]; h->s[i] = h->s[w]; h->s[w] = ts;
        int64_t ti = h->id[i]; h->id[i] = h->id[w]; h->id[w] = ti;
        i = w;
    }
}
static inline void fheap_push(fheap* h, float s, int64_t id) {
    if (h->n < h->k) {
        int i = h->n++;
        h->s[i] = s; h->id[i] = id;
        while (i > 0) {
            int p = (i - 1) / 2;
            if (fbetter(h->s[p], h->id[p], h->s[i], h->id[i], h->metric)) {
                float ts = h->s[i]; h->s[i] = h->s[p]; h->s[p] = ts;
                int64_t ti = h->id[i]; h->id[i] = h->id[p]; h->id[p] = ti;
                i = p;
            } else break;
        }
    } else {
        int improves = h->metric == ORC_METRIC_IP ? (s > h->s[0]) : (s < h->s[0]); /* strict */
        if (improves) { h->s[0] = s; h->id[0] = id; fheap_sift_down(h, 0); }
    }
}
static void fheap_drain(fheap* h, float* outS, int64_t* outI) {
    int n = h->n;
    for (int pos = n - 1; pos >= 0; --pos) {
        outS[pos] = h->s[0]; outI[pos] = h->id[0];
        h->n--;
        h->s[0] = h->s[h->n]; h->id[0] = h->id[h->n];
        fheap_sift_down(h, 0);
    }
}

/* sgemm-like block: out[a][j] = <q_a, x_j> for a < na, j < nb (fp32, 4x2 register tiles). */
static void ip_block(const float* q, int na, const float* x, int nb, int d, float* out, int ldo) {
    int a = 0;
    for (; a + 4 <= na; a += 4) {
        const float* q0 = q + (int64_t)a * d;
        const float* q1 = q0 + d; const float* q2 = q1 + d; const float* q3 = q2 + d;
        int j = 0;
        for (; j + 2 <= nb; j += 2) {
            const float* x0 = x + (int64_t)j * d; const float* x1 = x0 + d;
            v8f c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0}, c20 = {0}, c21 = {0}, c30 = {0}, c31 = {0};
            int i = 0;
            for (; i + 8 <= d; i += 8) {
                v8f b0, b1, a0, a1, a2, a3;
                memcpy(&b0, x0 + i, 32); memcpy(&b1, x1 + i, 32);
                memcpy(&a0, q0 + i, 32); memcpy(&a1, q1 + i, 32); memcpy(&a2, q2 + i, 32); memcpy(&a3, q3 + i, 32);
                c00 += a0 * b0; c01 += a0 * b1; c10 += a1 * b0; c11 += a1 * b1;
                c20 += a2 * b0; c21 += a2 * b1; c30 += a3 * b0; c31 += a3 * b1;
            }
            v8f* cs[8] = {&c00, &c01, &c10, &c11, &c20, &c21, &c30, &c31};
            for (int t = 0; t < 8; ++t) {
                v8f c = *cs[t];
                float m0 = c[0] + c[4], m1 = c[1] + c[5], m2 = c[2] + c[6], m3 = c[3] + c[7];
                float s = (m0 + m1) + (m2 + m3);
                int aa = a + t / 2, jj = j + (t & 1);
                for (int ii = i; ii < d; ++ii) s += q[(int64_t)aa * d + ii] * x[(int64_t)jj * d + ii];
                out[(int64_t)aa * ldo + jj] = s;
            }
        }
        for (; j < nb; ++j)
            for (int t = 0; t < 4; ++t) out[(int64_t)(a + t) * ldo + j] = fvec_ip(q + (int64_t)(a + t) * d, x + (int64_t)j * d, d);
    }
    for (; a < na; ++a)
        for (int j = 0; j < nb; ++j) out[(int64_t)a * ldo + j] = fvec_ip(q + (int64_t)a * d, x + (int64_t)j * d, d);
}

/* faiss IndexFlat{IP,L2}::search restated on fp32.  D/I are nq x k.  nthreads <= 0 -> all. */
void orc_knn_faiss_fp32(const float* x, int64_t N, int d, const float* q, int64_t nq, int k, int metric,
                        int nthreads, float* D, int64_t* I) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    int nthr = omp_get_max_threads();
#else
    int nthr = 1; (void)nthreads;
#endif
    const float worst = metric == ORC_METRIC_IP ? -FLT_MAX : FLT_MAX;
    if (nq < 20) {
        /* sequential path: faiss parallelises over queries only */
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t a = 0; a < nq; ++a) {
            float* hs = (float*)malloc(sizeof(float) * (size_t)k);
            int64_t* hi = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
            fheap h = {hs, hi, 0, k, metric};
            const float* qa = q + a * (int64_t)d;
            for (int64_t j = 0; j < N; ++j) {
                float s = metric == ORC_METRIC_IP ? fvec_ip(x + j * (int64_t)d, qa, d) : fvec_l2(x + j * (int64_t)d, qa, d);
                fheap_push(&h, s, j);
            }
            int got = h.n;
            fheap_drain(&h, D + a * k, I + a * k);
            for (int e = got; e < k; ++e) { D[a * k + e] = worst; I[a * k + e] = -1; }
            free(hs); free(hi);
        }
        return;
    }
    /* BLAS path: blocks of 4096 queries x 1024 rows; every thread owns a row range and its own
     * heaps, merged at the end (same result set as faiss' shared heaps). */
    const int BQ = 4096, BR = 1024;
    float* qn = NULL;
    float* xn = NULL;
    if (metric == ORC_METRIC_L2) {
        qn = (float*)malloc(sizeof(float) * (size_t)nq);
        xn = (float*)malloc(sizeof(float) * (size_t)N);
        for (int64_t a = 0; a < nq; ++a) qn[a] = fvec_ip(q + a * (int64_t)d, q + a * (int64_t)d, d);
#pragma omp parallel for schedule(static)
        for (int64_t j = 0; j < N; ++j) xn[j] = fvec_ip(x + j * (int64_t)d, x + j * (int64_t)d, d);
    }
    for (int64_t a0 = 0; a0 < nq; a0 += BQ) {
        int na = (int)((nq - a0) < BQ ? (nq - a0) : BQ);
        float* hs = (float*)malloc(sizeof(float) * (size_t)nthr * na * k);
        int64_t* hid = (int64_t*)malloc(sizeof(int64_t) * (size_t)nthr * na * k);
        int* hn = (int*)calloc((size_t)nthr * na, sizeof(int));
#pragma omp parallel
        {
            int t = 0, nt = 1;
#ifdef _OPENMP
            t = omp_get_thread_num(); nt = omp_get_num_threads();
#endif
            float* blk = (float*)malloc(sizeof(float) * (size_t)na * BR);
            int64_t nblk = (N + BR - 1) / BR;
            int64_t b_lo = nblk * t / nt, b_hi = nblk * (t + 1) / nt;
            for (int64_t b = b_lo; b < b_hi; ++b) {
                int64_t j0 = b * BR;
                int nb = (int)((N - j0) < BR ? (N - j0) : BR);
                ip_block(q + a0 * d, na, x + j0 * d, nb, d, blk, BR);
                for (int aa = 0; aa < na; ++aa) {
                    fheap h = {hs + ((size_t)t * na + aa) * k, hid + ((size_t)t * na + aa) * k,
                               hn[(size_t)t * na + aa], k, metric};
                    const float* row = blk + (int64_t)aa * BR;
                    for (int jj = 0; jj < nb; ++jj) {
                        float s = row[jj];
                        if (metric == ORC_METRIC_L2) s = qn[a0 + aa] + xn[j0 + jj] - 2.0f * s;
                        fheap_push(&h, s, j0 + jj);
                    }
                    hn[(size_t)t * na + aa] = h.n;
                }
            }
            free(blk);
        }
#pragma omp parallel for schedule(static)
        for (int aa = 0; aa < na; ++aa) {
            float* ms = (float*)malloc(sizeof(float) * (size_t)k);
            int64_t* mi = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
            fheap m = {ms, mi, 0, k, metric};
            for (int t = 0; t < nthr; ++t)
                for (int e = 0; e < hn[(size_t)t * na + aa]; ++e) {
                    float s = hs[((size_t)t * na + aa) * k + e];
                    int64_t id = hid[((size_t)t * na + aa) * k + e];
                    /* tie-aware merge (faiss heaps compare (score, id) via cmp2) */
                    if (m.n < m.k) fheap_push(&m, s, id);
                    else if (fbetter(s, id, m.s[0], m.id[0], metric)) { m.s[0] = s; m.id[0] = id; fheap_sift_down(&m, 0); }
                }
            int got = m.n;
            fheap_drain(&m, D + (a0 + aa) * k, I + (a0 + aa) * k);
            for (int e = got; e < k; ++e) { D[(a0 + aa) * k + e] = worst; I[(a0 + aa) * k + e] = -1; }
            free(ms); free(mi);
        }
        free(hs); free(hid); free(hn);
    }
    free(qn); free(xn);
}

/* number of OpenMP threads the oracle will use */
int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
