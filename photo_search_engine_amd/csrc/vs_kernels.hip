// vs_kernels.hip -- gfx950 (CDNA4) kernels of the exact flat k-NN backend.
//
// Pipeline of one search:
//   pack_q  -> screen (K1 MFMA bf16/f16, or K2 GEMV) -> merge (K3, 1-2 stages) -> refine (K5)
//
//   screen: streams the shard once from HBM, computes fp32 scores (bf16/f16 MFMA, or fp32 FMA),
//           and keeps per (workgroup, query) the top-Kp candidates by a running threshold;
//           survivors are rare after the first tiles, so the score matrix never leaves registers.
//   merge:  block-wide radix-bisection select of the best Kp keys of many partial lists.
//   refine: exact fp64 rescoring of the Kp survivors in the canonical expression tree
//           (oracle/vs_oracle.c canon_score), sort, exactness certificate, faiss-layout output.
//
// Candidate key (u64): (orderable fp32 score << 32) | (0xFFFFFFFF - local row id); larger is
// better, equal score -> lower id (faiss' effective tie order), 0 = empty.
#include "vs_internal.h"

#include <math.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <set>
#include <utility>

#include "vs_device.h"

namespace vs {

// ------------------------------------------------------------------------------------------------
// ingest: pack host/device fp32 rows into the tiled layout; synthetic rows; unpack
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t tiled_off(int64_t row, int i, int dpad, int es) {
    const int ce = CHB / es;  // (es is a compile-time constant at every call)
    return (row / TR) * (int64_t)TR * dpad * es + (int64_t)(i / ce) * TR * CHB + (row % TR) * CHB +
           (int64_t)(i % ce) * es;
}

// one wave per row; element i handled by lane i & 63 (the canonical fp32 order for sqn)
template <int DT>
__global__ void __launch_bounds__(256) k_pack_rows(const float* __restrict__ src, int64_t n, int d, int dpad,
                                                    uint8_t* __restrict__ data, int64_t lrow0, float* __restrict__ sqn,
                                                    unsigned* __restrict__ maxsq) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const float* s = src + r * (int64_t)d;
    const int64_t row = lrow0 + r;
    float ss = 0.0f;
    for (int i = lane; i < dpad; i += 64) {
        float v = i < d ? s[i] : 0.0f;
        float st = round_store<DT>(v, data + tiled_off(row, i, dpad, ES));
        ss = fmaf(st, st, ss);
    }
    ss = wave_sum_fp32_canon(ss);
    if (lane == 0) {
        sqn[row] = ss;
        atomicMax(maxsq, __float_as_uint(ss));
    }
}

// IVF ingest: the same packing into an arbitrary storage slot per row (list pages), recording
// the row's user id in slot_id
template <int DT>
__global__ void __launch_bounds__(256) k_pack_rows_map(const float* __restrict__ src, int64_t n, int d, int dpad,
                                                        uint8_t* __restrict__ data, const int64_t* __restrict__ slots,
                                                        float* __restrict__ sqn, unsigned* __restrict__ maxsq,
                                                        uint32_t* __restrict__ slot_id, int64_t id0) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const float* s = src + r * (int64_t)d;
    const int64_t row = slots[r];
    float ss = 0.0f;
    for (int i = lane; i < dpad; i += 64) {
        float v = i < d ? s[i] : 0.0f;
        float st = round_store<DT>(v, data + tiled_off(row, i, dpad, ES));
        ss = fmaf(st, st, ss);
    }
    ss = wave_sum_fp32_canon(ss);
    if (lane == 0) {
        sqn[row] = ss;
        slot_id[row] = (uint32_t)(id0 + r);
        atomicMax(maxsq, __float_as_uint(ss));
    }
}

// round fp32 values to the storage dtype in place (IVF: rows are assigned by their stored values)
template <int DT>
__global__ void __launch_bounds__(256) k_round_f32(float* __restrict__ x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = round_only<DT>(x[i]);
}

template <int DT>
__global__ void __launch_bounds__(256) k_synth_rows(uint64_t base, int64_t grow0, int64_t n, int d, int dpad,
                                                     uint8_t* __restrict__ data, int64_t lrow0, int normalize,
                                                     float* __restrict__ sqn, unsigned* __restrict__ maxsq) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const uint64_t ctr0 = (uint64_t)(grow0 + r) * (uint64_t)d;
    float nrm = 0.0f;
    if (normalize) {
        float part = 0.0f;
        for (int i = lane; i < d; i += 64) {
            float v = synth_raw(base, ctr0 + (uint64_t)i);
            part = fmaf(v, v, part);
        }
        nrm = sqrtf(wave_sum_fp32_canon(part));
    }
    const int64_t row = lrow0 + r;
    float ss = 0.0f;
    for (int i = lane; i < dpad; i += 64) {
        float v = 0.0f;
        if (i < d) {
            v = synth_raw(base, ctr0 + (uint64_t)i);
            if (normalize && nrm != 0.0f) v = v / nrm;
        }
        float st = round_store<DT>(v, data + tiled_off(row, i, dpad, ES));
        ss = fmaf(st, st, ss);
    }
    ss = wave_sum_fp32_canon(ss);
    if (lane == 0) {
        sqn[row] = ss;
        atomicMax(maxsq, __float_as_uint(ss));
    }
}

// same generator, row-major fp32 output (values rounded to DT), for synthetic query batches
template <int DT>
__global__ void __launch_bounds__(256) k_synth_f32(uint64_t base, int64_t grow0, int64_t n, int d, int normalize,
                                                    float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const uint64_t ctr0 = (uint64_t)(grow0 + r) * (uint64_t)d;
    float nrm = 0.0f;
    if (normalize) {
        float part = 0.0f;
        for (int i = lane; i < d; i += 64) {
            float v = synth_raw(base, ctr0 + (uint64_t)i);
            part = fmaf(v, v, part);
        }
        nrm = sqrtf(wave_sum_fp32_canon(part));
    }
    for (int i = lane; i < d; i += 64) {
        float v = synth_raw(base, ctr0 + (uint64_t)i);
        if (normalize && nrm != 0.0f) v = v / nrm;
        out[r * (int64_t)d + i] = round_only<DT>(v);
    }
}

template <int DT>
__global__ void __launch_bounds__(256) k_unpack_rows(const uint8_t* __restrict__ data, int64_t lrow0, int64_t n,
                                                      int d, int dpad, float* __restrict__ out) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t row = lrow0 + r;
    for (int i = lane; i < d; i += 64) out[r * (int64_t)d + i] = load_elem<DT>(data + tiled_off(row, i, dpad, ES));
}

template <int DT>
__global__ void __launch_bounds__(256) k_gather_rows(const uint8_t* __restrict__ data, const int64_t* __restrict__ ids,
                                                      int64_t n, int d, int dpad, float* __restrict__ out) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t row = ids[r];
    for (int i = lane; i < d; i += 64)
        out[r * (int64_t)d + i] = row < 0 ? 0.0f : load_elem<DT>(data + tiled_off(row, i, dpad, ES));
}

// ------------------------------------------------------------------------------------------------
// query packing
// ------------------------------------------------------------------------------------------------
// MFMA query tile [nks][256][32] in the corpus dtype; qinfo = (||q_hat||, ||q_hat - q||) in fp64,
// rounded up to fp32.  qidx (IVF list scans): tile row r is query qidx[r] of q, and its qinfo goes
// to qinfo[2 qidx[r]] as the max with what is there (the fp32 scan's values: a bound for both).
template <int DT>
__global__ void __launch_bounds__(256) k_pack_qtile(const float* __restrict__ q, int nqb, int d, int dpad,
                                                     uint8_t* __restrict__ qt, float* __restrict__ qinfo,
                                                     int* __restrict__ gcnt, u64* __restrict__ drop,
                                                     int* __restrict__ fails, const int* __restrict__ gate,
                                                     const int* __restrict__ qidx, int* __restrict__ gcnt2,
                                                     u64* __restrict__ drop2) {
    if (gate && *gate == 0) return;  // device fallback round with nothing to re-search
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= MFMA_QB) return;
    if (fails && r == 0 && lane == 0) fails[0] = fails[1] = 0;  // the block's certificate-failure counts
    if (gcnt && lane == 0) gcnt[r] = 0;  // survivor-list lengths of the screen that follows ...
    if (drop && lane == 0) drop[r] = 0ull;  // ... and its workgroups' drop bounds
    if (gcnt2 && lane == 0) {  // (and those of the device fallback round, which reuses this tile)
        gcnt2[r] = 0;
        drop2[r] = 0ull;
    }
    double n2 = 0.0, e2 = 0.0;
    const int64_t qr = (qidx && r < nqb) ? (int64_t)qidx[r] : (int64_t)r;
    constexpr int KE = DT == DT_F32 ? 16 : 32;  // elements per K-step (64 B per query row)
    constexpr int ES = DT == DT_F32 ? 4 : 2;
#pragma unroll 8
    for (int i = lane; i < dpad; i += 64) {
        float v = (r < nqb && i < d) ? q[qr * d + i] : 0.0f;
        float st = round_store<DT>(v, qt + (int64_t)(i / KE) * MFMA_QB * 64 + (int64_t)r * 64 + (i % KE) * ES);
        n2 += (double)st * st;
        double df = (double)st - (double)v;
        e2 += df * df;
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        n2 += __shfl_xor(n2, s, 64);
        e2 += __shfl_xor(e2, s, 64);
    }
    if (lane == 0 && r < nqb) {
        const float nq = (float)(sqrt(n2) * (1.0 + 1e-6)) + 1e-30f, eq = (float)(sqrt(e2) * (1.0 + 1e-6));
        if (qidx) {
            qinfo[2 * qr] = fmaxf(qinfo[2 * qr], nq);
            qinfo[2 * qr + 1] = fmaxf(qinfo[2 * qr + 1], eq);
        } else {
            qinfo[2 * r] = nq;
            qinfo[2 * r + 1] = eq;
        }
    }
}

// Split query tile of the mapped (IVF list) screen: up to 128 queries, query j = wn*64 + jj (jj < 64)
// as hi = round(q) in tile row wn*128 + (jj/16)*32 + jj%16 and lo = round(q - hi) 16 rows further,
// so the screen sums two MFMA accumulators per query.  Query j is q[qidx[j]]; its qinfo entry
// becomes the max of what is there and (||hi|| + ||lo||, ||q - hi - lo||) (fp64, rounded up).
// PLAIN: up to 256 queries, query j = hi alone in tile row j (qinfo: (||hi||, ||q - hi||)): half the
// MFMAs per query, a margin ~2^8 x wider (the refine's certificate takes it; re-search rounds pack
// split tiles).
// One launch packs every tile: tile y = blockIdx.y takes queries qidx[sinfo[2y] ..] (sinfo[2y + 1]
// of them) into qt + y * MFMA_QB * dpad * 2.
template <int DT, bool PLAIN>
__global__ void __launch_bounds__(256) k_pack_qtile_split(const float* __restrict__ q, const int* __restrict__ qidx,
                                                           const int* __restrict__ sinfo, int d, int dpad,
                                                           uint8_t* __restrict__ qt, float* __restrict__ qinfo) {
    qidx += sinfo[2 * blockIdx.y];
    const int nqb = sinfo[2 * blockIdx.y + 1];
    qt += (size_t)blockIdx.y * MFMA_QB * dpad * 2;
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);  // tile row
    if (c >= MFMA_QB) return;
    const int wn = c >> 7, ni = (c >> 4) & 7, part = PLAIN ? 0 : ni & 1;
    const int j = PLAIN ? c : wn * 64 + (ni >> 1) * 16 + (c & 15);
    const bool real = j < nqb;
    const int64_t qr = real ? (int64_t)qidx[j] : 0;
    double h2 = 0.0, l2 = 0.0, e2 = 0.0;
#pragma unroll 8
    for (int i = lane; i < dpad; i += 64) {
        const float v = (real && i < d) ? q[qr * d + i] : 0.0f;
        const float hi = round_only<DT>(v);
        const float lo = PLAIN ? 0.0f : round_only<DT>(v - hi);  // v - hi is exact in fp32
        round_store<DT>(part ? lo : hi, qt + (int64_t)(i >> 5) * MFMA_QB * 64 + (int64_t)c * 64 + (i & 31) * 2);
        h2 += (double)hi * hi;
        l2 += (double)lo * lo;
        const double df = (double)v - (double)hi - (double)lo;
        e2 += df * df;
    }
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        h2 += __shfl_xor(h2, sh, 64);
        l2 += __shfl_xor(l2, sh, 64);
        e2 += __shfl_xor(e2, sh, 64);
    }
    if (lane == 0 && real && part == 0) {
        const float nq = (float)((sqrt(h2) + sqrt(l2)) * (1.0 + 1e-6)) + 1e-30f, eq = (float)(sqrt(e2) * (1.0 + 1e-6));
        qinfo[2 * qr] = fmaxf(qinfo[2 * qr], nq);
        qinfo[2 * qr + 1] = fmaxf(qinfo[2 * qr + 1], eq);
    }
}

// ------------------------------------------------------------------------------------------------
// int8 screen copy (DESIGN §5 "int8 screen").  Per row, over its STORED values x: scale
// s = bf16(max|x| / 127), codes c = rint(x / s) in [-127, 127], and the bound
// beta = ||x - s c||_2 + eps_q ||s c|| (fp64, rounded up to bf16; eps_q: the query's share, see
// i8_eps_q); (s, beta) packed in one u32 per row (the screen
// epilogue reads 4 B per row).  Also the running maxima of ||s c|| and beta
// (maxes[0], maxes[1], fp32 bits) that bound the query-side and rounding terms of the refine's
// certificate.  The codes need not be the nearest: whatever rint gives, beta is measured.
// Layout: row tiles of TR rows, 64-element chunks, [chunk][row][64 B] -- one 16 KiB block per
// MFMA K-step, the same block geometry as the bf16 layout.
// ------------------------------------------------------------------------------------------------

// one wave per row
__device__ __forceinline__ uint32_t bf16_bits_up(float f) {  // smallest bf16 >= f (f >= 0, finite)
    const uint32_t u = __float_as_uint(f);
    return (u >> 16) + ((u & 0xFFFFu) ? 1u : 0u);
}

constexpr int GM_COLS = 1536;  // columns per pass of k_group_means (its LDS partial sums)
// Group residuals (inner-product int8 screens, DESIGN §5 "clustered corpora"): rows are coded as
// x = mu_g + r with mu_g the bf16-rounded mean of their group of I8_GROUP_ROWS consecutive rows, when
// that mean carries at least a quarter of the group's energy (a corpus inserted cluster by cluster);
// else mu_g = 0.  The error norm then scales with ||r||, not ||x||; the screen adds <mu_g, q> (fp32,
// k_group_dots) to every key of the group.  One block per group: the mean over the rows present,
// its bf16 rounding, the energy test; maxes[0] (fp32 bits) = the largest ||mu_g|| (rounded up),
// maxes[1] counts the groups with a mean.
template <int DT>
__global__ void __launch_bounds__(256) k_group_means(const uint8_t* __restrict__ data, int dpad, int d, int64_t g0,
                                                      int64_t n_rows, int dpad8, uint16_t* __restrict__ gmean,
                                                      unsigned* __restrict__ maxes) {
    // wave w sums rows w, w + 4, ... of the group; lane l columns l, l + 64, ... (one 128 B line of
    // the tiled layout per row and 64 columns at 16-bit): GM_COLS / 64 independent loads per row
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    constexpr int NC = GM_COLS / 64;
    __shared__ float part[4][GM_COLS];
    __shared__ float e2[4];
    __shared__ double m2w[4];
    const int64_t g = g0 + blockIdx.x;
    const int64_t lo = g * I8_GROUP_ROWS, hi = min(n_rows, lo + I8_GROUP_ROWS);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint16_t* dst = gmean + (size_t)g * dpad8;
    const float cnt = (float)(hi - lo);
    float x2 = 0.0f;
    double m2 = 0.0;  // ||mu||^2 of the stored bf16 means, exactly enough for the margin (fp64)
    for (int c0 = 0; c0 < dpad8; c0 += GM_COLS) {  // column blocks (d > GM_COLS)
        float s[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) s[c] = 0.0f;
        for (int64_t r = lo + w; r < hi; r += 4) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int i = c0 + 64 * c + lane;
                const float v = i < d ? load_elem<DT>(data + tiled_off(r, i, dpad, ES)) : 0.0f;
                s[c] += v;
                x2 += v * v;
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) part[w][64 * c + lane] = s[c];
        __syncthreads();
        for (int i = tid; i < GM_COLS && c0 + i < dpad8; i += 256) {
            const float t = part[0][i] + part[1][i] + part[2][i] + part[3][i];
            const uint16_t b = (c0 + i < d && cnt > 0.0f) ? f32_to_bf16_rne(t / cnt) : (uint16_t)0;
            dst[c0 + i] = b;
            const double mu = (double)bf16_bits_to_f32(b);
            m2 += mu * mu;
        }
        __syncthreads();
    }
    x2 = wave_sum_fp32_canon(x2);
    m2 = wave_sum_f64(m2);
    if (lane == 0) {
        e2[w] = x2;
        m2w[w] = m2;
    }
    __syncthreads();
    const double M2 = m2w[0] + m2w[1] + m2w[2] + m2w[3];
    const float X2 = e2[0] + e2[1] + e2[2] + e2[3];
    // a mean worth coding against: >= 1/4 of the group's mean row energy, over at least a tile of
    // rows (a few rows are their own mean, whatever the corpus) -- a heuristic choice: any mean,
    // zero included, gives exact keys
    const bool use = cnt >= (float)TR && M2 > 0.0 && (float)M2 * cnt >= 0.25f * X2;
    if (!use)
        for (int i = tid; i < dpad8; i += 256) dst[i] = 0;
    if (tid == 0 && use) {
        atomicMax(&maxes[0], __float_as_uint(f32_up(sqrt(M2) * (1.0 + 1e-9))));  // the margin's max ||mu||
        atomicAdd(&maxes[1], 1u);
    }
}

// The query side's int8 error ||q - t_q c_q|| is bounded per row, not per corpus: each row's bound
// word carries beta_x = ||x - s_x c_x|| + eps_q ||s_x c_x||, eps_q the typical relative int8 error of
// a d-vector (rms t / sqrt(12) per element, t = max / 127 ~ sqrt(2 ln 2d) sigma / 127), +10%; a
// query whose own error exceeds eps_q ||q|| pays the excess x max ||s_x c_x|| in its margin
// (k_pack_qtile_i8).  So a row far from its group mean widens only its own key, not every query's
// margin (cluster-boundary rows of group residuals: ||s_x c_x|| up to ~1.4 ||x||).
__host__ __device__ inline double i8_eps_q(int d) {
    return 1.1 * sqrt(2.0 * log(2.0 * (double)(d > 1 ? d : 1))) / (127.0 * 3.4641016151377544);
}

template <int DT>
__global__ void __launch_bounds__(256) k_quant_rows(const uint8_t* __restrict__ data, int dpad, int64_t r0, int64_t n,
                                                     int d, uint8_t* __restrict__ data8, int dpad8,
                                                     uint32_t* __restrict__ rsb, unsigned* __restrict__ maxes,
                                                     const uint16_t* __restrict__ gmean) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t row = r0 + r;
    // group residual: the codes quantise x - mu_g, computed exactly in fp64 (mu_g = 0: the row)
    const uint16_t* mu = gmean ? gmean + (size_t)(row / I8_GROUP_ROWS) * dpad8 : nullptr;
    auto resid = [&](int i) -> double {
        const double x = (double)load_elem<DT>(data + tiled_off(row, i, dpad, ES));
        return mu ? x - (double)bf16_bits_to_f32(mu[i]) : x;
    };
    float mx = 0.0f;
    for (int i = lane; i < d; i += 64) mx = fmaxf(mx, (float)fabs(resid(i)));
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s, 64));
    const uint32_t sbits = f32_to_bf16_rne(mx / 127.0f);
    const float sc = bf16_bits_to_f32(sbits);  // the scale as stored: codes and error use exactly it
    uint8_t* dst = data8 + (row / TR) * (int64_t)TR * dpad8 + (row % TR) * 64;
    double e2 = 0.0, c2 = 0.0, r2 = 0.0;
    for (int i = lane; i < dpad8; i += 64) {
        int c = 0;
        double x = 0.0;
        if (i < d) {
            x = resid(i);
            if (sc > 0.0f) c = max(-127, min(127, (int)rint(x / (double)sc)));
        }
        dst[(int64_t)(i >> 6) * TR * 64 + (i & 63)] = (uint8_t)(int8_t)c;
        // fp64: s c is exact; x - s c rounds at most once (relative 2^-53); with a group mean, x
        // itself (the stored value minus mu) may have rounded once too (|err| <= 2^-53 |x|): both are
        // covered by the norm's rounding-up below plus 2^-51 ||x||
        const double e = x - (double)sc * (double)c;
        e2 += e * e;
        c2 += (double)(c * c);
        r2 += x * x;
    }
    e2 = wave_sum_f64(e2);
    c2 = wave_sum_f64(c2);
    r2 = wave_sum_f64(r2);
    if (lane == 0) {
        const double xh = sqrt(c2) * (double)sc;  // ||s_x c_x|| (the query error's row factor)
        const uint32_t bbits = bf16_bits_up(f32_up((sqrt(e2) + i8_eps_q(d) * xh) * (1.0 + 1e-9) +
                                                   (mu ? sqrt(r2) * 4.440892098500626e-16 : 0.0)));
        rsb[row] = sbits | (bbits << 16);
        atomicMax(&maxes[0], __float_as_uint(f32_up(sqrt(c2) * (double)sc * (1.0 + 1e-9))));
        atomicMax(&maxes[1], bbits << 16);  // the fp32 bits of the bf16 bound
        atomicMax(&maxes[5], __float_as_uint(f32_up(sqrt(e2) * (1.0 + 1e-9))));  // max ||x - s c|| (GEMV depth)
    }
}

// T[g][q] = <mu_g, q> for the group means of the int8 copy (k_group_means) and a batch of fp32
// queries, by bf16 MFMA with each query split exactly into hi = bf16(q) + lo = bf16(q - hi): the
// products are exact in fp32, so |T - <mu_g, q>| <= (gamma_2d + 2^-16) ||mu_g|| ||q|| (|q - hi - lo|
// <= 2^-17 |q| elementwise) -- k_pack_qtile_i8 adds that to every query's margin.  One block per 16
// groups; wave w takes queries 64w .. 64w + 63 (four 16-column tiles), hi and lo into the same
// accumulators.  Groups without a mean (mu_g = 0) give T = 0.
__global__ void __launch_bounds__(256) k_group_dots(const uint16_t* __restrict__ gmean, int64_t ngroups, int dpad8,
                                                     const float* __restrict__ q, int nq, int d, float* __restrict__ T) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t g0 = (int64_t)blockIdx.x * 16;
    const int r16 = lane & 15, kc = (lane >> 4) * 8;
    const int64_t ga = min(g0 + r16, ngroups - 1);
    const uint16_t* arow = gmean + (size_t)ga * dpad8;
    floatx4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int k0 = 0; k0 < dpad8; k0 += 32) {
        const uint4 av = *(const uint4*)(arow + k0 + kc);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int qq = 64 * w + 16 * c + r16;
            uint32_t hi[4], lo[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = k0 + kc + 2 * e;
                const float v0 = (qq < nq && k < d) ? q[(int64_t)qq * d + k] : 0.0f;
                const float v1 = (qq < nq && k + 1 < d) ? q[(int64_t)qq * d + k + 1] : 0.0f;
                const uint32_t h0 = f32_to_bf16_rne(v0), h1 = f32_to_bf16_rne(v1);
                const uint32_t l0 = f32_to_bf16_rne(v0 - bf16_bits_to_f32(h0)), l1 = f32_to_bf16_rne(v1 - bf16_bits_to_f32(h1));
                hi[e] = h0 | (h1 << 16);
                lo[e] = l0 | (l1 << 16);
            }
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                             __builtin_bit_cast(bf16x8, make_uint4(hi[0], hi[1], hi[2], hi[3])),
                                                             acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                             __builtin_bit_cast(bf16x8, make_uint4(lo[0], lo[1], lo[2], lo[3])),
                                                             acc[c], 0, 0, 0);
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int qq = 64 * w + 16 * c + r16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t g = g0 + 4 * (lane >> 4) + j;
            if (g < ngroups) T[(size_t)g * MFMA_QB + qq] = qq < nq ? acc[c][j] : 0.0f;
        }
    }
}

// int8 query tile [nks8][256][64] (codes of q / t_q, t_q = max|q| / 127) for the int8 MFMA screen,
// one wave per query.  qfac = (t_q, ||q|| rounded up / t_q); qeps = the query-side margin of the
// screen key (key = s_x t_q <c_x, c_q> + beta_x ||q||, see k_screen_mfma):
//   true <x, q> <= s_x t_q <c_x, c_q> + ||x - s_x c_x|| ||q|| + ||s_x c_x|| ||q - t_q c_q|| + rounding
//               <= key + max ||s_x c_x|| max(0, ||q - t_q c_q|| - eps_q ||q||) + rounding <= key_score + qeps.
// Also zeroes the survivor-list lengths and the workgroup drop bounds of the screen that follows.
// NDT (bf16 / f16; 0 = none): also the device fallback round's native tile (NativeTile, the layout
// and qinfo of k_pack_qtile<NDT>), from the same loaded values -- the round's gated pack launch
// is then not needed.
template <int NDT>
__global__ void __launch_bounds__(256) k_pack_qtile_i8(const float* __restrict__ q, int nqb, int d, int dpad8,
                                                        uint8_t* __restrict__ qt, float2* __restrict__ qfac,
                                                        float* __restrict__ qeps, const unsigned* __restrict__ maxes,
                                                        int* __restrict__ gcnt, u64* __restrict__ drop,
                                                        int* __restrict__ fails, const unsigned* __restrict__ l2max,
                                                        float gamma, NativeTile nat) {
    // one workgroup per query (256 threads over its d elements; a query's pack is a chain of
    // reductions, so 4x the waves per query shorten the launch)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = blockIdx.x;
    __shared__ float s_mx[4];
    __shared__ double s_red[4][5];
    if (fails && r == 0 && tid == 0) fails[0] = fails[1] = 0;
    if (tid == 0) {
        gcnt[r] = 0;
        drop[r] = 0ull;
        if constexpr (NDT != 0) {
            nat.gcnt[r] = 0;
            nat.drop[r] = 0ull;
        }
    }
    // The codes need not be the nearest (the error norm below is measured from the codes chosen), so
    // v * (1 / t) replaces the division; d <= 2048 (the common case): the thread's values are loaded
    // once and kept in registers for the second pass.
    constexpr int PL = 8;
    float vv[PL];
    float mx = 0.0f;
    const bool cached = dpad8 <= 256 * PL && (NDT == 0 || nat.dpad <= 256 * PL);
    if (cached) {
#pragma unroll
        for (int j = 0; j < PL; ++j) {
            const int i = tid + 256 * j;
            vv[j] = (r < nqb && i < d) ? q[(int64_t)r * d + i] : 0.0f;
            mx = fmaxf(mx, fabsf(vv[j]));
        }
    } else if (r < nqb) {
        for (int i = tid; i < d; i += 256) mx = fmaxf(mx, fabsf(q[(int64_t)r * d + i]));
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s, 64));
    if (lane == 0) s_mx[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(s_mx[0], s_mx[1]), fmaxf(s_mx[2], s_mx[3]));
    const float t = mx / 127.0f;
    const float inv = t > 0.0f ? 1.0f / t : 0.0f;
    double e2 = 0.0, n2 = 0.0, c2 = 0.0;
    auto one = [&](int i, float v) {
        const int c = max(-127, min(127, (int)rintf(v * inv)));
        qt[(int64_t)(i >> 6) * MFMA_QB * 64 + (int64_t)r * 64 + (i & 63)] = (uint8_t)(int8_t)c;
        const double e = (double)v - (double)t * (double)c;
        e2 += e * e;
        n2 += (double)v * v;
        c2 += (double)(c * c);
    };
    if (cached) {
#pragma unroll
        for (int j = 0; j < PL; ++j) {
            const int i = tid + 256 * j;
            if (i < dpad8) one(i, vv[j]);
        }
    } else {
        for (int i = tid; i < dpad8; i += 256) one(i, (r < nqb && i < d) ? q[(int64_t)r * d + i] : 0.0f);
    }
    double n2n = 0.0, e2n = 0.0;
    if constexpr (NDT != 0) {  // the native tile (k_pack_qtile<NDT>'s layout and qinfo)
        auto nat_one = [&](int i, float v) {
            const float st = round_store<NDT>(v, nat.qt + (int64_t)(i >> 5) * MFMA_QB * 64 + (int64_t)r * 64 + (i & 31) * 2);
            n2n += (double)st * st;
            const double df = (double)st - (double)v;
            e2n += df * df;
        };
        if (cached) {
#pragma unroll
            for (int j = 0; j < PL; ++j) {
                const int i = tid + 256 * j;
                if (i < nat.dpad) nat_one(i, i < d ? vv[j] : 0.0f);
            }
        } else {
            for (int i = tid; i < nat.dpad; i += 256) nat_one(i, (r < nqb && i < d) ? q[(int64_t)r * d + i] : 0.0f);
        }
    }
    {  // the five sums over the workgroup (fp64), finished by thread 0
        const double v5[5] = {wave_sum_f64(e2), wave_sum_f64(n2), wave_sum_f64(c2), wave_sum_f64(n2n),
                              wave_sum_f64(e2n)};
        if (lane == 0)
#pragma unroll
            for (int j = 0; j < 5; ++j) s_red[w][j] = v5[j];
        __syncthreads();
        if (tid != 0) return;
        e2 = s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0];
        n2 = s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1];
        c2 = s_red[0][2] + s_red[1][2] + s_red[2][2] + s_red[3][2];
        n2n = s_red[0][3] + s_red[1][3] + s_red[2][3] + s_red[3][3];
        e2n = s_red[0][4] + s_red[1][4] + s_red[2][4] + s_red[3][4];
    }
    if constexpr (NDT != 0) {
        if (r < nqb) {
            nat.qinfo[2 * r] = (float)(sqrt(n2n) * (1.0 + 1e-6)) + 1e-30f;
            nat.qinfo[2 * r + 1] = (float)(sqrt(e2n) * (1.0 + 1e-6));
        }
    }
    if (r < nqb) {
        const float qn = f32_up(sqrt(n2) * (1.0 + 1e-9));
        const double eq = sqrt(e2) * (1.0 + 1e-9);
        const double qh = sqrt(c2) * (double)t * (1.0 + 1e-9);  // ||t_q c_q||
        const double X = (double)__uint_as_float(maxes[0]), B = (double)__uint_as_float(maxes[1]);
        // group residuals (inner product): the key adds T = fl<mu_g, q> (k_group_dots), within
        // (gamma_2d + 2^-16) ||mu_g|| ||q|| of the true dot; Mu = max ||mu_g|| (0 without them)
        const double Mu = (double)__uint_as_float(maxes[3]);
        // the key's fp32 evaluation t * fma(beta, fl(qn / t), fl(s * fl(acc))) [+ T]: <= 7 roundings
        // relative 2^-24 of |sigma| + beta qn [+ |T|] (|sigma| <= X ||t_q c_q||); 8 of them budgeted
        const double slop = 8.0 * 5.9604644775390625e-08 * (X * qh + B * (double)qn + Mu * (double)qn) + 1e-30 +
                            (2.02 * (double)gamma + 1.52587890625e-05) * Mu * (double)qn;
        // the screen computes key = t_q * (s_x acc + beta_x * (||q|| / t_q)); a zero query has t_q = 0
        // and every key 0
        qfac[r] = make_float2(t, t > 0.0f ? qn / t : 0.0f);
        // the rows' bound words cover eps_q ||q|| of this query's error (k_quant_rows); the excess
        // over it, times the largest ||s_x c_x||
        const double excess = fmax(0.0, eq - i8_eps_q(d) * sqrt(n2) * (1.0 - 1e-9));
        double e = X * excess + slop;
        if (l2max) {
            // L2 keys fl(2 fl(t v) - ||x||^2_fp32) bound 2 <x, q> - ||x||^2: twice the inner-product
            // margin, the fp32 norm's error (gamma_d ||x||^2, its canonical sum) and the key's last
            // rounding (relative 2^-24 of 2 (X ||t_q c_q|| + B ||q||) + ||x||^2)
            const double S = (double)__uint_as_float(l2max[0]);  // max ||x||^2 (fp32)
            e = 2.0 * e + ((double)gamma + 2.0 * 5.9604644775390625e-08) * S +
                2.0 * 5.9604644775390625e-08 * (X * qh + B * (double)qn);
            e *= 1.01;
        }
        qeps[r] = f32_up((e) * (1.0 + 1e-9));
    }
}

// GEMV queries: fp32, [nqpad][dpad] zero padded; q_hat = q
__global__ void __launch_bounds__(256) k_pack_qf32(const float* __restrict__ q, int nqb, int nqpad, int d, int dpad,
                                                    float* __restrict__ qp, float* __restrict__ qinfo,
                                                    int* __restrict__ ctr, int* __restrict__ fails,
                                                    u64* __restrict__ drop) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (drop && r < nqpad && lane == 0) drop[r] = 0ull;  // the GEMV screen's block drop bounds
    if (ctr && blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0;  // the GEMV screen's tile queue that follows
    if (fails && blockIdx.x == 0 && threadIdx.x == 0) fails[0] = fails[1] = 0;  // the block's certificate-failure counts
    if (r >= nqpad) return;
    double n2 = 0.0;
    for (int i = lane; i < dpad; i += 64) {
        float v = (r < nqb && i < d) ? q[(int64_t)r * d + i] : 0.0f;
        qp[(int64_t)r * dpad + i] = v;
        n2 += (double)v * v;
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) n2 += __shfl_xor(n2, s, 64);
    if (lane == 0 && r < nqb) {
        qinfo[2 * r] = (float)(sqrt(n2) * (1.0 + 1e-6)) + 1e-30f;
        qinfo[2 * r + 1] = 0.0f;
    }
}

}  // namespace vs
#include "vs_screen.h"
namespace vs {

// the K1 int8 inner-product direct screen's schedule (vs_set_k1_schedule; vs_screen.h screen_direct
// SCHED): 0 = barrier at the head of every K-step; 1 = the mid-step barrier (cfg3 K1 3.68 -> 3.50 ms,
// profiles/r06_k1_decomposition.json).  (The bf16 / f16 direct screen keeps the head barrier: the
// mid-step form measured no faster there, its loop bound by the half-line loads.)
static std::atomic<int> g_k1_sched{1};
void set_k1_schedule(int s) { g_k1_sched.store(s); }
int k1_schedule() { return g_k1_sched.load(std::memory_order_relaxed); }

bool i8_direct_ok(int dpad8) { return dpad8 % (64 * I8D_U) == 0 && dpad8 >= 2 * 64 * I8D_U; }
bool d16_direct_ok(int dpad) { return dpad % (CH * I8D_U) == 0 && dpad >= 2 * CH * I8D_U; }

// ... over group-residual codes (a corpus stored cluster by cluster): every key + <mu_g, q>
// (inner product; the seed pass adds the same terms to its maxima)
__global__ void __launch_bounds__(512, 2) k_screen_i8d_res(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT_I8, METRIC_IP, false, 16, true>(a, qt, nqb);
}
__global__ void __launch_bounds__(512, 2) k_screen_i8d_res_ms(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT_I8, METRIC_IP, false, 16, true, PR_NONE, 1>(a, qt, nqb);
}


// ------------------------------------------------------------------------------------------------
// K2: GEMV screen (any dtype, up to 8 queries per launch) -- HBM streaming, fp32 FMA
// ------------------------------------------------------------------------------------------------
// 256 threads, persistent over a contiguous tile range.  A row's piece of a chunk (one 128 B line;
// 64 B in the int8 screen copy) is LPR 16 B units, read by LPR consecutive lanes, so every
// wave-instruction is a contiguous 1 KiB piece.  int8: the fp32 dot of the codes with the fp32 query (no query
// quantisation), key = s_x * dot + beta_x * ||q|| (an upper bound of the true score up to fp32
// rounding, certified in k_refine).
// SPLIT: work items of 256 / SPLIT rows (a tile in SPLIT row blocks, each wave 64 / SPLIT rows of
// it): corpora of fewer tiles than resident blocks reach more CUs (cfg1: 40 tiles)
// QL: the queries staged in LDS once per workgroup (dynamic LDS, NQ x dpad fp32), read from there
// per chunk instead of from L1/L2: half the vector-memory instructions of the loop, and the query
// values no longer held across the unrolled chunks (fewer VGPRs)
template <int DT, int NQ, int SPLIT = 1, bool QL = false>
__global__ void __launch_bounds__(256) k_screen_gemv(ScreenArgs a, const float* __restrict__ qp, int nqb) {
    constexpr bool I8 = DT == DT_I8;
    constexpr int ES = DT == DT_F32 ? 4 : I8 ? 1 : 2;
    constexpr int CHK = I8 ? 64 : CHB / ES;  // elements per chunk
    constexpr int CB = CHK * ES;
    constexpr int LPR = CB / 16;
    constexpr int RPI = 64 / LPR;
    constexpr int EPU = 16 / ES;
    constexpr int RG = 64 / RPI / SPLIT;  // row groups per wave and item
    static_assert(RG >= 1 && 64 % (RPI * SPLIT) == 0, "split");
    constexpr int RB0 = (NQ <= 2) ? 8 : 4;  // rows per pass (register budget)
    constexpr int RB = RB0 < RG ? RB0 : RG;
    static_assert(RG % RB == 0, "row groups");

    __shared__ u64 thr_key[NQ];
    __shared__ float thr_f[NQ];
    __shared__ int cnt[NQ];
    __shared__ int red[8];
    __shared__ int tile_s;

    extern __shared__ __attribute__((aligned(16))) float qsh[];  // QL: [NQ][dpad]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int unit = lane % LPR, rsub = lane / LPR;
    const int blk = blockIdx.x;
    const int items = a.tiles * SPLIT;
    if constexpr (QL)
        for (int i = tid; i < NQ * a.dpad / 4; i += 256) ((float4*)qsh)[i] = ((const float4*)qp)[i];
    const int t0 = (int)((int64_t)items * blk / a.G);
    const int t1 = (int)((int64_t)items * (blk + 1) / a.G);
    if (tid < NQ) {
        const bool real = tid < nqb;
        thr_key[tid] = real ? 0ull : ~0ull;
        thr_f[tid] = real ? -INFINITY : INFINITY;
        cnt[tid] = 0;
    }
    __syncthreads();
    const int nch = a.dpad / CHK;
    const int64_t tbytes = (int64_t)TR * a.dpad * ES;
    u64* cand = a.cand + (size_t)blk * NQ * a.cap;
    const float epsq = I8 ? (float)(i8_eps_q(a.d) * (1.0 - 1e-6)) : 0.0f;  // (rounded below)
    const int trigger = a.cap - TR;

    // tiles: a static contiguous range, or (next_tile) one at a time from a work queue with a grid
    // of exactly the resident blocks, so no second partial round of blocks idles the HBM stream
    for (int it = 0;; ++it) {
        int item;
        if (a.next_tile) {
            if (tid == 0) tile_s = atomicAdd(a.next_tile, 1);
            __syncthreads();
            item = tile_s;
            __syncthreads();  // every thread has its item before tile_s is reused
            if (item >= items) break;  // block-uniform
        } else {
            item = t0 + it;
            if (item >= t1) break;
        }
        const int ti = item / SPLIT;
        const int wrow = (item % SPLIT) * (TR / SPLIT) + wid * (64 / SPLIT);  // the wave's first row
        const uint8_t* tb = a.corpus + (int64_t)ti * tbytes;
        const int64_t rowbase = (int64_t)ti * TR;
        for (int gb = 0; gb < RG / RB; ++gb) {
            float acc[RB][NQ];
            float cc2[RB];  // int8: sum of the codes' squares (||s_x c_x|| = s_x sqrt(cc2))
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                cc2[r] = 0.0f;
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) acc[r][qi] = 0.0f;
            }
            // (int8: 4 chunks per unrolled pass keep twice the loads in flight of the 64 B row
            // pieces: cfg2 GEMV 0.2834 -> 0.2806 ms, profiles/r06_ab_cfg2_gemv.txt)
            constexpr int CU = I8 ? 4 : 2;
#pragma unroll CU
            for (int c = 0; c < nch; ++c) {
                float qv[NQ][EPU];
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
                    const int64_t qo = (int64_t)qi * a.dpad + c * CHK + unit * EPU;
#pragma unroll
                    for (int h = 0; h < EPU / 4; ++h) {
                        float4 t;
                        if constexpr (QL) t = ((const float4*)(qsh + qo))[h];
                        else t = ((const float4*)(qp + qo))[h];
                        qv[qi][4 * h + 0] = t.x; qv[qi][4 * h + 1] = t.y;
                        qv[qi][4 * h + 2] = t.z; qv[qi][4 * h + 3] = t.w;
                    }
                }
                uint4 raw[RB];
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int rit = wrow + (gb * RB + r) * RPI + rsub;
                    // non-temporal: 1.04 -> 0.96-0.98 ms at cfg2 (74% -> 79-80% of HBM peak)
                    raw[r] = ld_nt16(tb + (int64_t)c * TR * CB + rit * CB + unit * 16);
                }
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    float xv[EPU];
                    unpack16<DT>(raw[r], xv);
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi)
#pragma unroll
                        for (int e = 0; e < EPU; ++e) acc[r][qi] = fmaf(xv[e], qv[qi][e], acc[r][qi]);
                    if constexpr (I8)
#pragma unroll
                        for (int e = 0; e < EPU; ++e) cc2[r] = fmaf(xv[e], xv[e], cc2[r]);
                }
            }
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
                    float v = acc[r][qi];
#pragma unroll
                    for (int s = 1; s < LPR; s <<= 1) v += __shfl_xor(v, s, 64);
                    acc[r][qi] = v;
                }
            if constexpr (I8)
#pragma unroll
                for (int r = 0; r < RB; ++r)
#pragma unroll
                    for (int s = 1; s < LPR; s <<= 1) cc2[r] += __shfl_xor(cc2[r], s, 64);
            if (unit == 0) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int rit = wrow + (gb * RB + r) * RPI + rsub;
                    const int64_t gr = rowbase + rit;
                    if (gr >= a.n_valid) continue;
                    float sq = 0.0f, rbeta = 0.0f;
                    if constexpr (I8) {
                        const uint32_t w = a.rsb[gr];
                        sq = __uint_as_float(w << 16);            // scale s_x
                        // the bound word less the query-error share it carries for the int8 MFMA
                        // screen (k_quant_rows): this screen's query is exact fp32.  ||s_x c_x|| from
                        // below (cc2's fp32 sum: relative error <= d 2^-24), so the result still
                        // bounds ||x - s_x c_x||
                        const float xh = sq * sqrtf(cc2[r]) * (1.0f - 3.0f * (float)a.dpad * 5.9604645e-08f - 1e-6f);
                        rbeta = fmaxf(0.0f, __uint_as_float(w & 0xFFFF0000u) - epsq * xh);
                    } else {
                        sq = a.metric == METRIC_L2 ? a.sqn[gr] : 0.0f;
                    }
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi) {
                        float sc = acc[r][qi];
                        if constexpr (I8) {
                            sc = fmaf(rbeta, a.qinfo[2 * qi], sq * sc);
                            if (a.metric == METRIC_L2) sc = 2.0f * sc - a.sqn[gr];
                        } else if (a.metric == METRIC_L2) {
                            sc = 2.0f * sc - sq;
                        }
                        if (sc >= thr_f[qi]) {
                            const u64 key = mk_key(sc, (uint32_t)gr);
                            if (key > thr_key[qi]) {
                                const int slot = atomicAdd(&cnt[qi], 1);
                                if (slot < a.cap) cand[(size_t)qi * a.cap + slot] = key;
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
        for (int qi = 0; qi < nqb; ++qi) {
            const int n = cnt[qi];
            if (n > trigger) {  // block-uniform
                u64* buf = cand + (size_t)qi * a.cap;
                const u64 t = block_kth_mem(buf, n, a.Kp, red);
                block_compact_mem(buf, buf, n, t, red);
                if (tid == 0) {
                    thr_key[qi] = t;
                    thr_f[qi] = key_score(t);
                    cnt[qi] = a.Kp;
                }
                __syncthreads();
            }
        }
    }
    __syncthreads();
    for (int qi = 0; qi < NQ; ++qi) {
        u64* pq = a.part + ((size_t)blk * NQ + qi) * a.Kp;
        u64* buf = cand + (size_t)qi * a.cap;
        int n = qi < nqb ? cnt[qi] : 0;
        u64 dropped = qi < nqb ? thr_key[qi] : 0ull;  // (rows below a compaction threshold were dropped)
        if (n > a.Kp) {
            const u64 t = block_kth_mem(buf, n, a.Kp, red);
            n = block_compact_mem(buf, pq, n, t, red);
            // keys below the Kp-th are dropped: its key bounds them (the refine's certificate
            // takes the largest such bound over blocks, ScreenArgs::drop)
            dropped = t > dropped ? t : dropped;
        } else {
            for (int j = tid; j < n; j += 256) pq[j] = buf[j];
        }
        for (int j = n + tid; j < a.Kp; j += 256) pq[j] = 0ull;
        if (a.drop && tid == 0 && dropped != 0ull) atomicMax(a.drop + qi, dropped);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// K6: IVF list scan -- the GEMV screen over the pages of one inverted list for the (few) queries
// that probe it.  At batch 256 / nprobe 32 / nlist 4096 a list is probed by ~2 queries, so each
// corpus byte feeds ~2 query dot products: HBM streaming, fp32 FMA, no MFMA.  256 threads,
// persistent over work items (list, page range, <= NQ queries); per (item, query) the best Kp
// keys (screen score, storage slot) are appended to the query's candidate list for k_refine.
// ------------------------------------------------------------------------------------------------
// One work item (list l, pages [p0, p1), nqi <= NQ queries) of the IVF scan, by one 256-thread
// block.  Shared state (thresholds, counts, query ids) is the caller's; the block is synchronised
// on entry and exit.  QL: the item's NQ queries staged in LDS (qsh, NQ x dpad fp32) and read from
// there per chunk, instead of 2 NQ global loads per lane and chunk beside the corpus loads.
template <int DT, int NQ, bool QL = false>
__device__ __forceinline__ void ivf_scan_item(const IvfScanArgs& a, const int* itm, u64* cand, u64* thr_key,
                                              float* thr_f, int* cnt, int* qid, int* red, int* off_s,
                                              float* qsh = nullptr) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    constexpr int CE = CHB / ES;  // elements per chunk
    constexpr int CB = CHB;
    constexpr int LPR = CB / 16;
    constexpr int RPI = 64 / LPR;
    constexpr int EPU = 16 / ES;
    constexpr int RG = 64 / RPI;
    constexpr int RB0 = (NQ <= 2) ? 8 : 4;  // rows per pass (register budget of the shared dyn kernel)
    constexpr int RB = RB0 < RG ? RB0 : RG;
    static_assert(RG % RB == 0, "row groups");
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int unit = lane % LPR, rsub = lane / LPR;
    const int nch = a.dpad / CE;
    const int64_t tbytes = (int64_t)TR * a.dpad * ES;
    const int trigger = a.cap - TR;
    const int l = itm[0], p0 = itm[1], p1 = itm[2], nqi = itm[3];
    if (tid < NQ) {
        const bool real = tid < nqi;
        thr_key[tid] = real ? 0ull : ~0ull;
        thr_f[tid] = real ? -INFINITY : INFINITY;
        cnt[tid] = 0;
        qid[tid] = real ? itm[4 + tid] : itm[4];
    }
    __syncthreads();
    if constexpr (QL) {  // (padding slots: copies of the item's first query, as qid)
        const int n4 = a.dpad / 4;
        for (int i = tid; i < NQ * n4; i += 256) {
            const int qi = i / n4, j = i - qi * n4;
            ((float4*)qsh)[i] = ((const float4*)(a.qp + (int64_t)qid[qi] * a.dpad))[j];
        }
        __syncthreads();
    }
    const int64_t ln = a.list_n[l];
    const int pbase = a.page_off[l];
    for (int p = p0; p < p1; ++p) {
        const int64_t page = a.list_pages[pbase + p];
        const int nvalid = (int)(ln - (int64_t)p * TR < TR ? ln - (int64_t)p * TR : TR);
        const uint8_t* tb = a.data + page * tbytes;
        const int64_t slot0 = page * TR;
        for (int gb = 0; gb < RG / RB; ++gb) {
            float acc[RB][NQ];
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) acc[r][qi] = 0.0f;
#pragma unroll 2
            for (int c = 0; c < nch; ++c) {
                float qv[NQ][EPU];
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
#pragma unroll
                    for (int h = 0; h < EPU / 4; ++h) {
                        float4 t;
                        if constexpr (QL) t = ((const float4*)(qsh + qi * a.dpad + c * CE + unit * EPU))[h];
                        else t = ((const float4*)(a.qp + (int64_t)qid[qi] * a.dpad + c * CE + unit * EPU))[h];
                        qv[qi][4 * h + 0] = t.x; qv[qi][4 * h + 1] = t.y;
                        qv[qi][4 * h + 2] = t.z; qv[qi][4 * h + 3] = t.w;
                    }
                }
                uint4 raw[RB];
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int rit = wid * 64 + (gb * RB + r) * RPI + rsub;
                    raw[r] = ld_nt16(tb + (int64_t)c * TR * CB + rit * CB + unit * 16);
                }
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    float xv[EPU];
                    unpack16<DT>(raw[r], xv);
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi)
#pragma unroll
                        for (int e = 0; e < EPU; ++e) acc[r][qi] = fmaf(xv[e], qv[qi][e], acc[r][qi]);
                }
            }
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
                    float v = acc[r][qi];
#pragma unroll
                    for (int s = 1; s < LPR; s <<= 1) v += __shfl_xor(v, s, 64);
                    acc[r][qi] = v;
                }
            if (unit == 0) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const int rit = wid * 64 + (gb * RB + r) * RPI + rsub;
                    if (rit >= nvalid) continue;  // page padding of the list's last page
                    const int64_t slot = slot0 + rit;
                    const float sq = a.metric == METRIC_L2 ? a.sqn[slot] : 0.0f;
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi) {
                        float sc = acc[r][qi];
                        if (a.metric == METRIC_L2) sc = 2.0f * sc - sq;
                        if (sc >= thr_f[qi]) {
                            const u64 key = mk_key(sc, (uint32_t)slot);
                            if (key > thr_key[qi]) {
                                const int s = atomicAdd(&cnt[qi], 1);
                                if (s < a.cap) cand[(size_t)qi * a.cap + s] = key;
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
        for (int qi = 0; qi < nqi; ++qi) {
            const int n = cnt[qi];
            if (n > trigger) {  // block-uniform
                u64* buf = cand + (size_t)qi * a.cap;
                const u64 t = block_kth_mem(buf, n, a.Kp, red);
                block_compact_mem(buf, buf, n, t, red);
                if (tid == 0) {
                    thr_key[qi] = t;
                    thr_f[qi] = key_score(t);
                    cnt[qi] = a.Kp;
                }
                __syncthreads();
            }
        }
    }
    __syncthreads();
    // flush: the item's best <= Kp keys per query, appended to the query's candidate list
    for (int qi = 0; qi < nqi; ++qi) {
        u64* buf = cand + (size_t)qi * a.cap;
        int n = cnt[qi] < a.cap ? cnt[qi] : a.cap;
        if (n > a.Kp) {
            const u64 t = block_kth_mem(buf, n, a.Kp, red);
            n = block_compact_mem(buf, buf, n, t, red);
        }
        if (tid == 0) *off_s = n ? atomicAdd(&a.gcnt[qid[qi]], n) : 0;
        __syncthreads();
        u64* dst = a.glist + (size_t)qid[qi] * a.lcap + *off_s;
        for (int j = tid; j < n; j += 256) dst[j] = buf[j];
        __syncthreads();
    }
}

// All query-count classes in ONE persistent launch with dynamic item fetch (an atomic counter):
// the host orders items most expensive class first, so no per-class launch tail idles the HBM
// stream and no block waits on a static share of heavier items.
template <int DT, bool QL>
__global__ void __launch_bounds__(256, 3) k_ivf_scan_dyn(IvfScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) float qsh[];  // QL: [IVF_QG][dpad]
    __shared__ u64 thr_key[IVF_QG];
    __shared__ float thr_f[IVF_QG];
    __shared__ int cnt[IVF_QG];
    __shared__ int qid[IVF_QG];
    __shared__ int red[8];
    __shared__ int off_s, item_s;
    u64* cand = a.cand + (size_t)blockIdx.x * IVF_QG * a.cap;
    for (;;) {
        __syncthreads();  // the previous item is flushed, item_s is free
        if (threadIdx.x == 0) item_s = atomicAdd(a.next_item, 1);
        __syncthreads();
        const int it = item_s;
        if (it >= a.n_items) break;  // block-uniform: every wave leaves here, the queue is drained
        const int* itm = a.items + (size_t)it * IVF_ITEM_INTS;
        const int nqi = itm[3];
        if (nqi <= 1) ivf_scan_item<DT, 1, QL>(a, itm, cand, thr_key, thr_f, cnt, qid, red, &off_s, qsh);
        else if (nqi <= 2) ivf_scan_item<DT, 2, QL>(a, itm, cand, thr_key, thr_f, cnt, qid, red, &off_s, qsh);
        else if (nqi <= 4) ivf_scan_item<DT, 4, QL>(a, itm, cand, thr_key, thr_f, cnt, qid, red, &off_s, qsh);
        else ivf_scan_item<DT, IVF_QG, QL>(a, itm, cand, thr_key, thr_f, cnt, qid, red, &off_s, qsh);
    }
}

template <int DT, int NQ>
__global__ void __launch_bounds__(256) k_ivf_scan(IvfScanArgs a) {
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    constexpr int CE = CHB / ES;  // elements per chunk
    constexpr int CB = CHB;
    constexpr int LPR = CB / 16;
    constexpr int RPI = 64 / LPR;
    constexpr int EPU = 16 / ES;
    constexpr int RG = 64 / RPI;
    constexpr int RB0 = (NQ <= 2) ? 8 : 4;
    constexpr int RB = RB0 < RG ? RB0 : RG;
    static_assert(RG % RB == 0, "row groups");

    __shared__ u64 thr_key[NQ];
    __shared__ float thr_f[NQ];
    __shared__ int cnt[NQ];
    __shared__ int qid[NQ];
    __shared__ int red[8];
    __shared__ int off_s;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int unit = lane % LPR, rsub = lane / LPR;
    const int nch = a.dpad / CE;
    const int64_t tbytes = (int64_t)TR * a.dpad * ES;
    u64* cand = a.cand + (size_t)blockIdx.x * NQ * a.cap;
    const int trigger = a.cap - TR;

    for (int it = blockIdx.x; it < a.n_items; it += gridDim.x) {
        const int* itm = a.items + (size_t)it * IVF_ITEM_INTS;
        const int l = itm[0], p0 = itm[1], p1 = itm[2], nqi = itm[3];
        __syncthreads();  // the previous item's buffers are flushed
        if (tid < NQ) {
            const bool real = tid < nqi;
            thr_key[tid] = real ? 0ull : ~0ull;
            thr_f[tid] = real ? -INFINITY : INFINITY;
            cnt[tid] = 0;
            qid[tid] = real ? itm[4 + tid] : itm[4];
        }
        __syncthreads();
        const int64_t ln = a.list_n[l];
        const int pbase = a.page_off[l];
        for (int p = p0; p < p1; ++p) {
            const int64_t page = a.list_pages[pbase + p];
            const int nvalid = (int)(ln - (int64_t)p * TR < TR ? ln - (int64_t)p * TR : TR);
            const uint8_t* tb = a.data + page * tbytes;
            const int64_t slot0 = page * TR;
            for (int gb = 0; gb < RG / RB; ++gb) {
                float acc[RB][NQ];
#pragma unroll
                for (int r = 0; r < RB; ++r)
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi) acc[r][qi] = 0.0f;
#pragma unroll 2
                for (int c = 0; c < nch; ++c) {
                    float qv[NQ][EPU];
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi) {
                        const float4* qs = (const float4*)(a.qp + (int64_t)qid[qi] * a.dpad + c * CE + unit * EPU);
#pragma unroll
                        for (int h = 0; h < EPU / 4; ++h) {
                            float4 t = qs[h];
                            qv[qi][4 * h + 0] = t.x; qv[qi][4 * h + 1] = t.y;
                            qv[qi][4 * h + 2] = t.z; qv[qi][4 * h + 3] = t.w;
                        }
                    }
                    uint4 raw[RB];
#pragma unroll
                    for (int r = 0; r < RB; ++r) {
                        const int rit = wid * 64 + (gb * RB + r) * RPI + rsub;
                        raw[r] = *(const uint4*)(tb + (int64_t)c * TR * CB + rit * CB + unit * 16);
                    }
#pragma unroll
                    for (int r = 0; r < RB; ++r) {
                        float xv[EPU];
                        unpack16<DT>(raw[r], xv);
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi)
#pragma unroll
                            for (int e = 0; e < EPU; ++e) acc[r][qi] = fmaf(xv[e], qv[qi][e], acc[r][qi]);
                    }
                }
#pragma unroll
                for (int r = 0; r < RB; ++r)
#pragma unroll
                    for (int qi = 0; qi < NQ; ++qi) {
                        float v = acc[r][qi];
#pragma unroll
                        for (int s = 1; s < LPR; s <<= 1) v += __shfl_xor(v, s, 64);
                        acc[r][qi] = v;
                    }
                if (unit == 0) {
#pragma unroll
                    for (int r = 0; r < RB; ++r) {
                        const int rit = wid * 64 + (gb * RB + r) * RPI + rsub;
                        if (rit >= nvalid) continue;  // page padding of the list's last page
                        const int64_t slot = slot0 + rit;
                        const float sq = a.metric == METRIC_L2 ? a.sqn[slot] : 0.0f;
#pragma unroll
                        for (int qi = 0; qi < NQ; ++qi) {
                            float sc = acc[r][qi];
                            if (a.metric == METRIC_L2) sc = 2.0f * sc - sq;
                            if (sc >= thr_f[qi]) {
                                const u64 key = mk_key(sc, (uint32_t)slot);
                                if (key > thr_key[qi]) {
                                    const int s = atomicAdd(&cnt[qi], 1);
                                    if (s < a.cap) cand[(size_t)qi * a.cap + s] = key;
                                }
                            }
                        }
                    }
                }
            }
            __syncthreads();
            for (int qi = 0; qi < nqi; ++qi) {
                const int n = cnt[qi];
                if (n > trigger) {  // block-uniform
                    u64* buf = cand + (size_t)qi * a.cap;
                    const u64 t = block_kth_mem(buf, n, a.Kp, red);
                    block_compact_mem(buf, buf, n, t, red);
                    if (tid == 0) {
                        thr_key[qi] = t;
                        thr_f[qi] = key_score(t);
                        cnt[qi] = a.Kp;
                    }
                    __syncthreads();
                }
            }
        }
        __syncthreads();
        // flush: the item's best <= Kp keys per query, appended to the query's candidate list
        for (int qi = 0; qi < nqi; ++qi) {
            u64* buf = cand + (size_t)qi * a.cap;
            int n = cnt[qi] < a.cap ? cnt[qi] : a.cap;
            if (n > a.Kp) {
                const u64 t = block_kth_mem(buf, n, a.Kp, red);
                n = block_compact_mem(buf, buf, n, t, red);
            }
            if (tid == 0) off_s = n ? atomicAdd(&a.gcnt[qid[qi]], n) : 0;
            __syncthreads();
            u64* dst = a.glist + (size_t)qid[qi] * a.lcap + off_s;
            for (int j = tid; j < n; j += 256) dst[j] = buf[j];
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// K3: merge of partial candidate lists (block-wide selection)
// ------------------------------------------------------------------------------------------------
// MERGE_E keys per thread: 4096 keys per block (16) or 8192 (32, screening depths above 2048)
template <int MERGE_E>
__global__ void __launch_bounds__(256) k_merge(const u64* __restrict__ in, int nseg, int qstride, int nq, int Kp,
                                               int spb, u64* __restrict__ out) {
    __shared__ int red[8];
    const int q = blockIdx.y, b = blockIdx.x, tid = threadIdx.x;
    const int s0 = b * spb;
    const int s1 = min(nseg, s0 + spb);
    const int n = (s1 - s0) * Kp;
    u64 keys[MERGE_E];
    int nvalid = 0;
#pragma unroll
    for (int e = 0; e < MERGE_E; ++e) {
        const int idx = tid + 256 * e;
        u64 k = 0ull;
        if (idx < n) {
            const int s = s0 + idx / Kp, j = idx % Kp;
            k = in[((size_t)s * qstride + q) * Kp + j];
        }
        keys[e] = k;
        nvalid += k != 0ull;
    }
    nvalid = wave_sum_i(nvalid);
    if ((tid & 63) == 0) red[tid >> 6] = nvalid;
    __syncthreads();
    int tot = 0;
    for (int i = 0; i < 4; ++i) tot += red[i];
    __syncthreads();
    const u64 t = tot > Kp ? block_kth<MERGE_E>(keys, Kp, red) : 1ull;
    u64* o = out + ((size_t)b * nq + q) * Kp;
    const int kept = block_write_kept<MERGE_E>(keys, t, o, red);
    for (int j = kept + tid; j < Kp; j += 256) o[j] = 0ull;
}


constexpr int RF_THREADS = 1024;  // 16 waves per query: Kp / 16 candidates per wave
constexpr int RF_E = 16;          // candidate keys per thread held in registers for the selection
constexpr int RF_WE = 32;         // lists up to 64 * RF_WE keys: threshold found by one wave
static_assert(64 * RF_WE == kRefineOneWaveKeys, "one-wave selection size");
static_assert(RF_THREADS * RF_E == kRefineRegKeys, "register selection size");

template <int DT, int METRIC, bool QLDS>
__device__ __forceinline__ void refine(const RefineArgs& a, int KP2) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    double* sc = (double*)smem;
    uint32_t* ids = (uint32_t*)(smem + (size_t)KP2 * 8);
    double* qs = (double*)(smem + (((size_t)KP2 * 12 + 7) & ~(size_t)7));  // 8-B aligned
    __shared__ int nv_s;
    __shared__ u64 minkey_s, thr_s;
    __shared__ double qq_s;
    __shared__ int red[2 * (RF_THREADS / 64)];
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NW = RF_THREADS / 64;
    // the best Kp keys of the candidate list, compacted into LDS (cq)
    // the query sits in LDS transposed, qs[e * ng + g] = q[8 g + e]: lane g of the exact scoring
    // reads element e of its 8-element group, so a wave's reads are contiguous (conflict-free)
    const int ng = (a.d + 7) >> 3;
    u64* cq = (u64*)(smem + (((size_t)KP2 * 12 + 7) & ~(size_t)7) + (QLDS ? (size_t)ng * 64 : 0));
    const u64* src = a.cand + (size_t)q * a.lcap;
    const int n = a.cand_n ? min(a.cand_n[q], a.lcap) : a.lcap;
    const float* qv = a.q + (int64_t)q * a.d;
    if (tid == 0) {
        nv_s = 0;
        minkey_s = ~0ull;
    }
    if constexpr (QLDS)
        for (int i = tid; i < a.d; i += RF_THREADS) qs[(i & 7) * ng + (i >> 3)] = (double)qv[i];
    int nkept;
    if (n <= RF_THREADS * RF_E) {
        u64 keys[RF_E];
#pragma unroll
        for (int e = 0; e < RF_E; ++e) {
            const int j = tid + RF_THREADS * e;
            keys[e] = j < n ? src[j] : 0ull;
        }
        // the best Kp..KP2 keys (any count in that range: the bisection stops early; every kept key
        // is scored, and the certificate uses the Kp-th best key below)
        u64 t = 1ull;
        if (n > KP2) {
            if (n <= 64 * RF_WE) {  // typical seeded list: one wave finds the threshold, no block barriers
                if (wid == 0) {
                    u64 wk[RF_WE];
#pragma unroll
                    for (int e = 0; e < RF_WE; ++e) {
                        const int j = lane + 64 * e;
                        wk[e] = j < n ? src[j] : 0ull;
                    }
                    const u64 tw = wave_kth_range<RF_WE>(wk, a.Kp, KP2);
                    if (lane == 0) thr_s = tw;
                }
                __syncthreads();
                t = thr_s;
            } else {
                // (the radix select takes exactly Kp at about the cost of a range: the one-wave
                // Kp-th search below is then not needed, and only Kp rows are scored)
                t = block_kth<RF_E>(keys, a.Kp, red);
            }
        }
        nkept = block_write_kept<RF_E>(keys, t, cq, red);
    } else {  // very long lists (unseeded screens of many workgroups): selection from memory
        const u64 t = block_kth_range_mem(src, n, a.Kp, KP2, red);
        nkept = block_compact_mem(src, cq, n, t, red);
    }
    __syncthreads();
    // the Kp-th best listed key bounds every listed row not kept and every row a screen block
    // dropped below its own Kp-th (a block's Kp-th key is at most the Kp-th over all lists); with
    // more than Kp kept it is found among the kept keys by one wave
    if (nkept > a.Kp && wid == 0) {
        const u64 kk = wave_kth_buf(cq, nkept, a.Kp);
        if (lane == 0) thr_s = kk;
    }
    int myv = 0;
    u64 mymin = ~0ull;
    for (int j = tid; j < nkept; j += RF_THREADS) {
        const u64 k = cq[j];
        ++myv;
        mymin = k < mymin ? k : mymin;
    }
    myv = wave_sum_i(myv);
    mymin = wave_min_u64(mymin);
    if (lane == 0) {
        atomicAdd(&nv_s, myv);
        atomicMin(&minkey_s, mymin);
    }
    if (wid == 1 && METRIC == METRIC_L2) {  // ||q||^2 for the L2 margin (staged query when in LDS)
        double s2 = 0.0;
        for (int i = lane; i < a.d; i += 64) {
            const double v = QLDS ? qs[(i & 7) * ng + (i >> 3)] : (double)qv[i];
            s2 += v * v;
        }
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) s2 += __shfl_xor(s2, s, 64);
        if (lane == 0) qq_s = s2;
    }
    __syncthreads();
    const int nv = nv_s;
    constexpr int RR = refine_rows<DT>();
    // split refine (a.nsplit > 1, blockIdx.y = slice): every workgroup of the query made the same
    // selection above; each scores its slice of cq into the query's global rows, the last to finish
    // gathers them and goes on alone
    const bool split = a.nsplit > 1;
    int jlo = 0, jhi = nv;
    if (split) {
        const int chunk = (nv + a.nsplit - 1) / a.nsplit;
        jlo = min(nv, (int)blockIdx.y * chunk);
        jhi = min(nv, jlo + chunk);
    }
    double* scw = split ? a.gsc + (size_t)q * KP2 : sc;
    uint32_t* idw = split ? a.gids + (size_t)q * KP2 : ids;
    for (int j = jlo + wid; j < jhi; j += RR * NW) {
        int64_t rr[RR];
#pragma unroll
        for (int i = 0; i < RR; ++i) rr[i] = j + i * NW < jhi ? (int64_t)key_id(cq[j + i * NW]) : -1;
        double s4[RR];
        exact_score_rows<DT, METRIC, QLDS, RR>(a.corpus, rr, qs, qv, a.d, a.dpad, lane, s4);
        if (lane == 0) {  // keys carry storage slots; IVF maps them to user ids (sort + output)
#pragma unroll
            for (int i = 0; i < RR; ++i)
                if (rr[i] >= 0) {
                    const uint32_t uid = a.idmap ? a.idmap[rr[i]] : (uint32_t)rr[i];
                    if (split) {  // (handed to the query's last workgroup: sc1 stores)
                        st_agent(scw + j + i * NW, s4[i]);
                        st_agent(idw + j + i * NW, uid);
                    } else {
                        scw[j + i * NW] = s4[i];
                        idw[j + i * NW] = uid;
                    }
                }
        }
    }
    if (split) {
        // the last of the query's workgroups takes over: sc1 stores above, every storing wave's
        // vmcnt(0), one agent-scope counter add per workgroup, sc1 loads (no cache fences)
        __shared__ int last_s;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            last_s = __hip_atomic_fetch_add(a.gdone + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                             (unsigned)(a.nsplit - 1) ? 1 : 0;
        __syncthreads();
        if (!last_s) return;
        for (int j = tid; j < nv; j += RF_THREADS) {
            sc[j] = ld_agent(scw + j);
            ids[j] = ld_agent(idw + j);
        }
        if (tid == 0) st_agent(a.gdone + q, 0u);  // ready for the next launch
    }
    const double worst = METRIC == METRIC_IP ? -INFINITY : INFINITY;
    for (int j = nv + tid; j < KP2; j += RF_THREADS) {
        sc[j] = worst;
        ids[j] = 0xFFFFFFFFu;
    }
    __syncthreads();
    sort_valid_best_first<METRIC>(sc, ids, nv, KP2);  // best first
    // exactness certificate: every non-candidate row has exact transformed score <= smin + eps
    if (tid == 0) {
        // rows outside the candidate set scored at most: the Kp-th best listed key (when the list
        // was cut to Kp), or a workgroup's compaction bound (deep searches keep MFMA_KP_MAX per
        // workgroup), whichever is larger
        u64 th = nv > a.Kp ? thr_s : nv == a.Kp ? minkey_s : 0ull;
        if (a.drop && a.drop[q] > th) th = a.drop[q];
        int cert = 1;
        if (a.optimistic && nv < a.Kp) cert = 0;  // an optimistic seed may have cut real candidates
        else if (th != 0ull && a.k > nv) cert = 0;
        else if (th != 0ull) {
            const double smin = (double)key_score(th);
            const double qh = (double)a.qinfo[2 * q], dq = (double)a.qinfo[2 * q + 1];
            const double xm = (double)a.xmax;
            double eps = ((double)a.gamma * qh + dq) * xm * 1.01 + 1e-30;
            if (a.i8max) {  // int8 GEMV keys: fp32 dot of the codes (gamma) + the key's 3 roundings
                const double X = (double)__uint_as_float(a.i8max[0]), B = (double)__uint_as_float(a.i8max[1]);
                eps = ((double)a.gamma * X + 3.0 * 5.9604644775390625e-08 * (X + B)) * qh * 1.01 + 1e-30;
            }
            double tk = sc[a.k - 1];
            if (a.metric == METRIC_L2) {
                eps = 2.0 * eps + ((double)a.gamma + 4.0 * 5.9604644775390625e-08) * (xm * xm + 2.0 * xm * qh) * 1.01 +
                      1e-12 * (qq_s + xm * xm);
                tk = qq_s - tk;
            }
            cert = tk > smin + eps ? 1 : 0;
        }
        if (a.cert) a.cert[q] = cert;
        if (!cert && a.uncert) atomicAdd(a.uncert, 1u);
        if (!cert && a.fails) atomicAdd(a.fails, 1);
    }
    for (int j = tid; j < a.k; j += RF_THREADS) {
        const size_t o = (size_t)q * a.k + j, ost = a.ostride > 1 ? (size_t)a.ostride : 1;
        if (j < nv) {
            if (a.D) a.D[o] = (float)sc[j];
            a.I[o * ost] = (int64_t)ids[j] + a.id_offset;
            if (a.S64) a.S64[o * ost] = sc[j];
        } else {
            if (a.D) a.D[o] = a.metric == METRIC_IP ? -3.402823466e+38f : 3.402823466e+38f;
            a.I[o * ost] = -1;
            if (a.S64) a.S64[o * ost] = a.metric == METRIC_IP ? -1.7976931348623157e308 : 1.7976931348623157e308;
        }
    }
}

template <int DT, int METRIC, bool QLDS>
__global__ void __launch_bounds__(RF_THREADS) k_refine(RefineArgs a, int KP2) {
    refine<DT, METRIC, QLDS>(a, KP2);
}
// the device fallback round's refine: only queries the first pass left uncertified (own symbol,
// as k_screen_mfma_redo)
template <int DT, int METRIC, bool QLDS>
__global__ void __launch_bounds__(RF_THREADS) k_refine_redo(RefineArgs a, int KP2) {
    if (*a.gate == 0 || a.cert[blockIdx.x] != 0) return;
    refine<DT, METRIC, QLDS>(a, KP2);
}

// ------------------------------------------------------------------------------------------------
// K5w: exact refine behind the int8 screen and the native MFMA screen's first passes (inner
// product) -- adaptive depth, two phases, one block per query.  The screen keys are within qeps of
// the true score from above: int8 keys are upper bounds, true <x, q> <= key_score + qeps[q]
// (k_pack_qtile_i8); native keys are within the native margin either way.
//  A: the best KA keys of the query's survivor list are scored exactly (canonical fp64); T' = the
//     k-th best of them is a lower bound of the final k-th best exact score T.
//  B: every other key with key_score >= T' - qeps could still reach T': those rows are scored too.
//     Every survivor left unscored has true < T' <= T.
//  Certificate: rows never listed (below the seed threshold thr0 or a workgroup's compaction bound
//  drop) have true <= key_score(max(thr0, drop)) + qeps, which must be < T; and the rows scored
//  must fit the block's RFW_CAP slots.
// ------------------------------------------------------------------------------------------------

// order-preserving block compaction of this thread's keys in [lo, hi) to ids[base + ...]; returns
// the block total
template <int E>
__device__ __forceinline__ int block_write_ids(const u64 (&keys)[E], u64 lo, u64 hi, uint32_t* out, int cap, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int c = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) c += (keys[e] >= lo && keys[e] < hi) ? 1 : 0;
    int incl = c;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        const int v = __shfl_up(incl, s, 64);
        if (lane >= s) incl += v;
    }
    if (lane == 63) red[w] = incl;
    __syncthreads();
    int base = 0, total = 0;
    for (int i = 0; i < nw; ++i) {
        if (i < w) base += red[i];
        total += red[i];
    }
    __syncthreads();
    int pos = base + incl - c;
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (keys[e] >= lo && keys[e] < hi) {
            if (pos < cap) out[pos] = key_id(keys[e]);
            ++pos;
        }
    return total;
}

// scores of ids[lo, hi) into sc[lo, hi): 16 waves, two rows in flight per wave.  L2: sc holds the
// negated canonical distance, so one order (higher first, ties to the lower id) serves both metrics
template <int DT, int METRIC, bool QLDS>
__device__ __forceinline__ void rfw_score(const RefineArgs& a, const uint32_t* ids, double* sc, int lo, int hi,
                                          const double* qs, const float* qv) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NW = RF_THREADS / 64;
    constexpr int RR = refine_rows<DT>();
    for (int j = lo + wid; j < hi; j += RR * NW) {
        int64_t rr[RR];
#pragma unroll
        for (int i = 0; i < RR; ++i) rr[i] = j + i * NW < hi ? (int64_t)ids[j + i * NW] : -1;
        double s4[RR];
        exact_score_rows<DT, METRIC, QLDS, RR>(a.corpus, rr, qs, qv, a.d, a.dpad, lane, s4);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < RR; ++i)
                if (rr[i] >= 0) sc[j + i * NW] = METRIC == METRIC_L2 ? -s4[i] : s4[i];
        }
    }
}

template <int DT, int METRIC, bool QLDS>
__global__ void __launch_bounds__(RF_THREADS) k_refine_wide(RefineArgs a, int KA) {
    constexpr bool L2 = METRIC == METRIC_L2;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    double* sc = (double*)smem;                                  // [RFW_CAP]
    uint32_t* ids = (uint32_t*)(smem + (size_t)RFW_CAP * 8);     // [RFW_CAP]
    double* qs = (double*)(smem + (size_t)RFW_CAP * 12);         // fp64 query, transposed groups
    __shared__ int red[2 * (RF_THREADS / 64)];
    __shared__ int nb_s;
    __shared__ double qq_s;
    const int q = blockIdx.x, tid = threadIdx.x;
    // a device fallback round: only the block's uncertified queries, and only when there are any
    if (a.redo && (*a.gate == 0 || a.cert[q] != 0)) return;
    const int ng = (a.d + 7) >> 3;
    const u64* src = a.cand + (size_t)q * a.lcap;
    const int n = min(a.cand_n[q], a.lcap);
    const float* qv = a.q + (int64_t)q * a.d;
    if constexpr (QLDS)
        for (int i = tid; i < a.d; i += RF_THREADS) qs[(i & 7) * ng + (i >> 3)] = (double)qv[i];
    // the key's margin: int8 keys carry theirs per query (upper bounds: true <= key + qeps); native
    // MFMA keys (qeps == null) are within the native screen's two-sided error of the true score
    // (the same bound as k_refine's certificate: fp32 accumulation + query rounding, times max ||x||)
    double eps = a.qeps ? (double)a.qeps[q]
                        : ((double)a.gamma * (double)a.qinfo[2 * q] + (double)a.qinfo[2 * q + 1]) *
                                  (double)a.xmax * 1.01 + 1e-30;
    // L2 (int8 keys of 2 <x, q> - ||x||^2, margin in qeps): the canonical distance D is compared with
    // the keys as ||q||^2 - D, whose fp64 evaluation adds ~1e-16 relative (budgeted 1e-12)
    double qq = 0.0;
    if constexpr (L2) {
        if (tid < 64) {
            double s2 = 0.0;
            for (int i = tid; i < a.d; i += 64) s2 += (double)qv[i] * (double)qv[i];
            s2 = wave_sum_f64(s2);
            if (tid == 0) qq_s = s2;
        }
        __syncthreads();
        qq = qq_s;
        eps += 1e-12 * (qq + (double)a.xmax * (double)a.xmax);
    }
    const double worst = -INFINITY;
    // ---- phase A: the best KA keys ----
    u64 keys[RF_E];
    const bool inreg = n <= RF_THREADS * RF_E;
    u64 tA = 1ull;  // keys >= tA form phase A
    int nA, nA2 = 1;
    if (a.phase != 2) {
#pragma unroll
    for (int e = 0; e < RF_E; ++e) {
        const int j = tid + RF_THREADS * e;
        keys[e] = (inreg && j < n) ? src[j] : 0ull;
    }
    // phase A: the best KA..rfw_ka_hi(KA) keys (any count in that range serves: T' and the phase-B
    // window follow from the rows actually scored, and the range stops the bisection early)
    if (n > KA) {
        const int Khi = rfw_ka_hi(KA);
        tA = inreg ? block_kth_range<RF_E>(keys, KA, Khi, red) : block_kth_range_mem(src, n, KA, Khi, red);
    }
    if (inreg) {
        nA = block_write_ids<RF_E>(keys, tA, ~0ull, ids, RFW_CAP, red);
    } else {  // very long lists: the phase-A set from memory (block_compact_mem writes keys)
        nA = 0;
        for (int r0 = 0; r0 < n; r0 += RF_THREADS) {
            const int j = r0 + tid;
            const u64 k = j < n ? src[j] : 0ull;
            const bool keep = k >= tA;
            const u64 m = __ballot(keep);
            if ((tid & 63) == 0) red[tid >> 6] = __popcll(m);
            __syncthreads();
            int wb = 0, tot = 0;
            for (int i = 0; i < RF_THREADS / 64; ++i) {
                if (i < (tid >> 6)) wb += red[i];
                tot += red[i];
            }
            __syncthreads();
            const int pos = nA + wb + lane_prefix(m);
            if (keep && pos < RFW_CAP) ids[pos] = key_id(k);
            nA += tot;
        }
    }
    nA = min(nA, RFW_CAP);
    __syncthreads();
    rfw_score<DT, METRIC, QLDS>(a, ids, sc, 0, nA, qs, qv);
    __syncthreads();
    while (nA2 < nA) nA2 <<= 1;
    for (int j = nA + tid; j < nA2; j += RF_THREADS) {
        sc[j] = worst;
        ids[j] = 0xFFFFFFFFu;
    }
    __syncthreads();
    sort_valid_best_first<METRIC_IP>(sc, ids, nA, nA2);  // phase A best first (nA2 <= RFW_CAP: KA <= RFW_CAP / 2)
    } else {  // phase 2: resume from the phase-1 state
        nA = a.pa_n[q];
        tA = a.pa_tA[q];
        while (nA2 < nA) nA2 <<= 1;
        for (int j = tid; j < nA2; j += RF_THREADS) {
            sc[j] = j < nA ? a.pa_sc[(size_t)q * a.pa_cap + j] : worst;
            ids[j] = j < nA ? a.pa_ids[(size_t)q * a.pa_cap + j] : 0xFFFFFFFFu;
        }
        __syncthreads();
    }
    if (a.phase == 1) {  // phase 1 ends here: its state, and its top-k for the exchange
        for (int j = tid; j < nA; j += RF_THREADS) {
            a.pa_sc[(size_t)q * a.pa_cap + j] = sc[j];
            a.pa_ids[(size_t)q * a.pa_cap + j] = ids[j];
        }
        if (tid == 0) {
            a.pa_n[q] = nA;
            a.pa_tA[q] = tA;
        }
        for (int j = tid; j < a.k; j += RF_THREADS) {
            const size_t o = (size_t)q * a.k + j, ost = a.ostride > 1 ? (size_t)a.ostride : 1;
            const double v = j < nA ? (L2 ? -sc[j] : sc[j]) : (L2 ? 1.7976931348623157e308 : -1.7976931348623157e308);
            if (a.D) a.D[o] = j < nA ? (float)v : (L2 ? 3.402823466e+38f : -3.402823466e+38f);
            a.I[o * ost] = j < nA ? (int64_t)ids[j] + a.id_offset : -1;
            if (a.S64) a.S64[o * ost] = v;
        }
        return;
    }
    // the exchange's floor: a lower bound of the global k-th best score (all shards' phase-1 rows)
    double floor_sc = -INFINITY;
    if (a.tfloor) {
        const double f = L2 ? -a.tfloor[(size_t)q * a.tfloor_k + a.tfloor_k - 1]
                            : a.tfloor[(size_t)q * a.tfloor_k + a.tfloor_k - 1];
        if (f > -1.7976931348623157e308) floor_sc = f;  // (padding -DBL_MAX / +DBL_MAX distance: none)
    }
    const double Tp = fmax(nA >= a.k ? sc[a.k - 1] : -INFINITY, floor_sc);
    // ---- phase B: keys in [tB, tA) whose bound reaches T' ----
    u64 tB = 1ull;
    if (Tp > -INFINITY) {
        const double TpK = L2 ? qq + Tp : Tp;  // T' in the keys' domain
        float f = (float)(TpK - eps);
        if ((double)f > TpK - eps) f = nextafterf(f, -INFINITY);  // round down: keys below tB score < T' - eps
        tB = (u64)ord_f32(f) << 32;
        if (tB == 0ull) tB = 1ull;
    }
    int nB = 0;
    if (tB < tA) {
        if (inreg) {
            // the keys are reloaded (L2-hot list) rather than held across phase A's scoring, where
            // their 32 VGPRs would push the gathers' registers into scratch
#pragma unroll
            for (int e = 0; e < RF_E; ++e) {
                const int j = tid + RF_THREADS * e;
                keys[e] = j < n ? __builtin_nontemporal_load(src + j) : 0ull;
            }
            nB = block_write_ids<RF_E>(keys, tB, tA, ids + nA2, RFW_CAP - nA2, red);
        } else {
            for (int r0 = 0; r0 < n; r0 += RF_THREADS) {
                const int j = r0 + tid;
                const u64 k = j < n ? src[j] : 0ull;
                const bool keep = k >= tB && k < tA;
                const u64 m = __ballot(keep);
                if ((tid & 63) == 0) red[tid >> 6] = __popcll(m);
                __syncthreads();
                int wb = 0, tot = 0;
                for (int i = 0; i < RF_THREADS / 64; ++i) {
                    if (i < (tid >> 6)) wb += red[i];
                    tot += red[i];
                }
                __syncthreads();
                const int pos = nB + wb + lane_prefix(m);
                if (keep && pos < RFW_CAP - nA2) ids[nA2 + pos] = key_id(k);
                nB += tot;
            }
        }
    }
    const bool overflow = nA2 + nB > RFW_CAP;
    nB = min(nB, RFW_CAP - nA2);
    __syncthreads();
    rfw_score<DT, METRIC, QLDS>(a, ids, sc, nA2, nA2 + nB, qs, qv);
    __syncthreads();
    // phase-B rows that beat T' join the phase-A list (order-preserving compaction in place)
    if (tid == 0) nb_s = 0;
    __syncthreads();
    for (int r0 = 0; r0 < nB; r0 += RF_THREADS) {
        const int j = r0 + tid;
        const bool keep = j < nB && !(sc[nA2 + j] < Tp);  // >= T' (T' = -inf: every row)
        const double s = keep ? sc[nA2 + j] : 0.0;
        const uint32_t id = keep ? ids[nA2 + j] : 0u;
        const u64 m = __ballot(keep);
        if ((tid & 63) == 0) red[tid >> 6] = __popcll(m);
        __syncthreads();
        int wb = 0, tot = 0;
        for (int i = 0; i < RF_THREADS / 64; ++i) {
            if (i < (tid >> 6)) wb += red[i];
            tot += red[i];
        }
        const int base = nb_s;
        __syncthreads();
        if (keep) {
            const int pos = nA + base + wb + lane_prefix(m);
            sc[pos] = s;
            ids[pos] = id;
        }
        if (tid == 0) nb_s = base + tot;
        __syncthreads();
    }
    const int nF = nA + nb_s;
    int nF2 = 1;
    while (nF2 < nF) nF2 <<= 1;
    for (int j = nF + tid; j < nF2; j += RF_THREADS) {
        sc[j] = worst;
        ids[j] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (nb_s > 0) sort_valid_best_first<METRIC_IP>(sc, ids, nF, nF2);
    // ---- certificate ----
    if (tid == 0) {
        u64 th = a.drop ? a.drop[q] : 0ull;
        if (a.thr0 && a.thr0[q] > th) th = a.thr0[q];
        int cert = overflow ? 0 : 1;
        if (cert && th != 0ull) {  // some rows were never listed
            // rows never listed score < T: below the k-th best of this shard's scored rows, or below
            // the exchange's floor (<= the global k-th best): in neither case in the global top-k
            const double Tl = fmax(nF >= a.k ? sc[a.k - 1] : -INFINITY, floor_sc);
            const double T = Tl > -INFINITY ? (L2 ? qq + Tl : Tl) : -INFINITY;
            cert = ((double)key_score(th) + eps < T) ? 1 : 0;
        }
        if (a.cert) a.cert[q] = cert;
        if (!cert && a.uncert) atomicAdd(a.uncert, 1u);
        if (!cert && a.fails) atomicAdd(a.fails, 1);
    }
    for (int j = tid; j < a.k; j += RF_THREADS) {
        const size_t o = (size_t)q * a.k + j, ost = a.ostride > 1 ? (size_t)a.ostride : 1;
        if (j < nF) {
            const double v = L2 ? -sc[j] : sc[j];
            if (a.D) a.D[o] = (float)v;
            a.I[o * ost] = (int64_t)ids[j] + a.id_offset;
            if (a.S64) a.S64[o * ost] = v;
        } else {
            if (a.D) a.D[o] = L2 ? 3.402823466e+38f : -3.402823466e+38f;
            a.I[o * ost] = -1;
            if (a.S64) a.S64[o * ost] = L2 ? 1.7976931348623157e308 : -1.7976931348623157e308;
        }
    }
}

// seed threshold from 16-row group maxima (one block per query): the rank-th largest maximum T
// has `rank` DISTINCT rows scoring >= T, so T never exceeds the true rank-th best screen score and
// the key just below every score >= T, (ord(T) << 32) | 0, is a valid starting threshold
// (rank = Kp: proven; rank < Kp: optimistic, checked by the refine certificate).
// Radix select over the block's value RANGE, one 256-thread block per query, maxima held in
// registers (VPT per thread): w = ord(v) - min, rounds of 8 bits from the top bit of max - min down
// (LDS histogram of the digit among the values matching the prefix so far, one wave scans the 256
// bins from the top) give the exact rank-th largest.  (Digits of the raw orderable value put all
// ~4k maxima -- one or two float exponents -- into one or two bins of the first two rounds, whose
// LDS atomics then serialise on a single address: 13 us per launch at the 8-shard step.)
constexpr int SEED_VPT = 16;  // up to 256 * 16 = 4096 maxima per query (2x / 4x variants below)
template <int VPT>
__global__ void __launch_bounds__(256) k_seed_select(const float* __restrict__ seedmax, int M, int nq, int rank,
                                                     u64* __restrict__ thr0) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_digit;
    __shared__ int s_rank;
    __shared__ unsigned s_mn[4], s_mx[4];
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    uint32_t v[VPT];
    unsigned mn = ~0u, mx = 0u;
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
        const int j = tid + 256 * e;
        v[e] = j < M ? ord_f32(seedmax[(size_t)q * M + j]) : 0u;
        if (j < M) {
            mn = min(mn, v[e]);
            mx = max(mx, v[e]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (unsigned)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    }
    if (lane == 0) {
        s_mn[tid >> 6] = mn;
        s_mx[tid >> 6] = mx;
    }
    __syncthreads();
    mn = min(min(s_mn[0], s_mn[1]), min(s_mn[2], s_mn[3]));
    mx = max(max(s_mx[0], s_mx[1]), max(s_mx[2], s_mx[3]));
    if (M < rank) {  // fewer than `rank` values: no threshold
        if (tid == 0) thr0[q] = 0ull;
        return;
    }
#pragma unroll
    for (int e = 0; e < VPT; ++e) v[e] -= mn;  // (padding: excluded by index below)
    const unsigned span = mx - mn;
    const int bits = span ? 32 - __builtin_clz(span) : 0;
    uint32_t prefix = 0u;
    int r = rank;
    for (int sh = bits - 8; sh > -8; sh -= 8) {
        // digit = bits [sh, sh + 8) of w (sh < 0: the low sh + 8 bits, left-aligned); the prefix
        // fixes the bits above sh + 8
        const uint32_t hmask = sh + 8 >= 32 ? 0u : ~0u << (sh + 8);
        hist[tid] = 0u;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < VPT; ++e)
            if (tid + 256 * e < M && (v[e] & hmask) == prefix)
                atomicAdd(&hist[(sh >= 0 ? v[e] >> sh : v[e] << -sh) & 255u], 1u);
        __syncthreads();
        if (tid < 64) {  // lane l holds bins 255-4l .. 252-4l (descending)
            unsigned c[4], sum = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                c[i] = hist[255 - 4 * lane - i];
                sum += c[i];
            }
            unsigned incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            const unsigned excl = incl - sum;
            const bool here = excl < (unsigned)r && incl >= (unsigned)r;
            if (here) {
                unsigned cum = excl;
                int i = 0;
                while (cum + c[i] < (unsigned)r) cum += c[i++];
                s_digit = 255u - 4u * lane - (unsigned)i;
                s_rank = r - (int)cum;
            }
        }
        __syncthreads();
        prefix |= sh >= 0 ? s_digit << sh : s_digit >> -sh;
        r = s_rank;
        __syncthreads();
    }
    if (tid == 0) {
        const uint32_t o = mn + prefix;
        const float T = unord_f32(o);
        thr0[q] = (o == 0u || T == -INFINITY) ? 0ull : ((u64)o << 32);
    }
}

// ------------------------------------------------------------------------------------------------
// merge of per-shard sorted results (after the RCCL all-gather)
// ------------------------------------------------------------------------------------------------
// one wave per query: lane g < G holds the head of shard list g; each of the k rounds picks the
// best head by a wave butterfly on (score, id) -- score desc (IP) / asc (L2), ties -> lower id --
// and the winning lane advances.  Lists end at their first id -1.
// Merge by rank (G * k <= kMergeRankMax, one 256-thread workgroup per query): the G lists go to
// LDS; every valid entry's output position is its index in its own list plus, for every other
// list, the number of that list's entries ahead of it -- a binary search, since each list is sorted
// under the same total order (score, then id, then list index) -- so no entry waits on another and
// the ~k dependent steps (each a global load) of k_merge_shards' wave-per-query merge are gone.
constexpr int kMergeRankMax = 4096;  // G * k entries (16 B each) in LDS
__global__ void __launch_bounds__(256) k_merge_shards_rank(int metric, const double* __restrict__ S_in,
                                                           const int64_t* __restrict__ I_in, int istride, int G,
                                                           int64_t nq, int k,
                                                           double* __restrict__ S_out, int64_t* __restrict__ I_out,
                                                           float* __restrict__ D_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    double* ss = (double*)smem;
    int64_t* si = (int64_t*)(smem + (size_t)G * k * 8);
    __shared__ int nval[64];
    const int64_t q = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = G * k;
    const bool ip = metric == METRIC_IP;
    if (tid < 64) nval[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
        const int g = i / k, j = i - g * k;
        const size_t o = (((size_t)g * nq + q) * k + j) * istride;
        const int64_t id = I_in[o];
        si[i] = id;
        ss[i] = id >= 0 ? S_in[o] : 0.0;
        if (id >= 0) atomicAdd(&nval[g], 1);  // (valid entries are each list's prefix)
    }
    __syncthreads();
    int total = 0;
    for (int g = 0; g < G; ++g) total += nval[g];
    for (int i = tid; i < n; i += 256) {
        const int g = i / k, j = i - g * k;
        if (j >= nval[g]) continue;
        const double s = ss[i];
        const int64_t id = si[i];
        int rank = j;
        for (int g2 = 0; g2 < G && rank < k; ++g2) {
            if (g2 == g) continue;
            const double* s2 = ss + (size_t)g2 * k;
            const int64_t* i2 = si + (size_t)g2 * k;
            int lo = 0, hi = nval[g2];
            while (lo < hi) {  // entries of list g2 ahead of (s, id, g)
                const int mid = (lo + hi) >> 1;
                const double sm = s2[mid];
                const bool ahead = sm != s ? (ip ? sm > s : sm < s) : (i2[mid] != id ? i2[mid] < id : g2 < g);
                if (ahead) lo = mid + 1;
                else hi = mid;
            }
            rank += lo;
        }
        if (rank < k) {
            const size_t oo = (size_t)q * k + rank;
            S_out[oo] = s;
            I_out[oo] = id;
            if (D_out) D_out[oo] = (float)s;
        }
    }
    for (int r = total + tid; r < k; r += 256) {  // every list exhausted: padding
        const size_t oo = (size_t)q * k + r;
        S_out[oo] = ip ? -1.7976931348623157e308 : 1.7976931348623157e308;
        I_out[oo] = -1;
        if (D_out) D_out[oo] = ip ? -3.402823466e+38f : 3.402823466e+38f;
    }
}

__global__ void __launch_bounds__(256) k_merge_shards(int metric, const double* __restrict__ S_in,
                                                      const int64_t* __restrict__ I_in, int istride, int G,
                                                      int64_t nq, int k,
                                                      double* __restrict__ S_out, int64_t* __restrict__ I_out,
                                                      float* __restrict__ D_out) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const double worst = metric == METRIC_IP ? -INFINITY : INFINITY;
    int pos = 0;
    double hs = worst;
    int64_t hi = -1;
    auto load_head = [&]() {
        hs = worst;
        hi = -1;
        if (lane < G && pos < k) {
            const size_t o = (((size_t)lane * nq + q) * k + pos) * istride;
            const int64_t id = I_in[o];
            if (id >= 0) {
                hs = S_in[o];
                hi = id;
            }
        }
    };
    load_head();
    for (int j = 0; j < k; ++j) {
        double bs = hs;
        int64_t bi = hi;
        int bl = hi >= 0 ? lane : 64;
#pragma unroll
        for (int sft = 32; sft > 0; sft >>= 1) {
            const double os = __shfl_xor(bs, sft, 64);
            const int64_t oi = __shfl_xor(bi, sft, 64);
            const int ol = __shfl_xor(bl, sft, 64);
            bool take;
            if (ol == 64) take = false;
            else if (bl == 64) take = true;
            else if (os != bs) take = metric == METRIC_IP ? os > bs : os < bs;
            else take = oi < bi;
            if (take) {
                bs = os;
                bi = oi;
                bl = ol;
            }
        }
        const size_t oo = (size_t)q * k + j;
        if (bl == 64) {  // every list exhausted: padding
            if (lane == 0) {
                S_out[oo] = metric == METRIC_IP ? -1.7976931348623157e308 : 1.7976931348623157e308;
                I_out[oo] = -1;
                if (D_out) D_out[oo] = metric == METRIC_IP ? -3.402823466e+38f : 3.402823466e+38f;
            }
            continue;
        }
        if (lane == 0) {
            S_out[oo] = bs;
            I_out[oo] = bi;
            if (D_out) D_out[oo] = (float)bs;
        }
        if (lane == bl) {
            ++pos;
            load_head();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
#define VS_DISPATCH_DT(dt, KERNEL, ...)                                       \
    do {                                                                      \
        if ((dt) == DT_F32) hipLaunchKernelGGL(KERNEL<DT_F32>, __VA_ARGS__);  \
        else if ((dt) == DT_BF16) hipLaunchKernelGGL(KERNEL<DT_BF16>, __VA_ARGS__); \
        else hipLaunchKernelGGL(KERNEL<DT_F16>, __VA_ARGS__);                 \
    } while (0)

static inline unsigned blocks4(int64_t n) { return (unsigned)((n + 3) / 4); }

hipError_t launch_pack_rows(int dt, const float* src, int64_t n, int d, int dpad, uint8_t* data, int64_t lrow0,
                            float* sqn, unsigned* maxsq, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_pack_rows, dim3(blocks4(n)), dim3(256), 0, st, src, n, d, dpad, data, lrow0, sqn, maxsq);
    return hipGetLastError();
}

hipError_t launch_synth_rows(int dt, uint64_t seed, int64_t grow0, int64_t n, int d, int dpad, uint8_t* data,
                             int64_t lrow0, int normalize, float* sqn, unsigned* maxsq, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    // base = splitmix64(seed), computed on the host exactly as the oracle does
    uint64_t x = seed + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    const uint64_t base = x ^ (x >> 31);
    const int64_t CHUNK = 1 << 22;  // rows per launch (grid-size bound)
    for (int64_t r0 = 0; r0 < n; r0 += CHUNK) {
        const int64_t m = n - r0 < CHUNK ? n - r0 : CHUNK;
        VS_DISPATCH_DT(dt, k_synth_rows, dim3(blocks4(m)), dim3(256), 0, st, base, grow0 + r0, m, d, dpad, data,
                       lrow0 + r0, normalize, sqn, maxsq);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

static inline uint64_t host_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

hipError_t launch_synth_f32(int dt, uint64_t seed, int64_t grow0, int64_t n, int d, int normalize, float* out,
                            hipStream_t st) {
    if (n <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_synth_f32, dim3(blocks4(n)), dim3(256), 0, st, host_splitmix64(seed), grow0, n, d, normalize,
                   out);
    return hipGetLastError();
}

hipError_t launch_unpack_rows(int dt, const uint8_t* data, int64_t lrow0, int64_t n, int d, int dpad, float* out,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_unpack_rows, dim3(blocks4(n)), dim3(256), 0, st, data, lrow0, n, d, dpad, out);
    return hipGetLastError();
}

hipError_t launch_gather_rows(int dt, const uint8_t* data, const int64_t* ids, int64_t n, int d, int dpad,
                              float* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_gather_rows, dim3(blocks4(n)), dim3(256), 0, st, data, ids, n, d, dpad, out);
    return hipGetLastError();
}

hipError_t launch_pack_qtile(int dt, const float* q, int nqb, int d, int dpad, uint8_t* qt, float* qinfo, int* gcnt,
                             u64* drop, hipStream_t st, int* fails, const int* gate, const int* qidx, int* gcnt2,
                             u64* drop2) {
    if ((gcnt2 == nullptr) != (drop2 == nullptr)) return hipErrorInvalidValue;
    if (dt == DT_F32)
        hipLaunchKernelGGL(k_pack_qtile<DT_F32>, dim3(MFMA_QB / 4), dim3(256), 0, st, q, nqb, d, dpad, qt, qinfo,
                           gcnt, drop, fails, gate, qidx, gcnt2, drop2);
    else if (dt == DT_BF16)
        hipLaunchKernelGGL(k_pack_qtile<DT_BF16>, dim3(MFMA_QB / 4), dim3(256), 0, st, q, nqb, d, dpad, qt, qinfo,
                           gcnt, drop, fails, gate, qidx, gcnt2, drop2);
    else
        hipLaunchKernelGGL(k_pack_qtile<DT_F16>, dim3(MFMA_QB / 4), dim3(256), 0, st, q, nqb, d, dpad, qt, qinfo,
                           gcnt, drop, fails, gate, qidx, gcnt2, drop2);
    return hipGetLastError();
}

hipError_t launch_pack_qtile_split(int dt, const float* q, const int* qidx, const int* sinfo, int ntiles, int d,
                                   int dpad, uint8_t* qt, float* qinfo, bool plain, hipStream_t st) {
    if (ntiles <= 0 || ntiles > 65535 || !qidx || !sinfo) return hipErrorInvalidValue;
    const dim3 grid(MFMA_QB / 4, ntiles);
#define VS_PACK_SPLIT(DT_, P_) \
    hipLaunchKernelGGL((k_pack_qtile_split<DT_, P_>), grid, dim3(256), 0, st, q, qidx, sinfo, d, dpad, qt, qinfo)
    if (dt == DT_BF16) {
        if (plain) VS_PACK_SPLIT(DT_BF16, true);
        else VS_PACK_SPLIT(DT_BF16, false);
    } else if (dt == DT_F16) {
        if (plain) VS_PACK_SPLIT(DT_F16, true);
        else VS_PACK_SPLIT(DT_F16, false);
    } else {
        return hipErrorInvalidValue;
    }
#undef VS_PACK_SPLIT
    return hipGetLastError();
}

hipError_t launch_group_means(int dt, const uint8_t* data, int dpad, int d, int64_t g0, int64_t ng, int64_t n_rows,
                              int dpad8, uint16_t* gmean, unsigned* maxes, hipStream_t st) {
    if (ng <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_group_means, dim3((unsigned)ng), dim3(256), 0, st, data, dpad, d, g0, n_rows, dpad8, gmean, maxes);
    return hipGetLastError();
}

hipError_t launch_group_dots(const uint16_t* gmean, int64_t ngroups, int dpad8, const float* q, int nq, int d, float* T,
                             hipStream_t st) {
    if (ngroups <= 0) return hipSuccess;
    if (nq > MFMA_QB || dpad8 % 64 != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_group_dots, dim3((unsigned)((ngroups + 15) / 16)), dim3(256), 0, st, gmean, ngroups, dpad8, q, nq,
                       d, T);
    return hipGetLastError();
}

hipError_t launch_quant_rows(int dt, const uint8_t* data, int dpad, int64_t r0, int64_t n, int d, uint8_t* data8,
                             int dpad8, uint32_t* rsb, unsigned* maxes, hipStream_t st, const uint16_t* gmean) {
    if (n <= 0) return hipSuccess;
    const int64_t CHUNK = 1 << 22;  // rows per launch (grid-size bound)
    for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
        const int64_t m = n - c0 < CHUNK ? n - c0 : CHUNK;
        VS_DISPATCH_DT(dt, k_quant_rows, dim3(blocks4(m)), dim3(256), 0, st, data, dpad, r0 + c0, m, d, data8, dpad8,
                       rsb, maxes, gmean);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_pack_qtile_i8(const float* q, int nqb, int d, int dpad8, uint8_t* qt, float2* qfac, float* qeps,
                                const unsigned* maxes, int* gcnt, u64* drop, hipStream_t st, int* fails,
                                const unsigned* l2max, float gamma, const NativeTile* nat) {
    const NativeTile none{};
    if (!nat) {
        hipLaunchKernelGGL(k_pack_qtile_i8<0>, dim3(MFMA_QB), dim3(256), 0, st, q, nqb, d, dpad8, qt, qfac, qeps,
                           maxes, gcnt, drop, fails, l2max, gamma, none);
        return hipGetLastError();
    }
    if (!nat->qt || !nat->qinfo || !nat->gcnt || !nat->drop || nat->dpad % 32 != 0) return hipErrorInvalidValue;
    if (nat->dt == DT_BF16)
        hipLaunchKernelGGL(k_pack_qtile_i8<DT_BF16>, dim3(MFMA_QB), dim3(256), 0, st, q, nqb, d, dpad8, qt, qfac,
                           qeps, maxes, gcnt, drop, fails, l2max, gamma, *nat);
    else if (nat->dt == DT_F16)
        hipLaunchKernelGGL(k_pack_qtile_i8<DT_F16>, dim3(MFMA_QB), dim3(256), 0, st, q, nqb, d, dpad8, qt, qfac,
                           qeps, maxes, gcnt, drop, fails, l2max, gamma, *nat);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_pack_qf32(const float* q, int nqb, int nqpad, int d, int dpad, float* qp, float* qinfo,
                            hipStream_t st, int* ctr, int* fails, u64* drop) {
    hipLaunchKernelGGL(k_pack_qf32, dim3(blocks4(nqpad)), dim3(256), 0, st, q, nqb, nqpad, d, dpad, qp, qinfo, ctr,
                       fails, drop);
    return hipGetLastError();
}

// Dynamic-LDS limit of a kernel, set once per (kernel, device) -- the attribute is per device, and
// several threads may launch at once (vs_multi runs one worker per device); thread-safe.
void set_lds_attr(const void* fn, int bytes) {  // (once per kernel and device)
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    if (!done.insert({fn, dev}).second) return;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipGetLastError();  // an attribute failure must not surface as the launch's error
}

template <int DT, int METRIC, bool SEED>
static void launch_mfma_one(const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    set_lds_attr((const void*)k_screen_mfma<DT, METRIC, SEED>, MF_LDS);
    if constexpr (!SEED && DT != DT_I8) set_lds_attr((const void*)k_screen_mfma_redo<DT, METRIC>, MF_LDS);
    if constexpr (!SEED && DT != DT_I8) {
        if (a.gate) {
            hipLaunchKernelGGL((k_screen_mfma_redo<DT, METRIC>), dim3(a.G), dim3(MF_THREADS), MF_LDS, st, a, qt, nqb);
            return;
        }
    }
    hipLaunchKernelGGL((k_screen_mfma<DT, METRIC, SEED>), dim3(a.G), dim3(MF_THREADS), MF_LDS, st, a, qt, nqb);
}
template <bool SEED>
static hipError_t launch_mfma_dt(int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    if (a.gate && (SEED || dt == DT_I8)) return hipErrorInvalidValue;  // fallback rounds: native main screen
    if (dt == DT_I8) {
        if (!a.rsb || !a.qfac || (a.metric == METRIC_L2 && !a.sqn)) return hipErrorInvalidValue;
        // group-residual keys (+ <mu_g, q>): the seed pass and the direct inner-product main pass only
        if (a.gT && (a.metric != METRIC_IP || !i8_direct_ok(a.dpad))) return hipErrorInvalidValue;
        if (!SEED && i8_direct_ok(a.dpad)) {  // the main pass: direct form (no seed-tile reuse)
            if (a.seed_acc || a.tile_stride != 0) return hipErrorInvalidValue;
            if (a.gT) {  // group residuals (inner product)
                if (a.metric != METRIC_IP) return hipErrorInvalidValue;
                void (*rf)(ScreenArgs, const uint8_t*, int) = k1_schedule() == 1 ? k_screen_i8d_res_ms : k_screen_i8d_res;
                set_lds_attr((const void*)rf, I8D_LDS + I8D_RES_LDS);
                hipLaunchKernelGGL(rf, dim3(a.G), dim3(MF_THREADS), I8D_LDS + I8D_RES_LDS, st, a, qt, nqb);
                return hipGetLastError();
            }
            // (the L2 form keeps the head barrier: under the mid-step schedule its ||x||^2 state
            // spills past the 256 VGPRs of two waves per SIMD)
            void (*fn)(ScreenArgs, const uint8_t*, int) =
                a.metric != METRIC_IP ? k_screen_i8d<METRIC_L2>
                                      : k1_schedule() == 1 ? k_screen_i8d_ms<METRIC_IP> : k_screen_i8d<METRIC_IP>;
            set_lds_attr((const void*)fn, I8D_LDS);
            hipLaunchKernelGGL(fn, dim3(a.G), dim3(MF_THREADS), I8D_LDS, st, a, qt, nqb);
            return hipGetLastError();
        }
        if (a.metric == METRIC_IP) launch_mfma_one<DT_I8, METRIC_IP, SEED>(a, qt, nqb, st);
        else launch_mfma_one<DT_I8, METRIC_L2, SEED>(a, qt, nqb, st);
    } else if ((dt == DT_BF16 || dt == DT_F16) && !SEED && !a.gate && d16_direct_ok(a.dpad)) {
        // the main pass of bf16 / f16 rows: direct form (no seed-tile reuse); fallback rounds keep
        // the tiled form
        if (a.seed_acc || a.tile_stride != 0 || (a.metric == METRIC_L2 && !a.sqn)) return hipErrorInvalidValue;
        void (*fn)(ScreenArgs, const uint8_t*, int) =
            dt == DT_BF16 ? (a.metric == METRIC_IP ? k_screen_d16<DT_BF16, METRIC_IP> : k_screen_d16<DT_BF16, METRIC_L2>)
                          : (a.metric == METRIC_IP ? k_screen_d16<DT_F16, METRIC_IP> : k_screen_d16<DT_F16, METRIC_L2>);
        set_lds_attr((const void*)fn, I8D_LDS);
        hipLaunchKernelGGL(fn, dim3(a.G), dim3(MF_THREADS), I8D_LDS, st, a, qt, nqb);
    } else if (dt == DT_BF16) {
        if (a.metric == METRIC_IP) launch_mfma_one<DT_BF16, METRIC_IP, SEED>(a, qt, nqb, st);
        else launch_mfma_one<DT_BF16, METRIC_L2, SEED>(a, qt, nqb, st);
    } else if (dt == DT_F16) {
        if (a.metric == METRIC_IP) launch_mfma_one<DT_F16, METRIC_IP, SEED>(a, qt, nqb, st);
        else launch_mfma_one<DT_F16, METRIC_L2, SEED>(a, qt, nqb, st);
    } else if (dt == DT_F32) {
        if (a.metric == METRIC_IP) launch_mfma_one<DT_F32, METRIC_IP, SEED>(a, qt, nqb, st);
        else launch_mfma_one<DT_F32, METRIC_L2, SEED>(a, qt, nqb, st);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_screen_mfma(int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    return launch_mfma_dt<false>(dt, a, qt, nqb, st);
}

template <int DT, int METRIC>
static void launch_mapped_one(const ScreenArgs& a, const uint8_t* qt, bool plain, hipStream_t st) {
    if (plain) {  // plain query tiles: the direct form only (checked by the caller)
        set_lds_attr((const void*)k_screen_d16_mapped<DT, METRIC, true>, I8D_LDS_MAP);
        hipLaunchKernelGGL((k_screen_d16_mapped<DT, METRIC, true>), dim3(a.G), dim3(MF_THREADS), I8D_LDS_MAP, st, a, qt, 0);
        return;
    }
    if (d16_direct_ok(a.dpad)) {  // the direct form (corpus fragments HBM -> VGPRs; narrow tiles inside)
        set_lds_attr((const void*)k_screen_d16_mapped<DT, METRIC, false>, I8D_LDS_MAP);
        hipLaunchKernelGGL((k_screen_d16_mapped<DT, METRIC, false>), dim3(a.G), dim3(MF_THREADS), I8D_LDS_MAP, st, a, qt, 0);
        return;
    }
    set_lds_attr((const void*)k_screen_mfma_mapped<DT, METRIC>, MF_LDS_MAP);
    hipLaunchKernelGGL((k_screen_mfma_mapped<DT, METRIC>), dim3(a.G), dim3(MF_THREADS), MF_LDS_MAP, st, a, qt, 0);
}
bool check_map_desc(const int* g, int64_t tmap_len, int n_qtiles, int64_t qmap_len, bool plain) {
    const int64_t tm_off = g[0], nt = g[1], t0 = g[2], nvalid = g[3], qti = g[4], qoff = g[5], nqb = g[6];
    // tiles [t0, t0 + nt) of a segment of nvalid rows, each holding at least one of its rows (the
    // kernel masks rows >= nvalid); page-table, query-tile and qmap slices in range
    return nt >= 1 && nt <= MFMA_MAP_TILES && tm_off >= 0 && tm_off + nt <= tmap_len && t0 >= 0 &&
           (t0 + nt - 1) * TR < nvalid && nvalid <= INT32_MAX && qti >= 0 && qti < n_qtiles && nqb >= 1 &&
           nqb <= (plain ? MFMA_QB : MFMA_QB / 2) && qoff >= 0 && qoff + nqb <= qmap_len;
}
hipError_t launch_screen_mfma_mapped(int dt, const ScreenArgs& a, const uint8_t* qt, bool plain, hipStream_t st) {
    // the launch contract the kernel relies on (descriptors: check_map_desc, by the caller)
    if (!a.tile_map || !a.qmap || !a.wg_desc || a.thr0 || a.seed_acc || a.tile_stride != 0 || a.gate || a.G <= 0 ||
        a.Kp > MFMA_KP_MAX || a.cap != MFMA_CAP || a.lcap < a.Kp || (plain && !d16_direct_ok(a.dpad)))
        return hipErrorInvalidValue;
    if (dt == DT_BF16) {
        if (a.metric == METRIC_IP) launch_mapped_one<DT_BF16, METRIC_IP>(a, qt, plain, st);
        else launch_mapped_one<DT_BF16, METRIC_L2>(a, qt, plain, st);
    } else if (dt == DT_F16) {
        if (a.metric == METRIC_IP) launch_mapped_one<DT_F16, METRIC_IP>(a, qt, plain, st);
        else launch_mapped_one<DT_F16, METRIC_L2>(a, qt, plain, st);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the GEMV's queries go to LDS (k_screen_gemv QL) when the padded class's fp32 rows fit this many
// bytes (one query up to d = 4096; occupancy below is taken at this size, which the VGPR budget
// limits before the LDS does)
constexpr size_t kGemvQlBytes = 16384;
static bool gemv_ql(int nqpad, int dpad) { return (size_t)nqpad * dpad * 4 <= kGemvQlBytes; }
template <int DT, bool QL>
static int gemv_occ(int nqpad) {
    int n = 0;
    hipError_t e = hipSuccess;
    const size_t lds = QL ? kGemvQlBytes : 0;
    switch (nqpad) {
        case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_screen_gemv<DT, 1, 1, QL>, 256, lds); break;
        case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_screen_gemv<DT, 2, 1, QL>, 256, lds); break;
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_screen_gemv<DT, 4, 1, QL>, 256, lds); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_screen_gemv<DT, 8, 1, QL>, 256, lds); break;
    }
    return e == hipSuccess && n > 0 ? n : 4;
}
template <int DT>
static int gemv_occ_dt(int q, bool ql) { return ql ? gemv_occ<DT, true>(q) : gemv_occ<DT, false>(q); }
int gemv_blocks_per_cu(int dt, int nqpad, int dpad) {
    static int cache[4][9][2] = {};  // benign race: idempotent
    const int q = nqpad <= 1 ? 1 : nqpad <= 2 ? 2 : nqpad <= 4 ? 4 : 8;
    const bool ql = gemv_ql(q, dpad);
    int& v = cache[dt][q][ql ? 1 : 0];
    if (!v)
        v = dt == DT_F32 ? gemv_occ_dt<DT_F32>(q, ql) : dt == DT_BF16 ? gemv_occ_dt<DT_BF16>(q, ql)
            : dt == DT_I8 ? gemv_occ_dt<DT_I8>(q, ql) : gemv_occ_dt<DT_F16>(q, ql);
    return v;
}

template <int DT, int SPLIT>
static void launch_gemv_split(const ScreenArgs& a, const float* qp, int nqb, int nqpad, hipStream_t st) {
    const int q = nqpad <= 1 ? 1 : nqpad <= 2 ? 2 : nqpad <= 4 ? 4 : 8;
    if (gemv_ql(q, a.dpad)) {  // the queries in LDS (k_screen_gemv QL)
        const size_t lds = (size_t)q * a.dpad * 4;
        switch (q) {
            case 1: hipLaunchKernelGGL((k_screen_gemv<DT, 1, SPLIT, true>), dim3(a.G), dim3(256), lds, st, a, qp, nqb); break;
            case 2: hipLaunchKernelGGL((k_screen_gemv<DT, 2, SPLIT, true>), dim3(a.G), dim3(256), lds, st, a, qp, nqb); break;
            case 4: hipLaunchKernelGGL((k_screen_gemv<DT, 4, SPLIT, true>), dim3(a.G), dim3(256), lds, st, a, qp, nqb); break;
            default: hipLaunchKernelGGL((k_screen_gemv<DT, 8, SPLIT, true>), dim3(a.G), dim3(256), lds, st, a, qp, nqb); break;
        }
        return;
    }
    switch (nqpad) {
        case 1: hipLaunchKernelGGL((k_screen_gemv<DT, 1, SPLIT>), dim3(a.G), dim3(256), 0, st, a, qp, nqb); break;
        case 2: hipLaunchKernelGGL((k_screen_gemv<DT, 2, SPLIT>), dim3(a.G), dim3(256), 0, st, a, qp, nqb); break;
        case 4: hipLaunchKernelGGL((k_screen_gemv<DT, 4, SPLIT>), dim3(a.G), dim3(256), 0, st, a, qp, nqb); break;
        default: hipLaunchKernelGGL((k_screen_gemv<DT, 8, SPLIT>), dim3(a.G), dim3(256), 0, st, a, qp, nqb); break;
    }
}
template <int DT>
static void launch_gemv_dt(const ScreenArgs& a, const float* qp, int nqb, int nqpad, hipStream_t st) {
    if (a.gemv_split == GEMV_SPLIT) launch_gemv_split<DT, GEMV_SPLIT>(a, qp, nqb, nqpad, st);
    else launch_gemv_split<DT, 1>(a, qp, nqb, nqpad, st);
}
hipError_t launch_screen_gemv(int dt, const ScreenArgs& a, const float* qp, int nqb, int nqpad, hipStream_t st) {
    if (dt == DT_I8 && (!a.rsb || !a.qinfo || (a.metric == METRIC_L2 && !a.sqn))) return hipErrorInvalidValue;
    if (a.gemv_split != 0 && a.gemv_split != 1 && a.gemv_split != GEMV_SPLIT) return hipErrorInvalidValue;
    if (dt == DT_F32) launch_gemv_dt<DT_F32>(a, qp, nqb, nqpad, st);
    else if (dt == DT_BF16) launch_gemv_dt<DT_BF16>(a, qp, nqb, nqpad, st);
    else if (dt == DT_I8) launch_gemv_dt<DT_I8>(a, qp, nqb, nqpad, st);
    else launch_gemv_dt<DT_F16>(a, qp, nqb, nqpad, st);
    return hipGetLastError();
}

hipError_t launch_merge(const u64* in, int nseg, int qstride, int nq, int Kp, u64* out, int* nseg_out,
                        hipStream_t st) {
    // >= 2 segments per block, so every stage shrinks the list count (Kp <= KP_MAX = 4096)
    const bool wide = Kp > 2048;
    const int spb = (256 * (wide ? 32 : 16)) / Kp;
    const int nb = (nseg + spb - 1) / spb;
    if (wide) hipLaunchKernelGGL(k_merge<32>, dim3(nb, nq), dim3(256), 0, st, in, nseg, qstride, nq, Kp, spb, out);
    else hipLaunchKernelGGL(k_merge<16>, dim3(nb, nq), dim3(256), 0, st, in, nseg, qstride, nq, Kp, spb, out);
    *nseg_out = nb;
    return hipGetLastError();
}

template <int DT, int METRIC, bool QLDS>
static void launch_refine_one(const RefineArgs& a, int nq, int KP2, size_t lds, hipStream_t st) {
    set_lds_attr((const void*)k_refine<DT, METRIC, QLDS>, 152 * 1024);
    set_lds_attr((const void*)k_refine_redo<DT, METRIC, QLDS>, 152 * 1024);
    if (a.redo) {
        hipLaunchKernelGGL((k_refine_redo<DT, METRIC, QLDS>), dim3(nq), dim3(RF_THREADS), lds, st, a, KP2);
        return;
    }
    const int ns = a.nsplit > 1 ? a.nsplit : 1;
    hipLaunchKernelGGL((k_refine<DT, METRIC, QLDS>), dim3(nq, ns), dim3(RF_THREADS), lds, st, a, KP2);
}

// Split a few-query refine over several workgroups per query when its rows (Kp per query) would
// otherwise take many serial gather rounds on one CU: >= 2 rounds (RR rows per wave x 16 waves)
// per workgroup, at most 32 per query, the whole grid within one wave of the chip.
int refine_split(int nq, int Kp, int dt, int num_cu) {
    const int per_round = (dt == DT_F32 ? 2 : 4) * (RF_THREADS / 64);
    // GEMV batches (<= 8 queries: the product's single-query call): half a scoring round per
    // workgroup -- a single query's Kp rows gathered by one CU were a chain of dependent rounds
    // (cfg2: 42 us for ~100 fp32 rows), and the gathers of a round still wait on their page
    // walks and lines for ~10 us, so more CUs each take fewer rows (one round: 3-4 us slower per
    // cfg2 step in the in-box A/B); MFMA batches: two rounds per workgroup
    int ns = nq <= GEMV_NQ_MAX ? (2 * Kp + per_round - 1) / per_round : Kp / (2 * per_round);
    ns = std::min(ns, 32);
    ns = std::min(ns, num_cu / std::max(nq, 1));
    return ns >= 2 ? ns : 1;
}

template <int DT>
static void launch_refine_dt(const RefineArgs& a, int nq, int KP2, size_t lds, bool qlds, hipStream_t st) {
    if (a.metric == METRIC_IP) {
        if (qlds) launch_refine_one<DT, METRIC_IP, true>(a, nq, KP2, lds, st);
        else launch_refine_one<DT, METRIC_IP, false>(a, nq, KP2, lds, st);
    } else {
        if (qlds) launch_refine_one<DT, METRIC_L2, true>(a, nq, KP2, lds, st);
        else launch_refine_one<DT, METRIC_L2, false>(a, nq, KP2, lds, st);
    }
}

hipError_t launch_refine(const RefineArgs& a, int nq, hipStream_t st) {
    if (a.redo && (!a.gate || !a.cert)) return hipErrorInvalidValue;
    if (a.nsplit > 1 && (a.redo || !a.gsc || !a.gids || !a.gdone)) return hipErrorInvalidValue;
    const int KP2 = refine_kp2(a.Kp);
    const size_t base = (size_t)KP2 * 12 + 8 + (size_t)KP2 * 8;  // scores, ids, (query), kept keys
    const size_t qbytes = (size_t)((a.d + 7) >> 3) * 64;    // fp64 query, transposed 8-element groups
    const bool qlds = base + qbytes <= 148 * 1024;  // query as fp64 in LDS when it fits
    const size_t lds = qlds ? base + qbytes : base;
    if (a.dt == DT_F32) launch_refine_dt<DT_F32>(a, nq, KP2, lds, qlds, st);
    else if (a.dt == DT_BF16) launch_refine_dt<DT_BF16>(a, nq, KP2, lds, qlds, st);
    else launch_refine_dt<DT_F16>(a, nq, KP2, lds, qlds, st);
    return hipGetLastError();
}

template <int DT, bool QLDS>
static void launch_refine_wide_one(const RefineArgs& a, int nq, int KA, size_t lds, hipStream_t st) {
    if (a.metric == METRIC_IP) {
        set_lds_attr((const void*)k_refine_wide<DT, METRIC_IP, QLDS>, 152 * 1024);
        hipLaunchKernelGGL((k_refine_wide<DT, METRIC_IP, QLDS>), dim3(nq), dim3(RF_THREADS), lds, st, a, KA);
    } else {
        set_lds_attr((const void*)k_refine_wide<DT, METRIC_L2, QLDS>, 152 * 1024);
        hipLaunchKernelGGL((k_refine_wide<DT, METRIC_L2, QLDS>), dim3(nq), dim3(RF_THREADS), lds, st, a, KA);
    }
}

hipError_t launch_refine_wide(const RefineArgs& a, int nq, int KA, hipStream_t st) {
    // L2: int8 keys only (their margin qeps covers the transformed key; native L2 uses k_refine)
    if ((a.metric != METRIC_IP && !(a.metric == METRIC_L2 && a.qeps)) || !(a.qeps || a.qinfo) || !a.cand_n ||
        KA <= 0 || 2 * KA > RFW_CAP || (a.redo && (!a.gate || !a.cert || a.phase != 0)))
        return hipErrorInvalidValue;
    const size_t base = (size_t)RFW_CAP * 12;
    const size_t qbytes = (size_t)((a.d + 7) >> 3) * 64;
    const bool qlds = base + qbytes <= 148 * 1024;
    const size_t lds = qlds ? base + qbytes : base;
    if (a.dt == DT_F32) {
        if (qlds) launch_refine_wide_one<DT_F32, true>(a, nq, KA, lds, st);
        else launch_refine_wide_one<DT_F32, false>(a, nq, KA, lds, st);
    } else if (a.dt == DT_BF16) {
        if (qlds) launch_refine_wide_one<DT_BF16, true>(a, nq, KA, lds, st);
        else launch_refine_wide_one<DT_BF16, false>(a, nq, KA, lds, st);
    } else {
        if (qlds) launch_refine_wide_one<DT_F16, true>(a, nq, KA, lds, st);
        else launch_refine_wide_one<DT_F16, false>(a, nq, KA, lds, st);
    }
    return hipGetLastError();
}

hipError_t launch_seed_mfma(int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    if (nqb > MFMA_QB || a.tile_stride <= 0 || !a.seedmax) return hipErrorInvalidValue;
    return launch_mfma_dt<true>(dt, a, qt, nqb, st);
}

hipError_t launch_seed_select(const float* seedmax, int M, int nq, int rank, u64* thr0, hipStream_t st) {
    if (rank <= 0) return hipErrorInvalidValue;
    const dim3 grid((unsigned)nq);
    if (M <= 256 * SEED_VPT)
        hipLaunchKernelGGL(k_seed_select<SEED_VPT>, grid, dim3(256), 0, st, seedmax, M, nq, rank, thr0);
    else if (M <= 256 * 2 * SEED_VPT)
        hipLaunchKernelGGL(k_seed_select<2 * SEED_VPT>, grid, dim3(256), 0, st, seedmax, M, nq, rank, thr0);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_pack_rows_map(int dt, const float* src, int64_t n, int d, int dpad, uint8_t* data,
                                const int64_t* slots, float* sqn, unsigned* maxsq, uint32_t* slot_id, int64_t id0,
                                hipStream_t st) {
    if (n <= 0) return hipSuccess;
    VS_DISPATCH_DT(dt, k_pack_rows_map, dim3(blocks4(n)), dim3(256), 0, st, src, n, d, dpad, data, slots, sqn, maxsq,
                   slot_id, id0);
    return hipGetLastError();
}

hipError_t launch_round_f32(int dt, float* x, int64_t n, hipStream_t st) {
    if (n <= 0 || dt == DT_F32) return hipSuccess;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (dt == DT_BF16) hipLaunchKernelGGL(k_round_f32<DT_BF16>, dim3(blocks), dim3(256), 0, st, x, n);
    else hipLaunchKernelGGL(k_round_f32<DT_F16>, dim3(blocks), dim3(256), 0, st, x, n);
    return hipGetLastError();
}

template <int DT>
static void launch_ivf_scan_dt(int nq_class, const IvfScanArgs& a, int grid, hipStream_t st) {
    switch (nq_class) {
        case 1: hipLaunchKernelGGL((k_ivf_scan<DT, 1>), dim3(grid), dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL((k_ivf_scan<DT, 2>), dim3(grid), dim3(256), 0, st, a); break;
        case 4: hipLaunchKernelGGL((k_ivf_scan<DT, 4>), dim3(grid), dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL((k_ivf_scan<DT, IVF_QG>), dim3(grid), dim3(256), 0, st, a); break;
    }
}
hipError_t launch_ivf_scan(int dt, int nq_class, const IvfScanArgs& a, int grid, hipStream_t st) {
    if (a.n_items <= 0 || grid <= 0) return hipSuccess;
    if (nq_class != 1 && nq_class != 2 && nq_class != 4 && nq_class != IVF_QG) return hipErrorInvalidValue;
    if (dt == DT_F32) launch_ivf_scan_dt<DT_F32>(nq_class, a, grid, st);
    else if (dt == DT_BF16) launch_ivf_scan_dt<DT_BF16>(nq_class, a, grid, st);
    else launch_ivf_scan_dt<DT_F16>(nq_class, a, grid, st);
    return hipGetLastError();
}

hipError_t launch_ivf_scan_dyn(int dt, const IvfScanArgs& a, int grid, hipStream_t st) {
    if (a.n_items <= 0 || grid <= 0) return hipSuccess;
    if (!a.next_item) return hipErrorInvalidValue;
    // the queries in LDS when an item's IVF_QG of them fit 48 KiB (3 resident workgroups per CU, as
    // the VGPR budget allows; d <= 1536)
    const size_t ql = (size_t)IVF_QG * a.dpad * 4;
    if (ql <= 48 * 1024) {
        if (dt == DT_F32) hipLaunchKernelGGL((k_ivf_scan_dyn<DT_F32, true>), dim3(grid), dim3(256), ql, st, a);
        else if (dt == DT_BF16) hipLaunchKernelGGL((k_ivf_scan_dyn<DT_BF16, true>), dim3(grid), dim3(256), ql, st, a);
        else hipLaunchKernelGGL((k_ivf_scan_dyn<DT_F16, true>), dim3(grid), dim3(256), ql, st, a);
        return hipGetLastError();
    }
    if (dt == DT_F32) hipLaunchKernelGGL((k_ivf_scan_dyn<DT_F32, false>), dim3(grid), dim3(256), 0, st, a);
    else if (dt == DT_BF16) hipLaunchKernelGGL((k_ivf_scan_dyn<DT_BF16, false>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_ivf_scan_dyn<DT_F16, false>), dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_merge_shards(int metric, const double* S_in, const int64_t* I_in, int G, int64_t nq, int k,
                               double* S_out, int64_t* I_out, float* D_out, hipStream_t st, int istride) {
    if (G > 64 || istride < 1) return hipErrorInvalidValue;
    if ((int64_t)G * k <= kMergeRankMax) {
        hipLaunchKernelGGL(k_merge_shards_rank, dim3((unsigned)nq), dim3(256), (size_t)G * k * 16, st, metric, S_in,
                           I_in, istride, G, nq, k, S_out, I_out, D_out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_merge_shards, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, st, metric, S_in, I_in, istride,
                       G, nq, k, S_out, I_out, D_out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// K7: HNSW graph search (host side vs_hnsw.hip) -- faiss HNSW::search restated
// (oracle/hnsw_oracle.py): greedy descent on the upper levels, then level 0 with a candidate set of
// capacity ef (popped entries stay and count in the stop test) and a result set of k.  One
// 1024-thread workgroup per query (the steps are dependent: 16 waves score a neighbour list in one
// or two rounds of 4 rows each, where 4 waves took up to 6 -- the step latency, not the bytes, sets
// the time).  Distances are exact_score_rows' canonical fp64 scores (IP:
// -score).  Both sets are sorted LDS arrays under (distance, id) and take a whole neighbour list
// per step: the new rows are scored by all 16 waves, rank-sorted, and merged (an element's new
// position = its index in its own list + its rank in the other, one binary search) -- the same
// decisions as faiss's array heaps whenever no two rows tie in distance.
// ------------------------------------------------------------------------------------------------
struct HnLds {
    double* qs;
    double* cd[2];
    int* ci[2];
    int* cv[2];
    double* rd[2];
    int* ri[2];
    double* bd;  // new rows: distances, ids (list order) ...
    int* bi;
    double* sd;  // ... rank-sorted
    int* si;
    int* bl;     // the raw neighbour list
};
__host__ __device__ inline size_t hn_layout(int d, int k, int ef, int nbmax, bool qlds, uint8_t* base, HnLds* L) {
    size_t off = 0;
    uint8_t* p[16];
    const size_t sz[16] = {qlds ? (size_t)((d + 7) >> 3) * 64 : 0,
                           (size_t)ef * 8, (size_t)ef * 8, (size_t)ef * 4, (size_t)ef * 4, (size_t)ef * 4, (size_t)ef * 4,
                           (size_t)k * 8, (size_t)k * 8, (size_t)k * 4, (size_t)k * 4,
                           (size_t)nbmax * 8, (size_t)nbmax * 4, (size_t)nbmax * 8, (size_t)nbmax * 4,
                           (size_t)nbmax * 4};
    for (int i = 0; i < 16; ++i) {
        p[i] = base + off;
        off += (sz[i] + 15) & ~(size_t)15;
    }
    if (L) {
        L->qs = (double*)p[0];
        L->cd[0] = (double*)p[1];
        L->cd[1] = (double*)p[2];
        L->ci[0] = (int*)p[3];
        L->ci[1] = (int*)p[4];
        L->cv[0] = (int*)p[5];
        L->cv[1] = (int*)p[6];
        L->rd[0] = (double*)p[7];
        L->rd[1] = (double*)p[8];
        L->ri[0] = (int*)p[9];
        L->ri[1] = (int*)p[10];
        L->bd = (double*)p[11];
        L->bi = (int*)p[12];
        L->sd = (double*)p[13];
        L->si = (int*)p[14];
        L->bl = (int*)p[15];
    }
    return off;
}
constexpr size_t HN_LDS_CAP = 160 * 1024 - 512;  // dynamic LDS left beside the kernel's static words
size_t hnsw_lds_bytes(int d, int k, int ef, int nbmax) {
    const size_t with_q = hn_layout(d, k, ef, nbmax, true, nullptr, nullptr);
    return with_q <= HN_LDS_CAP ? with_q : hn_layout(d, k, ef, nbmax, false, nullptr, nullptr);
}

__device__ __forceinline__ bool hn_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}
// entries of the sorted (distance, id) list [0, n) that precede (dv, iv)
__device__ __forceinline__ int hn_rank(const double* d, const int* id, int n, double dv, int iv) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (hn_less(d[mid], id[mid], dv, iv)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// entries of the sorted list [0, n) strictly closer than t (faiss MinimaxHeap::count_below)
__device__ __forceinline__ int hn_count_below(const double* d, int n, double t) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <int DT, int METRIC, bool QLDS>
__global__ void __launch_bounds__(HN_SEARCH_THREADS) k_hnsw_search(HnswArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NW = HN_SEARCH_THREADS / 64;
    constexpr bool IP = METRIC == METRIC_IP;
    __shared__ int s_m, s_imin, s_valid;
    __shared__ int s_new[NW], s_wj[NW];
    __shared__ double s_wd[NW];
    HnLds L;
    hn_layout(a.d, a.k, a.ef, a.nbmax, QLDS, smem, &L);
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ng = (a.d + 7) >> 3;
    const float* qv = a.q + (int64_t)q * a.d;
    uint32_t* vis = a.vis + (int64_t)q * a.vis_words;
    float* Dq = a.D + (int64_t)q * a.k;
    int64_t* Iq = a.I + (int64_t)q * a.k;
    if (a.entry < 0 || a.n == 0) {
        for (int j = tid; j < a.k; j += HN_SEARCH_THREADS) {
            Dq[j] = IP ? -__FLT_MAX__ : __FLT_MAX__;
            Iq[j] = -1;
        }
        return;
    }
    if constexpr (QLDS)
        for (int i = tid; i < a.d; i += HN_SEARCH_THREADS) L.qs[(i & 7) * ng + (i >> 3)] = (double)qv[i];

    // faiss distances of the rows bi[0 .. m) into bd (all waves, refine_rows rows per wave-step)
    auto score = [&](int m) {
        constexpr int RR = refine_rows<DT>();
        for (int j0 = wid * RR; j0 < m; j0 += NW * RR) {
            int64_t rr[RR];
#pragma unroll
            for (int i = 0; i < RR; ++i) rr[i] = j0 + i < m ? (int64_t)L.bi[j0 + i] : -1;
            double s[RR];
            exact_score_rows<DT, METRIC, QLDS, RR>(a.corpus, rr, L.qs, qv, a.d, a.dpad, lane, s);
            if (lane == 0)
#pragma unroll
                for (int i = 0; i < RR; ++i)
                    if (j0 + i < m) L.bd[j0 + i] = IP ? -s[i] : s[i];
        }
        __syncthreads();
    };
    // neighbour list of node v on level l into bl, up to its first -1; returns its length (uniform)
    auto load_list = [&](int v, int l) -> int {
        const int w = a.cum[l + 1] - a.cum[l];
        const int* src = a.neighbors + a.offsets[v] + a.cum[l];
        __syncthreads();
        if (tid == 0) s_m = w;
        __syncthreads();
        for (int t = tid; t < w; t += HN_SEARCH_THREADS) {
            const int u = src[t];
            L.bl[t] = u;
            if (u < 0) atomicMin(&s_m, t);
        }
        __syncthreads();
        return s_m;
    };

    // ---- upper levels: greedy descent (faiss greedy_update_nearest) ----
    int near = a.entry;
    if (tid == 0) L.bi[0] = near;
    __syncthreads();
    score(1);
    double dn = L.bd[0];
    for (int l = a.max_level; l >= 1; --l) {
        for (int64_t guard = 0; guard <= a.n; ++guard) {  // the distance strictly decreases
            const int m = load_list(near, l);
            for (int t = tid; t < m; t += HN_SEARCH_THREADS) L.bi[t] = L.bl[t];
            __syncthreads();
            score(m);
            // the first neighbour at the smallest distance (faiss: first strictly closer, in order)
            double bd = INFINITY;
            int bj = 0x7FFFFFFF;
            for (int t = tid; t < m; t += HN_SEARCH_THREADS) {
                const double v = L.bd[t];
                if (v < bd) {
                    bd = v;
                    bj = t;
                }
            }
#pragma unroll
            for (int sft = 32; sft > 0; sft >>= 1) {
                const double od = __shfl_xor(bd, sft, 64);
                const int oj = __shfl_xor(bj, sft, 64);
                if (od < bd || (od == bd && oj < bj)) {
                    bd = od;
                    bj = oj;
                }
            }
            if (lane == 0) {
                s_wd[wid] = bd;
                s_wj[wid] = bj;
            }
            __syncthreads();
            bd = s_wd[0];
            bj = s_wj[0];
            for (int w = 1; w < NW; ++w)
                if (s_wd[w] < bd || (s_wd[w] == bd && s_wj[w] < bj)) {
                    bd = s_wd[w];
                    bj = s_wj[w];
                }
            if (!(bj < m && bd < dn)) break;
            near = L.bi[bj];
            dn = bd;
        }
    }

    // ---- level 0 (faiss search_from_candidates) ----
    int cur = 0;
    __syncthreads();
    if (tid == 0) {
        L.cd[0][0] = dn;
        L.ci[0][0] = near;
        L.cv[0][0] = 1;
        L.rd[0][0] = dn;
        L.ri[0][0] = near;
        atomicOr(vis + (near >> 5), 1u << (near & 31));
    }
    int nc = 1, nres = 1, nvalid = 1;  // uniform
    for (int64_t step = 0; nvalid > 0 && step <= a.n; ++step) {
        // pop the closest valid candidate: the first valid entry of the sorted set
        if (tid == 0) {
            s_imin = 0x7FFFFFFF;
            s_valid = 0;
        }
        __syncthreads();
        for (int i = tid; i < nc; i += HN_SEARCH_THREADS)
            if (L.cv[cur][i]) {
                atomicMin(&s_imin, i);
                break;
            }
        __syncthreads();
        const int imin = s_imin;
        const double d0 = L.cd[cur][imin];
        const int v0 = L.ci[cur][imin];
        const int below = hn_count_below(L.cd[cur], nc, d0);  // popped entries included
        __syncthreads();
        if (tid == 0) L.cv[cur][imin] = 0;
        --nvalid;
        if (below >= a.ef_search) break;
        const int m = load_list(v0, 0);
        // visited test-and-set; the new neighbours compacted in list order into bi
        int nn = 0;
        for (int t0 = 0; t0 < m; t0 += HN_SEARCH_THREADS) {
            const int t = t0 + tid;
            bool isnew = false;
            int v = -1;
            if (t < m) {
                v = L.bl[t];
                const uint32_t bit = 1u << (v & 31);
                isnew = (atomicOr(vis + (v >> 5), bit) & bit) == 0u;
            }
            const u64 bal = __ballot(isnew);
            if (lane == 0) s_new[wid] = __popcll(bal);
            __syncthreads();
            int pre = 0, tot = 0;
            for (int w = 0; w < NW; ++w) {
                const int c = s_new[w];
                pre += w < wid ? c : 0;
                tot += c;
            }
            if (isnew) L.bi[nn + pre + lane_prefix(bal)] = v;
            nn += tot;
            __syncthreads();
        }
        if (nn == 0) continue;
        score(nn);
        for (int j = tid; j < nn; j += HN_SEARCH_THREADS) {  // rank sort by (distance, id)
            const double dj = L.bd[j];
            const int ij = L.bi[j];
            int r = 0;
            for (int i = 0; i < nn; ++i) r += hn_less(L.bd[i], L.bi[i], dj, ij) ? 1 : 0;
            L.sd[r] = dj;
            L.si[r] = ij;
        }
        __syncthreads();
        const int nxt = cur ^ 1;
        for (int i = tid; i < nres; i += HN_SEARCH_THREADS) {  // results: the best k of the union
            const int p = i + hn_rank(L.sd, L.si, nn, L.rd[cur][i], L.ri[cur][i]);
            if (p < a.k) {
                L.rd[nxt][p] = L.rd[cur][i];
                L.ri[nxt][p] = L.ri[cur][i];
            }
        }
        for (int j = tid; j < nn; j += HN_SEARCH_THREADS) {
            const int p = j + hn_rank(L.rd[cur], L.ri[cur], nres, L.sd[j], L.si[j]);
            if (p < a.k) {
                L.rd[nxt][p] = L.sd[j];
                L.ri[nxt][p] = L.si[j];
            }
        }
        int myvalid = 0;  // candidates: the best ef of the union, popped entries included
        for (int i = tid; i < nc; i += HN_SEARCH_THREADS) {
            const int p = i + hn_rank(L.sd, L.si, nn, L.cd[cur][i], L.ci[cur][i]);
            if (p < a.ef) {
                L.cd[nxt][p] = L.cd[cur][i];
                L.ci[nxt][p] = L.ci[cur][i];
                L.cv[nxt][p] = L.cv[cur][i];
                myvalid += L.cv[cur][i];
            }
        }
        for (int j = tid; j < nn; j += HN_SEARCH_THREADS) {
            const int p = j + hn_rank(L.cd[cur], L.ci[cur], nc, L.sd[j], L.si[j]);
            if (p < a.ef) {
                L.cd[nxt][p] = L.sd[j];
                L.ci[nxt][p] = L.si[j];
                L.cv[nxt][p] = 1;
                ++myvalid;
            }
        }
        myvalid = wave_sum_i(myvalid);
        if (lane == 0) atomicAdd(&s_valid, myvalid);
        __syncthreads();
        nvalid = s_valid;
        nres = min(nres + nn, a.k);
        nc = min(nc + nn, a.ef);
        cur = nxt;
        __syncthreads();  // s_valid read by every thread before the next step resets it
    }
    __syncthreads();
    for (int j = tid; j < a.k; j += HN_SEARCH_THREADS) {
        if (j < nres) {
            const double dv = L.rd[cur][j];
            Dq[j] = (float)(IP ? -dv : dv);
            Iq[j] = L.ri[cur][j];
        } else {
            Dq[j] = IP ? -__FLT_MAX__ : __FLT_MAX__;
            Iq[j] = -1;
        }
    }
}

template <int DT, int METRIC, bool QLDS>
static void launch_hnsw_one(const HnswArgs& a, int nq, size_t lds, hipStream_t st) {
    set_lds_attr((const void*)k_hnsw_search<DT, METRIC, QLDS>, (int)HN_LDS_CAP);
    hipLaunchKernelGGL((k_hnsw_search<DT, METRIC, QLDS>), dim3(nq), dim3(HN_SEARCH_THREADS), lds, st, a);
}
template <int DT>
static void launch_hnsw_dt(const HnswArgs& a, int nq, size_t lds, bool qlds, hipStream_t st) {
    if (a.metric == METRIC_IP) {
        if (qlds) launch_hnsw_one<DT, METRIC_IP, true>(a, nq, lds, st);
        else launch_hnsw_one<DT, METRIC_IP, false>(a, nq, lds, st);
    } else {
        if (qlds) launch_hnsw_one<DT, METRIC_L2, true>(a, nq, lds, st);
        else launch_hnsw_one<DT, METRIC_L2, false>(a, nq, lds, st);
    }
}
hipError_t launch_hnsw_search(const HnswArgs& a, int nq, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    if (a.k < 1 || a.ef < a.k || a.ef > HN_EF_MAX || a.nbmax > HN_NB_MAX || a.nbmax < 1) return hipErrorInvalidValue;
    const size_t lds = hnsw_lds_bytes(a.d, a.k, a.ef, a.nbmax);
    if (lds > HN_LDS_CAP) return hipErrorInvalidValue;
    const bool qlds = hn_layout(a.d, a.k, a.ef, a.nbmax, true, nullptr, nullptr) <= HN_LDS_CAP;
    if (a.dt == DT_F32) launch_hnsw_dt<DT_F32>(a, nq, lds, qlds, st);
    else if (a.dt == DT_BF16) launch_hnsw_dt<DT_BF16>(a, nq, lds, qlds, st);
    else if (a.dt == DT_F16) launch_hnsw_dt<DT_F16>(a, nq, lds, qlds, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// K8: HNSW neighbour selection (graph build; host side vs_hnsw.hip vs_hnsw_prune) -- faiss
// HNSW::shrink_neighbor_list restated (oracle/hnsw_oracle.py shrink_neighbor_list): a node's
// candidates in ascending (distance, id) order; a candidate is kept unless some already kept
// neighbour is strictly closer to it than the node is; stop at W kept.  Fewer than W candidates are
// kept whole (faiss returns early below max_size).  One 256-thread workgroup per node; distances
// are exact_score_rows' canonical fp64 scores (IP: -score) with the node's, then each tested
// candidate's, stored row staged in LDS as the query, so decisions equal the oracle's bit for bit.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline size_t hp_layout(int d, int C, int W, uint8_t* base, double** qs, double** cd, int** ci,
                                            double** sd, int** si, int** kept) {
    const size_t sz[6] = {(size_t)((d + 7) >> 3) * 64, (size_t)C * 8, (size_t)C * 4, (size_t)C * 8, (size_t)C * 4,
                          (size_t)W * 4};
    uint8_t* p[6];
    size_t off = 0;
    for (int i = 0; i < 6; ++i) {
        p[i] = base + off;
        off += (sz[i] + 15) & ~(size_t)15;
    }
    if (base) {
        *qs = (double*)p[0];
        *cd = (double*)p[1];
        *ci = (int*)p[2];
        *sd = (double*)p[3];
        *si = (int*)p[4];
        *kept = (int*)p[5];
    }
    return off;
}
size_t hnsw_prune_lds_bytes(int d, int C, int W) {
    return hp_layout(d, C, W, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
}

template <int DT, int METRIC>
__global__ void __launch_bounds__(HN_THREADS) k_hnsw_prune(HnswPruneArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NW = HN_THREADS / 64;
    constexpr int RR = refine_rows<DT>();
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    constexpr int CE = CHB / ES;
    constexpr bool IP = METRIC == METRIC_IP;
    __shared__ int s_m, s_bad[2];
    double *qs, *cd, *sd;
    int *ci, *si, *kept;
    hp_layout(a.d, a.C, a.W, smem, &qs, &cd, &ci, &sd, &si, &kept);
    const int node = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ng = (a.d + 7) >> 3;
    const int* cand = a.cand + (int64_t)node * a.C;
    int* out = a.out + (int64_t)node * a.W;
    // a stored row as the LDS query, in exact_score_rows' [e * ng + g] order
    auto stage_row = [&](int64_t r) {
        const uint8_t* rb = a.corpus + (r / TR) * (int64_t)TR * a.dpad * ES + (r % TR) * CHB;
        for (int i = tid; i < a.d; i += HN_THREADS)
            qs[(i & 7) * ng + (i >> 3)] = (double)load_elem<DT>(rb + (int64_t)(i / CE) * TR * CHB + (i % CE) * ES);
        __syncthreads();
    };
    if (tid == 0) s_m = a.C;
    __syncthreads();
    for (int j = tid; j < a.C; j += HN_THREADS) {
        const int v = cand[j];
        ci[j] = v;
        if (v < 0) atomicMin(&s_m, j);
    }
    stage_row(a.nodes[node]);  // (its barrier also publishes ci and s_m)
    const int m = s_m;
    // distances node -> candidates
    for (int j0 = wid * RR; j0 < m; j0 += NW * RR) {
        int64_t rr[RR];
#pragma unroll
        for (int i = 0; i < RR; ++i) rr[i] = j0 + i < m ? (int64_t)ci[j0 + i] : -1;
        double s[RR];
        exact_score_rows<DT, METRIC, true, RR>(a.corpus, rr, qs, nullptr, a.d, a.dpad, lane, s);
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < RR; ++i)
                if (j0 + i < m) cd[j0 + i] = IP ? -s[i] : s[i];
    }
    __syncthreads();
    for (int j = tid; j < m; j += HN_THREADS) {  // rank sort by (distance, id)
        const double dj = cd[j];
        const int ij = ci[j];
        int r = 0;
        for (int i = 0; i < m; ++i) r += hn_less(cd[i], ci[i], dj, ij) ? 1 : 0;
        sd[r] = dj;
        si[r] = ij;
    }
    __syncthreads();
    if (m < a.W) {
        for (int j = tid; j < a.W; j += HN_THREADS) out[j] = j < m ? si[j] : -1;
        return;
    }
    int nk = 0;  // uniform
    for (int i = 0; i < m && nk < a.W; ++i) {
        const int c = si[i];
        const double dq = sd[i];
        bool good = true;
        if (nk > 0) {
            stage_row(c);
            if (tid == 0) s_bad[0] = s_bad[1] = 0;
            __syncthreads();
            // kept neighbours in passes of NW * RR, stopping after the first pass that finds one
            // closer (the nearest kept ones come first, so most rejections end in pass one).  Pass
            // p raises flag p & 1: a fast wave's write in pass p + 1 cannot reach a slow wave still
            // reading pass p's flag, and that flag was 0 in pass p - 1 or the loop had ended
            int bad = 0;
            for (int p0 = 0, par = 0; p0 < nk; p0 += NW * RR, par ^= 1) {
                const int j0 = p0 + wid * RR;
                if (j0 < nk) {
                    int64_t rr[RR];
#pragma unroll
                    for (int t = 0; t < RR; ++t) rr[t] = j0 + t < nk ? (int64_t)kept[j0 + t] : -1;
                    double s[RR];
                    exact_score_rows<DT, METRIC, true, RR>(a.corpus, rr, qs, nullptr, a.d, a.dpad, lane, s);
                    bool closer = false;
#pragma unroll
                    for (int t = 0; t < RR; ++t) closer |= j0 + t < nk && (IP ? -s[t] : s[t]) < dq;
                    if (lane == 0 && closer) s_bad[par] = 1;
                }
                __syncthreads();
                bad = s_bad[par];  // (uniform: read after the barrier)
                if (bad) break;
            }
            good = bad == 0;
            __syncthreads();  // every thread has read its flag and qs before the next stage
        }
        if (good) {
            if (tid == 0) kept[nk] = c;
            ++nk;
            __syncthreads();
        }
    }
    for (int j = tid; j < a.W; j += HN_THREADS) out[j] = j < nk ? kept[j] : -1;
}

template <int DT>
static void launch_prune_dt(const HnswPruneArgs& a, int m, size_t lds, hipStream_t st) {
    if (a.metric == METRIC_IP) {
        set_lds_attr((const void*)k_hnsw_prune<DT, METRIC_IP>, (int)HN_LDS_CAP);
        hipLaunchKernelGGL((k_hnsw_prune<DT, METRIC_IP>), dim3(m), dim3(HN_THREADS), lds, st, a);
    } else {
        set_lds_attr((const void*)k_hnsw_prune<DT, METRIC_L2>, (int)HN_LDS_CAP);
        hipLaunchKernelGGL((k_hnsw_prune<DT, METRIC_L2>), dim3(m), dim3(HN_THREADS), lds, st, a);
    }
}
hipError_t launch_hnsw_prune(const HnswPruneArgs& a, int m, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    if (a.C < 1 || a.C > HP_C_MAX || a.W < 1 || a.W > HN_NB_MAX) return hipErrorInvalidValue;
    const size_t lds = hnsw_prune_lds_bytes(a.d, a.C, a.W);
    if (lds > HN_LDS_CAP) return hipErrorInvalidValue;
    if (a.dt == DT_F32) launch_prune_dt<DT_F32>(a, m, lds, st);
    else if (a.dt == DT_BF16) launch_prune_dt<DT_BF16>(a, m, lds, st);
    else if (a.dt == DT_F16) launch_prune_dt<DT_F16>(a, m, lds, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace vs
