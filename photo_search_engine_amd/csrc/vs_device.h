// vs_device.h -- device helpers shared by the gfx950 kernel sources of libvs (vs_kernels.hip,
// vs_fullscan.hip): orderable keys, dtype conversions, wave64 / block selection, and the exact
// canonical fp64 row scoring (bit-identical with oracle/vs_oracle.c).
#pragma once
#include "vs_internal.h"

#include <math.h>

namespace vs {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int intx4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// ------------------------------------------------------------------------------------------------
// scalar helpers (bit-identical with oracle/vs_oracle.c)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_f32(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
    uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    return __uint_as_float(u);
}
__device__ __forceinline__ u64 mk_key(float s, uint32_t id) {
    return ((u64)ord_f32(s) << 32) | (u64)(0xFFFFFFFFu - id);
}
__device__ __forceinline__ uint32_t key_id(u64 k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ float key_score(u64 k) { return unord_f32((uint32_t)(k >> 32)); }

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __forceinline__ uint16_t f32_to_f16_rne(float f) {
    uint32_t x = __float_as_uint(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return (uint16_t)(sign | (ax > 0x7F800000u ? 0x7E00u : 0x7C00u));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);
    if (ax < 0x38800000u) {
        float v = __uint_as_float(ax) * 16777216.0f;
        return (uint16_t)(sign | (uint32_t)rintf(v));
    }
    uint32_t e = (ax >> 23) - 127u + 15u;
    uint32_t mant = ax & 0x7FFFFFu;
    uint32_t r = (e << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) r++;
    return (uint16_t)(sign | r);
}
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float f16_bits_to_f32(uint32_t h) {
    _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)h);
    return (float)v;
}

template <int DT>
__device__ __forceinline__ float round_store(float v, uint8_t* p);
template <>
__device__ __forceinline__ float round_store<DT_F32>(float v, uint8_t* p) {
    *(float*)p = v;
    return v;
}
template <>
__device__ __forceinline__ float round_store<DT_BF16>(float v, uint8_t* p) {
    uint16_t h = f32_to_bf16_rne(v);
    *(uint16_t*)p = h;
    return bf16_bits_to_f32(h);
}
template <>
__device__ __forceinline__ float round_store<DT_F16>(float v, uint8_t* p) {
    uint16_t h = f32_to_f16_rne(v);
    *(uint16_t*)p = h;
    return f16_bits_to_f32(h);
}
template <int DT>
__device__ __forceinline__ float round_only(float v) {
    if constexpr (DT == DT_BF16) return bf16_bits_to_f32(f32_to_bf16_rne(v));
    else if constexpr (DT == DT_F16) return f16_bits_to_f32(f32_to_f16_rne(v));
    else return v;
}
template <int DT>
__device__ __forceinline__ float load_elem(const uint8_t* p) {
    if constexpr (DT == DT_F32) return *(const float*)p;
    else if constexpr (DT == DT_BF16) return bf16_bits_to_f32(*(const uint16_t*)p);
    else return f16_bits_to_f32(*(const uint16_t*)p);
}
// 16 B unit -> fp32 values (4 for f32, 8 for bf16/f16, 16 for the int8 screen copy)
template <int DT>
__device__ __forceinline__ void unpack16(const uint4 r, float* v) {
    if constexpr (DT == DT_F32) {
        v[0] = __uint_as_float(r.x); v[1] = __uint_as_float(r.y);
        v[2] = __uint_as_float(r.z); v[3] = __uint_as_float(r.w);
    } else if constexpr (DT == DT_BF16) {
        v[0] = __uint_as_float(r.x << 16); v[1] = __uint_as_float(r.x & 0xFFFF0000u);
        v[2] = __uint_as_float(r.y << 16); v[3] = __uint_as_float(r.y & 0xFFFF0000u);
        v[4] = __uint_as_float(r.z << 16); v[5] = __uint_as_float(r.z & 0xFFFF0000u);
        v[6] = __uint_as_float(r.w << 16); v[7] = __uint_as_float(r.w & 0xFFFF0000u);
    } else if constexpr (DT == DT_I8) {  // 16 int8 codes
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 * i + j] = (float)((int32_t)(w[i] << (24 - 8 * j)) >> 24);
    } else {
        v[0] = f16_bits_to_f32(r.x & 0xFFFFu); v[1] = f16_bits_to_f32(r.x >> 16);
        v[2] = f16_bits_to_f32(r.y & 0xFFFFu); v[3] = f16_bits_to_f32(r.y >> 16);
        v[4] = f16_bits_to_f32(r.z & 0xFFFFu); v[5] = f16_bits_to_f32(r.z >> 16);
        v[6] = f16_bits_to_f32(r.w & 0xFFFFu); v[7] = f16_bits_to_f32(r.w >> 16);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
#define SYNTH_SCALE ((float)(1.7320508075688772 / 4194304.0))
__device__ __forceinline__ float synth_raw(uint64_t base, uint64_t ctr) {
    uint64_t h1 = splitmix64(base + 2u * ctr);
    uint64_t h2 = splitmix64(base + 2u * ctr + 1u);
    uint32_t a = (uint32_t)(h1 & 0x3FFFFFu), b = (uint32_t)((h1 >> 22) & 0x3FFFFFu);
    uint32_t c = (uint32_t)(h2 & 0x3FFFFFu), d = (uint32_t)((h2 >> 22) & 0x3FFFFFu);
    int32_t s = (int32_t)(a + b + c + d) - (1 << 23);
    return (float)s * SYNTH_SCALE;
}

// ------------------------------------------------------------------------------------------------
// wave64 / block reductions and selection
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}
__device__ __forceinline__ float wave_sum_fp32_canon(float v) {
    // xor butterfly 32..1: identical expression tree to the oracle's part[j] + part[j ^ s]
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v = v + __shfl_xor(v, s, 64);
    return v;
}
__device__ __forceinline__ u64 wave_min_u64(u64 v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        u64 o = __shfl_xor(v, s, 64);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        u64 o = __shfl_xor(v, s, 64);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int lane_prefix(u64 mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// agent-scope relaxed stores / loads (global_store / global_load ... sc1): hand-offs between the
// workgroups of one launch without cache fences (MI355X_MICROARCH "valid forms": every handed-off
// byte stored and loaded sc1, every storing wave's vmcnt(0) before ONE lane's agent-scope counter
// add, the last adder told by the value its add returned, its waves loading after a barrier)
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// K-th largest key among the wave's keys (keys unique, 0 = empty, at least K non-empty).
// Bit-serial bisection with early exit once exactly K keys are >= the prefix.
template <int E>
__device__ __forceinline__ u64 wave_kth(const u64 (&keys)[E], int K) {
    u64 t = 0;
    for (int b = 63; b >= 0; --b) {
        const u64 cand = t | (1ull << b);
        int c = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) c += keys[e] >= cand ? 1 : 0;
        c = wave_sum_i(c);
        if (c >= K) {
            t = cand;
            if (c == K) break;
        }
    }
    return t;
}

// ... any threshold t with Klo <= #(keys >= t) <= Khi (the bisection stops at the first prefix
// whose count lands in the range; starts below the keys' common prefix)
template <int E>
__device__ __forceinline__ u64 wave_kth_range(const u64 (&keys)[E], int Klo, int Khi) {
    u64 kmax = 0ull, kmin = ~0ull;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        kmax = keys[e] > kmax ? keys[e] : kmax;
        kmin = (keys[e] != 0ull && keys[e] < kmin) ? keys[e] : kmin;
    }
    kmax = wave_max_u64(kmax);
    kmin = wave_min_u64(kmin);
    u64 t = 0;
    int bstart = 63;
    if (kmin != ~0ull && kmax != kmin) {
        bstart = 63 - __clzll((long long)(kmax ^ kmin));
        t = kmax & ~((2ull << bstart) - 1ull);
    }
    for (int b = bstart; b >= 0; --b) {
        const u64 cand = t | (1ull << b);
        int c = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) c += keys[e] >= cand ? 1 : 0;
        c = wave_sum_i(c);
        if (c >= Klo) {
            t = cand;
            if (c <= Khi) break;
        }
    }
    return t;
}
// K-th largest of n distinct keys in LDS / memory by ONE wave (no block barriers)
__device__ __forceinline__ u64 wave_kth_buf(const u64* buf, int n, int K) {
    const int lane = threadIdx.x & 63;
    u64 t = 0;
    for (int b = 63; b >= 0; --b) {
        const u64 cand = t | (1ull << b);
        int c = 0;
        for (int i = lane; i < n; i += 64) c += buf[i] >= cand ? 1 : 0;
        c = wave_sum_i(c);
        if (c >= K) {
            t = cand;
            if (c == K) break;
        }
    }
    return t;
}

// Over a whole block: a threshold t with Klo <= #(keys >= t) <= Khi (distinct keys, 0 = empty slot,
// Klo <= #keys; Khi = Klo: the Klo-th largest key).  Radix select over the keys' RANGE: w = key -
// min, rounds of 8 bits from the top bit of max - min (an LDS histogram of the digit among the keys
// matching the prefix so far; one wave scans the 256 bins from the top for the bin where the count
// reaches Klo), stopping at the first bin whose lower edge leaves at most Khi keys at or above it.
// The keys of a refine list span a narrow score range, so one or two rounds (3 barriers each)
// replace the ~25 one-barrier steps of a bit bisection (13 us of a phase-A refine at the 8-shard
// step).
template <int E>
__device__ __forceinline__ u64 block_kth_range(const u64 (&keys)[E], int Klo, int Khi, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __shared__ u64 mm[2 * 16];
    __shared__ unsigned hist[256];
    __shared__ int s_bin, s_above, s_cnt;
    (void)red;
    u64 kmax = 0ull, kmin = ~0ull;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        kmax = keys[e] > kmax ? keys[e] : kmax;
        kmin = (keys[e] != 0ull && keys[e] < kmin) ? keys[e] : kmin;
    }
    kmax = wave_max_u64(kmax);
    kmin = wave_min_u64(kmin);
    if (lane == 0) {
        mm[w] = kmax;
        mm[16 + w] = kmin;
    }
    __syncthreads();
    kmax = 0ull;
    kmin = ~0ull;
    for (int i = 0; i < nw; ++i) {
        kmax = mm[i] > kmax ? mm[i] : kmax;
        kmin = mm[16 + i] < kmin ? mm[16 + i] : kmin;
    }
    u64 t = kmin;
    if (kmin != ~0ull && kmax != kmin) {
        const u64 span = kmax - kmin;
        const int bits = 64 - __clzll((long long)span);
        u64 prefix = 0ull;
        int above = 0;  // keys above the prefix's range (counted in earlier rounds)
        for (int sh = bits - 8; sh > -8; sh -= 8) {
            const u64 hmask = sh + 8 >= 64 ? 0ull : ~0ull << (sh + 8);
            for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0u;
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const u64 x = keys[e] - kmin;
                if (keys[e] != 0ull && (x & hmask) == prefix)
                    atomicAdd(&hist[(unsigned)((sh >= 0 ? x >> sh : x << -sh) & 255ull)], 1u);
            }
            __syncthreads();
            if (w == 0) {  // lane l: bins 255-4l .. 252-4l (descending)
                unsigned c[4], sum = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    c[i] = hist[255 - 4 * lane - i];
                    sum += c[i];
                }
                unsigned incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const unsigned v = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += v;
                }
                const unsigned excl = incl - sum;
                const unsigned need = (unsigned)(Klo - above);
                const bool here = excl < need && incl >= need;
                if (here) {
                    unsigned cum = excl;
                    int i = 0;
                    while (cum + c[i] < need) cum += c[i++];
                    s_bin = 255 - 4 * lane - i;
                    s_above = above + (int)cum;
                    s_cnt = (int)c[i];
                }
                if (__ballot(here) == 0ull && lane == 0) {  // (fewer than Klo keys: the lowest bin)
                    s_bin = 0;
                    s_above = above;
                    s_cnt = 0;
                }
            }
            __syncthreads();
            const u64 b = (u64)s_bin;
            prefix |= sh >= 0 ? b << sh : b >> -sh;
            t = kmin + prefix;  // the bin's lower edge: s_above + s_cnt keys at or above it
            const int at = s_above + s_cnt;
            above = s_above;
            __syncthreads();  // (every wave has read the words before the next round rewrites them)
            if (at <= Khi || sh <= 0) break;
        }
    }
    __syncthreads();  // (every wave has read the shared words before the caller reuses them)
    return t;
}
// The K-th largest of the block's keys (distinct keys, K <= #keys); red: 2 x waves ints
template <int E>
__device__ __forceinline__ u64 block_kth(const u64 (&keys)[E], int K, int* red) {
    return block_kth_range<E>(keys, K, K, red);
}
// ... over keys in memory (lists longer than the registers hold)
__device__ __forceinline__ u64 block_kth_range_mem(const u64* buf, int n, int Klo, int Khi, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    u64 t = 0;
    for (int b = 63, par = 0; b >= 0; --b, par ^= 1) {
        const u64 cand = t | (1ull << b);
        int c = 0;
        for (int idx = threadIdx.x; idx < n; idx += blockDim.x) c += buf[idx] >= cand ? 1 : 0;
        c = wave_sum_i(c);
        if (lane == 0) red[par * nw + w] = c;
        __syncthreads();
        int tot = 0;
        for (int i = 0; i < nw; ++i) tot += red[par * nw + i];
        if (tot >= Klo) {
            t = cand;
            if (tot <= Khi) break;
        }
    }
    __syncthreads();  // (every wave has read red before its caller reuses it)
    return t;
}

// Write the block's keys >= t (t > 0) compactly to out[0..total), returns total.
template <int E>
__device__ __forceinline__ int block_write_kept(const u64 (&keys)[E], u64 t, u64* out, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int c = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) c += keys[e] >= t ? 1 : 0;
    int incl = c;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        int v = __shfl_up(incl, s, 64);
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
        if (keys[e] >= t) out[pos++] = keys[e];
    return total;
}

// K-th largest key of buf[0..n) by a 256-thread block, keys re-read from memory every bisection
// step (rare compaction path: keeps the streaming kernel's register budget small).
__device__ __forceinline__ u64 block_kth_mem(const u64* buf, int n, int K, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    u64 t = 0;
    for (int b = 63; b >= 0; --b) {
        const u64 cand = t | (1ull << b);
        int c = 0;
        for (int idx = threadIdx.x; idx < n; idx += blockDim.x) c += buf[idx] >= cand ? 1 : 0;
        c = wave_sum_i(c);
        if (lane == 0) red[w] = c;
        __syncthreads();
        int tot = 0;
        for (int i = 0; i < nw; ++i) tot += red[i];
        __syncthreads();
        if (tot >= K) {
            t = cand;
            if (tot == K) break;
        }
    }
    return t;
}
// Order-preserving compaction of src[0..n) keys >= t (t > 0) into dst[0..); dst may alias src
// (a kept key moves to a position <= its own, and every round reads before it writes).
__device__ __forceinline__ int block_compact_mem(const u64* src, u64* dst, int n, u64 t, int* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int base = 0;
    for (int r0 = 0; r0 < n; r0 += blockDim.x) {
        const int idx = r0 + threadIdx.x;
        const u64 k = idx < n ? src[idx] : 0ull;
        const bool keep = k >= t;
        const u64 m = __ballot(keep);
        if (lane == 0) red[w] = __popcll(m);
        __syncthreads();
        int wb = 0, tot = 0;
        for (int i = 0; i < nw; ++i) {
            if (i < w) wb += red[i];
            tot += red[i];
        }
        __syncthreads();
        if (keep) dst[base + wb + lane_prefix(m)] = k;
        base += tot;
    }
    return base;
}

__device__ __forceinline__ float f32_up(double v) {  // smallest fp32 >= v (v >= 0, finite)
    float f = (float)v;
    if ((double)f < v) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}

// ------------------------------------------------------------------------------------------------
// K5: exact refine -- canonical fp64 rescoring, sort, certificate, faiss-layout output
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool better_exact(double sa, uint32_t ia, double sb, uint32_t ib, int metric) {
    if (sa != sb) return metric == METRIC_IP ? (sa > sb) : (sa < sb);
    return ia < ib;
}

// Bitonic sort of (sc, ids)[0, n2) best first (n2 a power of two, padding = worst), the whole
// block taking part.  n2 <= blockDim.x: thread i keeps element i in registers; partners inside a
// wave (stride < 64) are exchanged by shuffles, wider ones through LDS (one barrier each way) --
// 3 barrier pairs for 256 elements instead of 36 barriers.  Larger n2: the LDS network.
template <int METRIC>
__device__ __forceinline__ void sort_best_first(double* sc, uint32_t* ids, int n2) {
    const int tid = threadIdx.x;
    if (n2 <= (int)blockDim.x) {
        const bool act = tid < n2;
        // (waves holding no element skip the shuffles -- they still meet every barrier)
        const bool wact = (tid & ~63) < n2;
        double s = act ? sc[tid] : 0.0;
        uint32_t id = act ? ids[tid] : 0u;
        for (int size = 2; size <= n2; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                double ps = 0.0;
                uint32_t pid = 0u;
                if (stride >= 64) {
                    __syncthreads();  // (every thread's previous read of its partner is done)
                    if (act) {
                        sc[tid] = s;
                        ids[tid] = id;
                    }
                    __syncthreads();
                    ps = act ? sc[tid ^ stride] : 0.0;
                    pid = act ? ids[tid ^ stride] : 0u;
                } else if (wact) {
                    ps = __shfl_xor(s, stride, 64);
                    pid = (uint32_t)__shfl_xor((int)id, stride, 64);
                }
                if (act) {
                    const bool up = (tid & size) == 0, lower = (tid & stride) == 0;
                    const bool pb = better_exact(ps, pid, s, id, METRIC);
                    if (lower == up ? pb : !pb) {
                        s = ps;
                        id = pid;
                    }
                }
            }
        }
        __syncthreads();
        if (act) {
            sc[tid] = s;
            ids[tid] = id;
        }
        __syncthreads();
        return;
    }
    for (int size = 2; size <= n2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < n2; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const double si = sc[i], sj = sc[j];
                    const uint32_t ii = ids[i], ij = ids[j];
                    const bool jb = better_exact(sj, ij, si, ii, METRIC);
                    if (up ? jb : !jb) {
                        sc[i] = sj; sc[j] = si;
                        ids[i] = ij; ids[j] = ii;
                    }
                }
            }
            __syncthreads();
        }
    }
}


// (sc, ids)[0, n) best first in place by rank (n <= blockDim.x; entries [n, n2) -- the caller's
// worst-score padding -- stay where they are): each entry's rank is the number of entries ahead of
// it under better_exact's order (IEEE compare, so -0 == +0; NaN ranked as the worst score; then
// the id; then the position, so equal entries keep distinct ranks), counted by NG groups of
// threads over a share of the entries each (8 broadcast LDS reads at a time, branch-free) and
// summed in LDS; then every entry moves to its rank.  A wave64 VALU op takes 4 cycles, so the
// count is spread over the whole block instead of one thread per entry (and ~log^2 n bitonic
// stages).  Larger n: the bitonic sort of all n2.
template <int METRIC>
__device__ __forceinline__ void sort_valid_best_first(double* sc, uint32_t* ids, int n, int n2) {
    if (n > (int)blockDim.x) {
        sort_best_first<METRIC>(sc, ids, n2);
        return;
    }
    __shared__ int rk[256];
    const int tid = threadIdx.x;
    int T = 64;  // threads per group: one per entry
    while (T < n) T <<= 1;
    const int NG = T <= 256 ? (int)blockDim.x / T : 1;
    const int e = tid & (T - 1), g = tid / T;
    const double worst = METRIC == METRIC_L2 ? INFINITY : -INFINITY;
    if (NG > 1) {
        for (int i = tid; i < T; i += blockDim.x) rk[i] = 0;
        __syncthreads();
    }
    double ms = 0.0;
    uint32_t mid = 0u;
    int rank = 0;
    const bool mine = e < n && g < NG;
    if (mine) {
        ms = sc[e];
        mid = ids[e];
        const double mk = ms == ms ? ms : worst;
        const int j0 = (int)((int64_t)n * g / NG), j1 = (int)((int64_t)n * (g + 1) / NG);
        for (int jb = j0; jb < j1; jb += 8) {
            double sv[8];
            uint32_t iv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = min(jb + u, j1 - 1);
                sv[u] = sc[j];
                iv[u] = ids[j];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = jb + u;
                const double k = sv[u] == sv[u] ? sv[u] : worst;
                const int gt = METRIC == METRIC_L2 ? (int)(k < mk) : (int)(k > mk);
                const int ahead = gt | ((int)(k == mk) & ((int)(iv[u] < mid) | ((int)(iv[u] == mid) & (int)(j < e))));
                rank += ahead & (int)(j < j1);
            }
        }
    }
    if (NG > 1) {
        if (mine && rank) atomicAdd(&rk[e], rank);
        __syncthreads();
        if (mine && g == 0) rank = rk[e];
    }
    __syncthreads();  // (every read of sc / ids is done)
    if (mine && g == 0) {
        sc[rank] = ms;
        ids[rank] = mid;
    }
    __syncthreads();
}

// Exact canonical fp64 scores of R stored rows at once (row[i] < 0: absent), query staged in LDS as
// fp64 (QLDS) or read from global fp32.  Lane l owns 8-element groups g = l, l+64, ... in ascending
// order and accumulates them sequentially, then an xor-butterfly 32..1 -- the expression tree of the
// oracle's orc_canon_scores (oracle/vs_oracle.c), so scores are bit-identical.  All R rows' gathers
// are issued before any is consumed (R rows of d x es bytes in flight per wave); a row's piece of a
// chunk is one 128 B line.
template <int DT>
constexpr int refine_rows() { return DT == DT_F32 ? 2 : 4; }  // (fp32 rows: twice the registers)
template <int DT, int METRIC, bool QLDS, int R>
__device__ __forceinline__ void exact_score_rows(const uint8_t* __restrict__ corpus, const int64_t (&row)[R],
                                                 const double* __restrict__ qs, const float* __restrict__ qg, int d,
                                                 int dpad, int lane, double (&out)[R]) {
#pragma clang fp contract(off)
    constexpr int ES = DT == DT_F32 ? 4 : 2;
    constexpr int NV = DT == DT_F32 ? 2 : 1;
    constexpr int RU = 3;
    constexpr int CE = CHB / ES;
    const uint8_t* rb[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int64_t r = row[i] >= 0 ? row[i] : row[0];
        rb[i] = corpus + (r / TR) * (int64_t)TR * dpad * ES + (r % TR) * CHB;
    }
    const int ng = (d + 7) >> 3;
    double acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = 0.0;
    for (int g0 = lane; g0 < ng; g0 += 64 * RU) {
        uint4 raw[RU][R][NV];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const int g = g0 + 64 * u;
            if (g < ng) {
                const int e0 = 8 * g;
                const int64_t off = (int64_t)(e0 / CE) * TR * CHB + (e0 % CE) * ES;
#pragma unroll
                for (int i = 0; i < R; ++i)
                    if (i == 0 || row[i] >= 0)
#pragma unroll
                        for (int v = 0; v < NV; ++v) raw[u][i][v] = *(const uint4*)(rb[i] + off + 16 * v);
            }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const int g = g0 + 64 * u;
            if (g < ng) {
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    if (i > 0 && row[i] < 0) continue;
                    float x[8];
#pragma unroll
                    for (int v = 0; v < NV; ++v) unpack16<DT>(raw[u][i][v], x + 4 * v);
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int ie = 8 * g + e;
                        if (ie < d) {
                            const double qq = QLDS ? qs[e * ng + g] : (double)qg[ie];
                            const double xa = (double)x[e];
                            if constexpr (METRIC == METRIC_IP) {
                                const double pa = xa * qq;
                                acc[i] = acc[i] + pa;
                            } else {
                                const double da = xa - qq;
                                const double pa = da * da;
                                acc[i] = acc[i] + pa;
                            }
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int sft = 32; sft > 0; sft >>= 1)
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const double o = __shfl_xor(acc[i], sft, 64);
            acc[i] = acc[i] + o;
        }
#pragma unroll
    for (int i = 0; i < R; ++i) out[i] = acc[i];
}

}  // namespace vs
