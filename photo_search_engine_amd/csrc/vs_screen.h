// vs_screen.h -- K1, the MFMA screens (tiled form screen_mfma, direct form screen_direct) as
// templates, shared by vs_kernels.hip (the product kernels) and vs_k1probe.hip (the diagnostic
// probe variants of the int8 direct screen, DESIGN §5 "Where K1 int8's time goes").
#pragma once
#include "vs_internal.h"
#include "vs_device.h"
#include "vs_i8_asm.h"

namespace vs {
// ------------------------------------------------------------------------------------------------
// K1: MFMA screen (bf16 / f16 rows, or the int8 screen copy; up to 256 queries per launch)
// ------------------------------------------------------------------------------------------------
// Workgroup = 512 threads = 8 waves (2 per SIMD), one per CU, persistent over a contiguous range
// of row tiles.  Output tile per tile pass: 256 corpus rows (M) x 256 queries (N), K = dpad.
// Waves 4(M) x 2(N): each wave 64 rows x 128 queries = 4 x 8 MFMA 16x16 tiles, 128 acc VGPRs.
//
// K-step = one 16 KiB block per operand: 256 rows x 64 B, i.e. 32 bf16/f16 elements
// (v_mfma_f32_16x16x32_{bf16,f16}) or 64 int8 elements (v_mfma_i32_16x16x64_i8, exact int32
// accumulation).  Both MFMAs take a lane's 16 B at (row lane & 15, piece lane >> 4) of a 64 B row
// chunk, so the two element types share the LDS image, the fragment reads and the C layout.  The
// blocks (the tile's rows, the query tile) are copied by LDS-DMA (global_load_lds_dwordx4, inline
// asm) into a 4-slot LDS ring MF_DEPTH = 3 K-steps ahead of the MFMAs.  Each K-step waits only for
// its own stage (counted s_waitcnt vmcnt, raw s_barrier), so three stages (48 KiB of corpus per
// CU) stay in flight across barriers.  The lane-linear LDS image is XOR-swizzled on the SOURCE
// address (64 B rows: 16 B piece p of row r holds chunk p ^ perm[(r >> 2) & 3]) so every
// ds_read_b128 fragment read is bank-conflict free.
constexpr int MF_SLOT = 32768;  // 16 KiB corpus + 16 KiB queries
constexpr int MF_SLOTS = 4;
constexpr int MF_DEPTH = MF_SLOTS - 1;
constexpr int MF_THREADS = 512;
constexpr int MF_POOL = 512;  // LDS insert pool of the loader waves (flushed by the writer waves)
constexpr int MF_SX = 8 * 64 * 8 * 4;  // per-wave insert staging: 64 lanes x 8 fp32 (slow path only)
constexpr int MF_QFAC = 256 * 8;       // int8 screen: (t_q, ||q|| / t_q) per query
constexpr int MF_ROWX = 2 * 256 * 4;   // per-row side data of two tiles (int8: scale | beta; L2: ||x||^2)
constexpr int MF_LDS = MF_SLOTS * MF_SLOT + 256 * 8 + 256 * 4 + 256 * 4 + 16 + MF_POOL * 8 + MF_POOL * 4 + MF_SX + MF_QFAC +
                       MF_ROWX;
static_assert(MF_LDS <= 160 * 1024, "LDS budget");
constexpr int MF_LDS_MAP = MF_LDS + MFMA_MAP_TILES * 4;  // mapped screen: + the workgroup's page table
static_assert(MF_LDS_MAP <= 160 * 1024, "LDS budget (mapped screen)");

typedef __attribute__((address_space(3))) uint8_t* lds_u8_t;

// LDS-DMA of 16 B per lane: LDS[m0 + lane*16] <- global[gptr].  Inline asm, so the compiler
// neither fences later ds_reads with vmcnt(0) (it cannot tell which LDS bytes a builtin DMA
// writes) nor drains it at barriers; the kernel counts these loads in its own s_waitcnt.
__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
// the same with the non-temporal hint (corpus blocks are read once per pass)
__device__ __forceinline__ void glds16_nt(const void* gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) { return (uint32_t)(uintptr_t)(lds_u8_t)(p); }

// swizzle: piece position of 16 B chunk c of LDS row r (64 B rows) = c ^ mf_swz(r)
__device__ __forceinline__ int mf_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// issue one K-step stage: waves 0-3 (the loader waves) issue 8 LDS-DMA instructions per thread
// (4 corpus + 4 query); waves 4-7 issue none.  Loader waves never store to global memory and the
// writer waves never load, so each wave's in-order vmcnt holds one kind of traffic: counted waits
// on the stage ring are never held up behind candidate stores.  Corpus rows are 1 << RS bytes
// apart (bf16 / f16: 128, the K-step reads the first or second 64 B of each row's line; int8: 64,
// contiguous); the LDS block is [row][64 B] either way.
template <int RS, int NLW>
__device__ __forceinline__ void mf_stage(const uint8_t* __restrict__ gA, const uint8_t* __restrict__ gB,
                                         uint32_t slot_base, int tid) {
    constexpr int NIT = 16 / NLW;  // DMA instructions per loader wave per operand
    const int w = tid >> 6, lane = tid & 63;
    if (w >= NLW) return;
    const uint32_t base = __builtin_amdgcn_readfirstlane(slot_base + (uint32_t)(w * 64 * 16));
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int g = it * (NLW * 64) + w * 64 + lane;
        const int row = g >> 2, pos = g & 3;
        // int8: each 64 B row piece is read once -> non-temporal; bf16 / f16: the line's other
        // half is read by the next K-step, so it must stay in L2 (default policy)
        if constexpr (RS == 6) glds16_nt(gA + ((size_t)row << RS) + (size_t)(pos ^ mf_swz(row)) * 16, base + it * NLW * 1024);
        else glds16(gA + ((size_t)row << RS) + (size_t)(pos ^ mf_swz(row)) * 16, base + it * NLW * 1024);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {  // the query tile is re-read by every CU: default policy (L2)
        const int g = it * (NLW * 64) + w * 64 + lane;
        const int row = g >> 2, pos = g & 3;
        const int src = (row << 2) + (pos ^ mf_swz(row));
        glds16(gB + (size_t)src * 16, base + it * NLW * 1024 + 16384);
    }
}

// wait until at most `ahead` younger stages (32 / NLW LDS-DMA each) of a loader wave are in
// flight, then barrier; other waves only drain their LDS traffic
template <int NLW>
__device__ __forceinline__ void mf_wait_barrier(int ahead, bool loader) {
    constexpr int P = 32 / NLW;
    if (!loader) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(3 * P) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * P) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(P) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void mf_barrier_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void mf_barrier_drain() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// one 16x16 MFMA tile step; the int8 form accumulates exact int32 (its bits live in the fp32
// accumulator registers and are converted in the epilogue)
template <int DT>
__device__ __forceinline__ floatx4 mfma16(const uint4 a, const uint4 b, floatx4 c) {
    if constexpr (DT == DT_I8)
        return __builtin_bit_cast(floatx4, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                               __builtin_bit_cast(intx4, a), __builtin_bit_cast(intx4, b),
                                               __builtin_bit_cast(intx4, c), 0, 0, 0));
    else if constexpr (DT == DT_BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                       0, 0, 0);
    else if constexpr (DT == DT_F32) {
        // fp32 rows (the fallback round of fp32 indexes, and their large batches): a 16 B fragment
        // holds 4 consecutive k of the K-step's 16, consumed by 4 16x16x4 MFMAs (MFMA k-slot g =
        // lane >> 4 is physical k 4g + e in MFMA e, for A and B alike)
        const floatx4 av = __builtin_bit_cast(floatx4, a), bv = __builtin_bit_cast(floatx4, b);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], c, 0, 0, 0);
        return __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], c, 0, 0, 0);
    }
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                      0, 0);
}

// one K-step: 4 A (corpus) + 8 B (query) fragments by ds_read_b128 at ONE per-lane offset plus
// immediates ((row >> 2) & 3 of every fragment row equals that of lane & 15), then 32 MFMAs
template <int DT>
__device__ __forceinline__ void mf_compute(const uint8_t* buf, floatx4 (&acc)[4][8], int wm, int wn, int lane_off) {
    uint4 af[4], bfr[8];
    const uint8_t* pa = buf + wm * 4096 + lane_off;
    const uint8_t* pb = buf + 16384 + wn * 8192 + lane_off;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) af[mi] = *(const uint4*)(pa + mi * 1024);
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) bfr[ni] = *(const uint4*)(pb + ni * 1024);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = mfma16<DT>(af[mi], bfr[ni], acc[mi][ni]);
}

// compact one (workgroup, query) candidate buffer to its best K keys (one wave); the new threshold
// is the workgroup's drop bound for the query, published to drop[] (the refine's certificate)
template <int E>
__device__ __forceinline__ void mf_wave_compact(u64* __restrict__ buf, int n, int K, u64* thr_key, float* thr_f,
                                                u64* drop, int lane) {
    u64 keys[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int idx = lane + 64 * e;
        keys[e] = idx < n ? buf[idx] : 0ull;
    }
    const u64 t = wave_kth<E>(keys, K);
    int base = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const bool keep = keys[e] >= t;
        const u64 m = __ballot(keep);
        const int pos = base + lane_prefix(m);
        if (keep) buf[pos] = keys[e];
        base += __popcll(m);
    }
    if (lane == 0) {
        *thr_key = t;
        *thr_f = key_score(t);
        if (drop) atomicMax(drop, t);
    }
}

// Flush of a workgroup's candidate buffers into the per-query survivor lists, once every buffer
// holds at most Kp keys (cnt[q] = its length).  Wave w owns queries w, w + 8, ... (32 per wave):
// lanes 0..31 reserve their queries' list space with one atomic each, issued together, and the
// wave's keys are then copied by one flat loop of independent loads and stores.  (One returning
// atomic and one dependent copy per query in turn -- with every workgroup flushing at the same
// moment onto the same 256 counters -- cost ~0.1 ms per launch: the screens' fixed overhead.)
template <bool MAP>
__device__ __forceinline__ void mf_flush_wave(const ScreenArgs& a, const u64* __restrict__ cand, const int* cnt,
                                              int nqb, int wid, int lane) {
    int n = 0, off = 0, qg = 0;
    const int q = wid + 8 * lane;
    if (lane < 32 && q < nqb) {
        n = min(cnt[q], min(a.cap, a.Kp));
        qg = MAP ? a.qmap[q] : q;
        if (n > 0) off = atomicAdd(&a.gcnt[qg], n);
    }
    int incl = n;
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) {
        const int v = __shfl_up(incl, sft, 64);
        if (lane >= sft) incl += v;
    }
    const int total = __shfl(incl, 63, 64);
    const int excl = incl - n;
    for (int t0 = 0; t0 < total; t0 += 64) {  // (wave-uniform trip count: every lane shuffles)
        const int t = t0 + lane;
        int lo = 0, hi = 31;  // the owner: the last lane whose exclusive prefix is <= t
#pragma unroll
        for (int step = 0; step < 5; ++step) {
            const int mid = (lo + hi + 1) >> 1;
            if (__shfl(excl, mid, 64) <= t) lo = mid;
            else hi = mid - 1;
        }
        const int j = t - __shfl(excl, lo, 64);
        const int o = __shfl(off, lo, 64);
        const int g = __shfl(qg, lo, 64);
        if (t < total) a.glist[(size_t)g * a.lcap + o + j] = cand[(size_t)(wid + 8 * lo) * a.cap + j];
    }
}

// SEED: the threshold-seed pass (one tile per workgroup, 16-row-group maxima of the keys only).
// Keys: bf16/f16 -> the fp32 MFMA score (L2: 2 x.q - ||x||^2); int8 -> the upper bound
// s_x t_q <c_x, c_q> + ||e_x|| ||q|| of the true inner product (the query-side error term is
// uniform over rows and sits in the refine's margin).
// MAP: the IVF list scan -- logical tile t of the launch is page a.tile_map[t] of a page pool (the
// workgroup's pages staged in LDS), keys carry storage slots, survivors go to glist row a.qmap[q].
template <int DT, int METRIC, bool SEED, bool MAP = false>
__device__ __forceinline__ void screen_mfma(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    constexpr bool I8 = DT == DT_I8;
    // int8 + L2: keys 2 (upper bound of <x, q>) - ||x||^2, the tile's ||x||^2 read by ordinary loads
    // in the epilogue (this form serves the seed pass and the main pass of d % 256 != 0; the direct
    // form k_screen_i8d stages them by LDS-DMA)
    constexpr bool I8L2 = I8 && METRIC == METRIC_L2;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    u64* thr_key = (u64*)(smem + MF_SLOTS * MF_SLOT);
    float* thr_f = (float*)(smem + MF_SLOTS * MF_SLOT + 256 * 8);
    int* cnt = (int*)(smem + MF_SLOTS * MF_SLOT + 256 * 12);
    int* flag = (int*)(smem + MF_SLOTS * MF_SLOT + 256 * 16);  // [1] pool count, [2 + tile parity] inserted
    u64* pool_key = (u64*)(smem + MF_SLOTS * MF_SLOT + 256 * 16 + 16);
    int* pool_q = (int*)(smem + MF_SLOTS * MF_SLOT + 256 * 16 + 16 + MF_POOL * 8);
    float* sx = (float*)(smem + MF_SLOTS * MF_SLOT + 256 * 16 + 16 + MF_POOL * 12) + (threadIdx.x >> 6) * 512 +
                (threadIdx.x & 63) * 8;
    float2* qfac = (float2*)(smem + MF_SLOTS * MF_SLOT + 256 * 16 + 16 + MF_POOL * 12 + MF_SX);
    uint32_t* rowx = (uint32_t*)(smem + MF_SLOTS * MF_SLOT + 256 * 16 + 16 + MF_POOL * 12 + MF_SX + MF_QFAC);

    // The LDS ring is written only by the inline-asm DMA: let the array escape into an asm with a
    // memory clobber, so the compiler must assume every later memory-clobbering asm (DMA issue,
    // barriers) may write it and can never fold the fragment reads away.
    asm volatile("; lds ring escapes: %0" ::"v"(smem) : "memory");
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid & 3, wn = wid >> 2;
    const int blk = blockIdx.x;
    int t0 = (int)((int64_t)a.tiles * blk / a.G);
    int t1 = (int)((int64_t)a.tiles * (blk + 1) / a.G);
    if (a.tile_stride > 0) {
        // seed pass: one tile per workgroup; with seed_acc, the first tile of the main pass's range
        // of this workgroup (same G), whose raw accumulators the main pass then reuses
        t0 = a.seed_acc ? (int)((int64_t)a.tiles * blk / a.G) : blk * a.tile_stride;
        t1 = t0 + 1 <= a.tiles ? t0 + 1 : a.tiles;
    }
    static_assert(!(MAP && SEED), "the mapped screen is unseeded");
    // a fallback round (gated) interleaves its tiles as the direct main passes do (workgroup blk:
    // tiles blk, blk + G, ...): a cluster stored contiguously then spreads over every workgroup's
    // MFMA_KP_MAX-deep lists instead of filling two or three of them, whose compaction bounds would
    // sit inside the query's top rows
    const bool ilv = !MAP && !SEED && a.gate != nullptr;
    if (ilv) {
        t0 = 0;
        t1 = a.tiles > blk ? (a.tiles - blk + a.G - 1) / a.G : 0;
    }
    int* tmap = (int*)(smem + MF_LDS);  // MAP: page of logical tile tbase + i
    if constexpr (MAP) {  // this workgroup's list segment, query tile and page table
        const int* dsc = a.wg_desc + (size_t)blk * MAP_DESC;
        const int tm_off = dsc[0], nt = dsc[1];
        t0 = dsc[2];
        t1 = t0 + nt;
        a.n_valid = dsc[3];
        qt += (size_t)dsc[4] * MFMA_QB * a.dpad * 2;
        a.qmap += dsc[5];
        nqb = dsc[6];
        for (int i = tid; i < nt; i += MF_THREADS) tmap[i] = a.tile_map[tm_off + i];
        __syncthreads();
    }
    const int tbase = t0;
    // storage tile of logical tile t
    auto phys = [&](int t) -> int64_t {
        if constexpr (MAP) return (int64_t)tmap[t - tbase];
        else return ilv ? (int64_t)blk + (int64_t)t * a.G : (int64_t)t;
    };
    const bool reuse = !MAP && !SEED && a.seed_acc != nullptr && t1 > t0;
    const int tseed = t0;
    if (reuse) ++t0;
    if (tid < 256) {
        // (a fallback round screens only the queries its first pass left uncertified)
        const bool real = tid < nqb && !(a.skip && a.skip[tid] != 0);
        const u64 k0 = real ? (a.thr0 ? a.thr0[tid] : 0ull) : ~0ull;
        thr_key[tid] = k0;
        thr_f[tid] = !real ? INFINITY : (k0 == 0ull ? -INFINITY : key_score(k0));
        cnt[tid] = 0;
        if constexpr (I8) qfac[tid] = real ? a.qfac[tid] : make_float2(0.0f, 0.0f);
    }
    if (tid == 0) {
        flag[0] = 0;
        flag[1] = 0;
        flag[2] = 0;
        flag[3] = 0;
    }
    constexpr bool F32 = DT == DT_F32;
    const int nks = a.dpad / (I8 ? 64 : F32 ? CH / 2 : CH);  // K-steps per tile (16 KiB each)
    const int64_t tbytes = (int64_t)TR * a.dpad * (I8 ? 1 : F32 ? 4 : 2);
    constexpr int RS = I8 ? 6 : 7;  // log2 of the corpus row stride within a chunk (see mf_stage)
    // waves issuing the stage DMAs (8 each per K-step): the loader waves.  Spreading them over all
    // 8 waves (4 each) measured slower for both screens (int8 K1 4.39 -> 4.54 ms, bf16 7.60 -> 7.94)
    constexpr int NLW = 4;
    // K-step ks of tile ti: int8 -> chunk ks (64 B per row); bf16 / f16 / fp32 -> half (ks & 1) of
    // chunk ks / 2 (128 B per row: 64 bf16 / 32 fp32 elements)
    auto kblock = [&](int ti, int ks) -> const uint8_t* {
        if constexpr (I8) return a.corpus + phys(ti) * tbytes + (int64_t)ks * 16384;
        else return a.corpus + phys(ti) * tbytes + (int64_t)(ks >> 1) * (TR * CHB) + (ks & 1) * 64;
    };
    const int S = (t1 - t0) * nks;
    u64* cand = a.cand + (size_t)blk * (MAP ? MFMA_QB / 2 : MFMA_QB) * a.cap;
    const int trigger = a.cap - TR;
    const uint32_t ring = lds_addr(smem);
    const int r16 = lane & 15;
    const int lane_off = r16 * 64 + (((lane >> 4) ^ mf_swz(r16)) << 4);

    floatx4 acc[4][8];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};

    // Per-row side data of a tile (int8: packed scale | error norm; L2: ||x||^2), 4 B per row = one
    // 1 KiB LDS-DMA by wave 0 into buffer (tile & 1), issued 3 K-steps before the tile's epilogue
    // (after the previous reader of that buffer, two tiles back): the counted wait of the
    // epilogue's K-step covers it, like a stage.  No ordinary global load in the K loop, so no
    // compiler-placed wait ever drains the in-flight stages.
    constexpr bool ROWX = I8 || METRIC == METRIC_L2;
    const uint32_t* rowsrc = I8 ? a.rsb : (const uint32_t*)a.sqn;
    auto rowx_issue = [&](int tile) {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr((const uint8_t*)(rowx + (tile & 1) * TR)));
        glds16(rowsrc + phys(tile) * TR + lane * 4, dst);
    };
    // the DMA for the epilogue at loop step j (if j ends a tile)
    auto rowx_rule = [&](int j) {
        if (j >= S) return;
        const int tile = t0 + j / nks;
        if (j % nks == nks - 1) rowx_issue(tile);
    };
    if constexpr (ROWX) {
        if (wid == 0) {
            if (reuse) {  // the seed tile's epilogue runs before the loop (below)
                rowx_issue(tseed);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            for (int j = 0; j < 3; ++j) rowx_rule(j);  // epilogues at loop steps 0..2
        }
        if (reuse) mf_barrier_lgkm();
    }

    // prologue: stages 0 .. DEPTH-1
    int iti = t0, iks = 0;  // (tile, k-step) of the next stage to issue
    for (int j = 0; j < MF_DEPTH && j < S; ++j) {
        mf_stage<RS, NLW>(kblock(iti, iks), qt + (int64_t)iks * 16384,
                 ring + (uint32_t)(j * MF_SLOT), tid);
        if (++iks == nks) { iks = 0; ++iti; }
    }
    int ti = t0, ks = 0;
    bool check_pending = false;
    // tile epilogue over the accumulators of tile `ti` (shared by the K loop and the seed tile)
    auto tile_epilogue = [&](const int ti) {
        // ---- fused top-k epilogue: threshold filter, rare inserts ----
        // Lane-derived indices come from an asm-opaque copy of the lane id, so the compiler
        // cannot hoist them out of the K loop (they would pin VGPRs the MFMA loop needs).
        if constexpr (SEED) {
            if (a.seed_acc) {  // raw accumulators of the tile, for the main pass to reuse
                // per lane 512 contiguous bytes: one base address, immediate offsets
                floatx4* dst = (floatx4*)(a.seed_acc + ((size_t)blk * MF_THREADS + tid) * 128);
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 8; ++ni) dst[mi * 8 + ni] = acc[mi][ni];
            }
        }
        int olane;
        asm volatile("v_mov_b32 %0, %1" : "=v"(olane) : "v"(lane));
        const int64_t rowbase = (MAP ? (int64_t)ti : phys(ti)) * TR;  // logical (the n_valid mask)
        const int64_t idbase = MAP ? phys(ti) * TR : rowbase;  // key ids: storage slots
        const int rid0 = wm * 64 + (olane >> 4) * 4;  // + mi*16 + r
        const int q0 = wn * 128 + (olane & 15);        // + ni*16
        // padding rows of the shard's last tile never qualify: NaN, not -inf (fmaxf skips it and
        // every `>= threshold` test fails, even against the unseeded threshold -inf; a -inf key
        // would enter the candidates and be rescored exactly as 0, beating all-negative scores)
        uint32_t bad = 0;
        if (rowbase + TR > a.n_valid) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (rowbase + rid0 + mi * 16 + r >= a.n_valid) bad |= 1u << (mi * 4 + r);
        }
        float sq[4][4], rb[4][4];  // L2: ||x||^2; int8: the row's scale and error norm (from LDS)
        float sq8[4][4];           // int8 + L2: ||x||^2
        if constexpr (I8L2) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gr = rowbase + rid0 + mi * 16 + r;
                    sq8[mi][r] = a.sqn[gr < a.n_valid ? gr : a.n_valid - 1];
                }
        }
        if constexpr (ROWX) {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const uint4 w = *(const uint4*)(rowx + (ti & 1) * TR + rid0 + mi * 16);
                const uint32_t w4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (I8) {
                        sq[mi][r] = __uint_as_float(w4[r] << 16);
                        rb[mi][r] = __uint_as_float(w4[r] & 0xFFFF0000u);
                    } else {
                        sq[mi][r] = __uint_as_float(w4[r]);
                    }
                }
            }
        }
        // MAP: the query tile holds (hi, lo) bf16/f16 parts of each query in column pairs (ni even /
        // odd), so a query's screen score is the sum of two accumulators (near-fp32 precision)
        constexpr int NCOL = MAP ? 4 : 8;
#pragma unroll
        for (int ni = 0; ni < NCOL; ++ni) {
            const int q = MAP ? wn * 64 + ni * 16 + (olane & 15) : q0 + ni * 16;
            // int8: values in the query's scaled domain v = s_x <c_x, c_q> + beta_x ||q|| / t_q (one
            // convert, one multiply, one fma per value, in packed pairs); the key is t_q * v
            float tq = 1.0f;
            float v[4][4];
            if constexpr (I8) {
                const float2 f = qfac[q];
                tq = f.x;
                const floatx2 u2 = {f.y, f.y};
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const floatx2 av = {(float)__float_as_int(acc[mi][ni][2 * h]),
                                            (float)__float_as_int(acc[mi][ni][2 * h + 1])};
                        const floatx2 s2 = {sq[mi][2 * h], sq[mi][2 * h + 1]};
                        const floatx2 b2 = {rb[mi][2 * h], rb[mi][2 * h + 1]};
                        const floatx2 vv = __builtin_elementwise_fma(b2, u2, av * s2);
                        v[mi][2 * h] = vv.x;
                        v[mi][2 * h + 1] = vv.y;
                    }
                if constexpr (I8L2) {  // the keys themselves: 2 t_q v - ||x||^2
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[mi][r] = __builtin_fmaf(2.0f, v[mi][r] * tq, -sq8[mi][r]);
                }
            } else {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float sc = MAP ? acc[mi][2 * ni][r] + acc[mi][2 * ni + 1][r] : acc[mi][ni][r];
                        if constexpr (METRIC == METRIC_L2) sc = 2.0f * sc - sq[mi][r];
                        v[mi][r] = sc;
                    }
            }
            if (bad) {  // the shard's last tile only
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (bad & (1u << (mi * 4 + r))) v[mi][r] = __builtin_nanf("");
            }
            float mx = -INFINITY;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r) mx = fmaxf(mx, v[mi][r]);
            if constexpr (I8 && !I8L2) mx *= tq;  // monotone: fl(t * max v) = max fl(t * v)
            // one compare per query column; the insert path runs only where something passes,
            // and then costs one LDS atomic per lane plus predicated stores
            if constexpr (SEED) {  // group g = wm*4 + lane/16 of the tile: 16 distinct rows
                // group residuals: + <mu_g, q> of the tile's group, as the main pass's keys
                // (fl(fl(t max v) + T) = max fl(fl(t v) + T): the seed is a real row's key)
                if constexpr (I8 && !I8L2)
                    if (a.gT) mx += a.gT[(size_t)((int64_t)ti * TR / I8_GROUP_ROWS) * MFMA_QB + q];
                a.seedmax[(size_t)q * (a.G * 16) + blk * 16 + wm * 4 + (olane >> 4)] = mx;
                continue;
            }
            const float tf = thr_f[q];
            if (mx >= tf) {
                const u64 tk = thr_key[q];
                uint32_t m = 0;
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (I8 && !I8L2) v[mi][r] *= tq;  // the keys' scores
                        m |= (v[mi][r] >= tf ? 1u : 0u) << (mi * 4 + r);  // ties below
                    }
                if (m) flag[2 + (ti & 1)] = 1;
                // Compact insert loop (not unrolled: an unrolled insert path for 8 columns x 16
                // values costs more in instruction fetch than the rare inserts themselves).  The
                // lane's values go through its LDS staging row, 8 at a time, so the loop can
                // index them.  Loader waves park keys in the LDS pool; writer waves store them to
                // the global candidate buffer.  (A younger VMEM op in a loader wave -- a pool
                // overflow store -- only makes its counted ring waits stricter, never looser.)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t mh = (m >> (8 * h)) & 0xFFu;
                    if (!mh) continue;
                    *(float4*)(sx) = make_float4(v[2 * h][0], v[2 * h][1], v[2 * h][2], v[2 * h][3]);
                    *(float4*)(sx + 4) = make_float4(v[2 * h + 1][0], v[2 * h + 1][1], v[2 * h + 1][2],
                                                     v[2 * h + 1][3]);
                    while (mh) {
                        const int j = __builtin_ctz(mh);
                        mh &= mh - 1u;
                        const int bit = 8 * h + j;
                        const u64 key = mk_key(sx[j], (uint32_t)(idbase + rid0 + (bit >> 2) * 16 + (bit & 3)));
                        if (key <= tk) continue;  // score == threshold and not ahead of it by id
                        if (wid < 4) {
                            const int slot = atomicAdd(&flag[1], 1);
                            if (slot < MF_POOL) {
                                pool_key[slot] = key;
                                pool_q[slot] = q;
                                continue;
                            }
                        }
                        const int slot = atomicAdd(&cnt[q], 1);
                        if (slot < a.cap) cand[(size_t)q * a.cap + slot] = key;
                    }
                }
            }
        }
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
        check_pending = !SEED;
    };
    if (reuse) {
        // the seed pass screened this workgroup's first tile (tseed) and left its raw accumulators:
        // run its epilogue now, while the DMAs of the next tile are already in flight
        const floatx4* src = (const floatx4*)(a.seed_acc + ((size_t)blk * MF_THREADS + tid) * 128);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = src[mi * 8 + ni];
        tile_epilogue(tseed);  // (its side data landed before the prologue stages were issued)
    }
    for (int s = 0; s < S; ++s) {
        const int left = S - 1 - s;
        mf_wait_barrier<NLW>(left < MF_DEPTH - 1 ? left : MF_DEPTH - 1, wid < NLW);
        const bool do_issue = s + MF_DEPTH < S;  // stage issued at step s: s + DEPTH
        if (do_issue) {
            mf_stage<RS, NLW>(kblock(iti, iks), qt + (int64_t)iks * 16384,
                     ring + (uint32_t)(((s + MF_DEPTH) % MF_SLOTS) * MF_SLOT), tid);
            if (++iks == nks) { iks = 0; ++iti; }
        }
        if constexpr (ROWX)
            if (wid == 0) rowx_rule(s + 3);
        mf_compute<DT>(smem + (s % MF_SLOTS) * MF_SLOT, acc, wm, wn, lane_off);
        if (ks == nks - 1) tile_epilogue(ti);
        // Deferred compaction check, after the NEXT K-step's barrier: by then every wave's
        // insert atomics of the finished tile are complete, and every wave reads all 256 LDS
        // counters, so the (rare) decision to compact is uniform without extra barriers.
        // (no check after the shard's last tile: the flush below compacts; capacity holds by the
        // invariant cnt <= cap - TR after every check, and one tile adds at most TR per query)
        // skipped when the finished tile inserted nothing anywhere in the workgroup (the common case
        // once the threshold is seeded): its parity flag was set before this step's barrier
        if (check_pending && ks != nks - 1 && flag[2 + ((ti - 1) & 1)] == 0) check_pending = false;
        if (check_pending && ks != nks - 1) {
            check_pending = false;
            // writer waves flush the loader waves' LDS pool into the global candidate buffers
            {
                int np = flag[1];
                np = np < MF_POOL ? np : MF_POOL;
                if (wid >= 4) {
                    for (int j = (wid - 4) * 64 + lane; j < np; j += 256) {
                        const int q = pool_q[j];
                        if (q < 0) continue;
                        const int slot = atomicAdd(&cnt[q], 1);
                        if (slot < a.cap) cand[(size_t)q * a.cap + slot] = pool_key[j];
                    }
                }
                mf_barrier_lgkm();  // every wave has read the tile's insert flag and the pool
                if (tid == 0) {
                    flag[1] = 0;
                    flag[2 + ((ti - 1) & 1)] = 0;
                }
            }
            int need = 0;
#pragma unroll
            for (int i = 0; i < 256 / 64; ++i) {
                const int q = lane + 64 * i;
                need |= (q < nqb && cnt[q] > trigger) ? 1 : 0;
            }
            if (__any(need)) {
                mf_barrier_drain();  // all candidate stores of all waves complete
                for (int q = wid; q < nqb; q += 8) {
                    const int n = cnt[q];
                    if (n > trigger) {
                        mf_wave_compact<MFMA_CAP / 64>(cand + (size_t)q * a.cap, n < a.cap ? n : a.cap, a.Kp,
                                                       &thr_key[q], &thr_f[q], a.drop ? a.drop + q : nullptr, lane);
                        if (lane == 0) cnt[q] = a.Kp;
                    }
                }
                mf_barrier_drain();  // counters / thresholds / compacted buffers published
            }
        }
        if (++ks == nks) { ks = 0; ++ti; }
    }
    if constexpr (SEED) return;  // no candidates (no DMA is in flight after the last K-step)
    // ---- flush: pool -> buffers, then the best <= Kp per query -> the query's survivor list ----
    mf_barrier_drain();
    {
        int np = flag[1];
        np = np < MF_POOL ? np : MF_POOL;
        if (wid >= 4) {
            for (int j = (wid - 4) * 64 + lane; j < np; j += 256) {
                const int q = pool_q[j];
                if (q < 0) continue;
                const int slot = atomicAdd(&cnt[q], 1);
                if (slot < a.cap) cand[(size_t)q * a.cap + slot] = pool_key[j];
            }
        }
    }
    mf_barrier_drain();
    // survivors (the workgroup's best <= Kp per query) appended to the query's compact list
    for (int q = wid; q < nqb; q += 8) {
        int n = cnt[q];
        if (n > a.cap) n = a.cap;
        if (n > a.Kp) {
            mf_wave_compact<MFMA_CAP / 64>(cand + (size_t)q * a.cap, n, a.Kp, &thr_key[q], &thr_f[q],
                                           a.drop ? a.drop + q : nullptr, lane);
            if (lane == 0) cnt[q] = a.Kp;  // (read back by this wave's flush: LDS order within a wave)
        }
    }
    mf_flush_wave<MAP>(a, cand, cnt, nqb, wid, lane);
}

// ------------------------------------------------------------------------------------------------
// K1 int8, direct form (k_screen_i8d): the main pass of the int8 screen when the K-steps per tile
// are a multiple of 4 (every d that is a multiple of 256, cfg3's 1536 included).  Same input,
// keys, candidate buffers and survivor lists as screen_mfma<DT_I8> (whose seed pass still seeds
// it); the operands move differently:
//   * each of the 8 waves owns 32 rows of the 256-row tile and all 256 query columns (2 x 16 MFMA
//     16x16 tiles, 128 accumulators);
//   * its corpus fragments go HBM -> VGPRs directly (global_load_dwordx4 nt, one 1 KiB fragment
//     per instruction), I8D_P K-steps ahead, into I8D_U rotating register sets: no LDS staging,
//     no LDS reads, no barrier wait on the corpus;
//   * only the query block (16 KiB per K-step, L2-resident, shared by every wave) goes through
//     an I8D_U-slot LDS ring by LDS-DMA, 2 instructions per wave, issued with the corpus loads;
//   * a K-step is one asm block (vs_i8_asm.h): 16 query-fragment reads kept 4 ahead of their
//     MFMA pairs, 32 MFMAs; the first K-step of a tile writes the accumulators (src2 = 0);
//   * one s_waitcnt vmcnt(2 * I8D_OPS) + s_barrier per K-step (the same count for every wave and
//     step: past the end the issue loads clamped dummy steps);
//   * tile epilogue: per lane 8 rows x 16 query columns; a column is tested by one upper bound of
//     its 8 keys (integer max, then the row scales' max / min and the error norms' max, all monotone
//     in fp32), and only a column whose bound reaches the query's threshold computes its 8 keys.
// Measured (scripts/k1_micro.hip, cfg3 shape): the loop alone runs at the HBM rate (2.53 ms,
// 6.1 TB/s) on all-zero operands; on random int8 codes the board holds ~1.6 GHz under the MFMA
// load and the loop takes ~3.5 ms (DESIGN §5 "power").
// ------------------------------------------------------------------------------------------------
constexpr int I8D_P = 3;            // K-steps of lead (measured: 3, 5 and 7 run at the same rate)
constexpr int I8D_U = I8D_P + 1;    // corpus register sets = query ring slots (nks % I8D_U == 0)
constexpr int I8D_OPS = 4;          // vector-memory ops per wave and K-step: 2 query DMAs + 2 corpus loads
constexpr int I8D_RING = I8D_U * 16384;
constexpr int I8D_REC = 64;  // per wave: staged (lane, column) records of the epilogue's per-row path
constexpr int I8D_LDS = I8D_RING + 256 * 8 + 256 * 4 + 256 * 4 + 16 + MF_POOL * 8 + MF_POOL * 4 +
                        8 * I8D_REC * 32 /* record accumulators */ + 256 * 16 /* qrec */ + MF_ROWX +
                        8 * I8D_REC * 4 /* record meta */ + MF_ROWX /* L2: ||x||^2 of two tiles */;
static_assert(I8D_LDS <= 160 * 1024, "LDS budget (direct int8 screen)");
static_assert(I8D_U == 4, "the K loop body and the vmcnt count are written for 4 slots");


// corpus fragment load: 16 B per lane into VGPRs, counted by the kernel's own s_waitcnt (inline
// asm: the compiler neither waits for it nor may read the registers before the wait below)
__device__ __forceinline__ void gld16_nt(intx4& v, const void* p) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
}
// 4 B per lane LDS-DMA (a tile's per-row side data: 64 rows per instruction)
__device__ __forceinline__ void glds4(const void* gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
// wait until at most 2 K-steps of this wave's loads are younger than the step's own, then barrier;
// the step's fragments are tied through the wait so nothing reads them before it
__device__ __forceinline__ void i8d_wait_barrier(intx4& a0, intx4& a1) {
    asm volatile("s_waitcnt vmcnt(%2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" : "+v"(a0), "+v"(a1) : "n"(2 * I8D_OPS)
                 : "memory");
}

// one K-step of the direct screen (the asm bodies of vs_i8_asm.h, chosen at compile time)
template <int DT, bool FIRST, int NG = 16>
__device__ __forceinline__ void d_step(intx4 (&acc)[2][16], intx4 (&bt)[4], uint32_t slot_lds, intx4& A0, intx4& A1) {
    if constexpr (NG == 4 && DT == DT_BF16) {  // narrow query tiles (4 column groups)
        if constexpr (FIRST) BFD_STEP0_N4(A0, A1);
        else BFD_STEP_N4(A0, A1);
    } else if constexpr (NG == 4) {
        static_assert(DT == DT_F16, "narrow tiles: bf16 / f16");
        if constexpr (FIRST) HFD_STEP0_N4(A0, A1);
        else HFD_STEP_N4(A0, A1);
    } else if constexpr (DT == DT_I8) {
        if constexpr (FIRST) I8D_STEP0(A0, A1);
        else I8D_STEP(A0, A1);
    } else if constexpr (DT == DT_BF16) {
        if constexpr (FIRST) BFD_STEP0(A0, A1);
        else BFD_STEP(A0, A1);
    } else {
        if constexpr (FIRST) HFD_STEP0(A0, A1);
        else HFD_STEP(A0, A1);
    }
}
// 16 B per lane into VGPRs with the default cache policy (bf16 / f16: a K-step reads one half of
// each row's 128 B line, the next K-step the other half, from L2)
__device__ __forceinline__ void gld16(intx4& v, const void* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}

constexpr int I8D_RES_LDS = 2 * MFMA_QB * 4;  // group residuals: <mu_g, q> of two tiles

// K-step kinds of the mid-step-barrier schedule (vs_i8_asm.h MS_*): F/N first K-step of a tile or
// not, O/P the step's first 4 fragment reads its own or prefetched, P/N prefetch the next step's
enum { MS_FON = 0, MS_NOP = 1, MS_NPP = 2, MS_NPN = 3 };
template <int DT, int KIND>
__device__ __forceinline__ void ms_step(intx4 (&acc)[2][16], intx4 (&bt)[4], uint32_t slot_lds, uint32_t next_lds,
                                        intx4& A0, intx4& A1, intx4& AN0, intx4& AN1, const uint8_t* qs0,
                                        const uint8_t* qs1, uint32_t ql0, uint32_t ql1, const uint8_t* cs) {
#define MS_KINDS(P_)                                                                  \
    do {                                                                              \
        if constexpr (KIND == MS_FON) P_##FON(A0, A1, AN0, AN1, qs0, qs1, ql0, ql1, cs); \
        else if constexpr (KIND == MS_NOP) P_##NOP(A0, A1, AN0, AN1, qs0, qs1, ql0, ql1, cs); \
        else if constexpr (KIND == MS_NPP) P_##NPP(A0, A1, AN0, AN1, qs0, qs1, ql0, ql1, cs); \
        else P_##NPN(A0, A1, AN0, AN1, qs0, qs1, ql0, ql1, cs);                        \
    } while (0)
    static_assert(DT == DT_I8, "the mid-step barrier: the int8 screen");
    MS_KINDS(MS_I8_);
#undef MS_KINDS
}

// The direct form for int8 codes (k_screen_i8d) and for bf16 / f16 rows (k_screen_d16): the same
// loop with the corpus dtype's MFMA.  16-bit rows: 32 elements per K-step, the K-step's 64 B of a
// row being one half of its 128 B line; native keys (fp32 score; L2: 2 score - ||x||^2); a column
// is tested by the max of its 8 keys.
// MAP: the IVF list scan over pages of a page pool (bf16 / f16), as screen_mfma's MAP form: the
// workgroup's descriptor (list segment, query tile, qmap slice), its page table in LDS (one lookup
// per tile), keys carrying storage slots, split (hi, lo) query columns summed in the epilogue.
// NG: query column groups of 16 (16 = the 256-column tile; 4 = a narrow tile of 64 columns for
// mapped scans of lists probed by <= 32 queries (<= 64 plain): a quarter of the MFMAs, and the query
// DMAs read only the tile's first 64 rows, so the L2 holds a quarter of each tile)
// PLAINQ (MAP only): the query tile holds one rounded copy of each query per column (k_pack_qtile_split
// <DT, true>): twice the queries per tile, no pair sums; the wider query-rounding margin is the
// refine's (qinfo).
// SCHED: 0 = one s_waitcnt + s_barrier at the head of every K-step, then the issue of the K-step 3
// ahead, then its MFMAs; 1 = the mid-step barrier (vs_i8_asm.h MS_*): the barrier sits between MFMA
// pairs 7 and 8 of a K-step and the issue of the K-step 3 ahead between pairs 8-11, and the next
// K-step's first fragment reads are issued at the end of the step, so the matrix pipe keeps working
// across every barrier (DESIGN §5 "K1 int8, mid-step barrier").
// PROBE (diagnostic builds of the loop, vs_k1probe.hip; 0 in the product): per workgroup
// s_memtime / s_memrealtime stamps around the loop into a.stamps, and PR_LOADS = the loads and the
// barriers only, PR_LDS = + the query-fragment reads, PR_MFMA = + the MFMAs (no epilogue), PR_FULL =
// the whole loop (the host sets every threshold to +inf: the epilogue's bound test, no survivor).
enum { PR_NONE = 0, PR_LOADS = 1, PR_LDS = 2, PR_MFMA = 3, PR_FULL = 4 };
template <int DT, int METRIC, bool MAP = false, int NG = 16, bool RES = false, int PROBE = PR_NONE, int SCHED = 0,
          bool PRIO = false, bool PLAINQ = false>
__device__ __forceinline__ void screen_direct(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    constexpr bool L2 = METRIC == METRIC_L2;
    constexpr bool I8 = DT == DT_I8;
    static_assert(!PLAINQ || MAP, "plain query tiles: mapped scans");
    constexpr bool SPLITQ = MAP && !PLAINQ;  // (hi, lo) column pairs per query
    static_assert(!(MAP && I8), "the mapped scan serves bf16 / f16 lists");
    static_assert(!RES || (I8 && !MAP && !L2), "group residuals: the int8 flat inner-product main pass");
    static_assert(NG == 16 || (NG == 4 && MAP), "narrow query tiles: mapped scans only");
    static_assert(SCHED == 0 || (I8 && !MAP && NG == 16), "the mid-step barrier: int8 flat shards");
    static_assert(SCHED == 0 || PROBE == PR_NONE || PROBE == PR_FULL, "the mid-step barrier: whole-loop probes");
    constexpr bool EPI = PROBE == PR_NONE || PROBE == PR_FULL;  // the tile epilogue runs
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* const sm = smem + I8D_RING;
    u64* thr_key = (u64*)sm;
    float* thr_f = (float*)(sm + 256 * 8);
    int* cnt = (int*)(sm + 256 * 12);
    int* flag = (int*)(sm + 256 * 16);  // [1] pool count, [2 + tile parity] inserted
    u64* pool_key = (u64*)(sm + 256 * 16 + 16);
    int* pool_q = (int*)(sm + 256 * 16 + 16 + MF_POOL * 8);
    // the wave's epilogue records: 8 accumulators (int) of one (lane, query column), and its meta
    intx4* rec = (intx4*)(sm + 256 * 16 + 16 + MF_POOL * 12) + (threadIdx.x >> 6) * I8D_REC * 2;
    float4* qrec = (float4*)(sm + 256 * 16 + 16 + MF_POOL * 12 + 8 * I8D_REC * 32);  // (t_q, ||q|| / t_q, thr, -)
    uint32_t* rowx = (uint32_t*)(sm + 256 * 16 + 16 + MF_POOL * 12 + 8 * I8D_REC * 32 + 256 * 16);
    int* rmeta = (int*)(sm + 256 * 16 + 16 + MF_POOL * 12 + 8 * I8D_REC * 32 + 256 * 16 + MF_ROWX) +
                 (threadIdx.x >> 6) * I8D_REC;
    // L2: the tiles' ||x||^2 (fp32, two tiles), the transformed key being 2 <x, q> - ||x||^2
    float* rowq = (float*)(sm + 256 * 16 + 16 + MF_POOL * 12 + 8 * I8D_REC * 32 + 256 * 16 + MF_ROWX + 8 * I8D_REC * 4);
    asm volatile("; lds ring escapes: %0" ::"v"(smem) : "memory");

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int blk = blockIdx.x;
    // The loop runs over j in [t0, t1).  Flat shards: workgroup blk takes tiles blk, blk + G, ...
    // (interleaved, so a corpus inserted cluster by cluster spreads every cluster over all the
    // workgroups instead of packing a query's whole top-k and its window into one workgroup's
    // 512-key lists); MAP: j is the list's logical tile, its page from the page table.
    int t0 = 0;
    int t1 = a.tiles > blk ? (a.tiles - blk + a.G - 1) / a.G : 0;
    int* tmap = (int*)(smem + I8D_LDS);  // MAP: page of logical tile t0 + i (published below)
    if constexpr (MAP) {
        const int* dsc = a.wg_desc + (size_t)blk * MAP_DESC;
        const int tm_off = dsc[0], nt = dsc[1];
        t0 = dsc[2];
        t1 = t0 + nt;
        a.n_valid = dsc[3];
        qt += (size_t)dsc[4] * MFMA_QB * a.dpad * 2;
        a.qmap += dsc[5];
        nqb = dsc[6];
        for (int i = tid; i < nt; i += MF_THREADS) tmap[i] = a.tile_map[tm_off + i];
    }
    const int tbase = t0;
    auto phys = [&](int t) -> int64_t {  // storage tile of loop index t
        if constexpr (MAP) return (int64_t)tmap[t - tbase];
        else return (int64_t)blk + (int64_t)t * a.G;
    };
    auto ltile = [&](int t) -> int64_t {  // logical tile of loop index t (its rows: the n_valid mask)
        if constexpr (MAP) return (int64_t)t;
        else return (int64_t)blk + (int64_t)t * a.G;
    };
    // RES: <mu_g, q> of the tile's group (two tiles, by parity), LDS-DMA'd by waves 4-7 one tile ahead
    // and copied into qrec[q].w at the tile's K-step 0
    float* const tlds = (float*)(smem + I8D_LDS);
    if (tid < 256) {
        const bool real = tid < nqb;
        const u64 k0 = real ? (a.thr0 ? a.thr0[tid] : 0ull) : ~0ull;
        thr_key[tid] = k0;
        const float tf = !real ? INFINITY : (k0 == 0ull ? -INFINITY : key_score(k0));
        thr_f[tid] = tf;
        cnt[tid] = 0;
        const float2 f = (I8 && real) ? a.qfac[tid] : make_float2(0.0f, 0.0f);
        qrec[tid] = make_float4(f.x, f.y, tf, 0.0f);
    }
    if (tid == 0) {
        flag[0] = 0;
        flag[1] = 0;
        flag[2] = 0;
        flag[3] = 0;
    }
    __syncthreads();
    uint64_t st_c0 = 0, st_r0 = 0;
    if constexpr (PROBE != PR_NONE) {
        st_c0 = __builtin_amdgcn_s_memtime();
        st_r0 = __builtin_amdgcn_s_memrealtime();
    }
    if constexpr (PRIO) {  // the second-dispatched half of the workgroup first at the matrix pipe
        if (__builtin_amdgcn_readfirstlane(tid >> 6) >= 4) __builtin_amdgcn_s_setprio(1);
    }
    const int nks = a.dpad / (I8 ? 64 : CH);
    const int64_t tbytes = (int64_t)TR * a.dpad * (I8 ? 1 : 2);
    u64* cand = a.cand + (size_t)blk * (SPLITQ ? MFMA_QB / 2 : MFMA_QB) * a.cap;
    const int trigger = a.cap - TR;
    const uint32_t ring = lds_addr(smem);
    const uint32_t rowx_lds = lds_addr((const uint8_t*)rowx);
    // this wave's side-data DMA (wave-uniform, scalar): source rows and LDS destination
    const int wid_s = __builtin_amdgcn_readfirstlane(wid);
    // (int8: waves 0-3 the (scale | beta) words, waves 4-7 ||x||^2 (L2) or the same words again;
    // 16-bit rows: ||x||^2 into rowx (L2 only))
    const bool sq_wave = L2 && (!I8 || wid_s >= 4);
    // (RES: waves 4-7 load the tile group's 1 KiB of <mu_g, q> instead of repeating the words)
    const bool t_wave = RES && wid_s >= 4;
    const uint32_t* const side_src = (t_wave ? (const uint32_t*)a.gT : sq_wave ? (const uint32_t*)a.sqn : a.rsb) + (wid_s & 3) * 64;
    const uint32_t side_dst = (t_wave ? lds_addr((const uint8_t*)tlds) : sq_wave && I8 ? lds_addr((const uint8_t*)rowq) : rowx_lds) +
                              (uint32_t)((wid_s & 3) * 256);
    const int r16 = lane & 15;
    const uint32_t lane_off = (uint32_t)(r16 * 64 + (((lane >> 4) ^ mf_swz(r16)) << 4));
    // lane's 16 B of the wave's first fragment (its second: 16 rows further)
    const int a_off = I8 ? wid * 2048 + r16 * 64 + (lane >> 4) * 16 : (wid * 32 + r16) * CHB + (lane >> 4) * 16;
    constexpr int A2 = I8 ? 1024 : 16 * CHB;

    intx4 A[I8D_U][2];  // corpus fragments of the K-steps in flight (set = K-step & 3)
    intx4 acc[2][16];   // acc[m][n][r]: row wid*32 + 16m + 4(lane >> 4) + r, query 16n + (lane & 15)
    intx4 bt[4];        // query fragments in flight (inside the asm block)

    // issue K-step (iti, iks) into register set SET = iks & 3 and ring slot SET: the tile's side
    // data first when it is the tile's last K-step, then the query block, then the corpus
    // fragments (dummy steps past the range reload the last tile: same op count every step)
    int iti = t0, iks = 0;
    int64_t pg = t1 > t0 ? phys(t0) : 0;  // storage tile of iti (MAP: looked up once per tile)
#define I8D_ISSUE(SET)                                                                                   \
    do {                                                                                                 \
        /* 4 waves cover the tile's 1 KiB of (scale | beta); waves 4-7 load its ||x||^2 (L2) or      \
           rewrite the same bytes (inner product): the same op count for every wave */                 \
        if ((I8 || L2) && iks == nks - 1 && iti < t1) {                                                  \
            if (!t_wave)                                                                                 \
                glds4(side_src + pg * TR + lane,                                                         \
                      __builtin_amdgcn_readfirstlane(side_dst + (uint32_t)((iti & 1) * 1024)));          \
            else /* RES: the NEXT tile's <mu_g, q> (read at its K-step 0; past the end: this one's) */    \
                glds4(side_src + ((iti + 1 < t1 ? phys(iti + 1) : pg) * TR / I8_GROUP_ROWS) * MFMA_QB + lane, \
                      __builtin_amdgcn_readfirstlane(side_dst + (uint32_t)(((iti + 1) & 1) * 1024)));    \
        }                                                                                                \
        const uint32_t qbase = __builtin_amdgcn_readfirstlane(ring + (uint32_t)((SET) * 16384 + wid * 1024)); \
        _Pragma("unroll") for (int it = 0; it < 2; ++it) {                                               \
            const int g = it * 512 + wid * 64 + lane;                                                    \
            const int row = g >> 2, pos = g & 3;                                                         \
            const int qrow = row & (NG * 16 - 1); /* (narrow tiles: rows >= 64 replaced by copies) */    \
            glds16(qt + (int64_t)iks * 16384 + (qrow << 6) + ((pos ^ mf_swz(qrow)) << 4), qbase + it * 8192); \
        }                                                                                                \
        const uint8_t* ab = a.corpus + pg * tbytes +                                                     \
                            (I8 ? (int64_t)iks * 16384 : (int64_t)(iks >> 1) * (TR * CHB) + (iks & 1) * 64) + a_off; \
        if (I8 || (iks & 1)) {  /* the line's last read: non-temporal */                                 \
            gld16_nt(A[SET][0], ab);                                                                     \
            gld16_nt(A[SET][1], ab + A2);                                                                \
        } else {                                                                                         \
            gld16(A[SET][0], ab);                                                                        \
            gld16(A[SET][1], ab + A2);                                                                   \
        }                                                                                                \
        if (++iks == nks) {                                                                              \
            iks = 0;                                                                                     \
            ++iti;                                                                                       \
            if (iti < t1) pg = phys(iti); /* (past the range: the last tile again, dummy steps) */       \
        }                                                                                                \
    } while (0)

    if (t1 > t0) {
        if constexpr (RES)  // the first tile's <mu_g, q> (later tiles': one tile ahead, in I8D_ISSUE)
            if (t_wave)
                glds4(side_src + (pg * TR / I8_GROUP_ROWS) * MFMA_QB + lane,
                      __builtin_amdgcn_readfirstlane(side_dst + (uint32_t)((t0 & 1) * 1024)));
        I8D_ISSUE(0);
        I8D_ISSUE(1);
        I8D_ISSUE(2);
    }
    bool check_pending = false;
    // one K-step: wait for its fragments + query block, barrier, issue the step 3 ahead, then the
    // MFMA block STEP_ (a static choice per call site: a runtime choice between asm variants makes
    // the register allocator shuffle the 128 accumulators)
#define I8D_BODY(U_, STEP_)                                                          \
    do {                                                                             \
        i8d_wait_barrier(A[U_][0], A[U_][1]);                                        \
        I8D_ISSUE(((U_) + I8D_P) & 3);                                               \
        const uint32_t slot_lds = ring + (uint32_t)((U_) * 16384) + lane_off;        \
        I8D_KSTEP(STEP_, A[U_][0], A[U_][1]);                                        \
    } while (0)
    // the K-step's reads and MFMAs (PROBE: the loads alone, or the fragment reads alone)
#define I8D_KSTEP(FIRST_, A0_, A1_)                                                  \
    do {                                                                             \
        if constexpr (PROBE == PR_LDS) {                                             \
            I8D_LDSONLY();                                                           \
        } else if constexpr (PROBE != PR_LOADS) {                                    \
            d_step<DT, FIRST_, NG>(acc, bt, slot_lds, A0_, A1_);                     \
        }                                                                            \
    } while (0)
    // the deferred compaction check of the previous tile (every wave's inserts of that tile complete)
    auto compaction_check = [&](int ti) {
        if (flag[2 + ((ti - 1) & 1)] != 0) {  // skipped when the tile inserted nothing
            // (thread-derived LDS addresses from an asm-opaque id: not hoisted out of the K loop,
            // where they would hold VGPRs across it)
            int otid;
            asm volatile("v_mov_b32 %0, %1" : "=v"(otid) : "v"(tid));
            int np = flag[1];
            np = np < MF_POOL ? np : MF_POOL;
            for (int j = otid; j < np; j += MF_THREADS) {  // the LDS pool -> candidate buffers
                const int q = pool_q[j];
                const int slot = atomicAdd(&cnt[q], 1);
                if (slot < a.cap) cand[(size_t)q * a.cap + slot] = pool_key[j];
            }
            // every wave has read the pool and the flag and done its counter atomics; the stores
            // stay in flight (vmcnt counts them in issue order behind the corpus loads, so the
            // counted corpus waits stay exact -- MI355X_MICROARCH.md, s_waitcnt)
            mf_barrier_lgkm();
            if (tid == 0) {
                flag[1] = 0;
                flag[2 + ((ti - 1) & 1)] = 0;
            }
            int need = 0;
#pragma unroll
            for (int i = 0; i < 256 / 64; ++i) {
                const int q = (otid & 63) + 64 * i;
                need |= (q < nqb && cnt[q] > trigger) ? 1 : 0;
            }
            if (__any(need)) {       // (uniform: every wave read the same counters)
                mf_barrier_drain();  // all candidate stores complete before a wave compacts a buffer
                for (int q = wid; q < nqb; q += 8) {
                    const int n = cnt[q];
                    if (n > trigger) {
                        mf_wave_compact<MFMA_CAP / 64>(cand + (size_t)q * a.cap, n < a.cap ? n : a.cap, a.Kp,
                                                       &thr_key[q], &thr_f[q], a.drop ? a.drop + q : nullptr,
                                                       lane);
                        if (lane == 0) {  // (lane 0 wrote the new threshold)
                            cnt[q] = a.Kp;
                            qrec[q].z = thr_f[q];
                        }
                    }
                }
                mf_barrier_drain();  // counters / thresholds / compacted buffers published
            }
        }
    };
    // SCHED 1: the operands of the issue of the K-step 3 ahead, made before the step's asm block (its
    // side-data DMA, once per tile, issued here); the counters advance as in I8D_ISSUE
    struct MsIssue {
        const uint8_t* qs0;
        const uint8_t* qs1;
        const uint8_t* cs;
        uint32_t ql0, ql1;
    };
    auto ms_prep = [&](int set) -> MsIssue {
        MsIssue r;
        if ((I8 || L2) && iks == nks - 1 && iti < t1) {  // (as I8D_ISSUE)
            if (!t_wave)
                glds4(side_src + pg * TR + lane, __builtin_amdgcn_readfirstlane(side_dst + (uint32_t)((iti & 1) * 1024)));
            else
                glds4(side_src + ((iti + 1 < t1 ? phys(iti + 1) : pg) * TR / I8_GROUP_ROWS) * MFMA_QB + lane,
                      __builtin_amdgcn_readfirstlane(side_dst + (uint32_t)(((iti + 1) & 1) * 1024)));
        }
        const uint32_t qbase = __builtin_amdgcn_readfirstlane(ring + (uint32_t)(set * 16384 + wid * 1024));
        r.ql0 = qbase;
        r.ql1 = __builtin_amdgcn_readfirstlane(qbase + 8192u);
        {
            const int g = wid * 64 + lane;
            const int row = g >> 2, pos = g & 3;
            r.qs0 = qt + (int64_t)iks * 16384 + (row << 6) + ((pos ^ mf_swz(row)) << 4);
            const int g1 = 512 + g;
            const int row1 = g1 >> 2, pos1 = g1 & 3;
            r.qs1 = qt + (int64_t)iks * 16384 + (row1 << 6) + ((pos1 ^ mf_swz(row1)) << 4);
        }
        r.cs = a.corpus + pg * tbytes +
               (I8 ? (int64_t)iks * 16384 : (int64_t)(iks >> 1) * (TR * CHB) + (iks & 1) * 64) + a_off;
        if (++iks == nks) {
            iks = 0;
            ++iti;
            if (iti < t1) pg = phys(iti);
        }
        return r;
    };
    // SCHED 1 K-step U_ (register set and ring slot U_, static) of kind KIND_ (vs_i8_asm.h MS_*)
#define I8D_MS(U_, KIND_)                                                                              \
    do {                                                                                               \
        asm volatile("s_waitcnt vmcnt(8)" : "+v"(A[U_][0]), "+v"(A[U_][1]) : : "memory");            \
        const MsIssue is_ = ms_prep(((U_) + I8D_P) & 3);                                               \
        ms_step<DT, KIND_>(acc, bt, ring + (uint32_t)((U_) * 16384) + lane_off,                \
                                                     ring + (uint32_t)((((U_) + 1) & 3) * 16384) + lane_off, \
                                                     A[U_][0], A[U_][1], A[((U_) + I8D_P) & 3][0],          \
                                                     A[((U_) + I8D_P) & 3][1], is_.qs0, is_.qs1, is_.ql0,   \
                                                     is_.ql1, is_.cs);                                     \
    } while (0)
    if constexpr (SCHED == 1) {
        // the issue above left K-steps 0..2 in flight; step 0's query block must have landed in every
        // wave before its first fragment read
        if (t1 > t0) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    }
    for (int ti = t0; ti < t1; ++ti) {
        if constexpr (SCHED == 1) {
            I8D_MS(0, MS_FON);
            if (check_pending) {
                check_pending = false;
                compaction_check(ti);
            }
            if constexpr (RES) {  // this tile's <mu_g, q> into qrec .w (every wave is past step 0's
                int otid;         // barrier: done with the previous tile's epilogue)
                asm volatile("v_mov_b32 %0, %1" : "=v"(otid) : "v"(tid));
                if (otid < MFMA_QB) qrec[otid].w = tlds[(ti & 1) * MFMA_QB + otid];
            }
            I8D_MS(1, MS_NOP);
            I8D_MS(2, MS_NPP);
            I8D_MS(3, MS_NPP);
            for (int ks0 = I8D_U; ks0 < nks - I8D_U; ks0 += I8D_U) {
                I8D_MS(0, MS_NPP);
                I8D_MS(1, MS_NPP);
                I8D_MS(2, MS_NPP);
                I8D_MS(3, MS_NPP);
            }
            I8D_MS(0, MS_NPP);
            I8D_MS(1, MS_NPP);
            I8D_MS(2, MS_NPP);
            I8D_MS(3, MS_NPN);
        } else {
        // K-steps 0..3: the first writes the accumulators; the deferred compaction check of the
        // previous tile runs after step 0's barrier (every wave's inserts of that tile complete)
        i8d_wait_barrier(A[0][0], A[0][1]);
        I8D_ISSUE(I8D_P);
        if (check_pending) {
            check_pending = false;
            compaction_check(ti);
        }
        if constexpr (RES) {  // this tile's <mu_g, q> into qrec .w (read by the epilogue, K-steps later)
            int otid;
            asm volatile("v_mov_b32 %0, %1" : "=v"(otid) : "v"(tid));
            if (otid < MFMA_QB) qrec[otid].w = tlds[(ti & 1) * MFMA_QB + otid];
        }
        {
            const uint32_t slot_lds = ring + lane_off;
            I8D_KSTEP(true, A[0][0], A[0][1]);
        }
        I8D_BODY(1, false);
        I8D_BODY(2, false);
        I8D_BODY(3, false);
        for (int ks0 = I8D_U; ks0 < nks; ks0 += I8D_U) {
            I8D_BODY(0, false);
            I8D_BODY(1, false);
            I8D_BODY(2, false);
            I8D_BODY(3, false);
        }
        }
        if constexpr (!EPI) continue;
        // the epilogue reads the last MFMAs' results (the hazard recognizer does not see the asm)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        // ---- tile epilogue ----
        // Per lane: 8 rows x 16 query columns.  A column is tested by ONE upper bound of its 8 keys;
        // the (lane, column) pairs that pass are staged as records in the wave's LDS buffer and their
        // keys are computed afterwards one record per lane (a column passes for a lane or two at a
        // time: per-column key code would run for the whole wave).
        int olane;  // asm-opaque lane id: lane-derived indices are not hoisted out of the K loop
        asm volatile("v_mov_b32 %0, %1" : "=v"(olane) : "v"(lane));
        const int64_t rowbase = ltile(ti) * TR;  // logical (the n_valid mask)
        const int64_t idbase = MAP ? phys(ti) * TR : rowbase;  // key ids (MAP: storage slots)
        const int qlane = olane & 15;  // + 16 n
        const uint32_t* rx = rowx + (ti & 1) * TR;
        // the shard's last tile: rows >= n_valid (garbage side data) never qualify -> no bound test,
        // every pair is staged, and the per-row path makes those rows NaN
        const bool edge = rowbase + TR > a.n_valid;
        // (L2) the tile's ||x||^2: int8 -> rowq, 16-bit rows -> rowx
        const float* rq = I8 ? rowq + (ti & 1) * TR : (const float*)rx;
        float smax = 0.0f, smin = 0.0f, bmax = 0.0f, sqmin = 0.0f;
        {
            const int rw0 = wid * 32 + (olane >> 4) * 4;
            if constexpr (I8) {
            const uint4 w0 = *(const uint4*)(rx + rw0), w1 = *(const uint4*)(rx + rw0 + 16);
            const uint32_t w8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            smax = smin = __uint_as_float(w8[0] << 16);
            bmax = __uint_as_float(w8[0] & 0xFFFF0000u);
#pragma unroll
            for (int j = 1; j < 8; ++j) {
                smax = fmaxf(smax, __uint_as_float(w8[j] << 16));
                smin = fminf(smin, __uint_as_float(w8[j] << 16));
                bmax = fmaxf(bmax, __uint_as_float(w8[j] & 0xFFFF0000u));
            }
            }
            if constexpr (L2) {
                const float4 n0 = *(const float4*)(rq + rw0), n1 = *(const float4*)(rq + rw0 + 16);
                sqmin = fminf(fminf(fminf(n0.x, n0.y), fminf(n0.z, n0.w)), fminf(fminf(n1.x, n1.y), fminf(n1.z, n1.w)));
            }
        }
        // keys of the staged records, one per lane; the record slot is reused as value staging
        auto drain = [&](int nrec) {
            __builtin_amdgcn_wave_barrier();
            if (lane < nrec) {
                const int meta = rmeta[lane];
                const int n = meta & 15, sl = meta >> 4;
                const int q = 16 * n + (sl & 15);
                const int r0 = wid * 32 + (sl >> 4) * 4;  // + 16 m + r
                const intx4 c0 = rec[2 * lane], c1 = rec[2 * lane + 1];
                const uint4 w0 = I8 ? *(const uint4*)(rx + r0) : make_uint4(0, 0, 0, 0);
                const uint4 w1 = I8 ? *(const uint4*)(rx + r0 + 16) : make_uint4(0, 0, 0, 0);
                const int cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                const uint32_t w8[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
                const float4 f = qrec[q];  // key = t_q * (s_x acc + beta_x ||q|| / t_q)
                float v[8];
                uint32_t mh = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int row = r0 + (j >> 2) * 16 + (j & 3);
                    float x = I8 ? __builtin_fmaf(__uint_as_float(w8[j] & 0xFFFF0000u), f.y,
                                                  (float)cc[j] * __uint_as_float(w8[j] << 16)) * f.x
                                 : __int_as_float(cc[j]);
                    if constexpr (L2) x = __builtin_fmaf(2.0f, x, -rq[row]);  // 2 <x, q> - ||x||^2
                    if constexpr (RES) x += f.w;  // + <mu_g, q>
                    v[j] = rowbase + row >= a.n_valid ? __builtin_nanf("") : x;
                    mh |= (v[j] >= f.z ? 1u : 0u) << j;  // (ties resolved by key below)
                }
                if (mh) {
                    flag[2 + (ti & 1)] = 1;
                    const u64 tk = thr_key[q];
                    float* sv = (float*)(rec + 2 * lane);
                    *(float4*)(sv) = make_float4(v[0], v[1], v[2], v[3]);
                    *(float4*)(sv + 4) = make_float4(v[4], v[5], v[6], v[7]);
                    while (mh) {  // compact insert loop: the LDS pool, a direct store when it is full
                        const int j = __builtin_ctz(mh);
                        mh &= mh - 1u;
                        const u64 key = mk_key(sv[j], (uint32_t)(idbase + r0 + (j >> 2) * 16 + (j & 3)));
                        if (key <= tk) continue;  // score == threshold and not ahead of it by id
                        const int ps = atomicAdd(&flag[1], 1);
                        if (ps < MF_POOL) {
                            pool_key[ps] = key;
                            pool_q[ps] = q;
                            continue;
                        }
                        const int slot = atomicAdd(&cnt[q], 1);
                        if (slot < a.cap) cand[(size_t)q * a.cap + slot] = key;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        };
        // split MAP: query p = columns 2p (hi) + 2p + 1 (lo): their fp32 sums, in place of the hi
        // column (p = 0..7: the 128 queries of the split tile; columns 8..15 then hold nothing used)
        constexpr int NCOL = SPLITQ ? NG / 2 : NG;
        if constexpr (SPLITQ) {
#pragma unroll
            for (int p = 0; p < NG / 2; ++p)
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[m][p][r] = __float_as_int(__int_as_float(acc[m][2 * p][r]) + __int_as_float(acc[m][2 * p + 1][r]));
        }
        // the bound test of all columns first (straight-line VALU, one bit per column)
        uint32_t gomask = 0;
#pragma unroll
        for (int n = 0; n < NCOL; ++n) {
            // bound of the column's 8 keys: max acc (exact int) -> fp32, times the rows' largest
            // (acc >= 0) or smallest (acc < 0) scale, plus the largest error norm; each step is
            // monotone, so a key that would pass implies a bound that passes
            const float4 f = qrec[16 * n + qlane];
            float b;
            if constexpr (I8) {
                const int mi = max(max(max(acc[0][n][0], acc[0][n][1]), max(acc[0][n][2], acc[0][n][3])),
                                   max(max(acc[1][n][0], acc[1][n][1]), max(acc[1][n][2], acc[1][n][3])));
                const float fm = (float)mi;
                b = __builtin_fmaf(bmax, f.y, fmaxf(smax * fm, smin * fm)) * f.x;
            } else {  // fp32 scores: the column's max
                b = fmaxf(fmaxf(fmaxf(__int_as_float(acc[0][n][0]), __int_as_float(acc[0][n][1])),
                                fmaxf(__int_as_float(acc[0][n][2]), __int_as_float(acc[0][n][3]))),
                          fmaxf(fmaxf(__int_as_float(acc[1][n][0]), __int_as_float(acc[1][n][1])),
                                fmaxf(__int_as_float(acc[1][n][2]), __int_as_float(acc[1][n][3]))));
            }
            if constexpr (L2) b = __builtin_fmaf(2.0f, b, -sqmin);  // (monotone: >= every row's key)
            if constexpr (RES) b += f.w;  // + <mu_g, q> (the tile's group: every row's)
            gomask |= (b >= f.z ? 1u : 0u) << n;
        }
        if (edge) gomask = (1u << NCOL) - 1u;
        int nrec = 0;  // wave-uniform
#pragma unroll
        for (int n = 0; n < NCOL; ++n) {
            const bool go = (gomask >> n) & 1u;
            const u64 bal = __ballot(go);
            if (bal == 0ull) continue;
            const int c = __popcll(bal);
            if (nrec + c > I8D_REC) {
                drain(nrec);
                nrec = 0;
            }
            if (go) {
                const int slot = nrec + lane_prefix(bal);
                rec[2 * slot] = acc[0][n];
                rec[2 * slot + 1] = acc[1][n];
                rmeta[slot] = n | (olane << 4);
            }
            nrec += c;
        }
        if (nrec) drain(nrec);
        check_pending = true;
    }
#undef I8D_ISSUE
#undef I8D_BODY
#undef I8D_KSTEP
#undef I8D_MS
    // ---- flush: pool -> buffers, then the best <= Kp per query -> the query's survivor list ----
    mf_barrier_drain();  // (also drains the dummy steps' loads)
    if constexpr (PROBE != PR_NONE) {  // the loop's stamps (diagnostic forms only): cycles, 100 MHz ticks
        const uint64_t st_c1 = __builtin_amdgcn_s_memtime();
        const uint64_t st_r1 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
            unsigned long long* st = a.stamps + (size_t)blk * 4;
            st[0] = st_c0;
            st[1] = st_c1;
            st[2] = st_r0;
            st[3] = st_r1;
        }
    }
    {
        int np = flag[1];
        np = np < MF_POOL ? np : MF_POOL;
        for (int j = tid; j < np; j += MF_THREADS) {
            const int q = pool_q[j];
            const int slot = atomicAdd(&cnt[q], 1);
            if (slot < a.cap) cand[(size_t)q * a.cap + slot] = pool_key[j];
        }
    }
    mf_barrier_drain();
    for (int q = wid; q < nqb; q += 8) {
        int n = cnt[q];
        if (n > a.cap) n = a.cap;
        if (n > a.Kp) {
            mf_wave_compact<MFMA_CAP / 64>(cand + (size_t)q * a.cap, n, a.Kp, &thr_key[q], &thr_f[q],
                                           a.drop ? a.drop + q : nullptr, lane);
            if (lane == 0) cnt[q] = a.Kp;  // (read back by this wave's flush: LDS order within a wave)
        }
    }
    mf_flush_wave<MAP>(a, cand, cnt, nqb, wid, lane);
}

template <int METRIC>
__global__ void __launch_bounds__(512, 2) k_screen_i8d(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT_I8, METRIC>(a, qt, nqb);
}
template <int DT, int METRIC>
__global__ void __launch_bounds__(512, 2) k_screen_d16(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT, METRIC>(a, qt, nqb);
}
// the int8 main passes under the mid-step-barrier schedule (SCHED 1; vs_set_k1_schedule)
template <int METRIC>
__global__ void __launch_bounds__(512, 2) k_screen_i8d_ms(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT_I8, METRIC, false, 16, false, PR_NONE, 1>(a, qt, nqb);
}

// One launch for every list scan: a workgroup whose query tile fits 64 columns runs the narrow
// form (32 queries x (hi, lo), or 64 plain queries: a quarter of the MFMAs, a quarter of the tile's
// L2 footprint), the others the full 256-column form (two separately allocated code paths; the
// choice is per workgroup, outside either K loop).
template <int DT, int METRIC, bool PLAINQ>
__global__ void __launch_bounds__(512, 2) k_screen_d16_mapped(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    if (a.wg_desc[(size_t)blockIdx.x * MAP_DESC + 6] <= (PLAINQ ? 64 : 32))
        screen_direct<DT, METRIC, true, 4, false, PR_NONE, 0, false, PLAINQ>(a, qt, nqb);
    else
        screen_direct<DT, METRIC, true, 16, false, PR_NONE, 0, false, PLAINQ>(a, qt, nqb);
}
constexpr int I8D_LDS_MAP = I8D_LDS + MFMA_MAP_TILES * 4;  // + the workgroup's page table
static_assert(I8D_LDS_MAP <= 160 * 1024, "LDS budget (direct mapped screen)");
// d16: K-steps of 32 elements per tile a multiple of 4 (and >= 8)

// 16 B streaming load with the non-temporal hint (corpus and list bytes are read once per pass)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const uint8_t* p) {
    const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int DT, int METRIC, bool SEED>
__global__ void __launch_bounds__(512, 2) k_screen_mfma(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_mfma<DT, METRIC, SEED>(a, qt, nqb);
}
// the device fallback round's screen (gated on the block's failure count): its own symbol, so a
// profile never averages its (almost always empty) launches with the main screen's
template <int DT, int METRIC>
__global__ void __launch_bounds__(512, 2) k_screen_mfma_redo(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    if (*a.gate == 0) return;
    screen_mfma<DT, METRIC, false>(a, qt, nqb);
}
// the IVF list scan's screen (MAP): its own symbol
template <int DT, int METRIC>
__global__ void __launch_bounds__(512, 2) k_screen_mfma_mapped(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_mfma<DT, METRIC, false, true>(a, qt, nqb);
}
}  // namespace vs
