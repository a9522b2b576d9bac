// vs_internal.h -- shared constants, HBM layout and kernel launchers of libvs (gfx950 only).
//
// HBM layout of a corpus shard ("row tiles"):
//   rows are grouped in tiles of TR = 256; a chunk is CE = CHB / es elements (32 fp32, 64 bf16 /
//   f16), one 128 B line per row; d is padded to dpad = roundup(d, CE) (>= 64);
//   inside a tile the matrix is stored chunk-major: [chunk c = i / CE][row r in tile][CE elements]
//   so element (r, i) of a tile lives at  c*(TR*CHB) + (r % TR)*CHB + (i % CE)*es.
// A row's piece of a chunk fills one 128 B line, so the exact-rescoring gather of a candidate row
// fetches only that row's bytes.  One MFMA K-step (256 rows x 32 bf16 elements) reads the
// 64 B half of every row's line (the next K-step the other half, from L2); every global load is
// a 16 B/lane piece of a 64 B run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "../../include/vs.h"

namespace vs {

constexpr int TR = 256;        // rows per tile
constexpr int CH = 32;         // elements per MFMA K-step (bf16 / f16: half a chunk)
constexpr int CHB = 128;       // bytes of a row's piece of one chunk: one 128 B line
constexpr int DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2;
constexpr int DT_I8 = 3;        // internal: the int8 screen copy (per-row scale, exact int32 MFMA)
constexpr int METRIC_IP = 0, METRIC_L2 = 1;

constexpr int MFMA_QB = 256;   // queries per MFMA screen launch
constexpr int MF_WG_THREADS = 512;  // MFMA screen workgroup (8 waves)
constexpr int MFMA_CAP = 768;  // candidate slots per (workgroup, query) in the MFMA screen
constexpr int MFMA_KP_MAX = 512;  // per-(workgroup, query) screening depth of the MFMA screen (= MFMA_CAP - TR:
                                  // a compacted buffer plus one tile fits); deeper searches keep 512 per
                                  // workgroup and certify against the workgroups' drop bounds
static_assert(MFMA_KP_MAX + TR <= MFMA_CAP, "MFMA screen: compaction invariant cnt <= cap - TR");
constexpr int GEMV_NQ_MAX = 8; // queries per GEMV screen launch
constexpr int GEMV_SPLIT = 4;   // row blocks per tile of the GEMV screen's small-corpus work items
constexpr int KP_MAX = 4096;   // largest screening depth (k <= 3276; k_refine sorts 4096 keys in LDS)
constexpr int SELECT_E = 16;   // keys per thread in block selection (256 threads -> 4096 keys)

inline int es_of(int dt) { return dt == DT_F32 ? 4 : 2; }
// padded dimension of the tiled layout: whole chunks, >= 2 MFMA K-steps per tile (the screen's
// deferred compaction check runs on the K-step after a tile's epilogue)
inline int pad_dim(int d, int dt) {
    const int ce = CHB / es_of(dt);
    return (int)std::max<int64_t>(((int64_t)d + ce - 1) / ce * ce, 2 * CH);
}
inline int64_t tile_bytes(int dpad, int dt) { return (int64_t)TR * dpad * es_of(dt); }
inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

constexpr int RFW_CAP = 8192;  // k_refine_wide: rows scored per query (fp64 score + id in LDS)
// k_refine_wide's phase A takes between KA and this many keys (the two-phase state holds as many):
// up to 1.5 KA, within KA's power of two (the phase-A sort's size stays what KA alone gives)
__host__ __device__ inline int rfw_ka_hi(int KA) {
    int p2 = 1;
    while (p2 < KA) p2 <<= 1;
    const int hi = KA + KA / 2 < p2 ? KA + KA / 2 : p2;
    return hi > KA ? hi : KA;
}

// screening depth: k plus a margin that certifies exactness for all but pathological inputs
inline int screen_depth(int k) {
    int kp = k + std::max(16, k / 4);
    kp = (int)round_up(kp, 16);
    return std::min(kp, KP_MAX);
}

// fp32 accumulation error factor of a d-term dot product (chains of <= d + 64 roundings)
inline float gamma_of(int d) {
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double n = (double)d + 64.0;
    return (float)(n * u / (1.0 - n * u));
}

// ---- errors: C++ exceptions inside the library, int codes + vs_last_error() at the ABI --------
struct VsError : std::runtime_error {
    int code;
    VsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
void set_last_error(const std::string& msg);  // thread-local message read by vs_last_error()

#define HIP_CHECK(expr)                                                                                    \
    do {                                                                                                   \
        hipError_t _e = (expr);                                                                            \
        if (_e != hipSuccess)                                                                              \
            throw ::vs::VsError(_e == hipErrorOutOfMemory ? VS_ERR_OOM : VS_ERR_DEVICE,                    \
                                std::string(#expr) + ": " + hipGetErrorString(_e));                        \
    } while (0)

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return VS_OK;
    } catch (const VsError& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return VS_ERR_INTERNAL;
    } catch (...) {
        set_last_error("unknown error");
        return VS_ERR_INTERNAL;
    }
}

// device buffer that only grows
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t want) {
        if (want <= bytes) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        HIP_CHECK(hipMalloc(&p, want));
        bytes = want;
    }
    template <typename T>
    T* as() const { return (T*)p; }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// two pinned host chunks + their "chunk consumed" events: double buffering of host <-> HBM copies
struct PinnedPair {
    float* host[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    size_t bytes = 0;
    void ensure(size_t want) {
        if (!done[0]) {
            HIP_CHECK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
        }
        if (want <= bytes) return;
        release_host();
        HIP_CHECK(hipHostMalloc((void**)&host[0], want, hipHostMallocDefault));
        HIP_CHECK(hipHostMalloc((void**)&host[1], want, hipHostMallocDefault));
        bytes = want;
    }
    void release_host() {
        for (float*& h : host) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
        }
        bytes = 0;
    }
    void release() {
        release_host();
        for (hipEvent_t& e : done) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// candidate key: (orderable score << 32) | (0xFFFFFFFF - local id); larger key = better,
// equal scores -> lower id first; key 0 = empty slot.
typedef unsigned long long u64;

struct ScreenArgs {
    const uint8_t* corpus;   // tiled shard
    int64_t n_valid;         // rows in the shard
    int tiles;               // ceil(n_valid / TR)
    int dpad, d;
    int metric;
    const float* sqn;        // per-row ||x||^2 (fp32) for L2 screening
    int Kp;                  // screening depth per (workgroup, query)
    int cap;                 // candidate buffer slots per (workgroup, query)
    u64* cand;               // [G][QB][cap]
    u64* part;               // [G][QB][Kp]
    int G;                   // workgroups
    int tile_stride;         // > 0: workgroup b screens only tile b*tile_stride (threshold seeding)
    const u64* thr0;         // [QB] initial per-query key threshold (keys > thr0 kept), or null
    float* seedmax;          // seed pass only: [QB][G*16] maxima of disjoint 16-row groups per query
    u64* glist;              // MFMA path output: per-query compact survivor list [QB][lcap] ...
    int* gcnt;               // ... with its length per query (zeroed by k_pack_qtile)
    int lcap;                // = G * Kp
    int* next_tile;          // GEMV: tile work-queue counter (zeroed before the launch); null = static ranges
    float* seed_acc;         // MFMA: [G][512 lanes][128] raw accumulators of each workgroup's seed tile (the
                             // first tile of its range): written by the seed pass, reused by the main pass
    const uint32_t* rsb;     // int8 screen, per row: bf16 scale s_x (x_hat = s_x * codes) in the low half,
                             // bf16 ||x - x_hat||_2 rounded up in the high half
    const float2* qfac;      // int8 screen: per query (t_q, ||q||), codes q_hat = t_q * int8
    const float* qinfo;      // int8 GEMV: per query [2q] = ||q|| rounded up (k_pack_qf32)
    u64* drop;               // MFMA: per query, max over workgroups of their compaction threshold
                             // (rows below it were dropped; zeroed by the query pack), or null
    const int* gate;         // device fallback round: the launch does nothing while *gate == 0 (no
                             // query of the block failed its certificate), or null = always run
    const int* tile_map;     // mapped screen (IVF list scan): page of logical tile t; keys carry
                             // storage slots page * TR + row, n_valid counts the list's rows
    const int* qmap;         // mapped screen: glist / gcnt row of a query (the workgroup's slice below)
    const int* skip;         // device fallback round: queries with skip[q] != 0 (certified by the first
                             // pass) are not screened (threshold +inf: no candidates), or null
    const int* wg_desc;      // mapped screen: per workgroup MAP_DESC ints {tile_map offset of its
                             // first tile, tiles, logical index of the first tile in its list
                             // segment, rows of that segment, query tile index, qmap offset, queries}
    int gemv_split;          // GEMV screen: 1 (or 0) = work items of whole tiles, GEMV_SPLIT = of
                             // 256 / GEMV_SPLIT rows (small corpora: more CUs)
    const float* gT;         // int8 group residuals: [group][QB] <mu_g, q> added to every key of the
                             // group's rows (the seed pass and k_screen_i8d_res), or null
    unsigned long long* stamps;  // diagnostic probe forms only (vs_k1probe.hip): per workgroup
                                 // {s_memtime, s_memrealtime} around the loop; null in the product
};
constexpr int MAP_DESC = 8;
constexpr int MFMA_MAP_TILES = 256;  // mapped screen: logical tiles per workgroup (its LDS page table)
int gemv_blocks_per_cu(int dt, int nqpad, int dpad);  // resident k_screen_gemv blocks per CU (occupancy API)

// ---- launchers (vs_kernels.hip) -------------------------------------------------------------
hipError_t launch_pack_rows(int dt, const float* src, int64_t n, int d, int dpad, uint8_t* data, int64_t lrow0,
                            float* sqn, unsigned* maxsq, hipStream_t st);
hipError_t launch_synth_rows(int dt, uint64_t seed, int64_t grow0, int64_t n, int d, int dpad, uint8_t* data,
                             int64_t lrow0, int normalize, float* sqn, unsigned* maxsq, hipStream_t st);
hipError_t launch_synth_f32(int dt, uint64_t seed, int64_t grow0, int64_t n, int d, int normalize, float* out,
                            hipStream_t st);
hipError_t launch_unpack_rows(int dt, const uint8_t* data, int64_t lrow0, int64_t n, int d, int dpad, float* out,
                              hipStream_t st);
hipError_t launch_gather_rows(int dt, const uint8_t* data, const int64_t* ids, int64_t n, int d, int dpad,
                              float* out, hipStream_t st);

// queries: MFMA tile (dtype, [nks][256][32]) or fp32 padded [NQ][dpad]; qinfo[q*2] = ||q_hat||,
// qinfo[q*2+1] = ||q_hat - q|| (upper bounds, fp32)
// fails (optional): zeroed -- the query block's certificate-failure count (RefineArgs::fails);
// gate (optional): as ScreenArgs::gate
// qidx (optional): tile row r packs query qidx[r] of q; qinfo is then indexed by qidx and max-combined
hipError_t launch_pack_qtile(int dt, const float* q, int nqb, int d, int dpad, uint8_t* qt, float* qinfo, int* gcnt,
                             u64* drop, hipStream_t st, int* fails = nullptr, const int* gate = nullptr,
                             const int* qidx = nullptr,
                             int* gcnt2 = nullptr, u64* drop2 = nullptr);
hipError_t launch_pack_qf32(const float* q, int nqb, int nqpad, int d, int dpad, float* qp, float* qinfo,
                            hipStream_t st, int* ctr = nullptr,  // ctr: zeroed (a screen's tile queue)
                            int* fails = nullptr, u64* drop = nullptr);  // drop: zeroed [nqpad]

hipError_t launch_screen_mfma(int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st);
// the direct K1 screens' schedule: 0 = barrier at the head of every K-step, 1 = mid-step barrier
void set_k1_schedule(int s);
int k1_schedule();
// diagnostic forms of the direct screen (vs_k1probe.hip): variant = VS_K1P_* (include/vs.h)
hipError_t launch_k1_probe(int variant, int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st);
// the int8 main pass runs the direct form (k_screen_i8d) for this int8 row stride (K-steps per tile
// a multiple of 4); it takes no seed-tile accumulators (ScreenArgs::seed_acc must be null)
bool i8_direct_ok(int dpad8);
// the same for bf16 / f16 rows (k_screen_d16: K-steps of 32 elements per tile a multiple of 4)
bool d16_direct_ok(int dpad);
// the same screen over pages of a page pool (IVF lists; bf16 / f16, unseeded, a.Kp <= MFMA_KP_MAX):
// a.G workgroups, each with its own descriptor (a.wg_desc): <= MFMA_MAP_TILES pages of one list
// (a.tile_map), one query tile of <= 128 split queries or <= 256 plain ones (qt + index * MFMA_QB *
// dpad * 2, made by launch_pack_qtile_split); survivors appended to glist rows a.qmap[...].
// Descriptors are validated on the host (check_map_desc) before the launch.  plain: the direct
// form only (d16_direct_ok).
hipError_t launch_screen_mfma_mapped(int dt, const ScreenArgs& a, const uint8_t* qt, bool plain, hipStream_t st);
// host check of one descriptor against the launch (tile map length, query tiles, qmap length)
bool check_map_desc(const int* desc, int64_t tmap_len, int n_qtiles, int64_t qmap_len, bool plain);
// every query tile of the launch at once: tile y packs the sinfo[2y + 1] (1..128 split, 1..256
// plain) queries qidx[sinfo[2y] ..] of q (host-checked by the caller)
hipError_t launch_pack_qtile_split(int dt, const float* q, const int* qidx, const int* sinfo, int ntiles, int d,
                                   int dpad, uint8_t* qt, float* qinfo, bool plain, hipStream_t st);
hipError_t launch_screen_gemv(int dt, const ScreenArgs& a, const float* qp, int nqb, int nqpad, hipStream_t st);

// one merge stage: in[(s*qstride + q)*Kp + j], s < nseg  ->  out[(b*nq + q)*Kp + j]
hipError_t launch_merge(const u64* in, int nseg, int qstride, int nq, int Kp, u64* out, int* nseg_out,
                        hipStream_t st);

constexpr int kRefineOneWaveKeys = 2048;  // = 64 * RF_WE: lists one wave of k_refine selects from
constexpr int kRefineRegKeys = 16384;     // = RF_THREADS * RF_E: lists k_refine selects from in registers
struct RefineArgs {
    const u64* cand;       // [nq][lcap] candidate keys: the first cand_n[q] (or, if cand_n is null,
    const int* cand_n;     //  all lcap, zero = empty) of each row; the refine keeps the best Kp
    int lcap;
    int Kp;
    const float* q;        // [nq][d] fp32 (original queries)
    int d, dpad, dt, metric;
    const uint8_t* corpus;
    const float* qinfo;    // [nq][2]
    float xmax;            // upper bound on ||x|| over the shard
    float gamma;           // fp32 accumulation error factor
    int k;
    int64_t n_valid;
    int64_t id_offset;
    float* D;              // [nq][k] (may be null)
    int64_t* I;            // [nq][k]
    double* S64;           // [nq][k] (may be null)
    int* cert;             // [nq] 1 = certified exact (may be null)
    unsigned* uncert;      // device counter (may be null)
    int optimistic;        // screened with an optimistic seed: fewer than Kp candidates = uncertified
    const float* qeps;     // int8 screen (k_refine_wide): per query, true score <= key_score + qeps
    const u64* drop;       // MFMA: per query, the workgroups' largest compaction threshold (or null)
    const u64* thr0;       // the screen's starting threshold per query (or null = none)
    const unsigned* i8max; // int8 GEMV screen: (max ||x_hat||, max beta) fp32 bits -> the certificate margin
    const uint32_t* idmap; // IVF: user id of every storage slot (keys carry slots); null = identity
    int* fails;            // first pass: count of the block's uncertified queries (the fallback's gate)
    int redo;              // device fallback round: only queries with cert[q] == 0 are refined (and
    const int* gate;       //  their outputs rewritten), nothing at all while *gate == 0
    int nsplit;            // k_refine, few queries with deep lists: > 1 workgroups per query each score
    double* gsc;           //  a slice of the kept rows into gsc / gids ([nq][KP2]); the last one to
    uint32_t* gids;        //  finish (gdone[q], zero between launches) sorts and certifies.  0/1 =
    unsigned* gdone;       //  one workgroup per query.
    // k_refine_wide in two launches around an exchange (the sharded step, vs_search_device_phase_a
    // / _phase_b): phase 1 scores the best KA keys and stops -- the top-k of them go to (D, I, S64)
    // for the exchange, the scored rows to pa_* -- and phase 2 resumes from pa_* with the floor
    // tfloor[q * tfloor_k + tfloor_k - 1] (a lower bound of the global k-th best score, metric
    // domain: IP score / L2 distance) raising T'.  0 = one launch (both phases).
    int phase;
    double* pa_sc;         // [nq][pa_cap] phase-1 scored rows (sorted, worst-padded), their ids,
    uint32_t* pa_ids;      //  count and phase-A key threshold
    int* pa_n;
    u64* pa_tA;
    int pa_cap;
    const double* tfloor;
    int tfloor_k;
    int ostride;           // I / S64 element stride (0/1 = separate arrays; 2 = interleaved (score bits, id))
};
// k_refine's kept-row capacity: a power of two >= 1.5 Kp (<= KP_MAX, >= Kp): its selection stops at
// any count of the best keys in [Kp, refine_kp2(Kp)], which ends the bisection early
inline int refine_kp2(int Kp) {
    const int want = std::max(Kp, std::min(KP_MAX, Kp + Kp / 2));
    int p = 1;
    while (p < want) p <<= 1;
    return p;
}
// workgroups per query of k_refine for a Kp-deep refine of nq queries (1 = no split)
int refine_split(int nq, int Kp, int dt, int num_cu);
hipError_t launch_refine(const RefineArgs& a, int nq, hipStream_t st);
// exact refine behind the int8 screen: adaptive two-phase depth (KA keys first), IP only
hipError_t launch_refine_wide(const RefineArgs& a, int nq, int KA, hipStream_t st);
// exact full scan of a shard for the queries no bounded screen could certify (vs_fullscan.hip):
// every row scored canonically, streamed through a running top-k (any number of ties)
struct FullScanArgs {
    const uint8_t* corpus;  // tiled shard
    int d, dpad, dt, metric;
    int64_t n_valid;
    const float* q;         // [nq][d] fp32 queries of the block
    int nq, k;
    int* cert;              // [nq]: queries with cert[q] == 0 are scanned (and set to 1)
    const int* gate;        // nothing at all while *gate == 0 (the fallback round's failure count), or null
    int64_t id_offset;
    float* D;               // [nq][k] (may be null)
    int64_t* I;             // [nq][k]
    double* S64;            // [nq][k] (may be null)
    int ostride;            // I / S64 element stride, as RefineArgs::ostride
    double* gsc;            // [nq][G][k] per-workgroup lists (full_scan_scratch_bytes)
    uint32_t* gid;
    unsigned* gdone;        // [nq] per-query completion counters, zero between launches
    unsigned* count;        // queries scanned (device counter), or null
    int G;                  // workgroups (row ranges)
    int all_queries;        // 1: scan every query of the block (cert is only written), no memset first
};
size_t full_scan_scratch_bytes(int nq, int G, int k);
void set_lds_attr(const void* fn, int bytes);  // max dynamic LDS of a kernel, set once per device
hipError_t launch_full_scan(const FullScanArgs& a, hipStream_t st);

constexpr int I8_GROUP_ROWS = 4096;  // rows per group of the int8 copy's group residuals (16 tiles)
constexpr int I8_MAX_K = 1024;  // largest k the int8 screen serves (k_refine_wide: 2 * KA <= RFW_CAP)
// int8 screen copy of stored rows [r0, r0 + n) (maxes[0..1]: running max ||x_hat||, max beta)
hipError_t launch_quant_rows(int dt, const uint8_t* data, int dpad, int64_t r0, int64_t n, int d, uint8_t* data8,
                             int dpad8, uint32_t* rsb, unsigned* maxes, hipStream_t st, const uint16_t* gmean = nullptr);
// group means of the int8 copy (groups [g0, g0 + ng) of I8_GROUP_ROWS rows, rows < n_rows; bf16
// [group][dpad8], zero where the mean is not worth coding against; maxes[0] = max ||mu|| (fp32
// bits), maxes[1] += groups with a mean) and their dots with a query batch (T [group][MFMA_QB])
hipError_t launch_group_means(int dt, const uint8_t* data, int dpad, int d, int64_t g0, int64_t ng, int64_t n_rows,
                              int dpad8, uint16_t* gmean, unsigned* maxes, hipStream_t st);
hipError_t launch_group_dots(const uint16_t* gmean, int64_t ngroups, int dpad8, const float* q, int nq, int d, float* T,
                             hipStream_t st);
// The device fallback round's native query tile, packed ahead by the first pass's query pack (so
// the gated round needs no pack launch of its own): the tile in the corpus dtype (bf16 / f16), its
// qinfo, and zeroed survivor-list lengths / drop bounds of the round's screen.
struct NativeTile {
    int dt;
    int dpad;
    uint8_t* qt;
    float* qinfo;
    int* gcnt;
    u64* drop;
};
hipError_t launch_pack_qtile_i8(const float* q, int nqb, int d, int dpad8, uint8_t* qt, float2* qfac, float* qeps,
                                const unsigned* maxes, int* gcnt, u64* drop, hipStream_t st, int* fails = nullptr,
                                const unsigned* l2max = nullptr, float gamma = 0.0f,
                                const NativeTile* nat = nullptr);

// ---- IVF-Flat (vs_ivf.hip) ---------------------------------------------------------------------
// Inverted lists are chains of pages: a page is one row tile (TR rows, the flat layout above) of
// a shared page pool; storage slot = page * TR + row.  A scan work item is (list, page range,
// up to IVF_QG queries probing that list).
constexpr int IVF_QG = 8;                       // queries per scan item
constexpr int IVF_ITEM_INTS = 4 + IVF_QG;       // list, page_begin, page_end, nq_item, query ids
struct IvfScanArgs {
    const uint8_t* data;       // page pool
    const float* sqn;          // ||x||^2 per slot (L2 screening)
    const float* qp;           // [nq][dpad] fp32 queries (k_pack_qf32)
    const int* items;          // [n_items][IVF_ITEM_INTS]
    int n_items;
    const int* list_pages;     // page table: pages of list l at list_pages[page_off[l] ...]
    const int* page_off;       // [nlist + 1]
    const int64_t* list_n;     // rows per list
    int dpad, metric, Kp, cap;
    u64* cand;                 // [gridDim][nq_item][cap] workspace
    u64* glist;                // per-query candidate lists [nq][lcap] (refine input) ...
    int* gcnt;                 // ... with their lengths (zeroed before the scan)
    int lcap;
    int* next_item;            // k_ivf_scan_dyn: work-queue counter (zeroed before the launch)
};
hipError_t launch_ivf_scan(int dt, int nq_class, const IvfScanArgs& a, int grid, hipStream_t st);
// every class in one launch, items fetched dynamically (nq_class of each item from its query count)
hipError_t launch_ivf_scan_dyn(int dt, const IvfScanArgs& a, int grid, hipStream_t st);
hipError_t launch_round_f32(int dt, float* x, int64_t n, hipStream_t st);  // in place, to the dtype's values
// pack fp32 rows into the slots slots[r] (slot_id[slot] = id0 + r); sqn / maxsq as k_pack_rows
hipError_t launch_pack_rows_map(int dt, const float* src, int64_t n, int d, int dpad, uint8_t* data,
                                const int64_t* slots, float* sqn, unsigned* maxsq, uint32_t* slot_id, int64_t id0,
                                hipStream_t st);

}  // namespace vs

#include <functional>
#include <shared_mutex>

struct vs_index;
namespace vs {
// the stored rows of a flat index as the kernels see them; read it (and launch on it) while holding
// flat_lock(ix) shared, the lock adds and resets take exclusively
struct FlatView {
    const uint8_t* data;
    int d, dpad, dtype, metric, device;
    int64_t ntotal;
};
FlatView flat_view(vs_index* ix);
std::shared_mutex& flat_lock(vs_index* ix);

// Host <-> HBM row streaming through two pinned host chunks (bulk add, persistence).
// add_rows_host appends n rows: fill(r0, m, dst) writes rows r0..r0+m-1 (fp32, row-major) into a
// pinned chunk while the copy engine and the pack kernel work on the previous one.  Takes the
// index's exclusive lock.
void add_rows_host(vs_index* ix, int64_t n, const std::function<void(int64_t, int64_t, float*)>& fill);
// read_rows_host streams rows i0..i0+n-1 as stored (dtype values widened to fp32): sink(r0, m, src)
// consumes one pinned chunk while the next is unpacked and copied.  Shared lock (concurrent with
// searches).
void read_rows_host(vs_index* ix, int64_t i0, int64_t n,
                    const std::function<void(int64_t, int64_t, const float*)>& sink);
int64_t stream_chunk_rows(int d);  // rows per pinned chunk (32 MiB of fp32)

// Exact top-k of device queries over a flat index, certificate failures re-searched (MFMA dtypes: by
// a gated fallback round on the device, then the gated exact full scan; async = no host sync).
// I_dev [nq][k], S64_dev optional.
// unres (optional): a device counter of this call's queries answered by the full scan, i.e. even
// the fallback round could not certify them (default: the index's counter behind vs_full_scan_count)
void search_exact_device(vs_index* ix, const float* q_dev, int64_t nq, int k, int64_t* I_dev, double* S64_dev,
                         hipStream_t st, float* D_dev = nullptr, int64_t id_offset = 0, bool async = false,
                         unsigned* unres = nullptr);
// drop rows [n, ntotal) of a flat index (rows are append-only: a failed multi-device add rolls back
// the shards that took their rows); the running maxima stay (they only widen certificate margins)
void truncate_rows(vs_index* ix, int64_t n);
unsigned* full_scan_counter(vs_index* ix);  // device word behind vs_full_scan_count
// S concurrent exact device searches over parts of one batch (own streams and workspaces;
// unres[i] counts part i's full-scanned queries)
void search_exact_device_parts(vs_index* ix, const float* q_dev, int64_t nq, int k, int64_t* I_dev,
                               hipStream_t* streams, int S, unsigned* unres);
// two-phase exact device search (vs_search_device_phase_a / _b)
bool two_phase_ok(const vs_index* ix, int64_t nq, int k);
vs_pending* search_phase_a(vs_index* ix, const float* q_dev, int64_t nq, int k, int world, int64_t id_offset,
                           double* S_a, int64_t* I_a, int stride, hipStream_t st);
// (unres: this call's counter of full-scanned queries, the fallback round could not certify them;
// null = the index's)
void search_phase_b(vs_pending* p, const double* floor_S, float* D, int64_t* I, double* S64, int stride,
                    hipStream_t st, unsigned* unres = nullptr);
void search_pending_free(vs_pending* p);
// seed pass: screen one tile per workgroup (tile_stride) and write per-query 16-row-group maxima
hipError_t launch_seed_mfma(int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st);
// thr0[q] = key just below the rank-th largest of the M group maxima of query q (0 if none)
hipError_t launch_seed_select(const float* seedmax, int M, int nq, int rank, u64* thr0, hipStream_t st);

hipError_t launch_merge_shards(int metric, const double* S_in, const int64_t* I_in, int G, int64_t nq, int k,
                               double* S_out, int64_t* I_out, float* D_out, hipStream_t st, int istride = 1);

// ---- HNSW graph search (vs_hnsw.hip) ---------------------------------------------
// faiss HNSW::search over a graph in faiss's layout (neighbors of node i on level l:
// neighbors[offsets[i] + cum[l] .. offsets[i] + cum[l + 1]), -1 padded), rows of a flat index,
// canonical fp64 distances.  One workgroup per query; the candidate and result heaps are sorted
// LDS arrays under (distance, id).
constexpr int HN_THREADS = 256;          // k_hnsw_prune: one workgroup per node
constexpr int HN_SEARCH_THREADS = 512;   // k_hnsw_search: one workgroup per query (8 waves score a list)
constexpr int HN_EF_MAX = 2048;  // largest max(efSearch, k)
constexpr int HN_NB_MAX = 1024;  // largest neighbour list of one level
struct HnswArgs {
    const uint8_t* corpus;       // flat index rows (tiled layout)
    int d, dpad, dt, metric;
    int64_t n;                   // rows (= graph nodes)
    const uint64_t* offsets;     // [n + 1]
    const int* neighbors;        // [offsets[n]]
    const int* cum;              // [max_level + 2] cumulative neighbour counts per level
    int entry, max_level;
    int nbmax;                   // widest level's neighbour count
    const float* q;              // [nq][d] fp32
    int k, ef_search, ef;        // ef = max(ef_search, k)
    uint32_t* vis;               // [nq][vis_words] visited bitmaps, zeroed before the launch
    int64_t vis_words;
    float* D;                    // [nq][k] scores (IP) / squared distances (L2), best first
    int64_t* I;                  // [nq][k] row ids, -1 padded
};
size_t hnsw_lds_bytes(int d, int k, int ef, int nbmax);  // dynamic LDS of one search workgroup
hipError_t launch_hnsw_search(const HnswArgs& a, int nq, hipStream_t st);

// faiss HNSW::shrink_neighbor_list per node (graph build): one workgroup per node
constexpr int HP_C_MAX = 2048;  // largest candidate list of one node
struct HnswPruneArgs {
    const uint8_t* corpus;  // flat index rows (tiled layout)
    int d, dpad, dt, metric;
    const int64_t* nodes;   // [m] row ids
    const int* cand;        // [m][C] distinct candidate row ids, -1 padded at the end
    int C, W;               // candidates per node, neighbours kept
    int* out;               // [m][W] kept ids best first, -1 padded
};
size_t hnsw_prune_lds_bytes(int d, int C, int W);
hipError_t launch_hnsw_prune(const HnswPruneArgs& a, int m, hipStream_t st);

}  // namespace vs
