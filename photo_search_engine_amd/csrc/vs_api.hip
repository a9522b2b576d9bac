// vs_api.hip -- C ABI of libvs (include/vs.h): index object, HBM residency, search orchestration.
//
// Replaces faiss.IndexFlatIP/IndexFlatL2 behind /root/reference/utils/vector_store.py
// (construct :79-81, add :164, search :191, reconstruct :207, ntotal :183/:271, clear :277).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/vs.h"
#include "vs_internal.h"

using namespace vs;

namespace {

thread_local std::string g_err;

// pinned staging per context for the host-buffer search (queries in, results out)
constexpr size_t kPinnedStageCap = 8u << 20;

// pinned host staging (grow-only): pageable hipMemcpyAsync is a staged, blocking copy
struct HostBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t want) {
        if (want <= bytes) return;
        release();
        HIP_CHECK(hipHostMalloc(&p, want, hipHostMallocDefault));
        bytes = want;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// per-call execution context: stream + workspace (pooled; one per concurrent search)
struct Ctx {
    hipStream_t stream = nullptr;
    // recorded behind the last lease's work on its caller's stream: the next lease (possibly on
    // another stream) waits on it before touching the workspace, so a device-API search that
    // returned with kernels still queued is never overwritten by the next caller's pack
    hipEvent_t idle = nullptr;
    bool pending = false;
    DevBuf qdev, qtile, qinfo, qpad, cand, part, merge_a, merge_b, outD, outI, outS, cert, thr0, seedmax, gcnt, gT;
    DevBuf qfac, qeps, drop;  // int8 screen: per-query code scale and norm, refine margin, drop bounds
    DevBuf fails;             // the current query block's certificate-failure counts: [0] first pass (the
                              // fallback round's gate), [1] fallback round (the full scan's gate)
    DevBuf fsc, fdone;        // full scan: per-workgroup lists of the block's queries, done counters
    DevBuf rsc, rdone;        // split refine: per-query scores + ids of the kept rows, done counters
    DevBuf pa;       // two-phase (sharded) search: the refine's phase-1 state between the launches
    DevBuf rows[2];  // read_rows_host: unpacked fp32 chunks
    DevBuf tilectr;  // GEMV screen: tile work-queue counter
    DevBuf seedacc;  // MFMA seed pass: raw accumulators of each workgroup's seed tile
    DevBuf outAll;   // vs_search: I (int64), D (fp32), certificates in one block: ONE D2H copy
    // the device fallback round's query tile, packed ahead by the block's first pass: 0 none (the
    // round packs it), 1 the native first pass's own tile (qtile), 2 the int8 pass's native copy
    // (qtile_n); the round's list counters are gcnt2 / drop2, zeroed by the same pack
    DevBuf qtile_n, gcnt2, drop2;
    int prepacked = 0;
    PinnedPair pin;  // read_rows_host: pinned landing chunks
    HostBuf hq;      // vs_search: the query batch, staged for the H2D copy
    HostBuf hout;    // vs_search: I (int64), D (fp32) and certificates land here; search_exact_device: certificates
    unsigned* unres = nullptr;  // this call's full-scan counter (device), instead of the index's
    ~Ctx() {
        for (DevBuf* b : {&qdev, &qtile, &qinfo, &qpad, &cand, &part, &merge_a, &merge_b, &outD, &outI, &outS, &cert, &thr0,
                          &gT, &seedmax, &gcnt, &rows[0], &rows[1], &tilectr, &seedacc, &outAll, &qfac, &qeps, &drop, &fails, &rsc, &rdone,
                          &pa, &fsc, &fdone})
            b->release();
        pin.release();
        hq.release();
        hout.release();
        if (idle) hipEventDestroy(idle);
        if (stream) hipStreamDestroy(stream);
    }
};

}  // namespace

void vs::set_last_error(const std::string& msg) { g_err = msg; }

constexpr int64_t kDefaultScanLimit = 192ll << 20;  // (the MALL holds such a corpus between calls)

struct vs_index {
    int d = 0, dpad = 0, metric = 0, dtype = 0, device = 0, es = 4;
    int num_cu = 256;
    int64_t ntotal = 0, cap_rows = 0;
    uint8_t* data = nullptr;
    float* sqn = nullptr;
    unsigned* d_maxsq = nullptr;
    unsigned* d_uncert = nullptr;
    unsigned* d_unres = nullptr;  // queries answered by the exact full scan (no bounded screen certified them)
    float maxsq = 0.0f;
    // int8 screen copy (VS_SCREEN_I8): codes in row tiles of 64-element chunks + per-row scale and
    // error norm; d_maxsq[2..3] = max ||x_hat||, max error norm (fp32 bits, certificate margins)
    int screen = VS_SCREEN_NATIVE;
    int dpad8 = 0;
    int64_t cap8 = 0;
    uint8_t* data8 = nullptr;
    uint32_t* rsb = nullptr;  // per row: bf16 scale | bf16 error norm (rounded up) << 16
    float i8_bmax = 0.0f;     // host copy of the largest row error norm (int8 GEMV depth)
    // group residuals (inner product, direct int8 screen): bf16 means of I8_GROUP_ROWS-row groups
    // [gcap][dpad8] the codes are taken against (zero for groups without a mean worth it);
    // d_maxsq[5] = max ||mu_g|| (fp32 bits), d_maxsq[6] = groups that have a mean
    uint16_t* gmean = nullptr;
    int64_t gcap = 0;
    bool i8_res = false;  // some group has a mean: the int8 screen adds <mu_g, q> to its keys
    hipStream_t own = nullptr;  // ingest stream
    DevBuf stage[2];            // add_rows_host: fp32 chunks on the device ...
    PinnedPair pin;             // ... and their pinned host sources
    std::shared_mutex rw;       // shared: search; exclusive: add/reset
    std::mutex pool_mtx;
    std::vector<Ctx*> pool_free;
    std::vector<Ctx*> pool_all;
    // timing (bench): events around the screen kernel
    std::atomic<bool> timing{false};
    std::mutex tmtx;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    // corpora of at most this many stored bytes answer calls of 1-2 queries with the exact full scan
    // alone (vs_set_scan_limit; 0 = never)
    std::atomic<int64_t> scan_limit{kDefaultScanLimit};
    int last_kernel_kind = 0;  // 1 = mfma, 2 = gemv, 3 = int8 mfma, 4 = int8 gemv, 5 = exact full scan
    // Screen health (first passes of MFMA batches): the certificate-failure count of a batch is read
    // back without a host wait (pinned word + event, observed by a later search).  A failed query
    // costs its block a full fallback round, so the index adapts to its corpus:
    //  * an int8 batch with failures doubles the int8 union (the rows listed above the seed), up
    //    to 2^kI8ScaleMax; one failing at that depth routes the next kI8RouteBatches searches to
    //    the native screen (score distributions denser than the int8 error window, e.g. tight
    //    clusters); kSeedRelax clean int8 batches halve the depth again;
    //  * a native batch with a failed query doubles the optimistic seed's depth (rows listed ahead
    //    of the refine), up to 2^kSeedScaleMax; kSeedRelax clean batches halve it again.
    std::mutex h_mu;
    unsigned* h_fails = nullptr;  // pinned
    hipEvent_t h_ev = nullptr;
    int h_pending = 0;          // 0 none, 1 int8 batch, 2 native batch in flight
    int h_nq = 0;               // queries of that batch
    int h_clean = 0;            // consecutive clean readbacks (past kHealthCleanRun: every kHealthStride-th batch read)
    unsigned h_seq = 0;         // batches noted since
    int i8_route = 0;           // searches still routed to the native screen
    int seed_log2 = 0, seed_clean = 0;
    int i8_log2 = 0, i8_clean = 0;  // int8 union depth: 2^i8_log2 times the target (dense corpora)
    int i8_route_log2 = 0;          // consecutive routings (each twice as long as the last)
};

vs::FlatView vs::flat_view(vs_index* ix) {
    return {ix->data, ix->d, ix->dpad, ix->dtype, ix->metric, ix->device, ix->ntotal};
}
std::shared_mutex& vs::flat_lock(vs_index* ix) { return ix->rw; }

namespace {

Ctx* acquire_ctx(vs_index* ix) {
    std::lock_guard<std::mutex> g(ix->pool_mtx);
    if (!ix->pool_free.empty()) {
        Ctx* c = ix->pool_free.back();
        ix->pool_free.pop_back();
        return c;
    }
    Ctx* c = new Ctx();
    ix->pool_all.push_back(c);  // owned by the pool from here on (freed by vs_destroy)
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&c->idle, hipEventDisableTiming));
    return c;
}
void release_ctx(vs_index* ix, Ctx* c) {
    std::lock_guard<std::mutex> g(ix->pool_mtx);
    ix->pool_free.push_back(c);
}
// A leased context works on `st` (null = the context's own stream): the lease first orders `st`
// behind the previous lease's work, and on release records the context's idle event on `st`.
struct CtxLease {
    vs_index* ix;
    Ctx* c;
    hipStream_t st;
    CtxLease(vs_index* i, hipStream_t s, bool own_stream) : ix(i), c(acquire_ctx(i)) {
        st = own_stream ? c->stream : s;
        if (c->pending) {
            hipError_t e = hipStreamWaitEvent(st, c->idle, 0);
            if (e != hipSuccess) {
                release_ctx(ix, c);
                HIP_CHECK(e);
            }
        }
    }
    ~CtxLease() {
        c->pending = hipEventRecord(c->idle, st) == hipSuccess;
        release_ctx(ix, c);
    }
};

void ensure_capacity_i8(vs_index* ix);

// exact: allocate exactly rows_needed (vs_reserve) instead of growing by 1.5x
void ensure_capacity(vs_index* ix, int64_t rows_needed, bool exact = false) {
    const int64_t want = round_up(rows_needed, TR);
    if (want <= ix->cap_rows) return;
    int64_t ncap = exact ? want : std::max(want, ix->cap_rows + ix->cap_rows / 2);
    ncap = round_up(ncap, TR);
    const int64_t tb = tile_bytes(ix->dpad, ix->dtype);
    uint8_t* nd = nullptr;
    float* ns = nullptr;
    HIP_CHECK(hipMalloc(&nd, (size_t)(ncap / TR) * tb));
    hipError_t e = hipMalloc(&ns, (size_t)ncap * sizeof(float));
    if (e != hipSuccess) {
        hipFree(nd);
        HIP_CHECK(e);
    }
    HIP_CHECK(hipMemsetAsync(nd, 0, (size_t)(ncap / TR) * tb, ix->own));
    HIP_CHECK(hipMemsetAsync(ns, 0, (size_t)ncap * sizeof(float), ix->own));
    if (ix->data && ix->ntotal > 0) {
        const int64_t used_tiles = (ix->ntotal + TR - 1) / TR;
        HIP_CHECK(hipMemcpyAsync(nd, ix->data, (size_t)used_tiles * tb, hipMemcpyDeviceToDevice, ix->own));
        HIP_CHECK(hipMemcpyAsync(ns, ix->sqn, (size_t)ix->ntotal * sizeof(float), hipMemcpyDeviceToDevice, ix->own));
    }
    HIP_CHECK(hipStreamSynchronize(ix->own));
    if (ix->data) hipFree(ix->data);
    if (ix->sqn) hipFree(ix->sqn);
    ix->data = nd;
    ix->sqn = ns;
    ix->cap_rows = ncap;
    ensure_capacity_i8(ix);
}

void free_i8(vs_index* ix) {
    if (ix->data8) (void)hipFree(ix->data8);
    if (ix->rsb) (void)hipFree(ix->rsb);
    if (ix->gmean) (void)hipFree(ix->gmean);
    ix->data8 = nullptr;
    ix->rsb = nullptr;
    ix->gmean = nullptr;
    ix->cap8 = 0;
    ix->gcap = 0;
    ix->i8_res = false;
}

// group residuals apply to inner-product indexes whose int8 main pass is the direct form
bool i8_groups_apply(const vs_index* ix) { return ix->metric == METRIC_IP && i8_direct_ok(ix->dpad8); }

// grow the int8 screen copy to ix->cap_rows rows (device copy of the rows present; the old and new
// arrays coexist only for the copy, as for the primary rows)
void ensure_capacity_i8(vs_index* ix) {
    if (ix->screen != VS_SCREEN_I8 || ix->cap8 >= ix->cap_rows) return;
    const int64_t ncap = ix->cap_rows;
    const size_t tb8 = (size_t)TR * ix->dpad8;
    uint8_t* nd = nullptr;
    uint32_t* nr = nullptr;
    uint16_t* ng = nullptr;
    const int64_t gcap = i8_groups_apply(ix) ? (ncap + I8_GROUP_ROWS - 1) / I8_GROUP_ROWS : 0;
    hipError_t e = hipMalloc(&nd, (size_t)(ncap / TR) * tb8);
    if (e == hipSuccess) e = hipMalloc(&nr, (size_t)ncap * sizeof(uint32_t));
    if (e == hipSuccess && gcap) e = hipMalloc(&ng, (size_t)gcap * ix->dpad8 * sizeof(uint16_t));
    if (e != hipSuccess) {
        if (nd) hipFree(nd);
        if (nr) hipFree(nr);
        HIP_CHECK(e);
    }
    if (ix->data8 && ix->ntotal > 0) {
        const int64_t used_tiles = (ix->ntotal + TR - 1) / TR;
        HIP_CHECK(hipMemcpyAsync(nd, ix->data8, (size_t)used_tiles * tb8, hipMemcpyDeviceToDevice, ix->own));
        HIP_CHECK(hipMemcpyAsync(nr, ix->rsb, (size_t)ix->ntotal * sizeof(uint32_t), hipMemcpyDeviceToDevice, ix->own));
        if (ng && ix->gmean) {
            const int64_t used_groups = (ix->ntotal + I8_GROUP_ROWS - 1) / I8_GROUP_ROWS;
            HIP_CHECK(hipMemcpyAsync(ng, ix->gmean, (size_t)used_groups * ix->dpad8 * sizeof(uint16_t),
                                     hipMemcpyDeviceToDevice, ix->own));
        }
    }
    HIP_CHECK(hipStreamSynchronize(ix->own));
    const bool res = ix->i8_res;
    free_i8(ix);
    ix->data8 = nd;
    ix->rsb = nr;
    ix->gmean = ng;
    ix->gcap = gcap;
    ix->i8_res = res;
    ix->cap8 = ncap;
}

// int8 screen copy of rows [r0, r0 + n) once they are packed (stream-ordered after the pack).  With
// group residuals, the groups the rows fall in get their means (re)computed over every row they
// hold now, and their rows are (re)quantised from the group's first row.
void quantize_rows(vs_index* ix, int64_t r0, int64_t n, hipStream_t st) {
    if (ix->screen != VS_SCREEN_I8 || n <= 0) return;
    if (ix->gmean) {
        // rows already searchable get new codes, bounds and group means: searches still queued on
        // other streams (device-API callers return before their kernels run) must finish first, or
        // one could read a row's new code with the old <mu_g, q> and its key would no longer bound
        // the score (the exclusive lock only orders host calls; vs_set_screen syncs likewise)
        if (r0 % I8_GROUP_ROWS != 0) HIP_CHECK(hipDeviceSynchronize());
        const int64_t g0 = r0 / I8_GROUP_ROWS, g1 = (r0 + n + I8_GROUP_ROWS - 1) / I8_GROUP_ROWS;
        HIP_CHECK(launch_group_means(ix->dtype, ix->data, ix->dpad, ix->d, g0, g1 - g0, r0 + n, ix->dpad8, ix->gmean,
                                     ix->d_maxsq + 5, st));
        n += r0 - g0 * I8_GROUP_ROWS;
        r0 = g0 * I8_GROUP_ROWS;
    }
    HIP_CHECK(launch_quant_rows(ix->dtype, ix->data, ix->dpad, r0, n, ix->d, ix->data8, ix->dpad8, ix->rsb,
                                ix->d_maxsq + 2, st, ix->gmean));
}

void refresh_maxsq(vs_index* ix) {
    unsigned bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIP_CHECK(hipMemcpyAsync(bits, ix->d_maxsq, sizeof(bits), hipMemcpyDeviceToHost, ix->own));
    HIP_CHECK(hipStreamSynchronize(ix->own));
    std::memcpy(&ix->maxsq, &bits[0], 4);
    std::memcpy(&ix->i8_bmax, &bits[7], 4);  // int8 copy: the largest ||x - s c|| (GEMV keys' error)
    ix->i8_res = ix->gmean != nullptr && bits[6] != 0;  // some group coded against its mean
}

// optimistic seed: a 16-row-group maximum of the strided tile sample, at the rank that leaves
// ~kOptimisticPassFactor * Kp corpus rows above it in expectation (the proven seed is rank Kp); a
// query left short is caught by the certificate and searched again with the proven seed
constexpr int kOptimisticSeedRank = 1;  // seed_rank argument: > 0 selects the optimistic rank
constexpr double kOptimisticPassFactor = 8.0;
constexpr int kOptimisticMinRank = 4;

// the seed pass screens each main-pass workgroup's first tile and the (native) main pass reuses
// its accumulators; the GEMV screen takes tiles from a work queue over its resident blocks (both
// measured faster than the alternatives they replaced)
constexpr bool seed_reuse() { return true; }
constexpr bool gemv_dyn() { return true; }

// The int8 pre-screen serves first passes of MFMA-sized batches (k <= I8_MAX_K) of an index with
// VS_SCREEN_I8; a query its certificate rejects is re-searched by the caller on the native path.
bool use_i8(const vs_index* ix, int nqb, int k) {
    if (ix->screen != VS_SCREEN_I8 || nqb <= GEMV_NQ_MAX || k > I8_MAX_K) return false;
    if (!ix->i8_res) return true;
    // group-residual codes: only the seed pass and the direct main pass add <mu_g, q> (else: native)
    const int64_t tiles = (ix->ntotal + TR - 1) / TR;
    const int64_t G = std::max<int64_t>(1, std::min<int64_t>(tiles, ix->num_cu));
    return tiles >= 4 * G;
}

constexpr int kF32MfmaMinQ = 64;     // fp32 native batches: MFMA screen from this many queries on
constexpr int kI8RouteBatches = 64;  // searches routed to the native screen after a failing int8 batch
constexpr int kSeedScaleMax = 6;     // native optimistic seed: at most 64x the default depth
constexpr int kSeedRelax = 64;       // clean native batches before the depth is halved again
constexpr int kI8ScaleMax = 4;       // int8 union: at most 16x its target before routing to native
constexpr int kI8RouteLog2Max = 6;   // routing stretches: at most 64 x kI8RouteBatches searches

// observe a completed failure-count readback (caller holds h_mu)
void health_poll(vs_index* ix) {
    if (ix->h_pending && hipEventQuery(ix->h_ev) == hipSuccess) {
        const unsigned f = *ix->h_fails;
        if (ix->h_pending == 1) {
            // an int8 batch with failures: a deeper union first (dense score distributions put
            // more rows inside the int8 error window), the native screen when even the deepest
            // union failed; clean batches relax the depth again
            // (a batch where over a quarter of the queries failed deepens two steps at once; each
            // routing that follows a failure at the deepest union lasts twice as long as the last,
            // up to 2^kI8RouteLog2Max times kI8RouteBatches, so a corpus the int8 window cannot
            // serve costs one failing batch per ever longer native stretch)
            if (f > 0) {
                if (ix->i8_log2 < kI8ScaleMax) {
                    ix->i8_log2 = std::min(kI8ScaleMax, ix->i8_log2 + (f > (unsigned)(ix->h_nq / 4) ? 2 : 1));
                } else {
                    ix->i8_route = kI8RouteBatches << ix->i8_route_log2;
                    ix->i8_route_log2 = std::min(ix->i8_route_log2 + 1, kI8RouteLog2Max);
                }
                ix->i8_clean = 0;
            } else {
                ix->i8_route_log2 = 0;
                if (ix->i8_log2 > 0 && ++ix->i8_clean >= kSeedRelax) {
                    --ix->i8_log2;
                    ix->i8_clean = 0;
                }
            }
        } else if (f > 0) {  // (one failed query costs its block a whole fallback screen: deepen)
            ix->seed_log2 = std::min(ix->seed_log2 + 1, kSeedScaleMax);
            ix->seed_clean = 0;
        } else if (ix->seed_log2 > 0 && ++ix->seed_clean >= kSeedRelax) {
            --ix->seed_log2;
            ix->seed_clean = 0;
        }
        ix->h_clean = f > 0 ? 0 : ix->h_clean + 1;
        ix->h_pending = 0;
    }
    (void)hipGetLastError();  // (hipEventQuery's "not ready" is no error)
}
// May this search use the int8 screen?  Consumes the routing state (one call per search).
bool i8_allowed(vs_index* ix) {
    if (ix->screen != VS_SCREEN_I8) return false;
    std::lock_guard<std::mutex> g(ix->h_mu);
    health_poll(ix);
    if (ix->i8_route > 0) {
        --ix->i8_route;
        return false;
    }
    return true;
}
// depth multiplier of the native optimistic seed
double seed_scale(vs_index* ix) {
    std::lock_guard<std::mutex> g(ix->h_mu);
    health_poll(ix);
    return (double)(1 << ix->seed_log2);
}
// after a first-pass batch (kind 1 int8, 2 native): read its failure count back behind it on the
// stream (one readback in flight per index)
// A long clean run reads back only every kHealthStride-th batch (a readback is a copy launch and ~10
// us of the 8-shard step); the first failing readback returns to every batch.
constexpr int kHealthCleanRun = 16;
constexpr unsigned kHealthStride = 4;
void health_note(vs_index* ix, Ctx* c, hipStream_t st, int kind, int nq) {
    std::lock_guard<std::mutex> g(ix->h_mu);
    if (ix->h_pending) return;
    if (ix->h_clean >= kHealthCleanRun && (++ix->h_seq % kHealthStride) != 0) return;
    if (!ix->h_fails) {
        HIP_CHECK(hipHostMalloc((void**)&ix->h_fails, sizeof(unsigned), hipHostMallocDefault));
        HIP_CHECK(hipEventCreateWithFlags(&ix->h_ev, hipEventDisableTiming));
    }
    HIP_CHECK(hipMemcpyAsync(ix->h_fails, c->fails.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipEventRecord(ix->h_ev, st));
    ix->h_pending = kind;
    ix->h_nq = nq;
}
// int8 GEMV screen depth.  Its keys carry the row error bound beta (~0.007-0.01 ||x|| ||q||), so the
// rows it must keep are those within ~beta of the k-th best.  For unit rows the scores are roughly
// N(0, 1/d) and the k-th best sits z = sqrt(2 ln(N / k)) deviations out, where the density grows by
// e^(z beta sqrt(d)) per beta: keep k times twice that (+64); deeper than kI8GemvMaxDepth, the
// native GEMV serves the query.  Data that defeat the estimate fail the certificate, not exactness.
constexpr int kI8GemvMaxDepth = 512;
int i8_gemv_depth(const vs_index* ix, int k) {
    const double z = std::sqrt(2.0 * std::log(std::max(2.0, (double)ix->ntotal / k)));
    const double g = std::exp(std::min(20.0, z * (double)ix->i8_bmax * std::sqrt((double)ix->d)));
    return (int)std::min<double>(KP_MAX, round_up((int64_t)std::ceil(2.0 * k * g + 64.0), 16));
}
// Union of survivors the int8 seed aims at (rows above the seeded threshold).  It must cover the
// refine's window -- every key within the int8 error budget of T', measured at ~7.5-10 k rows for
// unit-norm data -- or the certificate fails and the query is re-searched.  The seed is
// the rank-r maximum over S sampled rows, r = U S / N, so the count above it is U (1 +- ~1/sqrt r):
// take the smallest U whose 3-sigma low count still covers kI8Window * k rows, within
// [kI8UnionMin, kI8UnionMaxPerK * k].  Large shards need more margin (few sampled maxima per union
// row): cfg3's 10M rows -> ~41 k, the 8-GPU shard of 1.25M rows -> ~25 k (union sweep).
constexpr double kI8Window = 15.0;
constexpr double kI8UnionMaxPerK = 64.0;
constexpr double kI8UnionMin = 1024.0;
double i8_union_target(int k, double sampled, double n) {
    const double need = kI8Window * k;
    double u = std::max(need, kI8UnionMin);
    const double umax = std::max(kI8UnionMaxPerK * k, kI8UnionMin);
    while (u < umax) {
        const double r = u * sampled / n;
        if (r >= 9.0 && u * (1.0 - 3.0 / std::sqrt(r)) >= need) break;
        u *= 1.1;
    }
    return std::min(u, umax);
}

// int8 pre-screen of one query block: pack int8 query codes -> seed pass -> int8 MFMA screen with
// upper-bound keys -> adaptive exact refine (k_refine_wide).  q: device fp32 [nqb][d].
// phase 1 (two-phase sharded search, KA1 keys in phase A): stops after the refine's phase A and
// returns its arguments in *keep for vs_search_device_phase_b
void search_block_i8(vs_index* ix, Ctx* c, const float* q, int nqb, int k, float* D, int64_t* I, double* S64,
                     int* cert, int64_t id_offset, hipStream_t st, int phase = 0, int KA1 = 0,
                     RefineArgs* keep = nullptr, int ostride = 1, bool prepack = false, int kwin = 0) {
    const int64_t tiles = (ix->ntotal + TR - 1) / TR;
    ScreenArgs a{};
    a.corpus = ix->data8;
    a.n_valid = ix->ntotal;
    a.tiles = (int)tiles;
    a.dpad = ix->dpad8;
    a.d = ix->d;
    a.metric = ix->metric;  // L2: keys 2 (upper bound of <x, q>) - ||x||^2
    a.sqn = ix->sqn;
    a.Kp = MFMA_KP_MAX;  // per workgroup and query; the refine's depth is adaptive
    a.cap = MFMA_CAP;
    a.G = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, ix->num_cu));
    a.rsb = ix->rsb;
    c->qtile.ensure((size_t)MFMA_QB * ix->dpad8);
    c->qfac.ensure(sizeof(float2) * MFMA_QB);
    c->qeps.ensure(sizeof(float) * MFMA_QB);
    c->drop.ensure(sizeof(u64) * MFMA_QB);
    c->gcnt.ensure(sizeof(int) * MFMA_QB);
    c->fails.ensure(2 * sizeof(int));
    // threshold seeding: a seed pass + select before the main pass (>= 4 tiles per workgroup).
    // (Round 4 measured the alternative -- each workgroup of the direct main pass screening a sample
    // tile first and the workgroups selecting and adopting the seed among themselves, no extra
    // launches -- on MI355X: 0.19-0.23 ms slower per cfg3 batch (K1 3.96 vs 3.73 ms) and 0.2 ms at
    // the 8-shard's 1.25M rows, the tiles screened under provisional thresholds costing more than
    // the two launches, profiles/r04_seed_ab.txt; it was removed.)
    const bool seeded = tiles >= 4 * (int64_t)a.G;
    if (ix->i8_res && !(seeded && ix->metric == METRIC_IP && i8_direct_ok(ix->dpad8)))
        throw VsError(VS_ERR_INTERNAL, "group-residual int8 codes need the seeded direct pass");
    if (ix->i8_res) {  // <mu_g, q> of every group for this block's queries
        const int64_t ng = (ix->ntotal + I8_GROUP_ROWS - 1) / I8_GROUP_ROWS;
        c->gT.ensure((size_t)ng * MFMA_QB * sizeof(float));
        HIP_CHECK(launch_group_dots(ix->gmean, ng, ix->dpad8, q, nqb, ix->d, c->gT.as<float>(), st));
        a.gT = c->gT.as<float>();
    }
    // (a device fallback round follows: its native tile is packed here too, from the same loads)
    NativeTile nat{};
    c->prepacked = 0;
    if (prepack && (ix->dtype == DT_BF16 || ix->dtype == DT_F16)) {
        c->qtile_n.ensure((size_t)MFMA_QB * ix->dpad * ix->es);
        c->qinfo.ensure(sizeof(float) * 2 * MFMA_QB);
        c->gcnt2.ensure(sizeof(int) * MFMA_QB);
        c->drop2.ensure(sizeof(u64) * MFMA_QB);
        nat = NativeTile{ix->dtype, (int)ix->dpad, c->qtile_n.as<uint8_t>(), c->qinfo.as<float>(), c->gcnt2.as<int>(),
                         c->drop2.as<u64>()};
    }
    HIP_CHECK(launch_pack_qtile_i8(q, nqb, ix->d, ix->dpad8, c->qtile.as<uint8_t>(), c->qfac.as<float2>(),
                                   c->qeps.as<float>(), ix->d_maxsq + 2, c->gcnt.as<int>(), c->drop.as<u64>(), st,
                                   c->fails.as<int>(), ix->metric == METRIC_L2 ? ix->d_maxsq : nullptr,
                                   gamma_of(ix->d), nat.qt ? &nat : nullptr));
    if (nat.qt) c->prepacked = 2;
    a.qfac = c->qfac.as<float2>();
    a.drop = c->drop.as<u64>();
    a.lcap = a.G * a.Kp;
    c->cand.ensure((size_t)a.G * MFMA_QB * a.cap * sizeof(u64));
    c->part.ensure((size_t)MFMA_QB * a.lcap * sizeof(u64));
    a.cand = c->cand.as<u64>();
    a.glist = c->part.as<u64>();
    a.gcnt = c->gcnt.as<int>();
    a.thr0 = nullptr;
    auto seed_rank_of = [&](double sampled, int M) {
        double target = i8_union_target(kwin > 0 ? kwin : k, sampled, (double)ix->ntotal);
        {
            std::lock_guard<std::mutex> g(ix->h_mu);
            target *= (double)(1 << ix->i8_log2);
        }
        const double r = std::ceil(target * sampled / (double)ix->ntotal);
        return (int)std::min<double>(std::max<double>(r, (double)kOptimisticMinRank), (double)M);
    };
    if (seeded) {  // optimistic threshold seed from one tile per workgroup
        ScreenArgs sa = a;
        sa.G = std::min(sa.G, 512);
        sa.tile_stride = (int)(tiles / sa.G);
        // the direct main pass (k_screen_i8d) screens its whole range itself; the other form reuses
        // the seed tile's accumulators
        if (seed_reuse() && sa.G == a.G && !i8_direct_ok(ix->dpad8)) {
            c->seedacc.ensure((size_t)a.G * 128 * MF_WG_THREADS * sizeof(float));
            sa.seed_acc = c->seedacc.as<float>();
        }
        const int M = sa.G * 16;
        c->seedmax.ensure(sizeof(float) * MFMA_QB * M);
        sa.seedmax = c->seedmax.as<float>();
        HIP_CHECK(launch_seed_mfma(DT_I8, sa, c->qtile.as<uint8_t>(), nqb, st));
        c->thr0.ensure(sizeof(u64) * MFMA_QB);
        const int rank = seed_rank_of((double)sa.G * TR, M);
        HIP_CHECK(launch_seed_select(sa.seedmax, M, nqb, rank, c->thr0.as<u64>(), st));
        a.thr0 = c->thr0.as<u64>();
        a.seed_acc = sa.seed_acc;
    }
    const bool timing = ix->timing.load();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        HIP_CHECK(hipEventRecord(e0, st));
    }
    HIP_CHECK(launch_screen_mfma(DT_I8, a, c->qtile.as<uint8_t>(), nqb, st));
    if (timing) {
        HIP_CHECK(hipEventRecord(e1, st));
        std::lock_guard<std::mutex> g(ix->tmtx);
        ix->tev.emplace_back(e0, e1);
        ix->last_kernel_kind = 3;
    }
    RefineArgs r{};
    r.cand = a.glist;
    r.cand_n = a.gcnt;
    r.lcap = a.lcap;
    r.Kp = a.Kp;
    r.q = q;
    r.d = ix->d;
    r.dpad = ix->dpad;
    r.dt = ix->dtype;
    r.metric = ix->metric;
    r.xmax = (float)(std::sqrt((double)ix->maxsq) * (1.0 + 1e-5)) + 1e-30f;
    r.corpus = ix->data;
    r.k = k;
    r.n_valid = ix->ntotal;
    r.id_offset = id_offset;
    r.D = D;
    r.I = I;
    r.S64 = S64;
    r.cert = cert;
    r.uncert = ix->d_uncert;
    r.qeps = c->qeps.as<float>();
    r.drop = a.drop;
    r.thr0 = a.thr0;
    r.fails = c->fails.as<int>();
    r.ostride = ostride;
    if (phase == 1) {
        const int ka = KA1;
        const int kah = rfw_ka_hi(ka);  // (phase A keeps up to this many rows per query)
        c->pa.ensure((size_t)nqb * kah * 12 + (size_t)nqb * 16);
        r.phase = 1;
        r.pa_cap = kah;
        r.pa_sc = c->pa.as<double>();
        r.pa_ids = (uint32_t*)(r.pa_sc + (size_t)nqb * kah);
        r.pa_tA = (u64*)(r.pa_ids + (size_t)nqb * kah);
        r.pa_n = (int*)(r.pa_tA + nqb);
        HIP_CHECK(launch_refine_wide(r, nqb, ka, st));
        if (keep) *keep = r;
        return;
    }
    // (phase-A depths just under a power of two: the phase-A selection may stop anywhere up to
    // that power -- rfw_ka_hi -- instead of bisecting to an exact count)
    HIP_CHECK(launch_refine_wide(r, nqb, (int)round_up(2 * k + 24, 8), st));
}

// Enqueue one query block through screen -> merge -> refine.  q: device fp32 [nqb][d].
// seed_rank: 0 = proven (safe) seed, > 0 = optimistic seed at that sample rank (see k_seed_select)
// redo: the device fallback round of the block just searched (MFMA dtypes, unseeded screen): its
// three launches (pack, screen, refine) are gated on the block's failure count (c->fails) and the
// refine rewrites only the queries whose certificate failed; a query it cannot certify either
// counts in c->fails[1], the gate of the block's full scan (full_scan_block)
// prepack (first passes followed by their device fallback round): the round's native query tile
// and zeroed list counters are prepared by this pass's query pack (Ctx::prepacked)
void search_block(vs_index* ix, Ctx* c, const float* q, int nqb, int k, int Kp, float* D, int64_t* I, double* S64,
                  int* cert, int64_t id_offset, hipStream_t st, int seed_rank, bool redo = false,
                  bool allow_i8 = true, int ostride = 1, bool prepack = false) {
    if (!redo) c->prepacked = 0;
    if (seed_rank > 0 && allow_i8 && use_i8(ix, nqb, k)) {
        search_block_i8(ix, c, q, nqb, k, D, I, S64, cert, id_offset, st, 0, 0, nullptr, 1, prepack);
        health_note(ix, c, st, 1, nqb);
        return;
    }
    const int64_t tiles = (ix->ntotal + TR - 1) / TR;
    // (search_all makes blocks of > GEMV_NQ_MAX queries only where the MFMA screen serves them)
    const bool use_mfma = nqb > GEMV_NQ_MAX || redo;
    const int* gate = redo ? c->fails.as<int>() : nullptr;
    if (!redo) c->fails.ensure(2 * sizeof(int));
    // int8 screen, few queries: the GEMV streams the int8 copy (1 B per element) with the fp32
    // query; its keys carry the row error bound, so it screens deeper (first passes only)
    bool gemv_i8 = !use_mfma && seed_rank > 0 && ix->screen == VS_SCREEN_I8 && ix->data8 != nullptr && !ix->i8_res;
    if (gemv_i8) {
        const int kp8 = i8_gemv_depth(ix, k);
        gemv_i8 = kp8 <= kI8GemvMaxDepth;  // a single query's refine is one workgroup: deep lists cost
        if (gemv_i8) Kp = kp8;             // more than the int8 stream saves -> native GEMV
    }
    ScreenArgs a{};
    a.corpus = ix->data;
    a.n_valid = ix->ntotal;
    a.tiles = (int)tiles;
    a.dpad = ix->dpad;
    a.d = ix->d;
    a.metric = ix->metric;
    a.sqn = ix->sqn;
    // MFMA: each workgroup keeps its best min(Kp, MFMA_KP_MAX) per query; deeper screens certify
    // against the workgroups' compaction bounds (drop) in the refine.  First passes of inner-product
    // batches (adaptive refine below) keep MFMA_KP_MAX: a workgroup that holds many of a query's
    // best rows (a cluster inserted contiguously) then drops only rows far below the k-th best.
    // (the device fallback round too: its fixed-depth certificate needs two margins between the
    // k-th and the KP_MAX-th best, which a tight cluster -- scores denser than the bf16 query
    // rounding -- does not leave; the adaptive refine scores the rows inside one margin instead)
    const bool wide = use_mfma && ix->metric == METRIC_IP && k <= I8_MAX_K &&
                      (redo || refine_split(nqb, Kp, ix->dtype, ix->num_cu) <= 1);
    // (unseeded small shards -- under 4 tiles per workgroup -- keep max(128, 2 Kp) per workgroup:
    // MFMA_KP_MAX lists of every row there made the refine's selection the cost, 0.9 ms at 100k x
    // 4096 bf16, batch 256, k = 10; a workgroup holding more of a query's best rows fails its
    // certificate and the fallback round lists every row)
    const bool small_shard = tiles < 4 * (int64_t)ix->num_cu;
    a.Kp = use_mfma ? (wide ? (small_shard ? std::min(MFMA_KP_MAX, std::max(128, 2 * Kp)) : MFMA_KP_MAX)
                            : std::min(Kp, MFMA_KP_MAX))
                    : Kp;
    int QB;
    c->qinfo.ensure(sizeof(float) * 2 * MFMA_QB);
    // the screen's query tile and survivor-list counters (a fallback round prepared by its first pass:
    // the prepacked tile, counters gcnt2 / drop2, no pack launch)
    const int pre = redo ? c->prepacked : 0;
    c->prepacked = 0;
    const uint8_t* qtile = c->qtile.as<uint8_t>();
    int* gcnt = nullptr;
    u64* dropb = nullptr;
    if (use_mfma) {
        QB = MFMA_QB;
        a.cap = MFMA_CAP;
        a.G = (int)std::min<int64_t>(tiles, ix->num_cu);
        c->qtile.ensure((size_t)MFMA_QB * ix->dpad * ix->es);
        c->gcnt.ensure(sizeof(int) * MFMA_QB);
        c->drop.ensure(sizeof(u64) * MFMA_QB);
        qtile = c->qtile.as<uint8_t>();
        gcnt = c->gcnt.as<int>();
        dropb = c->drop.as<u64>();
        if (pre) {
            if (pre == 2) qtile = c->qtile_n.as<uint8_t>();
            gcnt = c->gcnt2.as<int>();
            dropb = c->drop2.as<u64>();
        } else {
            // a first pass whose fallback round follows zeroes that round's counters too
            const bool pp = prepack && !redo;
            if (pp) {
                c->gcnt2.ensure(sizeof(int) * MFMA_QB);
                c->drop2.ensure(sizeof(u64) * MFMA_QB);
            }
            HIP_CHECK(launch_pack_qtile(ix->dtype, q, nqb, ix->d, ix->dpad, c->qtile.as<uint8_t>(),
                                        c->qinfo.as<float>(), gcnt, dropb, st, redo ? nullptr : c->fails.as<int>(),
                                        gate, nullptr, pp ? c->gcnt2.as<int>() : nullptr,
                                        pp ? c->drop2.as<u64>() : nullptr));
            if (pp) c->prepacked = 1;
        }
    } else {
        QB = nqb <= 1 ? 1 : nqb <= 2 ? 2 : nqb <= 4 ? 4 : 8;
        a.cap = (int)round_up(Kp + 2 * TR, 256);
        const int sdt = gemv_i8 ? DT_I8 : ix->dtype;
        const int dpadq = gemv_i8 ? ix->dpad8 : ix->dpad;
        // work-queue tiles over exactly the resident blocks; a corpus of at most num_cu / 2 tiles
        // (cfg1: 40) would leave most CUs idle: its work items are quarter tiles (GEMV_SPLIT)
        const int64_t resident = (int64_t)ix->num_cu * (gemv_dyn() ? gemv_blocks_per_cu(sdt, QB, dpadq) : 8);
        a.gemv_split = tiles <= ix->num_cu / 2 ? GEMV_SPLIT : 1;
        a.G = (int)std::min<int64_t>(tiles * a.gemv_split, resident);
        // one query: each block keeps only Kb < Kp keys and publishes the key below which it dropped
        // rows (ScreenArgs::drop, the refine's certificate bound for them), so the G lists together
        // hold at most kRefineRegKeys keys -- the refine selects the best Kp from them in registers
        // and no k_merge launch runs (cfg2: 1024 blocks x 176 keys took a merge of 15 us).  A block
        // that drops a row the query needs fails the certificate; with ~Kp / G of the best rows per
        // block and Kb >= 16 that does not happen in practice.  First passes only (seed_rank > 0):
        // Kb does not grow with Kp, so the host API's 4x-deeper re-searches of a failed query (a
        // burst of near-duplicates in one block) keep whole Kp-deep lists and can certify it.
        if (nqb == 1 && seed_rank > 0 && ix->ntotal >= Kp) {
            const int kb = (int)std::max<int64_t>(16, (kRefineRegKeys / std::max(a.G, 1)) / 16 * 16);
            if (kb < Kp && (int64_t)a.G * kb <= kRefineRegKeys) {
                a.Kp = kb;
                a.cap = (int)round_up(kb + 2 * TR, 256);
                c->drop.ensure(sizeof(u64) * MFMA_QB);
                a.drop = c->drop.as<u64>();
            }
        }
        c->qpad.ensure((size_t)QB * dpadq * sizeof(float));
        int* ctr = nullptr;
        if (gemv_dyn()) {  // the work-queue counter is zeroed by the query pack (no separate memset)
            c->tilectr.ensure(sizeof(int));
            ctr = c->tilectr.as<int>();
        }
        HIP_CHECK(launch_pack_qf32(q, nqb, QB, ix->d, dpadq, c->qpad.as<float>(), c->qinfo.as<float>(), st, ctr,
                                   c->fails.as<int>(), a.drop));
        if (gemv_i8) {
            a.corpus = ix->data8;
            a.dpad = ix->dpad8;
            a.rsb = ix->rsb;
            a.qinfo = c->qinfo.as<float>();
        }
    }
    a.G = std::max(a.G, 1);
    a.gate = gate;
    if (redo && use_mfma) a.skip = cert;  // the fallback screens only the block's failed queries
    c->cand.ensure((size_t)a.G * QB * a.cap * sizeof(u64));
    c->part.ensure((size_t)a.G * QB * a.Kp * sizeof(u64));  // GEMV: [G][QB][Kp]; MFMA: [QB][G*Kp] survivor lists
    a.cand = c->cand.as<u64>();
    a.part = c->part.as<u64>();
    if (!use_mfma && gemv_dyn()) a.next_tile = c->tilectr.as<int>();
    if (use_mfma) {
        a.glist = c->part.as<u64>();
        a.gcnt = gcnt;
        a.lcap = a.G * a.Kp;
        a.drop = dropb;
    }

    // merge partial lists [nseg][qstride][Kp] down to one list per query (or, with stop_keys, to
    // the first round whose nseg * Kp <= stop_keys: one query's lists are then contiguous and the
    // refine selects the best Kp itself); returns it, nseg updated
    // (segments of a.Kp keys: the screen's per-block depth, = Kp whenever a merge runs)
    auto merge_all = [&](const u64* src, int& nseg, int qstride, int stop_keys) -> const u64* {
        const int W = a.Kp;
        const int spb = (256 * (W > 2048 ? 32 : 16)) / W;  // k_merge: 4096 / 8192 keys per block
        const size_t mbytes = (size_t)std::max(1, (nseg + spb - 1) / spb) * nqb * W * sizeof(u64);
        c->merge_a.ensure(mbytes);
        c->merge_b.ensure(mbytes);
        u64* bufs[2] = {c->merge_a.as<u64>(), c->merge_b.as<u64>()};
        int which = 0;
        while (nseg > 1 && (int64_t)nseg * W > stop_keys) {
            int nout = 0;
            HIP_CHECK(launch_merge(src, nseg, qstride, nqb, W, bufs[which], &nout, st));
            src = bufs[which];
            which ^= 1;
            nseg = nout;
            qstride = nqb;
        }
        return src;
    };

    // threshold seeding (MFMA path): screen one tile per CU, strided over the shard, keep only the
    // per-query maxima of 16-row groups, and start every workgroup of the main pass at the
    // rank-th largest of them (rank = Kp: proven lower bound; kOptimisticSeedRank: optimistic)
    a.tile_stride = 0;
    a.thr0 = nullptr;
    bool optimistic = false;
    // (not in a fallback round: its launches cost their dispatch on every call, and it rarely runs)
    if (use_mfma && !redo && tiles >= 4 * (int64_t)a.G) {
        ScreenArgs sa = a;
        sa.G = std::min(sa.G, 512);  // k_seed_select holds up to 8192 maxima per query
        sa.tile_stride = (int)(tiles / sa.G);
        // seed tile = the first tile of each main-pass workgroup; its raw accumulators are kept so
        // the main pass starts one tile later
        // (bf16 / f16 main passes in the direct form screen their whole range themselves)
        const bool direct = (ix->dtype == DT_BF16 || ix->dtype == DT_F16) && d16_direct_ok(ix->dpad);
        if (seed_reuse() && sa.G == a.G && !direct) {
            c->seedacc.ensure((size_t)a.G * 128 * MF_WG_THREADS * sizeof(float));
            sa.seed_acc = c->seedacc.as<float>();
        }
        const int M = sa.G * 16;
        c->seedmax.ensure(sizeof(float) * MFMA_QB * M);
        sa.seedmax = c->seedmax.as<float>();
        HIP_CHECK(launch_seed_mfma(ix->dtype, sa, c->qtile.as<uint8_t>(), nqb, st));
        c->thr0.ensure(sizeof(u64) * MFMA_QB);
        // optimistic rank: expected rows above the seed ~ rank * rows / sampled rows ~ 8 Kp
        int rank = Kp;
        if (seed_rank > 0) {
            const double sampled = (double)sa.G * TR;
            // deep screens aim lower (~12k listed rows per query), so the refine selects in registers
            const double factor = std::min(kOptimisticPassFactor, 12288.0 / Kp) * (wide ? seed_scale(ix) : 1.0);
            const double r = std::ceil(factor * Kp * sampled / (double)ix->ntotal);
            // floor: at rank 1 a sample maximum that falls inside the true top-Kp leaves fewer than
            // Kp survivors (probability ~Kp * sampled / N per query, ~2% at 100M rows); with >= 4
            // sampled rows required in the top-Kp the failure odds drop to ~(that)^4 / 24
            // (the fixed-depth refine needs rank <= Kp -- the proven seed -- for its certificate; the
            // adaptive refine's certificate checks the seed itself, so its rank may go deeper)
            rank = (int)std::min<double>(std::max<double>(r, (double)kOptimisticMinRank), wide ? (double)M : (double)Kp);
        }
        HIP_CHECK(launch_seed_select(sa.seedmax, M, nqb, rank, c->thr0.as<u64>(), st));
        a.thr0 = c->thr0.as<u64>();
        a.seed_acc = sa.seed_acc;
        optimistic = rank < Kp;
    }

    const bool timing = ix->timing.load() && !redo;  // (a fallback round is not the timed screen)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        HIP_CHECK(hipEventRecord(e0, st));
    }
    if (use_mfma) HIP_CHECK(launch_screen_mfma(ix->dtype, a, qtile, nqb, st));
    else HIP_CHECK(launch_screen_gemv(gemv_i8 ? DT_I8 : ix->dtype, a, c->qpad.as<float>(), nqb, QB, st));
    if (timing) {
        HIP_CHECK(hipEventRecord(e1, st));
        std::lock_guard<std::mutex> g(ix->tmtx);
        ix->tev.emplace_back(e0, e1);
        ix->last_kernel_kind = use_mfma ? 1 : gemv_i8 ? 4 : 2;
    }
    RefineArgs r{};
    if (use_mfma) {  // the refine selects the best Kp of each query's survivor list itself
        r.cand = a.glist;
        r.cand_n = a.gcnt;
        r.lcap = a.lcap;
    } else {  // GEMV: merge the per-block lists down to [q][Kp] (qstride nqb, or part[0] with QB)
        // one query (the product's call shape): stop the merge tree at <= kRefineRegKeys keys,
        // which the refine selects from in registers (one wave up to 2048; a k_merge launch costs
        // more than the block-wide selection above that).  Needs >= Kp non-empty keys among them,
        // which every round keeps when the shard has >= Kp rows.
        int nseg = a.G;
        const int stop = (nqb == 1 && ix->ntotal >= Kp) ? kRefineRegKeys : 0;
        r.cand = merge_all(a.part, nseg, QB, stop);
        r.cand_n = nullptr;
        r.lcap = nseg * a.Kp;
    }
    r.Kp = Kp;
    r.drop = a.drop;
    r.thr0 = a.thr0;  // (the adaptive refine's certificate: rows never listed scored <= thr0)
    r.i8max = gemv_i8 ? ix->d_maxsq + 2 : nullptr;
    r.q = q;
    r.d = ix->d;
    r.dpad = ix->dpad;
    r.dt = ix->dtype;
    r.metric = ix->metric;
    r.corpus = ix->data;
    r.qinfo = c->qinfo.as<float>();
    r.xmax = (float)(std::sqrt((double)ix->maxsq) * (1.0 + 1e-5)) + 1e-30f;
    r.gamma = gamma_of(ix->d);
    r.k = k;
    r.n_valid = ix->ntotal;
    r.id_offset = id_offset;
    r.D = D;
    r.I = I;
    r.S64 = S64;
    r.cert = cert;
    r.uncert = redo ? nullptr : ix->d_uncert;
    r.fails = c->fails.as<int>() + (redo ? 1 : 0);  // (a fallback round's failures gate the full scan)
    r.redo = redo ? 1 : 0;
    r.gate = gate;
    r.ostride = ostride;
    r.optimistic = optimistic ? 1 : 0;
    r.nsplit = redo ? 1 : refine_split(nqb, Kp, ix->dtype, ix->num_cu);
    if (r.nsplit > 1) {
        const int KP2 = refine_kp2(Kp);
        c->rsc.ensure((size_t)nqb * KP2 * 12);
        r.gsc = c->rsc.as<double>();
        r.gids = (uint32_t*)(r.gsc + (size_t)nqb * KP2);
        if (c->rdone.bytes < sizeof(unsigned) * MFMA_QB) {  // zeroed once; the last workgroup re-zeroes
            c->rdone.ensure(sizeof(unsigned) * MFMA_QB);
            HIP_CHECK(hipMemsetAsync(c->rdone.p, 0, c->rdone.bytes, st));
        }
        r.gdone = c->rdone.as<unsigned>();
    }
    // native MFMA first passes (inner product): the adaptive two-phase refine -- it scores every
    // listed row whose key is within the screen's margin of the k-th best, so dense score
    // distributions (clustered corpora) certify without a re-search; the fixed-depth refine's
    // certificate needs a gap of 2 margins between the k-th and the Kp-th best
    if (wide) {
        const int ka = redo ? screen_depth(k) : Kp;  // (a fallback round's Kp is the listing depth)
        HIP_CHECK(launch_refine_wide(r, nqb, (int)round_up(std::max(ka - 8, k + 24), 8), st));
        if (!redo) health_note(ix, c, st, 2, nqb);
        return;
    }
    HIP_CHECK(launch_refine(r, nqb, st));
}

// Depth of the device fallback round: the end of vs_search's host escalation (KP_MAX), within
// the shard.
int fallback_depth(const vs_index* ix) { return (int)std::min<int64_t>(KP_MAX, round_up(ix->ntotal, 16)); }

// The last tier: an exact full scan of the shard (vs_fullscan.hip) for the block's queries with
// cert[q] == 0 -- those no bounded screen could certify (more rows than KP_MAX tied within its
// margin, e.g. thousands of identical embeddings).  Every row is scored canonically and streamed
// through a running top-k, so the answer is faiss's (ties to the lowest ids) for any tie count.
// gate: the fallback round's failure count (c->fails[1]; the launch returns at once while it is
// 0), or null = run.  Scanned queries count in this call's counter or the index's d_unres.
constexpr int64_t kFullScanScratchMax = 512ll << 20;
constexpr int64_t kFullScanScratch = 32ll << 20;  // per-workgroup lists of one block, at most
// rows_per_wg: each workgroup's row range is at least this long (G = rows / rows_per_wg, <= CUs)
void full_scan_block(vs_index* ix, Ctx* c, const float* q, int nqb, int k, float* D, int64_t* I, double* S64,
                     int* cert, int64_t id_offset, hipStream_t st, const int* gate, int ostride = 1,
                     int rows_per_wg = TR, bool fallback = true, bool all_queries = false) {
    const int64_t ranges = (ix->ntotal + rows_per_wg - 1) / rows_per_wg;
    const int64_t per_wg = (int64_t)nqb * k * 12;
    // scratch: per workgroup one k-list per query of the block.  32 MiB serves ~100 workgroups at
    // 256 queries x k 100; deep lists (k in the thousands) may take up to kFullScanScratchMax so the
    // scan still reaches a quarter of the CUs (at 32 MiB, k = 3276 left it 3 workgroups)
    const int64_t budget = std::max<int64_t>(kFullScanScratch, std::min<int64_t>(kFullScanScratchMax,
                                                                                 per_wg * (ix->num_cu / 4)));
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(ix->num_cu, ranges), budget / per_wg));
    c->fsc.ensure(full_scan_scratch_bytes(nqb, G, k));
    if (c->fdone.bytes < sizeof(unsigned) * MFMA_QB) {  // zeroed once; each query's last workgroup re-zeroes
        c->fdone.ensure(sizeof(unsigned) * MFMA_QB);
        HIP_CHECK(hipMemsetAsync(c->fdone.p, 0, c->fdone.bytes, st));
    }
    FullScanArgs a{};
    a.corpus = ix->data;
    a.d = ix->d;
    a.dpad = ix->dpad;
    a.dt = ix->dtype;
    a.metric = ix->metric;
    a.n_valid = ix->ntotal;
    a.q = q;
    a.nq = nqb;
    a.k = k;
    a.cert = cert;
    a.gate = gate;
    a.id_offset = id_offset;
    a.D = D;
    a.I = I;
    a.S64 = S64;
    a.ostride = ostride;
    a.gsc = c->fsc.as<double>();
    a.gid = (uint32_t*)(a.gsc + (size_t)nqb * G * k);
    a.gdone = c->fdone.as<unsigned>();
    a.count = !fallback ? nullptr : c->unres ? c->unres : ix->d_unres;  // (a first pass is counted nowhere)
    a.G = G;
    a.all_queries = all_queries ? 1 : 0;
    HIP_CHECK(launch_full_scan(a, st));
}

// Full search of nq device queries; outputs device [nq][k].  device_fallback: every block's first
// pass is followed by its gated fallback round (no host round trip; MFMA dtypes only).
// (measured against the GEMV screen + refine, scripts/small_scan_timing.py: the scan wins up to
// ~190 MB at d >= 1536 and k = 10; more rows, smaller d or deeper k favour the screen)
constexpr int kSmallScanQ = 2;           // queries per call
constexpr int kSmallScanMaxK = 64;
constexpr int64_t kSmallScanMaxRows = 65536;
constexpr int kSmallScanRows = 64;       // rows per workgroup range
bool small_scan(const vs_index* ix, int64_t nq, int k) {
    return nq <= kSmallScanQ && k <= kSmallScanMaxK && ix->ntotal <= kSmallScanMaxRows &&
           (int64_t)ix->ntotal * ix->dpad * ix->es <= ix->scan_limit.load();
}

void search_all(vs_index* ix, Ctx* c, const float* q, int64_t nq, int k, int Kp, float* D, int64_t* I, double* S64,
                int* cert, int64_t id_offset, hipStream_t st, int seed_rank, bool device_fallback = false) {
    // One or two queries over a small corpus (the product's single-query call, BASELINE cfg1): the
    // exact full scan alone -- every row scored canonically in one launch, no screen, no refine, no
    // certificate to fail (measured: DESIGN §5 "Small corpora").  First passes only (seed_rank > 0):
    // a re-search of a certificate failure never reaches here, since this path has none.
    if (seed_rank > 0 && small_scan(ix, nq, k)) {
        int* cq = cert;
        if (!cq) {
            c->cert.ensure((size_t)nq * sizeof(int));
            cq = c->cert.as<int>();
        }
        const bool timing = ix->timing.load();
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (timing) {
            HIP_CHECK(hipEventCreate(&e0));
            HIP_CHECK(hipEventCreate(&e1));
            HIP_CHECK(hipEventRecord(e0, st));
        }
        full_scan_block(ix, c, q, (int)nq, k, D, I, S64, cq, id_offset, st, nullptr, 1, kSmallScanRows, false, true);
        if (timing) {
            HIP_CHECK(hipEventRecord(e1, st));
            std::lock_guard<std::mutex> g(ix->tmtx);
            ix->tev.emplace_back(e0, e1);
            ix->last_kernel_kind = 5;
        }
        return;
    }
    const bool i8 = seed_rank > 0 && i8_allowed(ix);  // (int8 screen on, and not routed away)
    const bool mfma_ok = (i8 && k <= I8_MAX_K) || ix->dtype != DT_F32;
    int64_t done = 0;
    while (done < nq) {
        const int64_t rem = nq - done;
        int nqb;
        // fp32 rows on the native screen: the fp32 MFMA (compute-bound, all 256 columns) pays from
        // ~kF32MfmaMinQ queries on; fewer take the GEMV, 8 queries per corpus pass
        if ((mfma_ok && rem > GEMV_NQ_MAX) || (!i8 && ix->dtype == DT_F32 && rem >= kF32MfmaMinQ))
            nqb = (int)std::min<int64_t>(rem, MFMA_QB);
        else nqb = (int)std::min<int64_t>(rem, GEMV_NQ_MAX);
        search_block(ix, c, q + done * ix->d, nqb, k, Kp, D ? D + done * k : nullptr, I + done * k,
                     S64 ? S64 + done * k : nullptr, cert ? cert + done : nullptr, id_offset, st, seed_rank, false, i8,
                     1, device_fallback && nqb > GEMV_NQ_MAX);
        if (device_fallback && nqb <= GEMV_NQ_MAX) {
            // a GEMV block (1-8 queries): a failed certificate goes straight to the full scan -- one
            // pass over the rows per failed query, about what the fallback round's MFMA screen costs
            // the block -- in ONE gated launch instead of four (the single-query step, cfg2)
            full_scan_block(ix, c, q + done * ix->d, nqb, k, D ? D + done * k : nullptr, I + done * k,
                            S64 ? S64 + done * k : nullptr, cert + done, id_offset, st, c->fails.as<int>());
        } else if (device_fallback) {
            search_block(ix, c, q + done * ix->d, nqb, k, std::max(Kp, fallback_depth(ix)), D ? D + done * k : nullptr,
                         I + done * k, S64 ? S64 + done * k : nullptr, cert + done, id_offset, st, 0, true);
            full_scan_block(ix, c, q + done * ix->d, nqb, k, D ? D + done * k : nullptr, I + done * k,
                            S64 ? S64 + done * k : nullptr, cert + done, id_offset, st, c->fails.as<int>() + 1);
        }
        done += nqb;
    }
}

void check_index(const vs_index* ix) {
    if (!ix) throw VsError(VS_ERR_ARG, "null index");
}

// Points a leased Ctx's full-scan counter at the caller's device word for one call, and
// clears it on every exit (exceptions included), before the Ctx returns to the pool: a later
// lease must never count into a buffer it does not own.
struct UnresScope {
    Ctx* c;
    UnresScope(Ctx* c_, unsigned* unres) : c(c_) { c->unres = unres; }
    ~UnresScope() { c->unres = nullptr; }
    UnresScope(const UnresScope&) = delete;
    UnresScope& operator=(const UnresScope&) = delete;
};

}  // namespace

// exact device search (vs_search_device_exact; the IVF coarse quantizer): like vs_search_device,
// but certificate failures are re-searched on the device, by each query block's gated fallback
// round at the deepest screen (KP_MAX, where vs_search's escalation ends; fp32 rows: the fp32 MFMA
// screen), and a query even that round cannot certify by the gated exact full scan of the shard
// (full_scan_block; counted in vs_full_scan_count).  async: no host round trip at all, the call
// returns with the work queued; otherwise the certificates are read back and checked.
void vs::search_exact_device(vs_index* ix, const float* q_dev, int64_t nq, int k, int64_t* I_dev, double* S64_dev,
                             hipStream_t st, float* D_dev, int64_t id_offset, bool async, unsigned* unres) {
    check_index(ix);
    if (nq <= 0) return;
    std::shared_lock<std::shared_mutex> lk(ix->rw);
    DeviceGuard dg(ix->device);
    if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");  // k > ntotal: -1 / worst-score padding
    CtxLease L(ix, st, false);
    Ctx* c = L.c;
    c->outD.ensure((size_t)nq * k * sizeof(float));
    c->cert.ensure((size_t)nq * sizeof(int));
    const int Kp = screen_depth(k);
    UnresScope us(c, unres);  // the caller's counter for this call only (the Ctx goes back to the pool)
    // every dtype has the on-device MFMA fallback round, queued behind each block's first pass
    search_all(ix, c, q_dev, nq, k, Kp, D_dev ? D_dev : c->outD.as<float>(), I_dev, S64_dev, c->cert.as<int>(),
               id_offset, st, kOptimisticSeedRank, true);
    if (async) return;
    c->hout.ensure((size_t)nq * sizeof(int));
    int* cert_h = (int*)c->hout.p;
    HIP_CHECK(hipMemcpyAsync(cert_h, c->cert.p, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    // (every block's full scan has run behind its fallback round: a query left uncertified here
    // would be a library error, so it is answered by a full scan of its own rather than trusted)
    for (int64_t qi = 0; qi < nq; ++qi) {
        if (cert_h[qi]) continue;
        int* cq = c->cert.as<int>() + qi;
        HIP_CHECK(hipMemsetAsync(cq, 0, sizeof(int), st));
        full_scan_block(ix, c, q_dev + qi * ix->d, 1, k, (D_dev ? D_dev : c->outD.as<float>()) + qi * k, I_dev + qi * k,
                        S64_dev ? S64_dev + qi * k : nullptr, cq, id_offset, st, nullptr);
        HIP_CHECK(hipMemcpyAsync(&cert_h[qi], cq, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        if (!cert_h[qi]) throw VsError(VS_ERR_INTERNAL, "full scan left a query uncertified");
    }
}

// S concurrent exact device searches over consecutive parts (whole query blocks) of one batch, each
// on its own stream with its own leased workspace (leases held together, so no two parts share a
// workspace and serialise on it); a part's full-scanned queries count in unres[part] (if given).  The IVF
// coarse assignment: one 256-row block of a small quantizer fills only nlist / 256 workgroups.
void vs::search_exact_device_parts(vs_index* ix, const float* q_dev, int64_t nq, int k, int64_t* I_dev,
                                   hipStream_t* streams, int S, unsigned* unres) {
    check_index(ix);
    if (nq <= 0) return;
    std::shared_lock<std::shared_mutex> lk(ix->rw);
    DeviceGuard dg(ix->device);
    if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
    std::vector<std::unique_ptr<CtxLease>> leases;
    for (int i = 0; i < S; ++i) leases.emplace_back(new CtxLease(ix, streams[i], false));
    const int Kp = screen_depth(k);
    const int64_t blocks = (nq + MFMA_QB - 1) / MFMA_QB;
    for (int i = 0; i < S; ++i) {
        const int64_t q0 = std::min(nq, blocks * i / S * MFMA_QB), q1 = std::min(nq, blocks * (i + 1) / S * MFMA_QB);
        if (q1 <= q0) continue;
        Ctx* c = leases[i]->c;
        c->outD.ensure((size_t)(q1 - q0) * k * sizeof(float));
        c->cert.ensure((size_t)(q1 - q0) * sizeof(int));
        UnresScope us(c, unres ? unres + i : nullptr);  // reset even if search_all throws
        search_all(ix, c, q_dev + q0 * ix->d, q1 - q0, k, Kp, c->outD.as<float>(), I_dev + q0 * k, nullptr,
                   c->cert.as<int>(), 0, streams[i], kOptimisticSeedRank, true);
    }
}

unsigned* vs::full_scan_counter(vs_index* ix) { return ix->d_unres; }

// ---- two-phase exact device search (the sharded step with a global T' exchange) ----
// Phase A of every shard scores the best KA keys of each query's survivor list; the shards exchange
// those top-k lists, and the merged k-th best (a lower bound of the global k-th best score) is the
// floor under which phase B scores nothing and the certificate needs nothing: each shard then
// scores about its share of the global refine window instead of a whole window of its own.
// Applies to one int8 MFMA block of a bf16/f16 index (static: the same answer on every rank of a
// collective); otherwise phase A runs the whole exact search and phase B returns its result.
struct vs_pending {
    vs_index* ix = nullptr;
    std::shared_lock<std::shared_mutex> lk;
    std::unique_ptr<CtxLease> L;
    hipStream_t st = nullptr;
    const float* q = nullptr;
    int64_t nq = 0;
    int k = 0, ka = 0, stride = 1;
    int64_t id_offset = 0;
    bool two = false;
    RefineArgs r{};
};

bool vs::two_phase_ok(const vs_index* ix, int64_t nq, int k) {
    return ix->screen == VS_SCREEN_I8 && nq > GEMV_NQ_MAX && nq <= MFMA_QB && k <= I8_MAX_K;
}

vs_pending* vs::search_phase_a(vs_index* ix, const float* q_dev, int64_t nq, int k, int world, int64_t id_offset,
                               double* S_a, int64_t* I_a, int stride, hipStream_t st) {
    check_index(ix);
    if (k <= 0 || nq <= 0 || world <= 0) throw VsError(VS_ERR_ARG, "nq, k and world must be > 0");
    if (stride < 1) throw VsError(VS_ERR_ARG, "stride must be >= 1");
    if (ix->ntotal == 0) throw VsError(VS_ERR_ARG, "index is empty");
    std::unique_ptr<vs_pending> p(new vs_pending());
    p->ix = ix;
    p->lk = std::shared_lock<std::shared_mutex>(ix->rw);
    DeviceGuard dg(ix->device);
    p->L.reset(new CtxLease(ix, st, false));
    Ctx* c = p->L->c;
    p->st = st;
    p->q = q_dev;
    p->nq = nq;
    p->k = k;
    p->id_offset = id_offset;
    if (!two_phase_ok(ix, nq, k)) throw VsError(VS_ERR_ARG, "two-phase search: not applicable (vs_two_phase_ok)");
    // (routed to the native screen, or group-residual codes on a shard too small for their seeded
    // direct pass: phase A runs the whole search -- a per-rank choice, the exchanges are the same)
    p->two = i8_allowed(ix) && use_i8(ix, (int)nq, k);
    c->cert.ensure((size_t)nq * sizeof(int));
    if (p->two) {
        // phase A's depth: twice a shard's expected share of the global top-k (+24), so the shards'
        // lists together hold the global k-th best of what they scored
        const int share = (k + world - 1) / world;
        p->ka = (int)std::min<int64_t>(round_up(2 * k + 24, 8), round_up(2 * share + 24, 8));
        // the seed's union covers this shard's share of the global window: phase B certifies the
        // unlisted rows against the global floor (~ the global k-th best), and the shard's rows
        // within the int8 error budget of it are ~1/world of the whole window (iid shards)
        search_block_i8(ix, c, q_dev, (int)nq, k, nullptr, I_a, S_a, c->cert.as<int>(), id_offset, st, 1, p->ka,
                        &p->r, stride, true, share);
    } else {
        c->outS.ensure((size_t)nq * k * sizeof(double));
        c->outI.ensure((size_t)nq * k * sizeof(int64_t));
        c->outD.ensure((size_t)nq * k * sizeof(float));
        search_all(ix, c, q_dev, nq, k, screen_depth(k), c->outD.as<float>(), c->outI.as<int64_t>(),
                   c->outS.as<double>(), c->cert.as<int>(), id_offset, st, kOptimisticSeedRank, true);
        HIP_CHECK(hipMemcpy2DAsync(S_a, (size_t)stride * 8, c->outS.p, 8, 8, (size_t)nq * k, hipMemcpyDeviceToDevice, st));
        HIP_CHECK(hipMemcpy2DAsync(I_a, (size_t)stride * 8, c->outI.p, 8, 8, (size_t)nq * k, hipMemcpyDeviceToDevice, st));
    }
    return p.release();
}

void vs::search_phase_b(vs_pending* p, const double* floor_S, float* D, int64_t* I, double* S64, int stride,
                        hipStream_t st, unsigned* unres) {
    std::unique_ptr<vs_pending> own(p);
    vs_index* ix = p->ix;
    DeviceGuard dg(ix->device);
    Ctx* c = p->L->c;
    if (st != p->st) {  // order the caller's stream behind phase A's work
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(e, p->st));
        HIP_CHECK(hipStreamWaitEvent(st, e, 0));
        (void)hipEventDestroy(e);
        p->L->st = st;
    }
    const int64_t nq = p->nq;
    const int k = p->k;
    if (stride < 1) throw VsError(VS_ERR_ARG, "stride must be >= 1");
    if (!p->two) {
        HIP_CHECK(hipMemcpy2DAsync(I, (size_t)stride * 8, c->outI.p, 8, 8, (size_t)nq * k, hipMemcpyDeviceToDevice, st));
        if (S64)
            HIP_CHECK(hipMemcpy2DAsync(S64, (size_t)stride * 8, c->outS.p, 8, 8, (size_t)nq * k, hipMemcpyDeviceToDevice, st));
        if (D) HIP_CHECK(hipMemcpyAsync(D, c->outD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToDevice, st));
        return;
    }
    RefineArgs r = p->r;
    r.phase = 2;
    r.tfloor = floor_S;
    r.tfloor_k = k;
    r.D = D;
    r.I = I;
    r.S64 = S64;
    r.ostride = stride;
    HIP_CHECK(launch_refine_wide(r, (int)nq, p->ka, st));
    health_note(ix, c, st, 1, (int)nq);
    // the block's gated fallback round (native screen, local certificate), as search_all's
    UnresScope us(c, unres);
    search_block(ix, c, p->q, (int)nq, k, std::max(screen_depth(k), fallback_depth(ix)), D, I, S64,
                 c->cert.as<int>(), p->id_offset, st, 0, true, true, stride);
    // and its gated full scan (the shard's own exact top-k; the floor is not needed for it)
    full_scan_block(ix, c, p->q, (int)nq, k, D, I, S64, c->cert.as<int>(), p->id_offset, st, c->fails.as<int>() + 1,
                    stride);
}

void vs::search_pending_free(vs_pending* p) { delete p; }

void vs::truncate_rows(vs_index* ix, int64_t n) {
    check_index(ix);
    std::unique_lock<std::shared_mutex> lk(ix->rw);
    if (n < 0 || n > ix->ntotal) throw VsError(VS_ERR_ARG, "truncate_rows: n outside [0, ntotal]");
    ix->ntotal = n;  // the rows behind stay allocated and are never read again (appends overwrite them)
}


int64_t vs::stream_chunk_rows(int d) { return std::max<int64_t>(1, (int64_t)(32 << 20) / ((int64_t)d * 4)); }

// Double-buffered host -> HBM ingest: chunk c is filled on the host (memcpy, file read) into pinned
// buffer c&1 while the copy engine and k_pack_rows still work on chunk c-1.  A pinned buffer is
// refilled only after the event recorded behind its previous pack has fired.
void vs::add_rows_host(vs_index* ix, int64_t n, const std::function<void(int64_t, int64_t, float*)>& fill) {
    check_index(ix);
    std::unique_lock<std::shared_mutex> lk(ix->rw);
    DeviceGuard dg(ix->device);
    if (ix->ntotal + n > (int64_t)0xFFFFFFF0LL) throw VsError(VS_ERR_ARG, "shard exceeds 2^32 rows");
    ensure_capacity(ix, ix->ntotal + n);
    const int64_t rpc = stream_chunk_rows(ix->d);
    const size_t cbytes = (size_t)std::min(n, rpc) * ix->d * sizeof(float);
    ix->pin.ensure(cbytes);
    ix->stage[0].ensure(cbytes);
    ix->stage[1].ensure(cbytes);
    try {
        for (int64_t c = 0, r0 = 0; r0 < n; ++c, r0 += rpc) {
            const int b = (int)(c & 1);
            const int64_t m = std::min(rpc, n - r0);
            if (c >= 2) HIP_CHECK(hipEventSynchronize(ix->pin.done[b]));
            fill(r0, m, ix->pin.host[b]);
            HIP_CHECK(hipMemcpyAsync(ix->stage[b].p, ix->pin.host[b], (size_t)m * ix->d * sizeof(float),
                                     hipMemcpyHostToDevice, ix->own));
            HIP_CHECK(launch_pack_rows(ix->dtype, ix->stage[b].as<float>(), m, ix->d, ix->dpad, ix->data,
                                       ix->ntotal + r0, ix->sqn, ix->d_maxsq, ix->own));
            HIP_CHECK(hipEventRecord(ix->pin.done[b], ix->own));
        }
        quantize_rows(ix, ix->ntotal, n, ix->own);
        HIP_CHECK(hipStreamSynchronize(ix->own));
    } catch (...) {
        (void)hipStreamSynchronize(ix->own);  // the pinned chunks may still be in flight
        throw;                                // ntotal unchanged: the packed rows stay invisible
    }
    ix->ntotal += n;
    refresh_maxsq(ix);
}

// Double-buffered HBM -> host export: chunk c is unpacked and copied into pinned buffer c&1 while
// the host consumes chunk c-1 (memcpy out, file write).
void vs::read_rows_host(vs_index* ix, int64_t i0, int64_t n,
                        const std::function<void(int64_t, int64_t, const float*)>& sink) {
    check_index(ix);
    std::shared_lock<std::shared_mutex> lk(ix->rw);
    if (i0 < 0 || n < 0 || i0 + n > ix->ntotal) throw VsError(VS_ERR_ARG, "reconstruct range out of bounds");
    if (n == 0) return;
    DeviceGuard dg(ix->device);
    CtxLease L(ix, nullptr, true);
    Ctx* c = L.c;
    const int64_t rpc = stream_chunk_rows(ix->d);
    const size_t cbytes = (size_t)std::min(n, rpc) * ix->d * sizeof(float);
    c->pin.ensure(cbytes);
    c->rows[0].ensure(cbytes);
    c->rows[1].ensure(cbytes);
    const int64_t nchunks = (n + rpc - 1) / rpc;
    auto enqueue = [&](int64_t ci) {
        const int b = (int)(ci & 1);
        const int64_t r0 = ci * rpc, m = std::min(rpc, n - r0);
        HIP_CHECK(launch_unpack_rows(ix->dtype, ix->data, i0 + r0, m, ix->d, ix->dpad, c->rows[b].as<float>(),
                                     c->stream));
        HIP_CHECK(hipMemcpyAsync(c->pin.host[b], c->rows[b].p, (size_t)m * ix->d * sizeof(float),
                                 hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(hipEventRecord(c->pin.done[b], c->stream));
    };
    try {
        enqueue(0);
        for (int64_t ci = 0; ci < nchunks; ++ci) {
            if (ci + 1 < nchunks) enqueue(ci + 1);  // pinned buffer (ci+1)&1 was drained at ci-1
            const int b = (int)(ci & 1);
            HIP_CHECK(hipEventSynchronize(c->pin.done[b]));
            const int64_t r0 = ci * rpc;
            sink(r0, std::min(rpc, n - r0), c->pin.host[b]);
        }
    } catch (...) {
        (void)hipStreamSynchronize(c->stream);
        throw;
    }
}

extern "C" {

const char* vs_last_error(void) { return g_err.c_str(); }
const char* vs_version(void) { return "libvs 0.1 (gfx950)"; }

int vs_create(int d, int metric, int dtype, int device, vs_index** out) {
    return guarded([&] {
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        *out = nullptr;
        if (d <= 0) throw VsError(VS_ERR_ARG, "dimension must be > 0");
        if (metric != VS_METRIC_IP && metric != VS_METRIC_L2) throw VsError(VS_ERR_ARG, "metric must be IP(0) or L2(1)");
        if (dtype < VS_DTYPE_F32 || dtype > VS_DTYPE_F16) throw VsError(VS_ERR_ARG, "dtype must be 0 (f32), 1 (bf16), 2 (f16)");
        int ndev = 0;
        hipError_t e = hipGetDeviceCount(&ndev);
        if (e != hipSuccess || ndev <= 0) throw VsError(VS_ERR_DEVICE, "no HIP device available (libvs needs an MI355X)");
        if (device < 0 || device >= ndev) throw VsError(VS_ERR_ARG, "device ordinal out of range");
        DeviceGuard dg(device);
        hipDeviceProp_t prop;
        HIP_CHECK(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            throw VsError(VS_ERR_DEVICE, std::string("libvs is built for gfx950, device is ") + prop.gcnArchName);
        vs_index* ix = new vs_index();
        ix->d = d;
        // >= 2 K-steps per tile: the MFMA screen's deferred compaction check runs on the K-step
        // after a tile's epilogue, so a one-step tile would never compact its candidate buffers
        ix->dpad = pad_dim(d, dtype);
        ix->metric = metric;
        ix->dtype = dtype;
        ix->device = device;
        ix->es = es_of(dtype);
        ix->num_cu = prop.multiProcessorCount;
        try {
            HIP_CHECK(hipStreamCreateWithFlags(&ix->own, hipStreamNonBlocking));
            // [0] max ||x||^2, [1] uncertified counter, [2..3] int8 screen maxima (fp32 bits),
            // [4] full-scan counter (vs_full_scan_count), [5..6] group residuals (max ||mu_g||,
            // groups with a mean), [7] max ||x - s c|| of the int8 codes
            HIP_CHECK(hipMalloc(&ix->d_maxsq, sizeof(unsigned) * 8));
            HIP_CHECK(hipMemset(ix->d_maxsq, 0, sizeof(unsigned) * 8));
            ix->d_uncert = ix->d_maxsq + 1;
            ix->d_unres = ix->d_maxsq + 4;
        } catch (...) {
            delete ix;
            throw;
        }
        *out = ix;
    });
}

void vs_destroy(vs_index* ix) {
    if (!ix) return;
    {
        DeviceGuard dg(ix->device);
        hipDeviceSynchronize();
        for (Ctx* c : ix->pool_all) delete c;
        for (auto& pr : ix->tev) {
            hipEventDestroy(pr.first);
            hipEventDestroy(pr.second);
        }
        ix->stage[0].release();
        ix->stage[1].release();
        ix->pin.release();
        if (ix->data) hipFree(ix->data);
        if (ix->sqn) hipFree(ix->sqn);
        if (ix->d_maxsq) hipFree(ix->d_maxsq);
        free_i8(ix);
        if (ix->own) hipStreamDestroy(ix->own);
        if (ix->h_ev) hipEventDestroy(ix->h_ev);
        if (ix->h_fails) hipHostFree(ix->h_fails);
    }
    delete ix;
}

int vs_reset(vs_index* ix) {
    return guarded([&] {
        check_index(ix);
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        ix->ntotal = 0;
        ix->maxsq = 0.0f;
        ix->i8_bmax = 0.0f;
        ix->i8_res = false;
        HIP_CHECK(hipMemsetAsync(ix->d_maxsq, 0, sizeof(unsigned), ix->own));
        HIP_CHECK(hipMemsetAsync(ix->d_maxsq + 2, 0, 2 * sizeof(unsigned), ix->own));
        HIP_CHECK(hipMemsetAsync(ix->d_maxsq + 5, 0, 3 * sizeof(unsigned), ix->own));
        HIP_CHECK(hipStreamSynchronize(ix->own));
    });
}

int vs_add(vs_index* ix, const float* x, int64_t n) {
    return guarded([&] {
        check_index(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x) throw VsError(VS_ERR_ARG, "x is null");
        const int64_t d = ix->d;
        add_rows_host(ix, n, [&](int64_t r0, int64_t m, float* dst) {
            std::memcpy(dst, x + r0 * d, (size_t)(m * d) * sizeof(float));
        });
    });
}

int vs_add_device(vs_index* ix, const float* x_dev, int64_t n, void* stream) {
    return guarded([&] {
        check_index(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x_dev) throw VsError(VS_ERR_ARG, "x_dev is null");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        if (ix->ntotal + n > (int64_t)0xFFFFFFF0LL) throw VsError(VS_ERR_ARG, "shard exceeds 2^32 rows");
        ensure_capacity(ix, ix->ntotal + n);
        // NULL is the legacy default stream (torch's default stream handle is 0), never the
        // index's private non-blocking stream: that one is unordered with the caller's producers
        hipStream_t st = (hipStream_t)stream;
        HIP_CHECK(launch_pack_rows(ix->dtype, x_dev, n, ix->d, ix->dpad, ix->data, ix->ntotal, ix->sqn, ix->d_maxsq, st));
        quantize_rows(ix, ix->ntotal, n, st);
        HIP_CHECK(hipStreamSynchronize(st));
        ix->ntotal += n;
        refresh_maxsq(ix);
    });
}

int vs_reserve(vs_index* ix, int64_t n) {
    return guarded([&] {
        check_index(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        if (ix->ntotal + n > (int64_t)0xFFFFFFF0LL) throw VsError(VS_ERR_ARG, "shard exceeds 2^32 rows");
        ensure_capacity(ix, ix->ntotal + n, true);
    });
}

int64_t vs_capacity(const vs_index* ix) { return ix ? ix->cap_rows : -1; }

int vs_add_synthetic(vs_index* ix, uint64_t seed, int64_t global_row0, int64_t n, int normalize) {
    return guarded([&] {
        check_index(ix);
        if (n < 0 || global_row0 < 0) throw VsError(VS_ERR_ARG, "bad synthetic range");
        if (n == 0) return;
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        if (ix->ntotal + n > (int64_t)0xFFFFFFF0LL) throw VsError(VS_ERR_ARG, "shard exceeds 2^32 rows");
        ensure_capacity(ix, ix->ntotal + n);
        HIP_CHECK(launch_synth_rows(ix->dtype, seed, global_row0, n, ix->d, ix->dpad, ix->data, ix->ntotal, normalize,
                                    ix->sqn, ix->d_maxsq, ix->own));
        quantize_rows(ix, ix->ntotal, n, ix->own);
        HIP_CHECK(hipStreamSynchronize(ix->own));
        ix->ntotal += n;
        refresh_maxsq(ix);
    });
}

int vs_synthesize(int device, uint64_t seed, int64_t global_row0, int64_t n, int d, int normalize, int dtype,
                  float* out_dev, void* stream) {
    return guarded([&] {
        if (n < 0 || d <= 0 || global_row0 < 0) throw VsError(VS_ERR_ARG, "bad synthetic shape");
        if (dtype < VS_DTYPE_F32 || dtype > VS_DTYPE_F16) throw VsError(VS_ERR_ARG, "bad dtype");
        if (n == 0) return;
        if (!out_dev) throw VsError(VS_ERR_ARG, "out_dev is null");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw VsError(VS_ERR_DEVICE, "no HIP device available");
        DeviceGuard dg(device);
        HIP_CHECK(launch_synth_f32(dtype, seed, global_row0, n, d, normalize, out_dev, (hipStream_t)stream));
    });
}

int vs_search_device(vs_index* ix, const float* q_dev, int64_t nq, int32_t k, float* D_dev, int64_t* I_dev,
                     double* S64_dev, int64_t id_offset, void* stream) {
    return guarded([&] {
        check_index(ix);
        if (nq < 0) throw VsError(VS_ERR_ARG, "nq must be >= 0");
        if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
        if (screen_depth(k) < k) throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
        if (nq == 0) return;
        if (!q_dev || !I_dev) throw VsError(VS_ERR_ARG, "null device buffer");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        // NULL is the legacy default stream (torch's default stream handle is 0), never the
        // index's private non-blocking stream: that one is unordered with the caller's producers
        hipStream_t st = (hipStream_t)stream;
        if (ix->ntotal == 0) throw VsError(VS_ERR_ARG, "index is empty");
        CtxLease L(ix, st, false);
        search_all(ix, L.c, q_dev, nq, k, screen_depth(k), D_dev, I_dev, S64_dev, nullptr, id_offset, st,
                   kOptimisticSeedRank);
    });
}

int vs_search_device_exact(vs_index* ix, const float* q_dev, int64_t nq, int32_t k, float* D_dev, int64_t* I_dev,
                           double* S64_dev, int64_t id_offset, void* stream) {
    return guarded([&] {
        check_index(ix);
        if (nq < 0) throw VsError(VS_ERR_ARG, "nq must be >= 0");
        if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
        if (screen_depth(k) < k) throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
        if (nq == 0) return;
        if (!q_dev || !I_dev) throw VsError(VS_ERR_ARG, "null device buffer");
        if (ix->ntotal == 0) throw VsError(VS_ERR_ARG, "index is empty");
        search_exact_device(ix, q_dev, nq, k, I_dev, S64_dev, (hipStream_t)stream, D_dev, id_offset, /*async*/ true);
    });
}

int vs_two_phase_ok(vs_index* ix, int64_t nq, int32_t k) {
    if (!ix) return VS_ERR_ARG;
    return two_phase_ok(ix, nq, k) ? 1 : 0;
}

int vs_search_device_phase_a(vs_index* ix, const float* q_dev, int64_t nq, int32_t k, int32_t world,
                             int64_t id_offset, double* S_a, int64_t* I_a, int32_t stride, void* stream,
                             vs_pending** out) {
    return guarded([&] {
        if (!out || !q_dev || !S_a || !I_a) throw VsError(VS_ERR_ARG, "null argument");
        *out = nullptr;
        if (screen_depth(k) < k) throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
        *out = search_phase_a(ix, q_dev, nq, k, world, id_offset, S_a, I_a, stride, (hipStream_t)stream);
    });
}

int vs_search_device_phase_b(vs_pending* p, const double* floor_S, float* D_dev, int64_t* I_dev, double* S64_dev,
                             int32_t stride, void* stream) {
    return guarded([&] {
        if (!p) throw VsError(VS_ERR_ARG, "null pending search");
        if (!floor_S || !I_dev) {
            search_pending_free(p);
            throw VsError(VS_ERR_ARG, "null device buffer");
        }
        search_phase_b(p, floor_S, D_dev, I_dev, S64_dev, stride, (hipStream_t)stream);
    });
}

void vs_search_pending_free(vs_pending* p) { search_pending_free(p); }

int vs_search(vs_index* ix, const float* q, int64_t nq, int32_t k, float* D, int64_t* I) {
    return guarded([&] {
        check_index(ix);
        if (nq < 0) throw VsError(VS_ERR_ARG, "nq must be >= 0");
        if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
        if (nq == 0) return;
        if (!q || !D || !I) throw VsError(VS_ERR_ARG, "null host buffer");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        const float fillD = ix->metric == VS_METRIC_IP ? -3.402823466e+38f : 3.402823466e+38f;
        if (ix->ntotal == 0) {
            for (int64_t i = 0; i < nq * k; ++i) {
                D[i] = fillD;
                I[i] = -1;
            }
            return;
        }
        // k beyond the rows present: search min(k, ntotal), pad the rest (faiss layout)
        const int kk = (int)std::min<int64_t>(k, ix->ntotal);
        if (kk > KP_MAX * 4 / 5) throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
        CtxLease L(ix, nullptr, true);
        Ctx* c = L.c;
        hipStream_t st = c->stream;
        // The caller's buffers are pageable: queries and results go through pinned staging of at
        // most kPinnedStageCap bytes per context, in chunks of queries (whole MFMA batches when a
        // chunk holds more than one), so a huge batch never pins its whole size for the index's life.
        const size_t per_q = std::max((size_t)ix->d * sizeof(float), (size_t)kk * (sizeof(int64_t) + sizeof(float)) + sizeof(int));
        int64_t chunk = std::max<int64_t>(1, (int64_t)(kPinnedStageCap / per_q));
        if (chunk >= MFMA_QB) chunk = chunk / MFMA_QB * MFMA_QB;
        chunk = std::min(chunk, nq);
        c->qdev.ensure((size_t)chunk * ix->d * sizeof(float));
        c->outD.ensure((size_t)kk * sizeof(float));
        c->outI.ensure((size_t)kk * sizeof(int64_t));
        c->cert.ensure(sizeof(int));
        c->hq.ensure((size_t)chunk * ix->d * sizeof(float));
        // device and pinned host blocks share one layout [I int64 | D fp32 | cert int]
        const size_t obytes_max = (size_t)chunk * kk * (sizeof(int64_t) + sizeof(float)) + (size_t)chunk * sizeof(int);
        c->hout.ensure(obytes_max);
        c->outAll.ensure(obytes_max);
        const int Kp = screen_depth(kk);
        for (int64_t q0 = 0; q0 < nq; q0 += chunk) {
            const int64_t m = std::min(chunk, nq - q0);
            std::memcpy(c->hq.p, q + q0 * ix->d, (size_t)m * ix->d * sizeof(float));
            HIP_CHECK(hipMemcpyAsync(c->qdev.p, c->hq.p, (size_t)m * ix->d * sizeof(float), hipMemcpyHostToDevice, st));
            const size_t obytes = (size_t)m * kk * (sizeof(int64_t) + sizeof(float)) + (size_t)m * sizeof(int);
            int64_t* Ik = (int64_t*)c->hout.p;
            float* Dk = (float*)(Ik + (size_t)m * kk);
            int* cert_h = (int*)(Dk + (size_t)m * kk);
            int64_t* Id = c->outAll.as<int64_t>();
            float* Dd = (float*)(Id + (size_t)m * kk);
            int* cert_d = (int*)(Dd + (size_t)m * kk);
            search_all(ix, c, c->qdev.as<float>(), m, kk, Kp, Dd, Id, nullptr, cert_d, 0, st, kOptimisticSeedRank);
            HIP_CHECK(hipMemcpyAsync(c->hout.p, c->outAll.p, obytes, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            // exactness certificate failed for some queries (near-ties deeper than the margin):
            // re-screen those queries one at a time with a 4x deeper candidate set; past the
            // deepest screen (more than KP_MAX rows tied within its margin) the exact full scan
            for (int64_t qi = 0; qi < m; ++qi) {
                int Kr = Kp;
                while (!cert_h[qi]) {
                    if (Kr < 0) throw VsError(VS_ERR_INTERNAL, "full scan left a query uncertified");
                    if (Kr >= KP_MAX || Kr >= ix->ntotal) {
                        HIP_CHECK(hipMemsetAsync(c->cert.p, 0, sizeof(int), st));
                        full_scan_block(ix, c, c->qdev.as<float>() + qi * ix->d, 1, kk, c->outD.as<float>(),
                                        c->outI.as<int64_t>(), nullptr, c->cert.as<int>(), 0, st, nullptr);
                        Kr = -1;
                    } else {
                        Kr = (int)std::min<int64_t>(std::min<int64_t>((int64_t)Kr * 4, KP_MAX), round_up(ix->ntotal, 16));
                        search_all(ix, c, c->qdev.as<float>() + qi * ix->d, 1, kk, Kr, c->outD.as<float>(),
                                   c->outI.as<int64_t>(), nullptr, c->cert.as<int>(), 0, st, /*safe seed*/ 0);
                    }
                    HIP_CHECK(hipMemcpyAsync(Dk + qi * kk, c->outD.p, kk * sizeof(float), hipMemcpyDeviceToHost, st));
                    HIP_CHECK(hipMemcpyAsync(Ik + qi * kk, c->outI.p, kk * sizeof(int64_t), hipMemcpyDeviceToHost, st));
                    HIP_CHECK(hipMemcpyAsync(&cert_h[qi], c->cert.p, sizeof(int), hipMemcpyDeviceToHost, st));
                    HIP_CHECK(hipStreamSynchronize(st));
                }
            }
            for (int64_t qi = 0; qi < m; ++qi)
                for (int j = 0; j < k; ++j) {
                    const int64_t o = (q0 + qi) * k + j;
                    if (j < kk) {
                        D[o] = Dk[qi * kk + j];
                        I[o] = Ik[qi * kk + j];
                    } else {
                        D[o] = fillD;
                        I[o] = -1;
                    }
                }
        }
    });
}

int vs_merge_shards_device(int metric, const double* S_in, const int64_t* I_in, int32_t in_stride, int G, int64_t nq,
                           int32_t k, double* S_out, int64_t* I_out, float* D_out, void* stream) {
    return guarded([&] {
        if (G <= 0 || G > 64) throw VsError(VS_ERR_ARG, "G must be in [1, 64]");
        if (k <= 0 || nq < 0) throw VsError(VS_ERR_ARG, "bad k / nq");
        if (in_stride < 1) throw VsError(VS_ERR_ARG, "in_stride must be >= 1");
        if (nq == 0) return;
        HIP_CHECK(launch_merge_shards(metric, S_in, I_in, G, nq, k, S_out, I_out, D_out, (hipStream_t)stream,
                                      in_stride));
    });
}

int vs_seed_select_device(int device, const float* maxima, int32_t M, int64_t nq, int32_t rank, uint64_t* thr,
                          void* stream) {
    return guarded([&] {
        if (M <= 0 || M > 8192 || rank < 1 || nq < 0) throw VsError(VS_ERR_ARG, "bad M / rank / nq");
        if (nq == 0) return;
        DeviceGuard dg(device);
        HIP_CHECK(launch_seed_select(maxima, M, (int)nq, rank, (u64*)thr, (hipStream_t)stream));
    });
}

int vs_reconstruct_n(vs_index* ix, int64_t i0, int64_t n, float* out) {
    return guarded([&] {
        check_index(ix);
        if (n == 0) return;
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        const int64_t d = ix->d;
        read_rows_host(ix, i0, n, [&](int64_t r0, int64_t m, const float* src) {
            std::memcpy(out + r0 * d, src, (size_t)(m * d) * sizeof(float));
        });
    });
}

int vs_reconstruct(vs_index* ix, int64_t id, float* out) { return vs_reconstruct_n(ix, id, 1, out); }

int64_t vs_ntotal(const vs_index* ix) { return ix ? ix->ntotal : -1; }
int vs_dim(const vs_index* ix) { return ix ? ix->d : -1; }
int vs_metric(const vs_index* ix) { return ix ? ix->metric : -1; }
int vs_dtype(const vs_index* ix) { return ix ? ix->dtype : -1; }
int vs_device(const vs_index* ix) { return ix ? ix->device : -1; }

int vs_set_screen(vs_index* ix, int screen) {
    return guarded([&] {
        check_index(ix);
        if (screen != VS_SCREEN_NATIVE && screen != VS_SCREEN_I8) throw VsError(VS_ERR_ARG, "screen must be 0 (native) or 1 (int8)");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        if (screen == ix->screen) return;
        if (screen == VS_SCREEN_NATIVE) {
            HIP_CHECK(hipDeviceSynchronize());  // searches in flight may still read the int8 copy
            free_i8(ix);
            ix->screen = VS_SCREEN_NATIVE;
            return;
        }
        ix->screen = VS_SCREEN_I8;
        ix->dpad8 = (int)std::max<int64_t>(round_up(ix->d, 64), 128);  // >= 2 K-steps per tile (see dpad)
        try {
            HIP_CHECK(hipMemsetAsync(ix->d_maxsq + 2, 0, 2 * sizeof(unsigned), ix->own));
            HIP_CHECK(hipMemsetAsync(ix->d_maxsq + 5, 0, 3 * sizeof(unsigned), ix->own));
            ensure_capacity_i8(ix);
            quantize_rows(ix, 0, ix->ntotal, ix->own);
            HIP_CHECK(hipStreamSynchronize(ix->own));
            refresh_maxsq(ix);
        } catch (...) {
            free_i8(ix);
            ix->screen = VS_SCREEN_NATIVE;
            throw;
        }
    });
}

int vs_screen(const vs_index* ix) { return ix ? ix->screen : -1; }

// the shared setup of the screen probes: the packed query tile (zeroed on request), every threshold at
// +inf, the candidate buffers; the caller holds the lease and the read lock
static ScreenArgs probe_setup(vs_index* ix, Ctx* c, const float* q_dev, int64_t nq, bool i8, bool zero_queries,
                              hipStream_t st, std::vector<u64>& thr) {
    const int nqb = (int)nq;
    const int64_t tiles = (ix->ntotal + TR - 1) / TR;
    ScreenArgs a{};
    a.n_valid = ix->ntotal;
    a.tiles = (int)tiles;
    a.d = ix->d;
    a.metric = ix->metric;
    a.sqn = ix->sqn;
    a.Kp = MFMA_KP_MAX;
    a.cap = MFMA_CAP;
    a.G = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, ix->num_cu));
    a.lcap = a.G * a.Kp;
    c->gcnt.ensure(sizeof(int) * MFMA_QB);
    c->drop.ensure(sizeof(u64) * MFMA_QB);
    c->fails.ensure(2 * sizeof(int));
    if (i8) {
        c->qtile.ensure((size_t)MFMA_QB * ix->dpad8);
        c->qfac.ensure(sizeof(float2) * MFMA_QB);
        c->qeps.ensure(sizeof(float) * MFMA_QB);
        HIP_CHECK(launch_pack_qtile_i8(q_dev, nqb, ix->d, ix->dpad8, c->qtile.as<uint8_t>(), c->qfac.as<float2>(),
                                       c->qeps.as<float>(), ix->d_maxsq + 2, c->gcnt.as<int>(), c->drop.as<u64>(), st,
                                       c->fails.as<int>(), ix->metric == METRIC_L2 ? ix->d_maxsq : nullptr,
                                       gamma_of(ix->d)));
        a.corpus = ix->data8;
        a.dpad = ix->dpad8;
        a.rsb = ix->rsb;
        a.qfac = c->qfac.as<float2>();
    } else {
        c->qtile.ensure((size_t)MFMA_QB * ix->dpad * ix->es);
        c->qinfo.ensure(sizeof(float) * 2 * MFMA_QB);
        HIP_CHECK(launch_pack_qtile(ix->dtype, q_dev, nqb, ix->d, ix->dpad, c->qtile.as<uint8_t>(),
                                    c->qinfo.as<float>(), c->gcnt.as<int>(), c->drop.as<u64>(), st));
        a.corpus = ix->data;
        a.dpad = ix->dpad;
    }
    if (zero_queries) HIP_CHECK(hipMemsetAsync(c->qtile.p, 0, c->qtile.bytes, st));
    // every query's threshold at the key of +inf: the bound test rejects every column, so the
    // launch is the K loop + the epilogue's bound test with no survivor to insert
    c->thr0.ensure(sizeof(u64) * MFMA_QB);
    thr.assign(MFMA_QB, 0xFF80000000000000ull);
    HIP_CHECK(hipMemcpyAsync(c->thr0.p, thr.data(), sizeof(u64) * MFMA_QB, hipMemcpyHostToDevice, st));
    a.thr0 = c->thr0.as<u64>();
    a.drop = c->drop.as<u64>();
    c->cand.ensure((size_t)a.G * MFMA_QB * a.cap * sizeof(u64));
    c->part.ensure((size_t)MFMA_QB * a.lcap * sizeof(u64));
    a.cand = c->cand.as<u64>();
    a.glist = c->part.as<u64>();
    a.gcnt = c->gcnt.as<int>();
    return a;
}

static void probe_checks(vs_index* ix, const float* q_dev, int64_t nq, int32_t screen, const void* out) {
    check_index(ix);
    if (!q_dev || !out || nq <= GEMV_NQ_MAX || nq > MFMA_QB) throw VsError(VS_ERR_ARG, "screen probe: 9..256 device queries");
    const bool i8 = screen == VS_SCREEN_I8;
    if (i8 && (ix->screen != VS_SCREEN_I8 || !ix->data8 || ix->i8_res || !i8_direct_ok(ix->dpad8)))
        throw VsError(VS_ERR_ARG, "screen probe: the int8 probe needs the int8 direct screen (no group residuals)");
    if (!i8 && !((ix->dtype == DT_BF16 || ix->dtype == DT_F16) && d16_direct_ok(ix->dpad)))
        throw VsError(VS_ERR_ARG, "screen probe: the native probe needs bf16 / f16 rows of the direct screen");
    if (ix->ntotal == 0) throw VsError(VS_ERR_ARG, "index is empty");
}

int vs_screen_probe(vs_index* ix, const float* q_dev, int64_t nq, int32_t screen, int32_t zero_queries, void* stream,
                    float* ms) {
    return guarded([&] {
        check_index(ix);
        probe_checks(ix, q_dev, nq, screen, ms);
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        const bool i8 = screen == VS_SCREEN_I8;
        hipStream_t st = (hipStream_t)stream;
        CtxLease L(ix, st, false);
        Ctx* c = L.c;
        const int nqb = (int)nq;
        std::vector<u64> thr;
        ScreenArgs a = probe_setup(ix, c, q_dev, nq, i8, zero_queries != 0, st, thr);
        // kProbeReps launches back to back (the cadence of the timed steps, no host gap between
        // them), each between its own events; the fastest one is reported
        constexpr int kProbeReps = 5;
        hipEvent_t ev[kProbeReps + 1];
        for (hipEvent_t& e : ev) HIP_CHECK(hipEventCreate(&e));
        hipError_t le = hipSuccess;
        HIP_CHECK(hipEventRecord(ev[0], st));
        for (int i = 0; i < kProbeReps && le == hipSuccess; ++i) {
            le = launch_screen_mfma(i8 ? DT_I8 : ix->dtype, a, c->qtile.as<uint8_t>(), nqb, st);
            HIP_CHECK(hipEventRecord(ev[i + 1], st));
        }
        HIP_CHECK(hipEventSynchronize(ev[kProbeReps]));  // (also keeps the host threshold array alive)
        float best = 0.0f;
        hipError_t te = hipSuccess;
        for (int i = 0; i < kProbeReps && te == hipSuccess; ++i) {
            float t = 0.0f;
            te = hipEventElapsedTime(&t, ev[i], ev[i + 1]);
            if (i == 0 || t < best) best = t;
        }
        for (hipEvent_t& e : ev) (void)hipEventDestroy(e);
        HIP_CHECK(le);
        HIP_CHECK(te);
        *ms = best;
    });
}

int vs_k1_probe(vs_index* ix, const float* q_dev, int64_t nq, int32_t screen, int32_t variant, int32_t zero_queries,
                int32_t reps, void* stream, float* ms, unsigned long long* stamps, int32_t* G_out) {
    return guarded([&] {
        check_index(ix);
        probe_checks(ix, q_dev, nq, screen, ms);
        if (!stamps || !G_out || reps < 1 || reps > 64) throw VsError(VS_ERR_ARG, "vs_k1_probe: 1..64 reps, stamps, G_out");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        const bool i8 = screen == VS_SCREEN_I8;
        if (ix->metric != METRIC_IP) throw VsError(VS_ERR_ARG, "vs_k1_probe: inner-product indexes");
        hipStream_t st = (hipStream_t)stream;
        CtxLease L(ix, st, false);
        Ctx* c = L.c;
        const int nqb = (int)nq;
        std::vector<u64> thr;
        ScreenArgs a = probe_setup(ix, c, q_dev, nq, i8, zero_queries != 0, st, thr);
        struct Stamps {  // (DevBuf frees nothing itself)
            DevBuf b;
            ~Stamps() { b.release(); }
        } stb;
        DevBuf& sbuf = stb.b;
        sbuf.ensure(sizeof(unsigned long long) * 4 * (size_t)a.G * (size_t)reps);
        std::vector<hipEvent_t> ev((size_t)reps + 1);
        for (hipEvent_t& e : ev) HIP_CHECK(hipEventCreate(&e));
        hipError_t le = hipSuccess;
        HIP_CHECK(hipEventRecord(ev[0], st));
        for (int r = 0; r < reps && le == hipSuccess; ++r) {
            a.stamps = sbuf.as<unsigned long long>() + (size_t)r * a.G * 4;
            le = launch_k1_probe(variant, i8 ? DT_I8 : ix->dtype, a, c->qtile.as<uint8_t>(), nqb, st);
            HIP_CHECK(hipEventRecord(ev[(size_t)r + 1], st));
        }
        HIP_CHECK(hipEventSynchronize(ev[(size_t)reps]));
        hipError_t te = hipSuccess;
        for (int r = 0; r < reps && te == hipSuccess && le == hipSuccess; ++r)
            te = hipEventElapsedTime(&ms[r], ev[(size_t)r], ev[(size_t)r + 1]);
        for (hipEvent_t& e : ev) (void)hipEventDestroy(e);
        if (le != hipSuccess) throw VsError(VS_ERR_ARG, "vs_k1_probe: variant not available for this screen / index");
        HIP_CHECK(te);
        HIP_CHECK(hipMemcpy(stamps, sbuf.p, sizeof(unsigned long long) * 4 * (size_t)a.G * (size_t)reps,
                            hipMemcpyDeviceToHost));
        *G_out = a.G;
    });
}

int vs_set_k1_schedule(int32_t schedule) {
    return guarded([&] {
        if (schedule != 0 && schedule != 1) throw VsError(VS_ERR_ARG, "K1 schedule: 0 or 1");
        set_k1_schedule(schedule);
    });
}
int vs_k1_schedule(void) { return k1_schedule(); }

int vs_set_scan_limit(vs_index* ix, int64_t bytes) {
    return guarded([&] {
        check_index(ix);
        if (bytes < 0) throw VsError(VS_ERR_ARG, "scan limit must be >= 0");
        ix->scan_limit.store(bytes);
    });
}

int vs_set_timing(vs_index* ix, int enable) {
    return guarded([&] {
        check_index(ix);
        ix->timing.store(enable != 0);
    });
}

int vs_timing_fetch(vs_index* ix, float* ms, int cap, int* kernel_kind) {
    int count = 0;
    int rc = guarded([&] {
        check_index(ix);
        DeviceGuard dg(ix->device);
        std::lock_guard<std::mutex> g(ix->tmtx);
        for (auto& pr : ix->tev) {
            HIP_CHECK(hipEventSynchronize(pr.second));
            float t = 0.0f;
            HIP_CHECK(hipEventElapsedTime(&t, pr.first, pr.second));
            if (ms && count < cap) ms[count] = t;
            ++count;
            hipEventDestroy(pr.first);
            hipEventDestroy(pr.second);
        }
        ix->tev.clear();
        if (kernel_kind) *kernel_kind = ix->last_kernel_kind;
    });
    return rc == VS_OK ? std::min(count, cap) : rc;
}

int64_t vs_host_staging_bytes(vs_index* ix) {
    if (!ix) return -1;
    std::lock_guard<std::mutex> g(ix->pool_mtx);
    int64_t b = 0;
    for (const Ctx* c : ix->pool_all) b += (int64_t)(c->hq.bytes + c->hout.bytes);
    return b;
}

int64_t vs_screen_copy_bytes(vs_index* ix) {
    if (!ix) return -1;
    if (!ix->data8) return 0;
    const int64_t rows = ix->cap8;
    return (rows / TR) * (int64_t)TR * ix->dpad8 + rows * (int64_t)sizeof(uint32_t) +
           ix->gcap * ix->dpad8 * (int64_t)sizeof(uint16_t);
}

int vs_screen_state(vs_index* ix, double* out, int cap) {
    return guarded([&] {
        check_index(ix);
        if (!out || cap < 0) throw VsError(VS_ERR_ARG, "null output");
        DeviceGuard dg(ix->device);
        HIP_CHECK(hipDeviceSynchronize());
        unsigned bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIP_CHECK(hipMemcpy(bits, ix->d_maxsq, sizeof(bits), hipMemcpyDeviceToHost));
        auto f = [&](int i) {
            float v;
            std::memcpy(&v, &bits[i], 4);
            return (double)v;
        };
        std::lock_guard<std::mutex> g(ix->h_mu);
        health_poll(ix);
        const double v[VS_SCREEN_STATE_N] = {(double)ix->screen, ix->i8_res ? 1.0 : 0.0, (double)bits[6], f(5), f(2),
                                             f(3), (double)ix->i8_log2, (double)ix->i8_route, (double)ix->seed_log2};
        for (int i = 0; i < cap && i < VS_SCREEN_STATE_N; ++i) out[i] = v[i];
    });
}

int64_t vs_full_scan_count(vs_index* ix) {
    int64_t v = -1;
    int rc = guarded([&] {
        check_index(ix);
        DeviceGuard dg(ix->device);
        HIP_CHECK(hipDeviceSynchronize());
        unsigned u = 0;
        HIP_CHECK(hipMemcpy(&u, ix->d_unres, sizeof(unsigned), hipMemcpyDeviceToHost));
        v = u;
    });
    return rc == VS_OK ? v : rc;
}

int64_t vs_uncertified_count(vs_index* ix) {
    int64_t v = -1;
    int rc = guarded([&] {
        check_index(ix);
        DeviceGuard dg(ix->device);
        HIP_CHECK(hipDeviceSynchronize());
        unsigned u = 0;
        HIP_CHECK(hipMemcpy(&u, ix->d_uncert, sizeof(unsigned), hipMemcpyDeviceToHost));
        v = u;
    });
    return rc == VS_OK ? v : rc;
}

}  // extern "C"
