// vs_multi.hip -- one exact flat index over several GPUs of ONE process (include/vs.h "multi-device").
//
// The reference builds one VectorStore in one process (/root/reference/main.py:59-68) over one
// faiss index (utils/vector_store.py:72-81).  This handle keeps that shape -- one object, host
// buffers in and out -- while the rows live on G devices:
//   * rows are dealt in chunks of C = 2^16 consecutive ids: chunk j lives on device j mod G, so
//     incremental adds (add_item, one row at a time) and bulk loads stay balanced, and the global
//     id of local row l of device g is ((l >> 16) * G + g) << 16 | (l & 0xFFFF) -- no id tables;
//   * a search runs every shard's exact search (vs_search_device_exact) concurrently, one host
//     worker and one stream per device; each shard maps its local ids to global ids on its device
//     and copies its (fp64 score, id) lists to device 0 over xGMI (peer copies); device 0 merges
//     the G sorted lists (k_merge_shards: score, then lower global id) and returns D / I;
//   * with the int8 screen on bf16 / f16 shards (vs_two_phase_ok) the search is the two-phase
//     step of the torch-distributed path: phase A on every device, the lists merged on device 0
//     into a floor that goes back to every device, phase B, then the same final merge.
// The merged order is total, so the result equals one index over all rows, bit for bit.
// Concurrency (the reference serves from Flask's threaded server, /root/reference/main.py:353):
// searches hold the handle's lock shared and lease a per-call context (streams, buffers, events,
// counters and one worker per device), so concurrent searches run concurrently on every device;
// adds, resets and screen switches take it exclusively.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "../../include/vs.h"
#include "vs_internal.h"

using namespace vs;

namespace {

constexpr int kChunkBits = 16;
constexpr int64_t kChunk = int64_t(1) << kChunkBits;

__global__ void __launch_bounds__(256) k_local_to_global(int64_t* __restrict__ I, int64_t n, int G, int g) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t l = I[i];
    if (l < 0) return;
    I[i] = ((((l >> kChunkBits) * G) + g) << kChunkBits) | (l & (kChunk - 1));
}

// persistent worker per device: run(job) hands a job to every worker and waits for all
struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
    std::vector<std::string> errs;
    std::vector<int> codes;

    explicit Pool(int n) : errs(n), codes(n, VS_OK) {
        for (int w = 0; w < n; ++w)
            th.emplace_back([this, w] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int)> j;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                    }
                    int code = VS_OK;
                    std::string msg;
                    try {
                        j(w);
                    } catch (const VsError& e) {
                        code = e.code;
                        msg = e.what();
                    } catch (const std::exception& e) {
                        code = VS_ERR_INTERNAL;
                        msg = e.what();
                    }
                    std::lock_guard<std::mutex> lk(mu);
                    codes[w] = code;
                    errs[w] = msg;
                    if (--pending == 0) done_cv.notify_all();
                }
            });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
    // runs f(w) on every worker w; rethrows the first worker failure
    void run(const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> lk(mu);
        job = f;
        pending = (int)th.size();
        ++gen;
        cv.notify_all();
        done_cv.wait(lk, [&] { return pending == 0; });
        for (size_t w = 0; w < th.size(); ++w)
            if (codes[w] != VS_OK) throw VsError(codes[w], "device shard " + std::to_string(w) + ": " + errs[w]);
    }
};

void throw_rc(int rc) {
    if (rc != VS_OK) throw VsError(rc, vs_last_error());
}

}  // namespace

// one search's resources on every device, leased per call
struct MCtx {
    std::vector<hipStream_t> st;
    std::vector<DevBuf> qdev, S, I;           // per device: queries, per-shard lists
    std::vector<DevBuf> floor;                // per device: the two-phase floor (device 0's merged phase-A lists)
    std::vector<hipEvent_t> ready;            // per device: its lists landed on device 0
    DevBuf gS, gI, oS, oI, oD;                // device 0: gathered [G][nq][k] lists, merged outputs
    DevBuf fS, fI, fD;                        // device 0: the merged phase-A lists (two-phase step)
    hipEvent_t floor_ready = nullptr;         // device 0: the floor is merged
    Pool* pool = nullptr;                     // one worker per device
};

struct vs_multi {
    int d = 0, metric = 0, dtype = 0, G = 0;
    std::vector<int> dev;
    std::vector<vs_index*> ix;
    int64_t ntotal = 0;
    std::shared_mutex rw;   // searches / reads shared; adds, resets, screen switches exclusive
    std::mutex pool_mu;     // the shared worker pool of the non-search jobs
    Pool* pool = nullptr;
    std::mutex ctx_mu;      // search contexts: every one ever made, the idle ones
    std::vector<MCtx*> ctx_all, ctx_idle;
};

namespace {

// rows [r0, r0 + n) of the global id space split into per-device contiguous pieces, in order
struct Piece {
    int g;
    int64_t src;  // offset (rows) into the caller's batch
    int64_t n;
};
std::vector<std::vector<Piece>> split_rows(int G, int64_t r0, int64_t n) {
    std::vector<std::vector<Piece>> out(G);
    int64_t i = 0;
    while (i < n) {
        const int64_t gid = r0 + i;
        const int64_t chunk = gid >> kChunkBits;
        const int64_t m = std::min(n - i, ((chunk + 1) << kChunkBits) - gid);
        out[(int)(chunk % G)].push_back({(int)(chunk % G), i, m});
        i += m;
    }
    return out;
}

void locate(const vs_multi* m, int64_t id, int* g, int64_t* local) {
    const int64_t chunk = id >> kChunkBits;
    *g = (int)(chunk % m->G);
    *local = ((chunk / m->G) << kChunkBits) | (id & (kChunk - 1));
}

}  // namespace

extern "C" {

namespace {

void destroy_ctx(vs_multi* m, MCtx* c) {
    delete c->pool;
    for (int g = 0; g < (int)c->st.size(); ++g) {
        DeviceGuard dg(m->dev[g]);
        if (c->st[g]) (void)hipStreamSynchronize(c->st[g]);
        for (DevBuf* b : {&c->qdev[g], &c->S[g], &c->I[g], &c->floor[g]}) b->release();
        if (c->ready[g]) (void)hipEventDestroy(c->ready[g]);
        if (c->st[g]) (void)hipStreamDestroy(c->st[g]);
    }
    if (!m->dev.empty()) {
        DeviceGuard dg(m->dev[0]);
        for (DevBuf* b : {&c->gS, &c->gI, &c->oS, &c->oI, &c->oD, &c->fS, &c->fI, &c->fD}) b->release();
        if (c->floor_ready) (void)hipEventDestroy(c->floor_ready);
    }
    delete c;
}

MCtx* make_ctx(vs_multi* m) {
    MCtx* c = new MCtx();
    const int G = m->G;
    c->st.assign(G, nullptr);
    c->ready.assign(G, nullptr);
    c->qdev.resize(G);
    c->S.resize(G);
    c->I.resize(G);
    c->floor.resize(G);
    try {
        for (int g = 0; g < G; ++g) {
            DeviceGuard dg(m->dev[g]);
            HIP_CHECK(hipStreamCreateWithFlags(&c->st[g], hipStreamNonBlocking));
            HIP_CHECK(hipEventCreateWithFlags(&c->ready[g], hipEventDisableTiming));
        }
        {
            DeviceGuard dg(m->dev[0]);
            HIP_CHECK(hipEventCreateWithFlags(&c->floor_ready, hipEventDisableTiming));
        }
        c->pool = new Pool(G);
    } catch (...) {
        destroy_ctx(m, c);
        throw;
    }
    return c;
}

// a search context for one call: an idle one, or a new one (concurrency grows the set)
struct CtxLease {
    vs_multi* m;
    MCtx* c;
    explicit CtxLease(vs_multi* mm) : m(mm), c(nullptr) {
        {
            std::lock_guard<std::mutex> lk(m->ctx_mu);
            if (!m->ctx_idle.empty()) {
                c = m->ctx_idle.back();
                m->ctx_idle.pop_back();
                return;
            }
        }
        c = make_ctx(m);
        std::lock_guard<std::mutex> lk(m->ctx_mu);
        m->ctx_all.push_back(c);
    }
    ~CtxLease() {
        std::lock_guard<std::mutex> lk(m->ctx_mu);
        m->ctx_idle.push_back(c);
    }
};

// Two-phase step over the devices (every shard non-empty and two_phase_ok): phase A on every
// device -> its lists (global ids) to device 0 -> merged there into the floor -> the floor to every
// device -> phase B (each shard's exact top-k, certified against the floor; its fallback round
// counts into this call's counter) -> the lists to device 0's gather buffers.  The caller merges
// them (the same final merge as the one-phase step).  A pending phase A is freed on every error.
void multi_search_two_phase(vs_multi* m, MCtx* c, const float* q, int64_t nq, int kk) {
    const int G = m->G;
    const size_t lb = (size_t)nq * kk;
    {
        DeviceGuard dg(m->dev[0]);
        c->fS.ensure(lb * sizeof(double));
        c->fI.ensure(lb * sizeof(int64_t));
        c->fD.ensure(lb * sizeof(float));
    }
    std::vector<vs_pending*> pend(G, nullptr);
    auto free_all = [&] {
        for (int g = 0; g < G; ++g) {
            if (pend[g]) {
                DeviceGuard dg(m->dev[g]);
                search_pending_free(pend[g]);
                pend[g] = nullptr;
            }
        }
    };
    try {
        c->pool->run([&](int g) {  // phase A
            DeviceGuard dg(m->dev[g]);
            hipStream_t s = c->st[g];
            c->qdev[g].ensure((size_t)nq * m->d * sizeof(float));
            c->S[g].ensure(lb * sizeof(double));
            c->I[g].ensure(lb * sizeof(int64_t));
            c->floor[g].ensure(lb * sizeof(double));
            HIP_CHECK(hipMemcpyAsync(c->qdev[g].p, q, (size_t)nq * m->d * sizeof(float), hipMemcpyHostToDevice, s));
            int64_t* Ig = c->I[g].as<int64_t>();
            pend[g] = search_phase_a(m->ix[g], c->qdev[g].as<float>(), nq, kk, G, 0, c->S[g].as<double>(), Ig, 1, s);
            hipLaunchKernelGGL(k_local_to_global, dim3((unsigned)((lb + 255) / 256)), dim3(256), 0, s, Ig, (int64_t)lb, G, g);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyPeerAsync(c->gS.as<double>() + lb * g, m->dev[0], c->S[g].p, m->dev[g], lb * sizeof(double), s));
            HIP_CHECK(hipMemcpyPeerAsync(c->gI.as<int64_t>() + lb * g, m->dev[0], Ig, m->dev[g], lb * sizeof(int64_t), s));
            HIP_CHECK(hipEventRecord(c->ready[g], s));
        });
        {  // the floor: the merged phase-A lists (a lower bound of every query's global k-th best)
            DeviceGuard dg(m->dev[0]);
            hipStream_t s0 = c->st[0];
            for (int g = 1; g < G; ++g) HIP_CHECK(hipStreamWaitEvent(s0, c->ready[g], 0));
            HIP_CHECK(launch_merge_shards(m->metric, c->gS.as<double>(), c->gI.as<int64_t>(), G, nq, kk, c->fS.as<double>(),
                                          c->fI.as<int64_t>(), c->fD.as<float>(), s0));
            HIP_CHECK(hipEventRecord(c->floor_ready, s0));
        }
        c->pool->run([&](int g) {  // phase B
            DeviceGuard dg(m->dev[g]);
            hipStream_t s = c->st[g];
            const double* fl = c->fS.as<double>();
            if (g != 0) {  // device 0's floor over xGMI
                HIP_CHECK(hipStreamWaitEvent(s, c->floor_ready, 0));
                HIP_CHECK(hipMemcpyPeerAsync(c->floor[g].p, m->dev[g], c->fS.p, m->dev[0], lb * sizeof(double), s));
                fl = c->floor[g].as<double>();
            }
            int64_t* Ig = c->I[g].as<int64_t>();
            vs_pending* p = pend[g];
            pend[g] = nullptr;  // (phase B frees it, on success and on every error)
            search_phase_b(p, fl, nullptr, Ig, c->S[g].as<double>(), 1, s);
            hipLaunchKernelGGL(k_local_to_global, dim3((unsigned)((lb + 255) / 256)), dim3(256), 0, s, Ig, (int64_t)lb, G, g);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyPeerAsync(c->gS.as<double>() + lb * g, m->dev[0], c->S[g].p, m->dev[g], lb * sizeof(double), s));
            HIP_CHECK(hipMemcpyPeerAsync(c->gI.as<int64_t>() + lb * g, m->dev[0], Ig, m->dev[g], lb * sizeof(int64_t), s));
            HIP_CHECK(hipEventRecord(c->ready[g], s));
        });
    } catch (...) {
        free_all();
        throw;
    }
}

}  // namespace

int vs_multi_create(int d, int metric, int dtype, int n_dev, const int* dev_ids, vs_multi** out) {
    return guarded([&] {
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        *out = nullptr;
        if (n_dev <= 0 || n_dev > 64 || !dev_ids) throw VsError(VS_ERR_ARG, "n_dev must be in [1, 64] with a device list");
        vs_multi* m = new vs_multi();
        m->d = d;
        m->metric = metric;
        m->dtype = dtype;
        m->G = n_dev;
        try {
            for (int g = 0; g < n_dev; ++g) {
                m->dev.push_back(dev_ids[g]);
                vs_index* x = nullptr;
                throw_rc(vs_create(d, metric, dtype, dev_ids[g], &x));
                m->ix.push_back(x);
                if (dev_ids[g] != dev_ids[0]) {
                    // xGMI peer paths both ways (best effort: copies work either way): the lists go
                    // device g -> device 0, the two-phase floor device 0 -> device g
                    for (int dir = 0; dir < 2; ++dir) {
                        const int from = dir == 0 ? dev_ids[g] : dev_ids[0], to = dir == 0 ? dev_ids[0] : dev_ids[g];
                        DeviceGuard dg(from);
                        int can = 0;
                        if (hipDeviceCanAccessPeer(&can, from, to) == hipSuccess && can)
                            (void)hipDeviceEnablePeerAccess(to, 0);  // (already enabled: ignored)
                        (void)hipGetLastError();
                    }
                }
            }
            m->pool = new Pool(n_dev);
        } catch (...) {
            vs_multi_destroy(m);
            throw;
        }
        *out = m;
    });
}

void vs_multi_destroy(vs_multi* m) {
    if (!m) return;
    for (MCtx* c : m->ctx_all) destroy_ctx(m, c);
    delete m->pool;
    for (int g = 0; g < (int)m->ix.size(); ++g) {
        DeviceGuard dg(m->dev[g]);
        (void)hipDeviceSynchronize();
        vs_destroy(m->ix[g]);
    }
    delete m;
}

namespace {
// append n global rows on the shards (add(g, piece) per shard piece, the devices in parallel); if
// any shard fails, the shards that took their rows are truncated back, so the shard row counts
// always match the chunk dealing of ntotal rows (global ids stay arithmetic); caller holds rw
// exclusively
void multi_append(vs_multi* m, int64_t n, const std::function<void(int, const Piece&)>& add) {
    const auto pieces = split_rows(m->G, m->ntotal, n);
    std::vector<int64_t> before(m->G);
    for (int g = 0; g < m->G; ++g) before[g] = vs_ntotal(m->ix[g]);
    try {
        std::lock_guard<std::mutex> pl(m->pool_mu);
        m->pool->run([&](int g) {
            for (const Piece& p : pieces[g]) add(g, p);
        });
    } catch (...) {
        for (int g = 0; g < m->G; ++g) {
            try {
                if (vs_ntotal(m->ix[g]) > before[g]) truncate_rows(m->ix[g], before[g]);
            } catch (...) {
            }
        }
        throw;
    }
    m->ntotal += n;
    const auto want = split_rows(m->G, 0, m->ntotal);
    for (int g = 0; g < m->G; ++g) {
        int64_t rows = 0;
        for (const Piece& p : want[g]) rows += p.n;
        if (vs_ntotal(m->ix[g]) != rows)
            throw VsError(VS_ERR_INTERNAL, "multi-device add: shard " + std::to_string(g) + " holds " +
                                               std::to_string(vs_ntotal(m->ix[g])) + " rows, expected " +
                                               std::to_string(rows));
    }
}
}  // namespace

int vs_multi_add(vs_multi* m, const float* x, int64_t n) {
    return guarded([&] {
        if (!m) throw VsError(VS_ERR_ARG, "null handle");
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x) throw VsError(VS_ERR_ARG, "x is null");
        std::unique_lock<std::shared_mutex> lk(m->rw);
        multi_append(m, n, [&](int g, const Piece& p) { throw_rc(vs_add(m->ix[g], x + p.src * m->d, p.n)); });
    });
}

int vs_multi_add_from_file(vs_multi* m, const char* path, int64_t byte_offset, int64_t n) {
    return guarded([&] {
        if (!m || !path) throw VsError(VS_ERR_ARG, "null argument");
        if (n < 0 || byte_offset < 0) throw VsError(VS_ERR_ARG, "bad range");
        if (n == 0) return;
        std::unique_lock<std::shared_mutex> lk(m->rw);
        multi_append(m, n, [&](int g, const Piece& p) {
            throw_rc(vs_add_from_file(m->ix[g], path, byte_offset + p.src * m->d * (int64_t)sizeof(float), p.n));
        });
    });
}

int vs_multi_write_rows_to_file(vs_multi* m, const char* path, int64_t byte_offset, int64_t i0, int64_t n) {
    return guarded([&] {
        if (!m || !path) throw VsError(VS_ERR_ARG, "null argument");
        if (i0 < 0 || n < 0 || i0 + n > m->ntotal) throw VsError(VS_ERR_ARG, "row range out of bounds");
        if (n == 0) return;
        std::shared_lock<std::shared_mutex> lk(m->rw);
        std::lock_guard<std::mutex> pl(m->pool_mu);
        const auto pieces = split_rows(m->G, i0, n);
        m->pool->run([&](int g) {  // disjoint file ranges: the devices write concurrently
            for (const Piece& p : pieces[g]) {
                int gg;
                int64_t local;
                locate(m, i0 + p.src, &gg, &local);
                throw_rc(vs_write_rows_to_file(m->ix[g], path, byte_offset + p.src * m->d * (int64_t)sizeof(float), local,
                                               p.n));
            }
        });
    });
}

int vs_multi_search(vs_multi* m, const float* q, int64_t nq, int32_t k, float* D, int64_t* I) {
    return guarded([&] {
        if (!m) throw VsError(VS_ERR_ARG, "null handle");
        if (nq < 0) throw VsError(VS_ERR_ARG, "nq must be >= 0");
        if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
        if (nq == 0) return;
        if (!q || !D || !I) throw VsError(VS_ERR_ARG, "null host buffer");
        std::shared_lock<std::shared_mutex> lk(m->rw);  // concurrent searches; adds wait
        const float fillD = m->metric == VS_METRIC_IP ? -3.402823466e+38f : 3.402823466e+38f;
        const int kk = (int)std::min<int64_t>(k, m->ntotal);
        if (kk == 0) {
            for (int64_t i = 0; i < nq * k; ++i) {
                D[i] = fillD;
                I[i] = -1;
            }
            return;
        }
        if (kk > KP_MAX * 4 / 5) throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
        const int G = m->G;
        const size_t lb = (size_t)nq * kk;
        CtxLease L(m);
        MCtx* c = L.c;
        {
            DeviceGuard dg(m->dev[0]);
            c->gS.ensure(lb * G * sizeof(double));
            c->gI.ensure(lb * G * sizeof(int64_t));
            c->oS.ensure(lb * sizeof(double));
            c->oI.ensure(lb * sizeof(int64_t));
            c->oD.ensure(lb * sizeof(float));
        }
        // the two-phase step (as the torch-distributed path's, photo_search_engine_amd/distributed.py):
        // every shard's phase A, the merged phase-A lists as a floor shared by all shards, then
        // each shard's phase B scores only its share of the global refine window
        bool two = G > 1;
        for (int g = 0; g < G && two; ++g) two = vs_ntotal(m->ix[g]) > 0 && two_phase_ok(m->ix[g], nq, kk);
        if (two) {
            multi_search_two_phase(m, c, q, nq, kk);
        } else {
        c->pool->run([&](int g) {
            DeviceGuard dg(m->dev[g]);
            hipStream_t s = c->st[g];
            c->qdev[g].ensure((size_t)nq * m->d * sizeof(float));
            c->S[g].ensure(lb * sizeof(double));
            c->I[g].ensure(lb * sizeof(int64_t));
            double* Sg = c->S[g].as<double>();
            int64_t* Ig = c->I[g].as<int64_t>();
            HIP_CHECK(hipMemcpyAsync(c->qdev[g].p, q, (size_t)nq * m->d * sizeof(float), hipMemcpyHostToDevice, s));
            if (vs_ntotal(m->ix[g]) > 0) {
                // exact per shard: uncertified screens are re-searched on this device, queued behind
                // the first pass (no host round trip): the fallback round, then the full scan
                search_exact_device(m->ix[g], c->qdev[g].as<float>(), nq, kk, Ig, Sg, s, nullptr, 0, /*async*/ true);
                hipLaunchKernelGGL(k_local_to_global, dim3((unsigned)((lb + 255) / 256)), dim3(256), 0, s, Ig,
                                   (int64_t)lb, G, g);
                HIP_CHECK(hipGetLastError());
            } else {  // an empty shard contributes only padding
                std::vector<double> ws(lb, m->metric == VS_METRIC_IP ? -1.7976931348623157e308 : 1.7976931348623157e308);
                std::vector<int64_t> wi(lb, -1);
                HIP_CHECK(hipMemcpyAsync(Sg, ws.data(), lb * sizeof(double), hipMemcpyHostToDevice, s));
                HIP_CHECK(hipMemcpyAsync(Ig, wi.data(), lb * sizeof(int64_t), hipMemcpyHostToDevice, s));
                HIP_CHECK(hipStreamSynchronize(s));  // (the host vectors go out of scope)
            }
            // this shard's lists into slot g of device 0's gather buffers (xGMI peer copy)
            HIP_CHECK(hipMemcpyPeerAsync(c->gS.as<double>() + lb * g, m->dev[0], Sg, m->dev[g], lb * sizeof(double), s));
            HIP_CHECK(hipMemcpyPeerAsync(c->gI.as<int64_t>() + lb * g, m->dev[0], Ig, m->dev[g], lb * sizeof(int64_t), s));
            HIP_CHECK(hipEventRecord(c->ready[g], s));
        });
        }
        DeviceGuard dg(m->dev[0]);
        hipStream_t s0 = c->st[0];
        for (int g = 1; g < G; ++g) HIP_CHECK(hipStreamWaitEvent(s0, c->ready[g], 0));
        HIP_CHECK(launch_merge_shards(m->metric, c->gS.as<double>(), c->gI.as<int64_t>(), G, nq, kk, c->oS.as<double>(),
                                      c->oI.as<int64_t>(), c->oD.as<float>(), s0));
        std::vector<float> Dk(lb);
        std::vector<int64_t> Ik(lb);
        HIP_CHECK(hipMemcpyAsync(Dk.data(), c->oD.p, lb * sizeof(float), hipMemcpyDeviceToHost, s0));
        HIP_CHECK(hipMemcpyAsync(Ik.data(), c->oI.p, lb * sizeof(int64_t), hipMemcpyDeviceToHost, s0));
        HIP_CHECK(hipStreamSynchronize(s0));  // (s0 waited for every shard's ready event)
        for (int64_t a = 0; a < nq; ++a)
            for (int j = 0; j < k; ++j) {
                D[a * k + j] = j < kk ? Dk[a * kk + j] : fillD;
                I[a * k + j] = j < kk ? Ik[a * kk + j] : -1;
            }
    });
}

int vs_multi_reconstruct_n(vs_multi* m, int64_t i0, int64_t n, float* out) {
    return guarded([&] {
        if (!m || !out) throw VsError(VS_ERR_ARG, "null argument");
        if (i0 < 0 || n < 0 || i0 + n > m->ntotal) throw VsError(VS_ERR_ARG, "reconstruct range out of bounds");
        if (n == 0) return;
        std::shared_lock<std::shared_mutex> lk(m->rw);
        std::lock_guard<std::mutex> pl(m->pool_mu);
        const auto pieces = split_rows(m->G, i0, n);
        m->pool->run([&](int g) {
            for (const Piece& p : pieces[g]) {
                int gg;
                int64_t local;
                locate(m, i0 + p.src, &gg, &local);
                throw_rc(vs_reconstruct_n(m->ix[g], local, p.n, out + p.src * m->d));
            }
        });
    });
}

int vs_multi_reset(vs_multi* m) {
    return guarded([&] {
        if (!m) throw VsError(VS_ERR_ARG, "null handle");
        std::unique_lock<std::shared_mutex> lk(m->rw);
        for (vs_index* x : m->ix) throw_rc(vs_reset(x));
        m->ntotal = 0;
    });
}

int vs_multi_set_screen(vs_multi* m, int screen) {
    return guarded([&] {
        if (!m) throw VsError(VS_ERR_ARG, "null handle");
        std::unique_lock<std::shared_mutex> lk(m->rw);
        std::lock_guard<std::mutex> pl(m->pool_mu);
        m->pool->run([&](int g) { throw_rc(vs_set_screen(m->ix[g], screen)); });
    });
}

int64_t vs_multi_ntotal(const vs_multi* m) { return m ? m->ntotal : -1; }
int vs_multi_ndev(const vs_multi* m) { return m ? m->G : -1; }
int64_t vs_multi_shard_rows(const vs_multi* m, int g) {
    return (m && g >= 0 && g < m->G) ? vs_ntotal(m->ix[g]) : -1;
}

}  // extern "C"
