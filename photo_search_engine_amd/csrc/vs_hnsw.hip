// vs_hnsw.hip -- HNSW graph search of libvs (include/vs.h "HNSW graph search").
//
// The reference's index_type="hnsw" is faiss.IndexHNSWFlat (/root/reference/utils/vector_store.py
// :73-78), searched at :191.  A vs_hnsw holds a graph in faiss's HNSW layout over the rows of a
// flat vs_index on that index's device; vs_hnsw_search runs k_hnsw_search (vs_kernels.hip: faiss
// HNSW::search with the flat path's exact canonical distances, one workgroup per query) in chunks
// of queries, each with its own zeroed visited bitmap.  Results equal oracle/hnsw_oracle.py.
// vs_hnsw_prune runs k_hnsw_prune (faiss HNSW::shrink_neighbor_list, the graph build's neighbour
// selection) for a batch of nodes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/vs.h"
#include "vs_internal.h"

using namespace vs;

struct vs_hnsw {
    vs_index* ix = nullptr;  // not owned
    int device = 0;
    int64_t n = 0;
    int entry = -1, max_level = -1, nbmax = 1;
    DevBuf offsets, neighbors, cum, vis, qdev, outD, outI, ppos, pval;
    std::vector<int32_t> levels_h, cum_h;  // host copies: vs_hnsw_patch validates against them
    std::vector<uint64_t> offsets_h;
    hipStream_t st = nullptr;
    std::mutex mtx;  // searches on one handle are serialised (shared workspaces)
};

namespace {

constexpr size_t kVisitedBytes = 256u << 20;  // visited bitmaps of one query chunk

void fail(const std::string& m) { throw VsError(VS_ERR_ARG, "hnsw graph: " + m); }

// validate a faiss-layout graph and return its neighbour array with every list cut at its first
// -1 and later duplicates dropped (-1 padded): both leave every faiss search unchanged
std::vector<int32_t> checked_neighbors(int64_t n, const int32_t* levels, const uint64_t* offsets,
                                       const int32_t* neighbors, const int32_t* cum, int n_cum, int entry,
                                       int max_level, int* nbmax) {
    if (n_cum < 2 || cum[0] != 0) fail("cum_nneighbor_per_level must start at 0 and cover a level");
    const int nlev = n_cum - 1;
    *nbmax = 1;
    for (int l = 0; l < nlev; ++l) {
        if (cum[l + 1] < cum[l]) fail("cum_nneighbor_per_level must not decrease");
        *nbmax = std::max(*nbmax, cum[l + 1] - cum[l]);
    }
    if (*nbmax > HN_NB_MAX) fail("a level holds more than " + std::to_string(HN_NB_MAX) + " neighbours");
    if (n == 0) {
        if (entry != -1) fail("an empty graph has entry point -1");
        return {};
    }
    if (entry < 0 || entry >= n) fail("entry point out of range");
    if (offsets[0] != 0) fail("offsets[0] must be 0");
    for (int64_t i = 0; i < n; ++i) {
        if (levels[i] < 1 || levels[i] > nlev) fail("node level out of range");
        if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] != (uint64_t)cum[levels[i]])
            fail("offsets do not match the node levels");
    }
    if (max_level != levels[entry] - 1) fail("max_level must be the entry point's top level");
    std::vector<int32_t> out(offsets[n], -1);
    std::vector<int64_t> seen(n, -1);  // last (node, level) stamp that listed each id
    for (int64_t i = 0; i < n; ++i)
        for (int l = 0; l < levels[i]; ++l) {
            const uint64_t b = offsets[i] + cum[l], e = offsets[i] + cum[l + 1];
            const int64_t stamp = i * nlev + l;
            uint64_t w = b;
            for (uint64_t j = b; j < e; ++j) {
                const int32_t v = neighbors[j];
                if (v < 0) break;
                if (v >= n) fail("neighbour id out of range");
                if (levels[v] <= l) fail("a neighbour is listed on a level above its own");
                if (seen[v] == stamp) continue;
                seen[v] = stamp;
                out[w++] = v;
            }
        }
    return out;
}

__global__ void __launch_bounds__(256) k_scatter_i32(int32_t* __restrict__ dst, const uint64_t* __restrict__ pos,
                                                     const int32_t* __restrict__ val, int64_t m) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < m) dst[pos[i]] = val[i];
}

}  // namespace

extern "C" {

int vs_hnsw_create(vs_index* index, int64_t n, const int32_t* levels, const uint64_t* offsets,
                   const int32_t* neighbors, const int32_t* cum, int32_t n_cum, int32_t entry_point,
                   int32_t max_level, vs_hnsw** out) {
    return guarded([&] {
        if (!index || !out || n < 0 || !cum || (n > 0 && (!levels || !offsets || !neighbors)))
            throw VsError(VS_ERR_ARG, "vs_hnsw_create: bad arguments");
        *out = nullptr;
        const FlatView fv = flat_view(index);
        int nbmax = 1;
        const std::vector<int32_t> nb =
            checked_neighbors(n, levels, offsets, neighbors, cum, n_cum, entry_point, max_level, &nbmax);
        DeviceGuard g(fv.device);
        vs_hnsw* h = new vs_hnsw();
        try {
            h->ix = index;
            h->device = fv.device;
            h->n = n;
            h->entry = n ? entry_point : -1;
            h->max_level = n ? max_level : -1;
            h->nbmax = nbmax;
            h->levels_h.assign(levels, levels + n);
            h->offsets_h.assign(offsets, offsets + (n > 0 ? n + 1 : 0));
            h->cum_h.assign(cum, cum + n_cum);
            HIP_CHECK(hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking));
            if (n > 0) {
                h->offsets.ensure((size_t)(n + 1) * 8);
                h->neighbors.ensure(std::max<size_t>(nb.size(), 1) * 4);
                HIP_CHECK(hipMemcpyAsync(h->offsets.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, h->st));
                if (!nb.empty())
                    HIP_CHECK(hipMemcpyAsync(h->neighbors.p, nb.data(), nb.size() * 4, hipMemcpyHostToDevice, h->st));
            }
            h->cum.ensure((size_t)n_cum * 4);
            HIP_CHECK(hipMemcpyAsync(h->cum.p, cum, (size_t)n_cum * 4, hipMemcpyHostToDevice, h->st));
            HIP_CHECK(hipStreamSynchronize(h->st));
        } catch (...) {
            vs_hnsw_destroy(h);
            throw;
        }
        *out = h;
    });
}

void vs_hnsw_destroy(vs_hnsw* h) {
    if (!h) return;
    {
        DeviceGuard g(h->device);
        if (h->st) (void)hipStreamSynchronize(h->st);
        for (DevBuf* b : {&h->offsets, &h->neighbors, &h->cum, &h->vis, &h->qdev, &h->outD, &h->outI, &h->ppos, &h->pval})
            b->release();
        if (h->st) (void)hipStreamDestroy(h->st);
    }
    delete h;
}

int64_t vs_hnsw_ntotal(const vs_hnsw* h) { return h ? h->n : -1; }

int vs_hnsw_patch(vs_hnsw* h, int64_t m, const uint64_t* pos, const int32_t* val, int32_t entry_point,
                  int32_t max_level) {
    return guarded([&] {
        if (!h || m < 0 || (m > 0 && (!pos || !val))) throw VsError(VS_ERR_ARG, "vs_hnsw_patch: bad arguments");
        const int64_t n = h->n;
        if (n == 0) {
            if (m > 0) fail("an empty graph has no neighbour slots");
            return;
        }
        if (entry_point < 0 || entry_point >= n) fail("entry point out of range");
        if (max_level != h->levels_h[entry_point] - 1) fail("max_level must be the entry point's top level");
        const int nlev = (int)h->cum_h.size() - 1;
        // every slot and id is checked here: the search kernel follows them.  A patch rewrites whole
        // (node, level) lists -- every slot of each list it touches (a slot given twice must carry
        // the same id) -- and each list in the form vs_hnsw_create leaves: distinct ids, then -1s
        std::vector<std::pair<uint64_t, int32_t>> pv((size_t)m);
        for (int64_t i = 0; i < m; ++i) {
            if (pos[i] >= h->offsets_h[n]) fail("patch position out of range");
            pv[(size_t)i] = {pos[i], val[i]};
        }
        std::sort(pv.begin(), pv.end());
        size_t w = 0;
        for (size_t i = 0; i < pv.size(); ++i) {
            if (w > 0 && pv[w - 1].first == pv[i].first) {
                if (pv[w - 1].second != pv[i].second) fail("one neighbour slot patched with two ids");
                continue;
            }
            pv[w++] = pv[i];
        }
        pv.resize(w);
        std::vector<int32_t> ids;
        for (size_t i = 0; i < pv.size();) {
            const uint64_t p0 = pv[i].first;
            const int64_t node = (int64_t)(std::upper_bound(h->offsets_h.begin(), h->offsets_h.end(), p0) -
                                           h->offsets_h.begin()) - 1;
            const uint64_t rel = p0 - h->offsets_h[node];
            int l = 0;
            while (l + 1 < nlev && rel >= (uint64_t)h->cum_h[l + 1]) ++l;
            const uint64_t lo = h->offsets_h[node] + (uint64_t)h->cum_h[l];
            const uint64_t hi = h->offsets_h[node] + (uint64_t)h->cum_h[l + 1];
            if (p0 != lo || i + (hi - lo) > pv.size() || pv[i + (hi - lo) - 1].first != hi - 1)
                fail("a patch must rewrite whole neighbour lists");
            ids.clear();
            bool ended = false;
            for (uint64_t j = 0; j < hi - lo; ++j) {
                const int32_t v = pv[i + j].second;
                if (v < -1 || v >= n) fail("neighbour id out of range");
                if (v == -1) {
                    ended = true;
                    continue;
                }
                if (ended) fail("a neighbour id after the list's -1 terminator");
                if (h->levels_h[v] <= l) fail("a neighbour is listed on a level above its own");
                ids.push_back(v);
            }
            std::sort(ids.begin(), ids.end());
            if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) fail("a neighbour listed twice in one list");
            i += hi - lo;
        }
        std::lock_guard<std::mutex> lk(h->mtx);
        DeviceGuard g(h->device);
        if (m > 0) {
            h->ppos.ensure((size_t)m * 8);
            h->pval.ensure((size_t)m * 4);
            HIP_CHECK(hipMemcpyAsync(h->ppos.p, pos, (size_t)m * 8, hipMemcpyHostToDevice, h->st));
            HIP_CHECK(hipMemcpyAsync(h->pval.p, val, (size_t)m * 4, hipMemcpyHostToDevice, h->st));
            // (the synchronisation below keeps the caller's pos / val alive for the copies)
            hipLaunchKernelGGL(k_scatter_i32, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, h->st,
                               h->neighbors.as<int32_t>(), h->ppos.as<uint64_t>(), h->pval.as<int32_t>(), m);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipStreamSynchronize(h->st));
        }
        h->entry = entry_point;
        h->max_level = max_level;
    });
}

int vs_hnsw_search(vs_hnsw* h, const float* q, int64_t nq, int32_t k, int32_t ef_search, float* D, int64_t* I) {
    return guarded([&] {
        if (!h || nq < 0 || k < 1 || ef_search < 1 || (nq > 0 && (!q || !D || !I)))
            throw VsError(VS_ERR_ARG, "vs_hnsw_search: bad arguments");
        const int ef = std::max(ef_search, k);
        if (ef > HN_EF_MAX) throw VsError(VS_ERR_ARG, "vs_hnsw_search: max(ef_search, k) > 2048");
        if (nq == 0) return;
        std::lock_guard<std::mutex> lk(h->mtx);
        std::shared_lock<std::shared_mutex> rl(flat_lock(h->ix));
        const FlatView fv = flat_view(h->ix);
        // rows are append-only, so a graph over the first h->n rows stays valid while rows are
        // added behind it (the host searches those exactly and merges); fewer rows = a reset index
        if (fv.ntotal < h->n)
            throw VsError(VS_ERR_ARG, "vs_hnsw_search: the graph covers " + std::to_string(h->n) +
                                          " rows, the index holds only " + std::to_string(fv.ntotal));
        if (hnsw_lds_bytes(fv.d, k, ef, h->nbmax) > 160 * 1024 - 512)
            throw VsError(VS_ERR_ARG, "vs_hnsw_search: k / ef_search too large for one workgroup's LDS");
        DeviceGuard g(h->device);
        const int64_t words = std::max<int64_t>(1, (h->n + 31) / 32);
        const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>({nq, 4096, (int64_t)(kVisitedBytes / (words * 4))}));
        h->vis.ensure((size_t)(chunk * words * 4));
        h->qdev.ensure((size_t)(chunk * fv.d * 4));
        h->outD.ensure((size_t)(chunk * k * 4));
        h->outI.ensure((size_t)(chunk * k * 8));
        HnswArgs a{};
        a.corpus = fv.data;
        a.d = fv.d;
        a.dpad = fv.dpad;
        a.dt = fv.dtype;
        a.metric = fv.metric;
        a.n = h->n;
        a.offsets = h->offsets.as<uint64_t>();
        a.neighbors = h->neighbors.as<int>();
        a.cum = h->cum.as<int>();
        a.entry = h->entry;
        a.max_level = h->max_level;
        a.nbmax = h->nbmax;
        a.k = k;
        a.ef_search = ef_search;
        a.ef = ef;
        a.vis = h->vis.as<uint32_t>();
        a.vis_words = words;
        a.q = h->qdev.as<float>();
        a.D = h->outD.as<float>();
        a.I = h->outI.as<int64_t>();
        for (int64_t q0 = 0; q0 < nq; q0 += chunk) {
            const int64_t m = std::min(chunk, nq - q0);
            HIP_CHECK(hipMemcpyAsync(h->qdev.p, q + q0 * fv.d, (size_t)(m * fv.d * 4), hipMemcpyHostToDevice, h->st));
            HIP_CHECK(hipMemsetAsync(h->vis.p, 0, (size_t)(m * words * 4), h->st));
            HIP_CHECK(launch_hnsw_search(a, (int)m, h->st));
            HIP_CHECK(hipMemcpyAsync(D + q0 * k, h->outD.p, (size_t)(m * k * 4), hipMemcpyDeviceToHost, h->st));
            HIP_CHECK(hipMemcpyAsync(I + q0 * k, h->outI.p, (size_t)(m * k * 8), hipMemcpyDeviceToHost, h->st));
            HIP_CHECK(hipStreamSynchronize(h->st));
        }
    });
}

int vs_hnsw_prune(vs_index* index, int64_t m, const int64_t* nodes, const int32_t* cand, int32_t C, int32_t W,
                  int32_t* out) {
    return guarded([&] {
        if (!index || m < 0 || C < 1 || W < 1 || (m > 0 && (!nodes || !cand || !out)))
            throw VsError(VS_ERR_ARG, "vs_hnsw_prune: bad arguments");
        if (C > HP_C_MAX || W > HN_NB_MAX)
            throw VsError(VS_ERR_ARG, "vs_hnsw_prune: C <= " + std::to_string(HP_C_MAX) + " and W <= " +
                                          std::to_string(HN_NB_MAX));
        if (m == 0) return;
        std::shared_lock<std::shared_mutex> rl(flat_lock(index));
        const FlatView fv = flat_view(index);
        if (hnsw_prune_lds_bytes(fv.d, C, W) > 160 * 1024 - 512)
            throw VsError(VS_ERR_ARG, "vs_hnsw_prune: d / C too large for one workgroup's LDS");
        // every id is checked here: the kernel gathers rows by them
        for (int64_t i = 0; i < m; ++i) {
            if (nodes[i] < 0 || nodes[i] >= fv.ntotal) throw VsError(VS_ERR_ARG, "vs_hnsw_prune: node id out of range");
            const int32_t* c = cand + i * C;
            bool pad = false;
            for (int j = 0; j < C; ++j) {
                if (c[j] < 0) pad = true;
                else if (pad || c[j] >= fv.ntotal)
                    throw VsError(VS_ERR_ARG, "vs_hnsw_prune: candidate ids in range, -1 padding only at the end");
            }
        }
        DeviceGuard g(fv.device);
        hipStream_t st = nullptr;
        HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        DevBuf dn, dc, dout;
        try {
            const int64_t chunk = std::min<int64_t>(m, std::max<int64_t>(1, (int64_t)(256u << 20) / ((int64_t)C * 4)));
            dn.ensure((size_t)chunk * 8);
            dc.ensure((size_t)chunk * C * 4);
            dout.ensure((size_t)chunk * W * 4);
            HnswPruneArgs a{};
            a.corpus = fv.data;
            a.d = fv.d;
            a.dpad = fv.dpad;
            a.dt = fv.dtype;
            a.metric = fv.metric;
            a.nodes = dn.as<int64_t>();
            a.cand = dc.as<int>();
            a.C = C;
            a.W = W;
            a.out = dout.as<int>();
            for (int64_t i0 = 0; i0 < m; i0 += chunk) {
                const int64_t mm = std::min(chunk, m - i0);
                HIP_CHECK(hipMemcpyAsync(dn.p, nodes + i0, (size_t)mm * 8, hipMemcpyHostToDevice, st));
                HIP_CHECK(hipMemcpyAsync(dc.p, cand + i0 * C, (size_t)mm * C * 4, hipMemcpyHostToDevice, st));
                HIP_CHECK(launch_hnsw_prune(a, (int)mm, st));
                HIP_CHECK(hipMemcpyAsync(out + i0 * W, dout.p, (size_t)mm * W * 4, hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
            }
        } catch (...) {
            (void)hipStreamSynchronize(st);
            for (DevBuf* b : {&dn, &dc, &dout}) b->release();
            (void)hipStreamDestroy(st);
            throw;
        }
        for (DevBuf* b : {&dn, &dc, &dout}) b->release();
        HIP_CHECK(hipStreamDestroy(st));
    });
}

}  // extern "C"
