// vs_ivf.hip -- IVF-Flat index of libvs (include/vs.h, "IVF-Flat"; SURVEY.md §8 f2, BASELINE cfg5).
//
// The reference has flat and HNSW indexes only (/root/reference/utils/vector_store.py:51-53,72-81);
// this is the faiss IndexIVFFlat design rebuilt for one MI355X:
//   * coarse quantizer: an exact flat libvs index over the nlist centroids (vs_index, MFMA/GEMV
//     screen + exact refine), used for row assignment (k=1) and query probing (k=nprobe);
//   * inverted lists: chains of pages in ONE HBM page pool; a page is one row tile of the flat
//     layout (TR rows, chunk-major), so every scan read is a full coalesced 1 KiB wave piece.
//     slot = page * TR + row; slot_id[slot] = user id (insertion order);
//   * search: exact probe -> host inversion into (list, page range, <= IVF_QG queries) work items
//     -> k_ivf_scan (GEMV screen, fused threshold top-Kp) -> k_refine (exact fp64 rescoring, slot ->
//     id map, certificate) -> uncertified queries re-searched with a 4x deeper screen.
// Results equal oracle/ivf_oracle.py bit for bit (ids and fp64 scores).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <vector>

#include "../../include/vs.h"
#include "vs_internal.h"

using namespace vs;

struct vs_ivf {
    int d = 0, dpad = 0, nlist = 0, metric = 0, dtype = 0, device = 0, es = 4, num_cu = 256;
    vs_index* coarse = nullptr;
    bool trained = false;
    // page pool
    uint8_t* data = nullptr;
    float* sqn = nullptr;
    uint32_t* slot_id = nullptr;
    int64_t cap_pages = 0, used_pages = 0;
    unsigned* d_flags = nullptr;  // [0] max ||x||^2 bits, [1] uncertified-query counter
    float maxsq = 0.0f;
    std::vector<std::vector<int>> pages;  // page chain of every list
    std::vector<int64_t> list_n;          // rows of every list
    std::vector<int64_t> id_slot;         // storage slot of every id
    int64_t ntotal = 0;
    // device copy of the page tables (CSR), refreshed lazily after adds
    DevBuf d_page_off, d_list_pages, d_list_n;
    std::vector<int> page_off_h;  // host copy of d_page_off
    bool csr_dirty = true;
    // workspaces (add: exclusive lock; search / reconstruct: search_mtx)
    DevBuf tmp_rows, slots, assign_ids;
    DevBuf qdev, probes, items, qp, qinfo, cand, glist, gcnt, cert, outD, outI, rec, next_item;
    DevBuf mqidx, mqtile, mcand, mdesc;
    std::vector<int> desc_h;  // MFMA list scans: workgroup descriptors (MAP_DESC ints each), then
    int n_mdesc = 0;          // per query tile (offset into mqidx, queries)
    DevBuf rq, rD, rI, rS;  // re-search of uncertified queries: gathered queries and their outputs  // MFMA list scans: query indices, query tile, workspaces
    int scan_mode = VS_IVF_SCAN_AUTO;
    int qtile_mode = VS_IVF_QTILE_SPLIT;  // MFMA list scans' first-pass query tiles
    int last_mfma_lists = 0;  // first pass of the last search: MFMA list scans ...
    int last_uncert = 0;      // ... and queries its certificate rejected (re-searched deeper)
    int cur_mfma_lists = 0;
    double last_bytes[2] = {0.0, 0.0}, cur_bytes[2] = {0.0, 0.0};  // pages read by the MFMA / GEMV scans
    std::vector<int64_t> probes_h;
    std::vector<int> cert_h;
    hipStream_t own = nullptr;
    // coarse assignment of added rows: kAssignStreams concurrent exact searches (one 256-row block
    // of the coarse quantizer fills only nlist / 256 workgroups)
    hipStream_t astream[8] = {};
    hipEvent_t aev[9] = {};
    std::shared_mutex rw;
    std::mutex search_mtx;
    std::atomic<bool> timing{false};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
    std::vector<double> tbytes;
};

namespace {

constexpr int kPagesPerItem = 16;  // scan work item: up to 16 pages (4096 rows) of one list (8: +2%, 32: +0.7% scan time)

void check_ivf(const vs_ivf* ix) {
    if (!ix) throw VsError(VS_ERR_ARG, "null IVF index");
}

// A list probed by nql queries costs the GEMV scan ceil(nql / IVF_QG) reads of its pages (items of
// <= 8 queries, each re-reading the list from HBM); the MFMA screen reads them once per query tile
// (qb = 128 split or 256 plain queries), in the one launch shared by all MFMA scans.  Rates
// measured on MI355X: GEMV scan ~76% of HBM peak on evenly probed lists, bf16 MFMA screen ~50%.
bool mfma_scan_pays(const vs_ivf* ix, int64_t np, int nql, int qb) {
    if (ix->dtype == DT_F32 || nql <= 1 || ix->scan_mode == VS_IVF_SCAN_GEMV) return false;
    if (ix->scan_mode == VS_IVF_SCAN_MFMA) return true;
    const double B = (double)tile_bytes(ix->dpad, ix->dtype);
    const double t_gemv = (double)((nql + IVF_QG - 1) / IVF_QG) * (double)np * B / 6.0e12;
    const double t_mfma = (double)((nql + qb - 1) / qb) * (double)np * B / 4.0e12;
    return t_mfma < t_gemv;
}

int64_t rows_per_chunk(int d) { return std::max<int64_t>(1, (int64_t)(256 << 20) / ((int64_t)d * 4)); }

void ensure_pages(vs_ivf* ix, int64_t need) {
    if (need <= ix->cap_pages) return;
    const int64_t ncap = std::max(need, ix->cap_pages + ix->cap_pages / 4);
    const int64_t tb = tile_bytes(ix->dpad, ix->dtype);
    uint8_t* nd = nullptr;
    float* ns = nullptr;
    uint32_t* ni = nullptr;
    HIP_CHECK(hipMalloc(&nd, (size_t)ncap * tb));
    hipError_t e = hipMalloc(&ns, (size_t)ncap * TR * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&ni, (size_t)ncap * TR * sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipFree(nd);
        if (ns) (void)hipFree(ns);
        HIP_CHECK(e);
    }
    HIP_CHECK(hipMemsetAsync(nd, 0, (size_t)ncap * tb, ix->own));
    HIP_CHECK(hipMemsetAsync(ns, 0, (size_t)ncap * TR * sizeof(float), ix->own));
    HIP_CHECK(hipMemsetAsync(ni, 0xFF, (size_t)ncap * TR * sizeof(uint32_t), ix->own));
    if (ix->used_pages > 0) {
        HIP_CHECK(hipMemcpyAsync(nd, ix->data, (size_t)ix->used_pages * tb, hipMemcpyDeviceToDevice, ix->own));
        HIP_CHECK(hipMemcpyAsync(ns, ix->sqn, (size_t)ix->used_pages * TR * sizeof(float), hipMemcpyDeviceToDevice,
                                 ix->own));
        HIP_CHECK(hipMemcpyAsync(ni, ix->slot_id, (size_t)ix->used_pages * TR * sizeof(uint32_t),
                                 hipMemcpyDeviceToDevice, ix->own));
    }
    HIP_CHECK(hipStreamSynchronize(ix->own));
    if (ix->data) (void)hipFree(ix->data);
    if (ix->sqn) (void)hipFree(ix->sqn);
    if (ix->slot_id) (void)hipFree(ix->slot_id);
    ix->data = nd;
    ix->sqn = ns;
    ix->slot_id = ni;
    ix->cap_pages = ncap;
}

void refresh_maxsq(vs_ivf* ix) {
    unsigned bits = 0;
    HIP_CHECK(hipMemcpyAsync(&bits, ix->d_flags, sizeof(unsigned), hipMemcpyDeviceToHost, ix->own));
    HIP_CHECK(hipStreamSynchronize(ix->own));
    std::memcpy(&ix->maxsq, &bits, 4);
}

void upload_csr(vs_ivf* ix, hipStream_t st) {
    if (!ix->csr_dirty) return;
    std::vector<int>& off = ix->page_off_h;
    std::vector<int> flat;
    off.assign(ix->nlist + 1, 0);
    for (int l = 0; l < ix->nlist; ++l) {
        off[l + 1] = off[l] + (int)ix->pages[l].size();
        flat.insert(flat.end(), ix->pages[l].begin(), ix->pages[l].end());
    }
    if (flat.empty()) flat.push_back(0);
    ix->d_page_off.ensure(off.size() * sizeof(int));
    ix->d_list_pages.ensure(flat.size() * sizeof(int));
    ix->d_list_n.ensure((size_t)ix->nlist * sizeof(int64_t));
    HIP_CHECK(hipMemcpyAsync(ix->d_page_off.p, off.data(), off.size() * sizeof(int), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(ix->d_list_pages.p, flat.data(), flat.size() * sizeof(int), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(ix->d_list_n.p, ix->list_n.data(), (size_t)ix->nlist * sizeof(int64_t),
                             hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));  // host vectors above are temporaries
    ix->csr_dirty = false;
}

// list id of every row: exact best centroid of its stored (dtype-rounded) values
// (fill(r0, m, dst) writes rows r0.. as device fp32)
template <typename Fill>
void assign_rows(vs_ivf* ix, int64_t n, Fill&& fill, int64_t* lists_host) {
    const int64_t rpc = rows_per_chunk(ix->d);
    ix->tmp_rows.ensure((size_t)std::min(n, rpc) * ix->d * sizeof(float));
    ix->assign_ids.ensure((size_t)std::min(n, rpc) * sizeof(int64_t));
    constexpr int S = 8;  // concurrent searches of the coarse quantizer (streams)
    if (!ix->astream[0]) {
        for (int i = 0; i < S; ++i) HIP_CHECK(hipStreamCreateWithFlags(&ix->astream[i], hipStreamNonBlocking));
        for (int i = 0; i <= S; ++i) HIP_CHECK(hipEventCreateWithFlags(&ix->aev[i], hipEventDisableTiming));
    }
    for (int64_t r0 = 0; r0 < n; r0 += rpc) {
        const int64_t m = std::min(rpc, n - r0);
        fill(r0, m, ix->tmp_rows.as<float>());
        // a row goes to the best centroid of its STORED values (the dtype-rounded row)
        HIP_CHECK(launch_round_f32(ix->dtype, ix->tmp_rows.as<float>(), m * ix->d, ix->own));
        HIP_CHECK(hipEventRecord(ix->aev[S], ix->own));
        // the chunk in S parts of whole 256-row blocks, each an exact device search on its own
        // stream (no host round trip: every query certified by its first pass, the device fallback
        // round or the full scan -- a row tied between centroids goes to the lowest id, as in faiss)
        for (int i = 0; i < S; ++i) HIP_CHECK(hipStreamWaitEvent(ix->astream[i], ix->aev[S], 0));
        search_exact_device_parts(ix->coarse, ix->tmp_rows.as<float>(), m, 1, ix->assign_ids.as<int64_t>(),
                                  ix->astream, S, nullptr);
        for (int i = 0; i < S; ++i) {
            HIP_CHECK(hipEventRecord(ix->aev[i], ix->astream[i]));
            HIP_CHECK(hipStreamWaitEvent(ix->own, ix->aev[i], 0));
        }
        HIP_CHECK(hipMemcpyAsync(lists_host + r0, ix->assign_ids.p, (size_t)m * sizeof(int64_t),
                                 hipMemcpyDeviceToHost, ix->own));
        HIP_CHECK(hipStreamSynchronize(ix->own));
    }
}

template <typename Fill>
void add_rows(vs_ivf* ix, int64_t n, Fill&& fill) {
    if (!ix->trained) throw VsError(VS_ERR_ARG, "IVF index is not trained (set its centroids first)");
    if (ix->ntotal + n > (int64_t)0xFFFFFFF0LL) throw VsError(VS_ERR_ARG, "IVF index exceeds 2^32 rows");
    std::vector<int64_t> lists((size_t)n);
    assign_rows(ix, n, fill, lists.data());
    // destinations: append to each list's last page, new pages from the pool (committed at the end)
    std::vector<std::vector<int>> pages = ix->pages;
    std::vector<int64_t> list_n = ix->list_n;
    int64_t used = ix->used_pages;
    std::vector<int64_t> slot((size_t)n);
    for (int64_t r = 0; r < n; ++r) {
        const int64_t l = lists[r];
        if (l < 0 || l >= ix->nlist) throw VsError(VS_ERR_INTERNAL, "coarse assignment out of range");
        if (list_n[l] % TR == 0) {
            if (used >= (int64_t)1 << 31) throw VsError(VS_ERR_ARG, "IVF page pool exceeds 2^31 pages");
            pages[l].push_back((int)used++);
        }
        slot[r] = (int64_t)pages[l].back() * TR + list_n[l] % TR;
        ++list_n[l];
    }
    ensure_pages(ix, used);
    const int64_t rpc = rows_per_chunk(ix->d);
    ix->slots.ensure((size_t)std::min(n, rpc) * sizeof(int64_t));
    for (int64_t r0 = 0; r0 < n; r0 += rpc) {
        const int64_t m = std::min(rpc, n - r0);
        fill(r0, m, ix->tmp_rows.as<float>());
        HIP_CHECK(hipMemcpyAsync(ix->slots.p, slot.data() + r0, (size_t)m * sizeof(int64_t), hipMemcpyHostToDevice,
                                 ix->own));
        HIP_CHECK(launch_pack_rows_map(ix->dtype, ix->tmp_rows.as<float>(), m, ix->d, ix->dpad, ix->data,
                                       ix->slots.as<int64_t>(), ix->sqn, ix->d_flags, ix->slot_id, ix->ntotal + r0,
                                       ix->own));
        HIP_CHECK(hipStreamSynchronize(ix->own));  // slot staging reuse
    }
    ix->pages.swap(pages);
    ix->list_n.swap(list_n);
    ix->used_pages = used;
    ix->id_slot.insert(ix->id_slot.end(), slot.begin(), slot.end());
    ix->ntotal += n;
    ix->csr_dirty = true;
    refresh_maxsq(ix);
}

// one search pass at screening depth Kp; outputs device [nq][k]; cert_dev [nq]
void search_core(vs_ivf* ix, const float* q_dev, int64_t nq, int k, int nprobe, int Kp, float* D, int64_t* I,
                 double* S64, int* cert_dev, hipStream_t st, bool first_pass) {
    // 1. probes: exact top-nprobe centroids of every query
    ix->probes.ensure((size_t)nq * nprobe * sizeof(int64_t));
    search_exact_device(ix->coarse, q_dev, nq, nprobe, ix->probes.as<int64_t>(), nullptr, st);
    ix->probes_h.resize((size_t)nq * nprobe);
    HIP_CHECK(hipMemcpyAsync(ix->probes_h.data(), ix->probes.p, ix->probes_h.size() * sizeof(int64_t),
                             hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    upload_csr(ix, st);  // page tables (and page_off_h) current
    // 2. work items (list, page range, <= IVF_QG queries), grouped by query-count class
    std::vector<std::vector<int>> lq((size_t)ix->nlist);
    for (int64_t q = 0; q < nq; ++q)
        for (int p = 0; p < nprobe; ++p) {
            const int64_t l = ix->probes_h[(size_t)q * nprobe + p];
            if (l < 0 || l >= ix->nlist) throw VsError(VS_ERR_INTERNAL, "probe out of range");
            lq[l].push_back((int)q);
        }
    const int classes[4] = {1, 2, 4, IVF_QG};
    std::vector<int> cls_items[4];
    std::vector<int64_t> per_q((size_t)nq, 0);  // candidate keys each query's list can receive
    double bytes = 0.0;
    // MFMA list scans: one query tile (<= qb queries, offset q0 into mq) over a list: split (hi, lo)
    // tiles of 128 queries (margin ~2^-17 ||q|| ||x||), or in the first pass under
    // VS_IVF_QTILE_PLAIN, plain tiles where the direct form serves (256 queries a tile, one MFMA
    // column per query; their query-rounding margin, ~2^-9 ||q|| ||x||, goes to the certificate;
    // cfg5 Zipf 1.1: scans 1.4% faster, but one query in 256 fails the wider margin and its
    // re-search -- every probed list scanned again for it -- costs 4.4 ms).
    struct MScan { int l, q0, nqb; };
    std::vector<MScan> mscans;
    std::vector<int> mq;  // query indices of every MFMA scan's block
    int64_t mtiles = 0;   // pages all MFMA scans read
    const bool mfma_ok = Kp <= MFMA_KP_MAX;
    const bool plain = first_pass && ix->qtile_mode == VS_IVF_QTILE_PLAIN && d16_direct_ok(ix->dpad);
    const int qb = plain ? MFMA_QB : MFMA_QB / 2;
    for (int l = 0; l < ix->nlist; ++l) {
        const int nql = (int)lq[l].size();
        const int np = (int)ix->pages[l].size();
        if (nql == 0 || np == 0) continue;
        bytes += (double)ix->list_n[l] * ix->d * ix->es;
        if (mfma_ok && mfma_scan_pays(ix, np, nql, qb)) {
            for (int b0 = 0; b0 < nql; b0 += qb) {
                const int nb = std::min(qb, nql - b0);
                mscans.push_back({l, (int)mq.size(), nb});
                mq.insert(mq.end(), lq[l].begin() + b0, lq[l].begin() + b0 + nb);
                mtiles += np;
            }
            continue;
        }
        for (int g0 = 0; g0 < nql; g0 += IVF_QG) {
            const int gq = std::min(IVF_QG, nql - g0);
            const int c = gq <= 1 ? 0 : gq <= 2 ? 1 : gq <= 4 ? 2 : 3;
            for (int pb = 0; pb < np; pb += kPagesPerItem) {
                const int pe = std::min(np, pb + kPagesPerItem);
                std::vector<int>& v = cls_items[c];
                v.push_back(l);
                v.push_back(pb);
                v.push_back(pe);
                v.push_back(gq);
                for (int j = 0; j < IVF_QG; ++j) v.push_back(j < gq ? lq[l][g0 + j] : -1);
                for (int j = 0; j < gq; ++j) per_q[lq[l][g0 + j]] += Kp;
            }
        }
    }
    // (algorithmic bytes above: every probed list read once; the GEMV scan re-reads a list per
    // query group, the MFMA scan per 128-query block -- that extra traffic is not algorithmic)
    // The MFMA scans run as ONE launch of ~2 workgroups per CU (one resident per CU, LDS-bound), each
    // over a chunk of one scan's pages with that scan's query tile -- re-read from L2 once per page.
    // XCD grouping: workgroups b and b + 8 share an XCD and its 4 MB L2 (blocks are dealt round-robin
    // over the 8 XCDs; observed placement, used for speed only), so the scans are dealt to 8 groups
    // in order of size, each group filled to 1/8 of the pages (a scan larger than that spans groups),
    // and group x's W chunks take descriptor slots x, x + 8, x + 16, ...: an XCD then holds the query
    // tiles of ~1/8 of the scans instead of all of them (mapped-scan traffic 1.116x -> see DESIGN §7c).
    std::vector<int>& desc = ix->desc_h;
    desc.clear();
    if (!mscans.empty()) {
        constexpr int NX = 8;
        struct Seg { int si, p0, p1; };  // pages [p0, p1) of scan si
        std::vector<int> order((size_t)mscans.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
            return ix->pages[mscans[x].l].size() > ix->pages[mscans[y].l].size();
        });
        std::vector<std::vector<Seg>> grp(NX);
        std::vector<int64_t> gp(NX, 0);
        {
            const int64_t target = (mtiles + NX - 1) / NX;
            int x = 0;
            for (int si : order) {
                const int np = (int)ix->pages[mscans[si].l].size();
                int p0 = 0;
                while (p0 < np) {
                    if (x < NX - 1 && gp[x] >= target) ++x;
                    const int take = x < NX - 1 ? (int)std::min<int64_t>(np - p0, std::max<int64_t>(1, target - gp[x])) : np - p0;
                    grp[x].push_back({si, p0, p0 + take});
                    gp[x] += take;
                    p0 += take;
                }
            }
        }
        // W chunks per group: ~2 workgroups per CU in all, at most MFMA_MAP_TILES pages each, at least
        // one per segment
        int W = std::max(1, (2 * ix->num_cu + NX - 1) / NX);
        for (int x = 0; x < NX; ++x) {
            W = std::max<int>(W, (int)grp[x].size());
            W = std::max<int>(W, (int)((gp[x] + MFMA_MAP_TILES - 1) / MFMA_MAP_TILES));
        }
        struct Wg { int nt, tm_off, t0, nvalid, qti, qoff, nqb; };
        std::vector<std::vector<Wg>> gw(NX);
        for (int x = 0; x < NX; ++x) {
            if (grp[x].empty()) continue;
            // chunks per segment: proportional to its pages (>= 1, <= its pages, <= 256 pages each)
            const int nseg = (int)grp[x].size();
            std::vector<int> w(nseg);
            int sum = 0;
            for (int i = 0; i < nseg; ++i) {
                const int64_t len = grp[x][i].p1 - grp[x][i].p0;
                const int64_t lo = (len + MFMA_MAP_TILES - 1) / MFMA_MAP_TILES;
                w[i] = (int)std::min<int64_t>(len, std::max<int64_t>(lo, (int64_t)std::llround((double)W * len / (double)gp[x])));
                sum += w[i];
            }
            for (bool grew = true; sum < W && grew;) {  // top up (largest pages per chunk first)
                grew = false;
                int best = -1;
                double bpc = 0.0;
                for (int i = 0; i < nseg; ++i) {
                    const int len = grp[x][i].p1 - grp[x][i].p0;
                    if (w[i] < len && (double)len / w[i] > bpc) {
                        bpc = (double)len / w[i];
                        best = i;
                    }
                }
                if (best >= 0) {
                    ++w[best];
                    ++sum;
                    grew = true;
                }
            }
            for (bool shrank = true; sum > W && shrank;) {  // trim (smallest pages per chunk first)
                shrank = false;
                int best = -1;
                double bpc = 1e300;
                for (int i = 0; i < nseg; ++i) {
                    const int len = grp[x][i].p1 - grp[x][i].p0;
                    const int lo = (len + MFMA_MAP_TILES - 1) / MFMA_MAP_TILES;
                    if (w[i] > std::max(1, lo) && (double)len / w[i] < bpc) {
                        bpc = (double)len / w[i];
                        best = i;
                    }
                }
                if (best >= 0) {
                    --w[best];
                    --sum;
                    shrank = true;
                }
            }
            for (int i = 0; i < nseg; ++i) {
                const Seg& g = grp[x][i];
                const MScan& m = mscans[g.si];
                const int64_t len = g.p1 - g.p0;
                for (int c = 0; c < w[i]; ++c) {
                    const int t0 = g.p0 + (int)(len * c / w[i]), t1 = g.p0 + (int)(len * (c + 1) / w[i]);
                    gw[x].push_back({t1 - t0, ix->page_off_h[m.l] + t0, t0, (int)ix->list_n[m.l], g.si, m.q0, m.nqb});
                }
                for (int j = 0; j < m.nqb; ++j) per_q[mq[m.q0 + j]] += w[i] * Kp;
            }
            std::stable_sort(gw[x].begin(), gw[x].end(), [](const Wg& a_, const Wg& b_) { return a_.nt > b_.nt; });
        }
        // slot 8 j + x <- group x's j-th chunk (a group short of chunks: the others close ranks)
        std::vector<Wg> wgs;
        size_t maxlen = 0;
        for (auto& v : gw) maxlen = std::max(maxlen, v.size());
        for (size_t j = 0; j < maxlen; ++j)
            for (int x = 0; x < NX; ++x)
                if (j < gw[x].size()) wgs.push_back(gw[x][j]);
        ix->n_mdesc = (int)wgs.size();
        const int64_t tmap_len = ix->page_off_h.back();
        for (const Wg& w : wgs) {
            const int g[MAP_DESC] = {w.tm_off, w.nt, w.t0, w.nvalid, w.qti, w.qoff, w.nqb, 0};
            if (!check_map_desc(g, tmap_len, (int)mscans.size(), (int64_t)mq.size(), plain))
                throw VsError(VS_ERR_INTERNAL, "IVF MFMA scan: invalid workgroup descriptor");
            desc.insert(desc.end(), g, g + MAP_DESC);
        }
        for (const MScan& m : mscans) {  // the query tiles' (offset into mq, queries), after the descriptors
            if (m.nqb < 1 || m.nqb > qb || m.q0 < 0 || m.q0 + m.nqb > (int)mq.size())
                throw VsError(VS_ERR_INTERNAL, "IVF MFMA scan: invalid query tile");
            desc.push_back(m.q0);
            desc.push_back(m.nqb);
        }
    }
    int64_t max_keys = Kp;
    for (int64_t v : per_q) max_keys = std::max(max_keys, v);
    if (max_keys > (int64_t)1 << 30) throw VsError(VS_ERR_ARG, "IVF candidate lists exceed 2^30 keys per query");
    const int lcap = (int)max_keys;
    ix->cur_mfma_lists = (int)mscans.size();
    {
        const double B = (double)tile_bytes(ix->dpad, ix->dtype);
        double gp = 0.0;
        for (auto& v : cls_items)
            for (size_t i = 0; i < v.size(); i += IVF_ITEM_INTS) gp += (double)(v[i + 2] - v[i + 1]);
        ix->cur_bytes[0] = (double)mtiles * B;
        ix->cur_bytes[1] = gp * B;
    }
    size_t total_ints = 0;
    for (auto& v : cls_items) total_ints += v.size();
    ix->items.ensure(std::max<size_t>(total_ints, 1) * sizeof(int));
    // one dynamic launch takes the items most expensive class first (measured faster than one
    // launch per class)
    constexpr bool dyn = true;
    {
        std::vector<int> all;
        all.reserve(total_ints);
        if (dyn)
            for (int c = 3; c >= 0; --c) all.insert(all.end(), cls_items[c].begin(), cls_items[c].end());
        else
            for (auto& v : cls_items) all.insert(all.end(), v.begin(), v.end());
        if (!all.empty())
            HIP_CHECK(hipMemcpyAsync(ix->items.p, all.data(), all.size() * sizeof(int), hipMemcpyHostToDevice, st));
        if (!mq.empty()) {
            ix->mqidx.ensure(mq.size() * sizeof(int));
            HIP_CHECK(hipMemcpyAsync(ix->mqidx.p, mq.data(), mq.size() * sizeof(int), hipMemcpyHostToDevice, st));
            ix->mdesc.ensure(desc.size() * sizeof(int));
            HIP_CHECK(hipMemcpyAsync(ix->mdesc.p, desc.data(), desc.size() * sizeof(int), hipMemcpyHostToDevice, st));
        }
        HIP_CHECK(hipStreamSynchronize(st));  // `all` and `mq` are temporaries
    }
    // 3. queries fp32 padded, ||q|| for the certificate
    ix->qp.ensure((size_t)nq * ix->dpad * sizeof(float));
    ix->qinfo.ensure((size_t)nq * 2 * sizeof(float));
    HIP_CHECK(launch_pack_qf32(q_dev, (int)nq, (int)nq, ix->d, ix->dpad, ix->qp.as<float>(), ix->qinfo.as<float>(), st));
    // 4. list scans
    ix->glist.ensure((size_t)nq * lcap * sizeof(u64));
    ix->gcnt.ensure((size_t)nq * sizeof(int));
    HIP_CHECK(hipMemsetAsync(ix->gcnt.p, 0, (size_t)nq * sizeof(int), st));
    IvfScanArgs a{};
    a.data = ix->data;
    a.sqn = ix->sqn;
    a.qp = ix->qp.as<float>();
    a.list_pages = ix->d_list_pages.as<int>();
    a.page_off = ix->d_page_off.as<int>();
    a.list_n = ix->d_list_n.as<int64_t>();
    a.dpad = ix->dpad;
    a.metric = ix->metric;
    a.Kp = Kp;
    a.cap = (int)round_up(Kp + 2 * TR, 256);
    a.glist = ix->glist.as<u64>();
    a.gcnt = ix->gcnt.as<int>();
    a.lcap = lcap;
    // persistent scan workgroups: 8 per CU (32 waves) keep enough 16 B loads in flight per CU
    constexpr int grid_per_cu = 8;
    const int max_grid = ix->num_cu * grid_per_cu;
    ix->cand.ensure((size_t)max_grid * IVF_QG * a.cap * sizeof(u64));
    a.cand = ix->cand.as<u64>();
    const bool timing = first_pass && ix->timing.load();  // (re-search rounds are not the timed scan)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        HIP_CHECK(hipEventRecord(e0, st));
    }
    // Both scans at once when both have work: the GEMV scan (HBM-bound, 8 small workgroups per CU)
    // on a side stream beside the MFMA scan (power-bound, one LDS-heavy workgroup per CU), so the
    // chip streams the GEMV lists while the MFMAs run instead of after them; they share only the
    // per-query list counters (atomics) and write disjoint candidate slots.
    const int n_dyn_items = (int)(total_ints / IVF_ITEM_INTS);
    const bool concurrent = dyn && !mscans.empty() && n_dyn_items > 0;
    hipStream_t dst = st;
    if (concurrent) {
        if (!ix->astream[0]) {
            for (int i = 0; i < 8; ++i) HIP_CHECK(hipStreamCreateWithFlags(&ix->astream[i], hipStreamNonBlocking));
            for (int i = 0; i <= 8; ++i) HIP_CHECK(hipEventCreateWithFlags(&ix->aev[i], hipEventDisableTiming));
        }
        dst = ix->astream[0];
        ix->next_item.ensure(sizeof(int));
        HIP_CHECK(hipMemsetAsync(ix->next_item.p, 0, sizeof(int), st));
        HIP_CHECK(hipEventRecord(ix->aev[0], st));  // fork: queries packed, list counters zeroed
        HIP_CHECK(hipStreamWaitEvent(dst, ix->aev[0], 0));
        a.next_item = ix->next_item.as<int>();
        a.items = ix->items.as<int>();
        a.n_items = n_dyn_items;
        HIP_CHECK(launch_ivf_scan_dyn(ix->dtype, a, std::min(a.n_items, max_grid), dst));
        HIP_CHECK(hipEventRecord(ix->aev[1], dst));
    }
    // lists probed by many queries: the MFMA screen over their pages (unseeded; every workgroup
    // appends its best Kp per query to the query's list, which the refine cuts to Kp)
    if (!mscans.empty()) {
        const size_t qtb = (size_t)MFMA_QB * ix->dpad * 2;  // one query tile
        ix->mqtile.ensure(qtb * mscans.size());
        const int G = ix->n_mdesc;
        ix->mcand.ensure((size_t)G * qb * MFMA_CAP * sizeof(u64));
        // the query tiles (and their queries' margins in qinfo), one launch
        HIP_CHECK(launch_pack_qtile_split(ix->dtype, q_dev, ix->mqidx.as<int>(), ix->mdesc.as<int>() + (size_t)G * MAP_DESC,
                                          (int)mscans.size(), ix->d, ix->dpad, ix->mqtile.as<uint8_t>(),
                                          ix->qinfo.as<float>(), plain, st));
        ScreenArgs sa{};
        sa.corpus = ix->data;
        sa.dpad = ix->dpad;
        sa.d = ix->d;
        sa.metric = ix->metric;
        sa.sqn = ix->sqn;
        sa.Kp = Kp;
        sa.cap = MFMA_CAP;
        sa.cand = ix->mcand.as<u64>();
        sa.G = G;
        sa.glist = ix->glist.as<u64>();
        sa.gcnt = ix->gcnt.as<int>();
        sa.lcap = lcap;
        sa.tile_map = ix->d_list_pages.as<int>();
        sa.qmap = ix->mqidx.as<int>();
        sa.wg_desc = ix->mdesc.as<int>();
        HIP_CHECK(launch_screen_mfma_mapped(ix->dtype, sa, ix->mqtile.as<uint8_t>(), plain, st));
    }
    size_t off = 0;
    if (concurrent) {
        HIP_CHECK(hipStreamWaitEvent(st, ix->aev[1], 0));  // join
    } else if (dyn) {
        ix->next_item.ensure(sizeof(int));
        HIP_CHECK(hipMemsetAsync(ix->next_item.p, 0, sizeof(int), st));
        a.next_item = ix->next_item.as<int>();
        a.items = ix->items.as<int>();
        a.n_items = (int)(total_ints / IVF_ITEM_INTS);
        if (a.n_items > 0) HIP_CHECK(launch_ivf_scan_dyn(ix->dtype, a, std::min(a.n_items, max_grid), st));
    }
    for (int c = 0; c < 4 && !dyn; ++c) {
        const int n_items = (int)(cls_items[c].size() / IVF_ITEM_INTS);
        a.items = ix->items.as<int>() + off;
        a.n_items = n_items;
        off += cls_items[c].size();
        if (n_items == 0) continue;
        HIP_CHECK(launch_ivf_scan(ix->dtype, classes[c], a, std::min(n_items, max_grid), st));
    }
    if (timing) {
        HIP_CHECK(hipEventRecord(e1, st));
        ix->tev.emplace_back(e0, e1);
        ix->tbytes.push_back(bytes);
    }
    // 5. exact refine over each query's candidate list (slots -> user ids)
    RefineArgs r{};
    r.cand = ix->glist.as<u64>();
    r.cand_n = ix->gcnt.as<int>();
    r.lcap = lcap;
    r.Kp = Kp;
    r.q = q_dev;
    r.d = ix->d;
    r.dpad = ix->dpad;
    r.dt = ix->dtype;
    r.metric = ix->metric;
    r.corpus = ix->data;
    r.qinfo = ix->qinfo.as<float>();
    r.xmax = (float)(std::sqrt((double)ix->maxsq) * (1.0 + 1e-5)) + 1e-30f;
    r.gamma = gamma_of(ix->d);
    r.k = k;
    r.n_valid = ix->ntotal;
    r.id_offset = 0;
    r.D = D;
    r.I = I;
    r.S64 = S64;
    r.cert = cert_dev;
    r.uncert = ix->d_flags + 1;
    r.optimistic = 0;
    r.idmap = ix->slot_id;
    HIP_CHECK(launch_refine(r, (int)nq, st));
}

void fill_padding(vs_ivf* ix, int64_t nq, int k, float* D, int64_t* I, double* S64, hipStream_t st) {
    const size_t n = (size_t)nq * k;
    std::vector<int64_t> hi(n, -1);
    HIP_CHECK(hipMemcpyAsync(I, hi.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, st));
    if (D) {
        std::vector<float> hd(n, ix->metric == VS_METRIC_IP ? -3.402823466e+38f : 3.402823466e+38f);
        HIP_CHECK(hipMemcpyAsync(D, hd.data(), n * sizeof(float), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    if (S64) {
        std::vector<double> hs(n, ix->metric == VS_METRIC_IP ? -1.7976931348623157e308 : 1.7976931348623157e308);
        HIP_CHECK(hipMemcpyAsync(S64, hs.data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    HIP_CHECK(hipStreamSynchronize(st));
}

// full search with certificate retries (caller holds the locks)
void search_locked(vs_ivf* ix, const float* q_dev, int64_t nq, int k, int nprobe, float* D, int64_t* I, double* S64,
                   hipStream_t st) {
    if (ix->ntotal == 0) {
        fill_padding(ix, nq, k, D, I, S64, st);
        return;
    }
    nprobe = std::min(nprobe, ix->nlist);
    const int Kp = screen_depth(k);
    ix->cert.ensure((size_t)nq * sizeof(int));
    search_core(ix, q_dev, nq, k, nprobe, Kp, D, I, S64, ix->cert.as<int>(), st, true);
    ix->cert_h.resize((size_t)nq);
    HIP_CHECK(hipMemcpyAsync(ix->cert_h.data(), ix->cert.p, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    std::vector<int> fail;
    for (int64_t qi = 0; qi < nq; ++qi)
        if (!ix->cert_h[qi]) fail.push_back((int)qi);
    ix->last_mfma_lists = ix->cur_mfma_lists;
    ix->last_bytes[0] = ix->cur_bytes[0];
    ix->last_bytes[1] = ix->cur_bytes[1];
    ix->last_uncert = (int)fail.size();
    // uncertified queries: re-searched together, 4x deeper per round (their probed lists scanned
    // once per round for all of them, on the MFMA screen where that pays)
    const size_t ko = (size_t)k;
    int Kr = Kp;
    while (!fail.empty()) {
        if (Kr >= KP_MAX) throw VsError(VS_ERR_UNCERTIFIED, "exactness certificate failed at maximum screening depth");
        Kr = std::min(Kr * 4, KP_MAX);
        const int nf = (int)fail.size();
        ix->rq.ensure((size_t)nf * ix->d * sizeof(float));
        ix->rI.ensure((size_t)nf * ko * sizeof(int64_t));
        if (D) ix->rD.ensure((size_t)nf * ko * sizeof(float));
        if (S64) ix->rS.ensure((size_t)nf * ko * sizeof(double));
        for (int j = 0; j < nf; ++j)
            HIP_CHECK(hipMemcpyAsync(ix->rq.as<float>() + (size_t)j * ix->d, q_dev + (size_t)fail[j] * ix->d,
                                     (size_t)ix->d * sizeof(float), hipMemcpyDeviceToDevice, st));
        search_core(ix, ix->rq.as<float>(), nf, k, nprobe, Kr, D ? ix->rD.as<float>() : nullptr, ix->rI.as<int64_t>(),
                    S64 ? ix->rS.as<double>() : nullptr, ix->cert.as<int>(), st, false);
        for (int j = 0; j < nf; ++j) {
            const size_t o = (size_t)fail[j] * ko, r = (size_t)j * ko;
            HIP_CHECK(hipMemcpyAsync(I + o, ix->rI.as<int64_t>() + r, ko * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
            if (D) HIP_CHECK(hipMemcpyAsync(D + o, ix->rD.as<float>() + r, ko * sizeof(float), hipMemcpyDeviceToDevice, st));
            if (S64)
                HIP_CHECK(hipMemcpyAsync(S64 + o, ix->rS.as<double>() + r, ko * sizeof(double), hipMemcpyDeviceToDevice, st));
        }
        ix->cert_h.resize((size_t)nf);
        HIP_CHECK(hipMemcpyAsync(ix->cert_h.data(), ix->cert.p, (size_t)nf * sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        std::vector<int> still;
        for (int j = 0; j < nf; ++j)
            if (!ix->cert_h[j]) still.push_back(fail[j]);
        fail.swap(still);
    }
}

void check_search_args(const vs_ivf* ix, int64_t nq, int32_t k, int32_t nprobe) {
    check_ivf(ix);
    if (nq < 0) throw VsError(VS_ERR_ARG, "nq must be >= 0");
    if (k <= 0) throw VsError(VS_ERR_ARG, "k must be > 0");
    if (screen_depth(k) < k || k > KP_MAX * 4 / 5)
        throw VsError(VS_ERR_ARG, "k too large (max " + std::to_string(KP_MAX * 4 / 5) + ")");
    if (nprobe <= 0) throw VsError(VS_ERR_ARG, "nprobe must be > 0");
    if (!ix->trained) throw VsError(VS_ERR_ARG, "IVF index is not trained (set its centroids first)");
}

}  // namespace

extern "C" {

int vs_ivf_create(int d, int nlist, int metric, int dtype, int device, vs_ivf** out) {
    return guarded([&] {
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        *out = nullptr;
        if (d <= 0) throw VsError(VS_ERR_ARG, "dimension must be > 0");
        if (nlist <= 0) throw VsError(VS_ERR_ARG, "nlist must be > 0");
        if (metric != VS_METRIC_IP && metric != VS_METRIC_L2) throw VsError(VS_ERR_ARG, "metric must be IP(0) or L2(1)");
        if (dtype < VS_DTYPE_F32 || dtype > VS_DTYPE_F16) throw VsError(VS_ERR_ARG, "dtype must be 0 (f32), 1 (bf16), 2 (f16)");
        vs_index* coarse = nullptr;
        int rc = vs_create(d, metric, dtype, device, &coarse);
        if (rc != VS_OK) throw VsError(rc, std::string("coarse quantizer: ") + vs_last_error());
        vs_ivf* ix = new vs_ivf();
        ix->coarse = coarse;
        ix->d = d;
        ix->dpad = pad_dim(d, dtype);
        ix->nlist = nlist;
        ix->metric = metric;
        ix->dtype = dtype;
        ix->device = device;
        ix->es = es_of(dtype);
        ix->pages.resize((size_t)nlist);
        ix->list_n.assign((size_t)nlist, 0);
        try {
            DeviceGuard dg(device);
            hipDeviceProp_t prop;
            HIP_CHECK(hipGetDeviceProperties(&prop, device));
            ix->num_cu = prop.multiProcessorCount;
            HIP_CHECK(hipStreamCreateWithFlags(&ix->own, hipStreamNonBlocking));
            HIP_CHECK(hipMalloc(&ix->d_flags, sizeof(unsigned) * 2));
            HIP_CHECK(hipMemset(ix->d_flags, 0, sizeof(unsigned) * 2));
        } catch (...) {
            vs_ivf_destroy(ix);
            throw;
        }
        *out = ix;
    });
}

void vs_ivf_destroy(vs_ivf* ix) {
    if (!ix) return;
    {
        DeviceGuard dg(ix->device);
        (void)hipDeviceSynchronize();
        for (DevBuf* b : {&ix->d_page_off, &ix->d_list_pages, &ix->d_list_n, &ix->tmp_rows, &ix->slots, &ix->assign_ids,
                          &ix->qdev, &ix->probes, &ix->items, &ix->qp, &ix->qinfo, &ix->cand, &ix->glist, &ix->gcnt,
                          &ix->cert, &ix->outD, &ix->outI, &ix->rec, &ix->next_item})
            b->release();
        for (auto& pr : ix->tev) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        if (ix->data) (void)hipFree(ix->data);
        if (ix->sqn) (void)hipFree(ix->sqn);
        if (ix->slot_id) (void)hipFree(ix->slot_id);
        if (ix->d_flags) (void)hipFree(ix->d_flags);
        if (ix->own) (void)hipStreamDestroy(ix->own);
        for (hipStream_t& a : ix->astream)
            if (a) (void)hipStreamDestroy(a);
        for (hipEvent_t& e : ix->aev)
            if (e) (void)hipEventDestroy(e);
    }
    vs_destroy(ix->coarse);
    delete ix;
}

int vs_ivf_set_centroids(vs_ivf* ix, const float* c) {
    return guarded([&] {
        check_ivf(ix);
        if (!c) throw VsError(VS_ERR_ARG, "centroids are null");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        if (ix->ntotal > 0) throw VsError(VS_ERR_ARG, "IVF index is not empty: reset() before setting centroids");
        int rc = vs_reset(ix->coarse);
        if (rc == VS_OK) rc = vs_add(ix->coarse, c, ix->nlist);
        if (rc != VS_OK) throw VsError(rc, std::string("coarse quantizer: ") + vs_last_error());
        ix->trained = true;
    });
}

int vs_ivf_get_centroids(vs_ivf* ix, float* out) {
    return guarded([&] {
        check_ivf(ix);
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        if (!ix->trained) throw VsError(VS_ERR_ARG, "IVF index is not trained (set its centroids first)");
        const int rc = vs_reconstruct_n(ix->coarse, 0, ix->nlist, out);
        if (rc != VS_OK) throw VsError(rc, vs_last_error());
    });
}

int vs_ivf_is_trained(const vs_ivf* ix) { return ix ? (ix->trained ? 1 : 0) : -1; }

int vs_ivf_assign(vs_ivf* ix, const float* x, int64_t n, int64_t* lists) {
    return guarded([&] {
        check_ivf(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x || !lists) throw VsError(VS_ERR_ARG, "null host buffer");
        if (!ix->trained) throw VsError(VS_ERR_ARG, "IVF index is not trained (set its centroids first)");
        std::unique_lock<std::shared_mutex> lk(ix->rw);  // shares the add workspaces
        DeviceGuard dg(ix->device);
        const int d = ix->d;
        assign_rows(ix, n,
                    [&](int64_t r0, int64_t m, float* dst) {
                        HIP_CHECK(hipMemcpyAsync(dst, x + r0 * d, (size_t)m * d * sizeof(float), hipMemcpyHostToDevice,
                                                 ix->own));
                    },
                    lists);
    });
}

int vs_ivf_add(vs_ivf* ix, const float* x, int64_t n) {
    return guarded([&] {
        check_ivf(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x) throw VsError(VS_ERR_ARG, "x is null");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        const int d = ix->d;
        add_rows(ix, n, [&](int64_t r0, int64_t m, float* dst) {
            HIP_CHECK(hipMemcpyAsync(dst, x + r0 * d, (size_t)m * d * sizeof(float), hipMemcpyHostToDevice, ix->own));
        });
    });
}

int vs_ivf_add_device(vs_ivf* ix, const float* x_dev, int64_t n, void* stream) {
    return guarded([&] {
        check_ivf(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        if (!x_dev) throw VsError(VS_ERR_ARG, "x_dev is null");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        // the producer's writes land first (NULL = the legacy default stream, torch's default)
        HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
        const int d = ix->d;
        add_rows(ix, n, [&](int64_t r0, int64_t m, float* dst) {
            HIP_CHECK(hipMemcpyAsync(dst, x_dev + r0 * d, (size_t)m * d * sizeof(float), hipMemcpyDeviceToDevice,
                                     ix->own));
        });
    });
}

int vs_ivf_reserve(vs_ivf* ix, int64_t n) {
    return guarded([&] {
        check_ivf(ix);
        if (n < 0) throw VsError(VS_ERR_ARG, "n must be >= 0");
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        // n more rows need at most ceil(n / TR) new pages plus one partly filled page per list
        ensure_pages(ix, ix->used_pages + (n + TR - 1) / TR + ix->nlist);
    });
}

int vs_ivf_add_synthetic(vs_ivf* ix, uint64_t seed, int64_t global_row0, int64_t n, int normalize) {
    return guarded([&] {
        check_ivf(ix);
        if (n < 0 || global_row0 < 0) throw VsError(VS_ERR_ARG, "bad synthetic range");
        if (n == 0) return;
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        add_rows(ix, n, [&](int64_t r0, int64_t m, float* dst) {
            // unrounded fp32 rows; k_pack_rows_map rounds to the index dtype exactly as k_synth_rows does
            HIP_CHECK(launch_synth_f32(DT_F32, seed, global_row0 + r0, m, ix->d, normalize, dst, ix->own));
        });
    });
}

int vs_ivf_search_device(vs_ivf* ix, const float* q_dev, int64_t nq, int32_t k, int32_t nprobe, float* D_dev,
                         int64_t* I_dev, double* S64_dev, void* stream) {
    return guarded([&] {
        check_search_args(ix, nq, k, nprobe);
        if (nq == 0) return;
        if (!q_dev || !I_dev) throw VsError(VS_ERR_ARG, "null device buffer");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        std::lock_guard<std::mutex> sg(ix->search_mtx);
        DeviceGuard dg(ix->device);
        search_locked(ix, q_dev, nq, k, nprobe, D_dev, I_dev, S64_dev, (hipStream_t)stream);  // NULL: legacy default
    });
}

int vs_ivf_search(vs_ivf* ix, const float* q, int64_t nq, int32_t k, int32_t nprobe, float* D, int64_t* I) {
    return guarded([&] {
        check_search_args(ix, nq, k, nprobe);
        if (nq == 0) return;
        if (!q || !D || !I) throw VsError(VS_ERR_ARG, "null host buffer");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        std::lock_guard<std::mutex> sg(ix->search_mtx);
        DeviceGuard dg(ix->device);
        hipStream_t st = ix->own;
        ix->qdev.ensure((size_t)nq * ix->d * sizeof(float));
        ix->outD.ensure((size_t)nq * k * sizeof(float));
        ix->outI.ensure((size_t)nq * k * sizeof(int64_t));
        HIP_CHECK(hipMemcpyAsync(ix->qdev.p, q, (size_t)nq * ix->d * sizeof(float), hipMemcpyHostToDevice, st));
        search_locked(ix, ix->qdev.as<float>(), nq, k, nprobe, ix->outD.as<float>(), ix->outI.as<int64_t>(), nullptr,
                      st);
        HIP_CHECK(hipMemcpyAsync(D, ix->outD.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipMemcpyAsync(I, ix->outI.p, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
    });
}

int vs_ivf_reconstruct(vs_ivf* ix, int64_t id, float* out) {
    return guarded([&] {
        check_ivf(ix);
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        if (id < 0 || id >= ix->ntotal) throw VsError(VS_ERR_ARG, "reconstruct id out of bounds");
        std::lock_guard<std::mutex> sg(ix->search_mtx);
        DeviceGuard dg(ix->device);
        ix->rec.ensure((size_t)ix->d * sizeof(float));
        HIP_CHECK(launch_unpack_rows(ix->dtype, ix->data, ix->id_slot[(size_t)id], 1, ix->d, ix->dpad,
                                     ix->rec.as<float>(), ix->own));
        HIP_CHECK(hipMemcpyAsync(out, ix->rec.p, (size_t)ix->d * sizeof(float), hipMemcpyDeviceToHost, ix->own));
        HIP_CHECK(hipStreamSynchronize(ix->own));
    });
}

int vs_ivf_list_sizes(vs_ivf* ix, int64_t* out) {
    return guarded([&] {
        check_ivf(ix);
        if (!out) throw VsError(VS_ERR_ARG, "out is null");
        std::shared_lock<std::shared_mutex> lk(ix->rw);
        std::copy(ix->list_n.begin(), ix->list_n.end(), out);
    });
}

int vs_ivf_reset(vs_ivf* ix) {
    return guarded([&] {
        check_ivf(ix);
        std::unique_lock<std::shared_mutex> lk(ix->rw);
        DeviceGuard dg(ix->device);
        for (auto& p : ix->pages) p.clear();
        std::fill(ix->list_n.begin(), ix->list_n.end(), 0);
        ix->id_slot.clear();
        ix->used_pages = 0;
        ix->ntotal = 0;
        ix->maxsq = 0.0f;
        ix->csr_dirty = true;
        HIP_CHECK(hipMemsetAsync(ix->d_flags, 0, sizeof(unsigned), ix->own));
        HIP_CHECK(hipStreamSynchronize(ix->own));
    });
}

int64_t vs_ivf_ntotal(const vs_ivf* ix) { return ix ? ix->ntotal : -1; }
int vs_ivf_nlist(const vs_ivf* ix) { return ix ? ix->nlist : -1; }

int vs_ivf_set_timing(vs_ivf* ix, int enable) {
    return guarded([&] {
        check_ivf(ix);
        ix->timing.store(enable != 0);
    });
}

int vs_ivf_set_scan(vs_ivf* ix, int mode) {
    return guarded([&] {
        check_ivf(ix);
        if (mode != VS_IVF_SCAN_AUTO && mode != VS_IVF_SCAN_GEMV && mode != VS_IVF_SCAN_MFMA)
            throw VsError(VS_ERR_ARG, "unknown IVF scan mode");
        std::lock_guard<std::mutex> g(ix->search_mtx);
        ix->scan_mode = mode;
    });
}

int vs_ivf_set_query_tiles(vs_ivf* ix, int mode) {
    return guarded([&] {
        check_ivf(ix);
        if (mode != VS_IVF_QTILE_PLAIN && mode != VS_IVF_QTILE_SPLIT) throw VsError(VS_ERR_ARG, "unknown IVF query-tile mode");
        std::lock_guard<std::mutex> g(ix->search_mtx);
        ix->qtile_mode = mode;
    });
}

int vs_ivf_last_search_stats(const vs_ivf* ix, int* mfma_lists, int* uncertified, double* bytes_read) {
    return guarded([&] {
        check_ivf(ix);
        if (mfma_lists) *mfma_lists = ix->last_mfma_lists;
        if (uncertified) *uncertified = ix->last_uncert;
        if (bytes_read) {
            bytes_read[0] = ix->last_bytes[0];
            bytes_read[1] = ix->last_bytes[1];
        }
    });
}

int vs_ivf_timing_fetch(vs_ivf* ix, float* ms, double* bytes_scanned, int cap) {
    int count = 0;
    int rc = guarded([&] {
        check_ivf(ix);
        std::lock_guard<std::mutex> sg(ix->search_mtx);
        DeviceGuard dg(ix->device);
        for (size_t i = 0; i < ix->tev.size(); ++i) {
            auto& pr = ix->tev[i];
            HIP_CHECK(hipEventSynchronize(pr.second));
            float t = 0.0f;
            HIP_CHECK(hipEventElapsedTime(&t, pr.first, pr.second));
            if (count < cap) {
                if (ms) ms[count] = t;
                if (bytes_scanned) bytes_scanned[count] = ix->tbytes[i];
            }
            ++count;
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        ix->tev.clear();
        ix->tbytes.clear();
    });
    return rc == VS_OK ? std::min(count, cap) : rc;
}

}  // extern "C"
