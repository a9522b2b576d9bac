// vs_fullscan.hip -- the last tier of the exactness fallback: an exact full scan of the shard.
//
// Every screen of libvs lists a bounded number of candidate rows per query (KP_MAX = 4096 in the
// deepest fallback round), and its certificate proves that no unlisted row can enter the top-k.
// When more rows than that tie (or nearly tie) at the k-th best score -- thousands of identical
// photo embeddings -- no bounded list can hold them, and faiss still answers: IndexFlatIP /
// IndexFlatL2 return the k lowest ids among equal scores (/root/reference/utils/vector_store.py:191,
// pinned by /root/reference/tests/test_searcher.py:323-350).  This kernel gives that answer for any
// number of ties: every row of the shard is scored exactly (the canonical fp64 expression tree of
// exact_score_rows, bit-identical with the oracle) and streamed through a bounded running top-k
// under the total order (score desc / distance asc, then id asc).
//
// One launch handles every query of a block whose cert[q] is 0 (optionally gated on a device count,
// so the launch returns at once when no query needs it).  Workgroup b scans the contiguous row range
// [n b / G, n (b + 1) / G): rows are scored 32 at a time (8 waves x RR rows), the ones that beat the
// workgroup's current k-th best go to an LDS batch, and a full batch is sorted (bitonic) and merged
// into the workgroup's sorted list by rank (each element's new position = its index + its rank in
// the other list).  Within a range rows come in id order, so once the list is full a row tied with
// the k-th best never enters it: the memory stays O(k) however many rows tie.  Each workgroup writes
// its list to global scratch; the last one to finish (device-scope fence + per-query counter, re-
// zeroed by it) merges the G sorted lists -- only each list's prefix that beats the running k-th
// best is read -- and writes the faiss-layout result and cert[q] = 1.
#include "vs_device.h"

namespace vs {

constexpr int FS_THREADS = 512;
constexpr int FS_NW = FS_THREADS / 64;
constexpr int FS_B = 512;  // candidate batch merged into a workgroup's list at once (= FS_THREADS)
static_assert(FS_B == FS_THREADS, "the batch sort keeps one element per thread");

__device__ __forceinline__ bool fs_better(double sa, uint32_t ia, double sb, uint32_t ib) {
    return sa != sb ? sa > sb : ia < ib;
}
// entries of the best-first list (sc, id)[0, n) better than (s, i)
__device__ __forceinline__ int fs_rank(const double* sc, const uint32_t* id, int n, double s, uint32_t i) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (fs_better(sc[mid], id[mid], s, i)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

struct FsLists {
    double* lsc[2];
    uint32_t* lid[2];
    double* bsc;
    uint32_t* bid;
};

// merge the best-first batch (bsc, bid)[0, nb) into list `cur` (nl entries), keeping the best k in
// list cur ^ 1; every thread updates cur / nl alike
__device__ __forceinline__ void fs_merge(const FsLists& L, int& cur, int& nl, int nb, int k) {
    const int tid = threadIdx.x;
    const double* asc = L.lsc[cur];
    const uint32_t* aid = L.lid[cur];
    double* osc = L.lsc[cur ^ 1];
    uint32_t* oid = L.lid[cur ^ 1];
    for (int i = tid; i < nb; i += FS_THREADS) {
        const double s = L.bsc[i];
        const uint32_t id = L.bid[i];
        const int p = i + fs_rank(asc, aid, nl, s, id);
        if (p < k) {
            osc[p] = s;
            oid[p] = id;
        }
    }
    for (int j = tid; j < nl; j += FS_THREADS) {
        const double s = asc[j];
        const uint32_t id = aid[j];
        const int p = j + fs_rank(L.bsc, L.bid, nb, s, id);
        if (p < k) {
            osc[p] = s;
            oid[p] = id;
        }
    }
    __syncthreads();
    cur ^= 1;
    nl = min(k, nl + nb);
}

// sort the batch's nb entries (by rank; the bitonic network over the next power of two, worst-padded,
// past one entry per thread) and merge them in
__device__ __forceinline__ void fs_sort_merge(const FsLists& L, int& cur, int& nl, int nb, int k) {
    int n2 = 1;
    while (n2 < nb) n2 <<= 1;
    for (int j = nb + (int)threadIdx.x; j < n2; j += FS_THREADS) {
        L.bsc[j] = -INFINITY;
        L.bid[j] = 0xFFFFFFFFu;
    }
    __syncthreads();
    sort_valid_best_first<METRIC_IP>(L.bsc, L.bid, nb, n2);
    fs_merge(L, cur, nl, nb, k);
}

// rows per wave in flight: twice the refine's (one workgroup per CU here, so the registers are there)
template <int DT>
constexpr int fs_rows() { return DT == DT_F32 ? 4 : 8; }

// (the hand-off of the workgroups' lists to the last one: st_agent / ld_agent, vs_device.h)

template <int DT, int METRIC, bool QLDS>
__global__ void __launch_bounds__(FS_THREADS) k_full_scan(FullScanArgs a, int KL) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.gate && *a.gate == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int b = blockIdx.x, G = gridDim.x;
    const int ng = (a.d + 7) >> 3;
    FsLists L;
    L.lsc[0] = (double*)smem;
    L.lsc[1] = L.lsc[0] + KL;
    L.bsc = L.lsc[1] + KL;
    double* qs = L.bsc + FS_B;
    L.lid[0] = (uint32_t*)(qs + (QLDS ? (size_t)ng * 8 : 0));
    L.lid[1] = L.lid[0] + KL;
    L.bid = L.lid[1] + KL;
    __shared__ int go_s, nb_s, last_s;
    __shared__ int red_s[FS_NW];
    constexpr int RR = fs_rows<DT>();
    const int k = a.k;
    const int64_t r0 = a.n_valid * b / G, r1 = a.n_valid * (b + 1) / G;
    for (int q = 0; q < a.nq; ++q) {
        __syncthreads();  // (the previous query's readers of qs / the lists are done)
        if (tid == 0) {
            go_s = (a.all_queries || a.cert[q] == 0) ? 1 : 0;
            nb_s = 0;
        }
        __syncthreads();
        if (!go_s) continue;
        const float* qv = a.q + (int64_t)q * a.d;
        if constexpr (QLDS)
            for (int i = tid; i < a.d; i += FS_THREADS) qs[(i & 7) * ng + (i >> 3)] = (double)qv[i];
        __syncthreads();
        int cur = 0, nl = 0;
        for (int64_t base = r0; base < r1; base += FS_NW * RR) {
            int64_t rr[RR];
#pragma unroll
            for (int i = 0; i < RR; ++i) {
                const int64_t r = base + wid + (int64_t)i * FS_NW;
                rr[i] = r < r1 ? r : -1;
            }
            if (rr[0] >= 0) {  // (wave-uniform)
                double s4[RR];
                exact_score_rows<DT, METRIC, QLDS, RR>(a.corpus, rr, qs, qv, a.d, a.dpad, lane, s4);
                if (lane == 0) {
                    const bool full = nl >= k;
                    const double ts = full ? L.lsc[cur][k - 1] : 0.0;
                    const uint32_t ti = full ? L.lid[cur][k - 1] : 0u;
#pragma unroll
                    for (int i = 0; i < RR; ++i) {
                        if (rr[i] < 0) continue;
                        const double s = METRIC == METRIC_L2 ? -s4[i] : s4[i];
                        const uint32_t id = (uint32_t)rr[i];
                        if (!full || fs_better(s, id, ts, ti)) {
                            const int slot = atomicAdd(&nb_s, 1);
                            L.bsc[slot] = s;
                            L.bid[slot] = id;
                        }
                    }
                }
            }
            __syncthreads();
            const int nb = nb_s;
            if (nb > FS_B - FS_NW * RR || base + FS_NW * RR >= r1) {
                if (nb > 0) fs_sort_merge(L, cur, nl, nb, k);
                if (tid == 0) nb_s = 0;
                __syncthreads();
            }
        }
        // this workgroup's list -> scratch; the last workgroup of the query merges all of them
        double* gs = a.gsc + ((size_t)q * G + b) * k;
        uint32_t* gi = a.gid + ((size_t)q * G + b) * k;
        for (int j = tid; j < k; j += FS_THREADS) {
            st_agent(gs + j, j < nl ? L.lsc[cur][j] : -INFINITY);
            st_agent(gi + j, j < nl ? L.lid[cur][j] : 0xFFFFFFFFu);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every storing wave, before the add)
        __syncthreads();
        if (tid == 0)
            last_s = __hip_atomic_fetch_add(a.gdone + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                             (unsigned)(G - 1) ? 1 : 0;
        __syncthreads();
        if (!last_s) continue;
        // The other lists as one flat array [G][k].  First a floor: the k-th best of the G lists'
        // heads (k distinct rows at least that good, so no entry below it can be in the top-k).  Then
        // FS_B entries at a time (the next chunk's loads in flight): entries at least as good as the
        // floor that beat the running k-th best are appended to the batch; a batch that would
        // overflow, and the last one, are sorted and merged (few entries pass the floor).
        {
            const double* vs_ = a.gsc + (size_t)q * G * k;
            const uint32_t* vi = a.gid + (size_t)q * G * k;
            const int total = G * k;
            // every load of the first FS_PF chunks (and the heads) issued before any is used
            constexpr int FS_PF = 8;
            auto fetch = [&](int j, double& s, uint32_t& id) {
                s = -INFINITY;
                id = 0xFFFFFFFFu;
                if (j < total && j / k != b) {
                    s = ld_agent(vs_ + j);
                    id = ld_agent(vi + j);
                }
            };
            double ps[FS_PF];
            uint32_t pi[FS_PF];
#pragma unroll
            for (int c = 0; c < FS_PF; ++c) fetch(c * FS_B + tid, ps[c], pi[c]);
            int h2 = 1;
            while (h2 < G) h2 <<= 1;
            for (int g = tid; g < h2; g += FS_THREADS) {
                double s = -INFINITY;
                uint32_t id = 0xFFFFFFFFu;
                if (g < G) {
                    if (g == b) {
                        if (nl > 0) {
                            s = L.lsc[cur][0];
                            id = L.lid[cur][0];
                        }
                    } else {
                        s = ld_agent(vs_ + (size_t)g * k);
                        id = ld_agent(vi + (size_t)g * k);
                    }
                }
                L.bsc[g] = s;
                L.bid[g] = id;
            }
            __syncthreads();
            sort_valid_best_first<METRIC_IP>(L.bsc, L.bid, G, h2);
            const bool has_floor = G >= k && L.bid[k - 1] != 0xFFFFFFFFu;
            const double fs = has_floor ? L.bsc[k - 1] : -INFINITY;
            const uint32_t fi = has_floor ? L.bid[k - 1] : 0xFFFFFFFFu;
            __syncthreads();  // (every thread has the floor before the batch is reused)
            int nb = 0;  // entries waiting in the batch (block-uniform)
            for (int c0 = 0, ci = 0; c0 < total; c0 += FS_B, ++ci) {
                const int slot = ci % FS_PF;
                double s = 0.0;
                uint32_t id = 0u;
#pragma unroll
                for (int c = 0; c < FS_PF; ++c)
                    if (c == slot) {
                        s = ps[c];
                        id = pi[c];
                    }
                if (slot == FS_PF - 1)  // this group of chunks is in registers: fetch the next group
#pragma unroll
                    for (int c = 0; c < FS_PF; ++c) fetch(c0 + (c + 1) * FS_B + tid, ps[c], pi[c]);
                bool ok = id != 0xFFFFFFFFu;
                if (ok && has_floor) ok = !fs_better(fs, fi, s, id);  // not below the floor
                if (ok && nl >= k) ok = fs_better(s, id, L.lsc[cur][k - 1], L.lid[cur][k - 1]);
                const u64 m = __ballot(ok);
                if (lane == 0) red_s[wid] = __popcll(m);
                __syncthreads();
                int wb = 0, cnt = 0;
                for (int i = 0; i < FS_NW; ++i) {
                    if (i < wid) wb += red_s[i];
                    cnt += red_s[i];
                }
                if (nb + cnt > FS_B) {  // (block-uniform) make room
                    fs_sort_merge(L, cur, nl, nb, k);
                    nb = 0;
                }
                if (ok) {
                    const int pos = nb + wb + lane_prefix(m);
                    L.bsc[pos] = s;
                    L.bid[pos] = id;
                }
                nb += cnt;
                __syncthreads();
            }
            if (nb > 0) fs_sort_merge(L, cur, nl, nb, k);
        }
        const size_t ost = a.ostride > 1 ? (size_t)a.ostride : 1;
        for (int j = tid; j < k; j += FS_THREADS) {
            const size_t o = (size_t)q * k + j;
            if (j < nl) {
                const double v = METRIC == METRIC_L2 ? -L.lsc[cur][j] : L.lsc[cur][j];
                if (a.D) a.D[o] = (float)v;
                a.I[o * ost] = (int64_t)L.lid[cur][j] + a.id_offset;
                if (a.S64) a.S64[o * ost] = v;
            } else {
                if (a.D) a.D[o] = METRIC == METRIC_L2 ? 3.402823466e+38f : -3.402823466e+38f;
                a.I[o * ost] = -1;
                if (a.S64) a.S64[o * ost] = METRIC == METRIC_L2 ? 1.7976931348623157e308 : -1.7976931348623157e308;
            }
        }
        if (tid == 0) {
            a.cert[q] = 1;
            st_agent(a.gdone + q, 0u);  // ready for the next launch
            if (a.count) atomicAdd(a.count, 1u);
        }
    }
}

template <int DT, int METRIC, bool QLDS>
static void launch_full_scan_one(const FullScanArgs& a, int KL, size_t lds, hipStream_t st) {
    set_lds_attr((const void*)k_full_scan<DT, METRIC, QLDS>, 152 * 1024);
    hipLaunchKernelGGL((k_full_scan<DT, METRIC, QLDS>), dim3(a.G), dim3(FS_THREADS), lds, st, a, KL);
}

template <int DT>
static void launch_full_scan_dt(const FullScanArgs& a, int KL, size_t lds, bool qlds, hipStream_t st) {
    if (a.metric == METRIC_IP) {
        if (qlds) launch_full_scan_one<DT, METRIC_IP, true>(a, KL, lds, st);
        else launch_full_scan_one<DT, METRIC_IP, false>(a, KL, lds, st);
    } else {
        if (qlds) launch_full_scan_one<DT, METRIC_L2, true>(a, KL, lds, st);
        else launch_full_scan_one<DT, METRIC_L2, false>(a, KL, lds, st);
    }
}

size_t full_scan_scratch_bytes(int nq, int G, int k) { return (size_t)nq * G * k * 12; }

hipError_t launch_full_scan(const FullScanArgs& a, hipStream_t st) {
    if (a.nq <= 0 || a.k <= 0 || a.k > KP_MAX || a.G <= 0 || a.G > FS_B || a.n_valid <= 0 || !a.cert || !a.I || !a.gsc || !a.gid ||
        !a.gdone || !a.q || !a.corpus)
        return hipErrorInvalidValue;
    int KL = 64;
    while (KL < a.k) KL <<= 1;
    const size_t base = (size_t)KL * 24 + (size_t)FS_B * 12;
    const size_t qbytes = (size_t)((a.d + 7) >> 3) * 64;
    const bool qlds = base + qbytes <= 148 * 1024;
    const size_t lds = qlds ? base + qbytes : base;
    if (a.dt == DT_F32) launch_full_scan_dt<DT_F32>(a, KL, lds, qlds, st);
    else if (a.dt == DT_BF16) launch_full_scan_dt<DT_BF16>(a, KL, lds, qlds, st);
    else if (a.dt == DT_F16) launch_full_scan_dt<DT_F16>(a, KL, lds, qlds, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace vs
