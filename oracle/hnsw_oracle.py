"""TEST INFRASTRUCTURE ONLY -- CPU oracle for HNSW graph search.

Only ``tests/`` may import this module, and only as the checker.  The product
(``photo_search_engine_amd``) never does.

The reference builds ``faiss.IndexHNSWFlat(d, M, metric)`` for ``index_type="hnsw"`` and sets
``hnsw.efConstruction`` / ``hnsw.efSearch`` (/root/reference/utils/vector_store.py:73-78), then
calls ``index.search`` (``:191``).  faiss is third-party (``faiss-cpu>=1.7.0``,
/root/reference/requirements.txt:5), neither vendored nor installed, so its published search
algorithm is restated here (faiss/impl/HNSW.cpp ``HNSW::search``, ``greedy_update_nearest``,
``search_from_candidates``, ``MinimaxHeap``; faiss/utils/Heap.h ``heap_push`` / ``heap_pop`` /
``heap_replace_top`` with the ``CMax::cmp2`` id tie-break; faiss/IndexHNSW.cpp: inner-product
distances are negated so that smaller is better, and negated back on output):

1. ``nearest = entry_point``; on every level ``max_level .. 1`` the greedy descent moves to the
   first strictly closer neighbour until none is (no visited table);
2. level 0: a ``MinimaxHeap`` of capacity ``ef = max(efSearch, k)`` seeded with ``nearest``;
   repeatedly pop its closest valid entry ``v0`` (distance ``d0``), stop when at least
   ``efSearch`` heap entries -- popped ones included -- are closer than ``d0``, else every
   unvisited neighbour of ``v0`` (list order, up to the first -1) is marked visited, scored,
   offered to the result max-heap (size k, admission ``d < D[0]``) and pushed on the candidates
   (when full: rejected if ``d >= max``, else the max is evicted);
3. results sorted best first (``heap_reorder``: ascending distance, ties by id), padded with
   id -1 and -FLT_MAX (IP) / FLT_MAX (L2), the flat path's padding.

Distances here are the flat path's canonical fp64 scores (``oracle.canon_scores``: IP -> -score,
L2 -> squared distance), not faiss's fp32 SIMD sums -- the same exactness contract as the flat
search.  ``search_faiss`` restates the array heaps literally; ``search`` states the same procedure
with the heaps as ordered multisets under the total order (distance, id), which is what the HIP
kernel implements.  The two take identical decisions whenever no two distinct rows are at exactly
equal distance from a query (faiss's choice among exact ties depends on its heap array layout);
tests/test_hnsw_oracle.py checks that they agree.  Parity with faiss itself is unpinned (faiss is
absent); the reference's own HNSW file (tests/golden/ref_photo_search.index, 77 rows, M=48) is
searched by both.
"""
from __future__ import annotations

import bisect
import math
from typing import Tuple

import numpy as np

from . import oracle as O


# ---------------------------------------------------------------------------------------------
# graph layout helpers (faiss HNSW: neighbors of node i on level l are
# neighbors[offsets[i] + cum[l] : offsets[i] + cum[l + 1]], -1 padded)
# ---------------------------------------------------------------------------------------------
def neighbor_list(graph: dict, node: int, level: int):
    off = int(graph["offsets"][node])
    cum = graph["cum_nneighbor_per_level"]
    out = []
    for j in range(off + int(cum[level]), off + int(cum[level + 1])):
        v = int(graph["neighbors"][j])
        if v < 0:
            break
        out.append(v)
    return out


def _distances(x_stored, q, metric) -> np.ndarray:
    """faiss HNSW distance of every (query, row): IP -> -canonical score, L2 -> canonical."""
    S = O.canon_scores(x_stored, q, metric)
    return -S if O._metric(metric) == O.METRIC_IP else S


_FLT_MAX = float(np.finfo(np.float32).max)  # faiss heap neutral (Limits<float>::max), as the flat path


def _output(res, k: int, metric):
    """Sorted (distance, id) pairs -> faiss layout (D fp64 score, I) padded with -1 / -+FLT_MAX."""
    ip = O._metric(metric) == O.METRIC_IP
    S = np.full(k, -_FLT_MAX if ip else _FLT_MAX, dtype=np.float64)
    I = np.full(k, -1, dtype=np.int64)
    for j, (dv, v) in enumerate(res[:k]):
        S[j] = -dv if ip else dv
        I[j] = v
    return S, I


def _greedy_upper(graph, dist_row, nearest: int):
    d_nearest = dist_row[nearest]
    for level in range(int(graph["max_level"]), 0, -1):
        while True:
            prev = nearest
            for v in neighbor_list(graph, nearest, level):
                dv = dist_row[v]
                if dv < d_nearest:
                    nearest, d_nearest = v, dv
            if nearest == prev:
                break
    return nearest, d_nearest


# ---------------------------------------------------------------------------------------------
# literal restatement: faiss array heaps
# ---------------------------------------------------------------------------------------------
def _cmp2(a, b, ia, ib) -> bool:  # CMax<T, TI>::cmp2
    return a > b or (a == b and ia > ib)


def _heap_push(k, val, ids, v, i):  # k = size after the push (faiss passes ++k); 1-based inside
    j = k
    while j > 1:
        f = j >> 1
        if not _cmp2(v, val[f - 1], i, ids[f - 1]):
            break
        val[j - 1], ids[j - 1] = val[f - 1], ids[f - 1]
        j = f
    val[j - 1], ids[j - 1] = v, i


def _sift_down(k, val, ids, v, i):
    j = 1
    while True:
        j1 = j << 1
        j2 = j1 + 1
        if j1 > k:
            break
        if j2 == k + 1 or _cmp2(val[j1 - 1], val[j2 - 1], ids[j1 - 1], ids[j2 - 1]):
            if _cmp2(v, val[j1 - 1], i, ids[j1 - 1]):
                break
            val[j - 1], ids[j - 1] = val[j1 - 1], ids[j1 - 1]
            j = j1
        else:
            if _cmp2(v, val[j2 - 1], i, ids[j2 - 1]):
                break
            val[j - 1], ids[j - 1] = val[j2 - 1], ids[j2 - 1]
            j = j2
    return j


def _heap_pop(k, val, ids):  # k = size before the pop
    v, i = val[k - 1], ids[k - 1]
    j = _sift_down(k, val, ids, v, i)
    val[j - 1], ids[j - 1] = val[k - 1], ids[k - 1]


def _heap_replace_top(k, val, ids, v, i):
    j = _sift_down(k, val, ids, v, i)
    val[j - 1], ids[j - 1] = v, i


class _MinimaxHeap:
    def __init__(self, n: int):
        self.n, self.k, self.nvalid = n, 0, 0
        self.ids = [-1] * n
        self.dis = [math.inf] * n

    def push(self, i, v):
        if self.k == self.n:
            if v >= self.dis[0]:
                return
            if self.ids[0] != -1:
                self.nvalid -= 1
            _heap_pop(self.k, self.dis, self.ids)
            self.k -= 1
        self.k += 1
        _heap_push(self.k, self.dis, self.ids, v, i)
        self.nvalid += 1

    def pop_min(self):
        i = self.k - 1
        while i >= 0 and self.ids[i] == -1:
            i -= 1
        if i < 0:
            return -1, math.inf
        imin, vmin = i, self.dis[i]
        i -= 1
        while i >= 0:
            if self.ids[i] != -1 and self.dis[i] < vmin:
                vmin, imin = self.dis[i], i
            i -= 1
        ret = self.ids[imin]
        self.ids[imin] = -1
        self.nvalid -= 1
        return ret, vmin

    def count_below(self, t) -> int:
        return sum(1 for i in range(self.k) if self.dis[i] < t)


def _search_one_faiss(graph, dist_row, k: int, ef_search: int):
    n = len(dist_row)
    if int(graph["entry_point"]) < 0 or n == 0:
        return []
    nearest, d_nearest = _greedy_upper(graph, dist_row, int(graph["entry_point"]))
    cand = _MinimaxHeap(max(ef_search, k))
    cand.push(nearest, d_nearest)
    D = [math.inf] * k
    I = [-1] * k
    nres = 0
    visited = np.zeros(n, dtype=bool)
    for i in range(cand.k):  # search_from_candidates: the seeds enter the results
        v1, dv = cand.ids[i], cand.dis[i]
        if nres < k:
            nres += 1
            _heap_push(nres, D, I, dv, v1)
        elif dv < D[0]:
            _heap_replace_top(nres, D, I, dv, v1)
        visited[v1] = True
    while cand.nvalid > 0:
        v0, d0 = cand.pop_min()
        if cand.count_below(d0) >= ef_search:
            break
        for v1 in neighbor_list(graph, v0, 0):
            if visited[v1]:
                continue
            visited[v1] = True
            dv = dist_row[v1]
            if nres < k:
                nres += 1
                _heap_push(nres, D, I, dv, v1)
            elif dv < D[0]:
                _heap_replace_top(nres, D, I, dv, v1)
            cand.push(v1, dv)
    # heap_reorder: pops in cmp2 order -> ascending (distance, id)
    return sorted((D[j], I[j]) for j in range(nres))


def search_faiss(x_stored, graph: dict, q, k: int, ef_search: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """faiss ``IndexHNSWFlat.search`` restated with its array heaps: (S fp64 nq x k, I nq x k)."""
    q = np.atleast_2d(np.asarray(q, dtype=np.float32))
    Dm = _distances(x_stored, q, metric)
    S = np.empty((q.shape[0], k), dtype=np.float64)
    I = np.empty((q.shape[0], k), dtype=np.int64)
    for r in range(q.shape[0]):
        S[r], I[r] = _output(_search_one_faiss(graph, Dm[r], k, ef_search), k, metric)
    return S, I


# ---------------------------------------------------------------------------------------------
# ordered-multiset statement (the HIP kernel's): heaps as sorted lists under (distance, id)
# ---------------------------------------------------------------------------------------------
def _search_one(graph, dist_row, k: int, ef_search: int):
    n = len(dist_row)
    if int(graph["entry_point"]) < 0 or n == 0:
        return []
    nearest, d_nearest = _greedy_upper(graph, dist_row, int(graph["entry_point"]))
    ef = max(ef_search, k)
    cand = [(d_nearest, nearest, True)]  # sorted by (distance, id); popped entries stay (valid False)
    res = [(d_nearest, nearest)]
    visited = np.zeros(n, dtype=bool)
    visited[nearest] = True
    while any(c[2] for c in cand):
        j = next(i for i, c in enumerate(cand) if c[2])
        d0, v0, _ = cand[j]
        cand[j] = (d0, v0, False)
        if bisect.bisect_left([c[0] for c in cand], d0) >= ef_search:
            break
        for v1 in neighbor_list(graph, v0, 0):
            if visited[v1]:
                continue
            visited[v1] = True
            e = (dist_row[v1], v1)
            bisect.insort(res, e)
            del res[k:]
            bisect.insort(cand, (e[0], e[1], True))
            del cand[ef:]
    return res


def search(x_stored, graph: dict, q, k: int, ef_search: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """HNSW search with ordered-multiset heaps (the HIP kernel's statement): (S fp64, I)."""
    q = np.atleast_2d(np.asarray(q, dtype=np.float32))
    Dm = _distances(x_stored, q, metric)
    S = np.empty((q.shape[0], k), dtype=np.float64)
    I = np.empty((q.shape[0], k), dtype=np.int64)
    for r in range(q.shape[0]):
        S[r], I[r] = _output(_search_one(graph, Dm[r], k, ef_search), k, metric)
    return S, I


# ---------------------------------------------------------------------------------------------
# test graphs
# ---------------------------------------------------------------------------------------------
def _default_probas(M: int):
    """faiss ``HNSW::set_default_probas(M, 1 / log(M))``: level probabilities and cumulative
    neighbour counts (2M on level 0, M above)."""
    lm = 1.0 / math.log(M)
    probas, cum, level = [], [0], 0
    while True:
        p = math.exp(-level / lm) * (1.0 - math.exp(-1.0 / lm))
        if p < 1e-9:
            break
        probas.append(p)
        cum.append(cum[-1] + (2 * M if level == 0 else M))
        level += 1
    return np.array(probas, dtype="<f8"), np.array(cum, dtype="<i4")


def layered_knn_graph(x_stored, M: int, metric="ip", seed: int = 1, level_mult=None) -> dict:
    """A multi-level graph in faiss's HNSW layout for exercising the search (test-only): node
    levels drawn as faiss does (``-log(U) * 1/ln(M)``, seeded numpy RNG -- not faiss's generator),
    and on every level each node's neighbours are its exact nearest nodes of that level (2M on
    level 0, M above), best first, -1 padded."""
    x = np.asarray(x_stored, dtype=np.float32)
    n = x.shape[0]
    probas, cum = _default_probas(M)
    rng = np.random.default_rng(seed)
    lm = (1.0 / math.log(M)) if level_mult is None else level_mult
    lev = np.minimum((-np.log(rng.random(n)) * lm).astype(np.int64), len(cum) - 2)
    levels = lev + 1
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(cum[levels].astype(np.uint64))
    nb = np.full(int(offsets[-1]), -1, dtype=np.int32)
    S = O.canon_scores(x, x, metric)
    ip = O._metric(metric) == O.METRIC_IP
    for level in range(int(lev.max()) + 1):
        members = np.nonzero(lev >= level)[0]
        width = int(cum[level + 1] - cum[level])
        for i in members:
            others = members[members != i]
            s = S[i, others]
            order = np.lexsort((others, -s if ip else s))[:width]
            base = int(offsets[i]) + int(cum[level])
            nb[base:base + len(order)] = others[order]
    top = int(lev.max())
    entry = int(np.nonzero(lev == top)[0][0])
    return {"assign_probas": probas, "cum_nneighbor_per_level": cum, "levels": levels.astype(np.int32),
            "offsets": offsets, "neighbors": nb, "entry_point": entry, "max_level": top,
            "efConstruction": 40, "efSearch": 16, "upper_beam": 1}


def has_exact_ties(x_stored, q, metric="ip") -> bool:
    """True if some query is at exactly equal distance from two distinct rows."""
    Dm = _distances(x_stored, np.atleast_2d(np.asarray(q, dtype=np.float32)), metric)
    return any(len(np.unique(r)) != len(r) for r in Dm)


# ---------------------------------------------------------------------------------------------
# graph build: faiss's neighbour-selection heuristic
# ---------------------------------------------------------------------------------------------
def shrink_neighbor_list(dist, node: int, cand, W: int):
    """faiss ``HNSW::shrink_neighbor_list`` (faiss/impl/HNSW.cpp; reached from ``add_links_starting_
    from`` and ``add_link`` through the static overload that returns early when fewer than
    ``max_size`` candidates are offered): candidates in ascending (distance to ``node``, id) order,
    one kept unless an already kept neighbour is strictly closer to it than ``node`` is, stopping
    at ``W`` kept.  ``dist[a, b]`` = distance with ``a`` as the query and ``b`` as the row (the
    flat path's canonical fp64 value; IP: -score).  faiss orders equal distances by its heap; the
    (distance, id) order here is what the HIP kernel (k_hnsw_prune) implements."""
    cand = [int(c) for c in cand if c >= 0]
    if len(cand) < W:
        return sorted(cand, key=lambda c: (dist[node, c], c))
    order = sorted(cand, key=lambda c: (dist[node, c], c))
    kept = []
    for c in order:
        dq = dist[node, c]
        if all(not (dist[c, r] < dq) for r in kept):
            kept.append(c)
            if len(kept) >= W:
                break
    return kept


HP_C_MAX = 2048  # largest candidate list of one node (include/vs.h vs_hnsw_prune)


def select_level(dist, members, cand_lists, W: int, cmax: int = HP_C_MAX):
    """One level of the batch build (photo_search_engine_amd/hnsw.py ``select_level``): every member's
    forward list = shrink(its candidates, W) (faiss, on inserting a node: shrink its efConstruction
    candidates to the level's width); then every member j receives the reverse links i -> j and
    keeps its forward list followed by the new sources in ascending id, unpruned while that fits W
    (faiss ``add_link`` appends while a list has room), else shrunk to W over the union (faiss
    ``add_link`` on a full list); a union longer than ``cmax`` is cut there first."""
    members = [int(v) for v in members]
    F = {v: shrink_neighbor_list(dist, v, cand_lists[i], W) for i, v in enumerate(members)}
    R = {v: [] for v in members}
    for i in members:
        for j in F[i]:
            R[j].append(i)
    out = {}
    for j in members:
        fs = set(F[j])
        U = (F[j] + [i for i in R[j] if i not in fs])[:cmax]
        out[j] = U if len(U) <= W else shrink_neighbor_list(dist, j, U, W)
    return out


def heuristic_graph(x_stored, M: int, ef_construction: int, metric="ip", levels=None, seed: int = 12345) -> dict:
    """The graph ``VectorStore._build_graph`` writes, restated: node levels as it draws them
    (numpy's generator, ``seed``; or ``levels``, 1-based), and on every level each
    member's candidates are its exact max(efConstruction, width) nearest members (itself excluded,
    ties -> lower id), then :func:`select_level`.  Entry point: the first node of the top level."""
    x = np.asarray(x_stored, dtype=np.float32)
    n = x.shape[0]
    probas, cum = _default_probas(M)
    if levels is None:
        f = np.random.default_rng(seed).random(n)
        lev = np.full(n, len(probas) - 1, dtype=np.int64)
        open_ = np.ones(n, dtype=bool)
        for level, p in enumerate(probas):
            hit = open_ & (f < p)
            lev[hit] = level
            open_ &= ~hit
            f[open_] -= p
    else:
        lev = np.asarray(levels, dtype=np.int64) - 1
    dist = _distances(x, x, metric)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(cum[lev + 1].astype(np.uint64))
    nb = np.full(int(offsets[-1]), -1, dtype=np.int32)
    top = int(lev.max()) if n else -1
    for level in range(top + 1):
        members = np.nonzero(lev >= level)[0]
        width = int(cum[level + 1] - cum[level])
        C = min(max(ef_construction, width), members.shape[0] - 1, HP_C_MAX)
        cands = []
        for i in members:
            others = members[members != i]
            order = np.lexsort((others, dist[i, others]))[:C]
            cands.append(others[order])
        sel = select_level(dist, members, cands, width)
        for i in members:
            base = int(offsets[i]) + int(cum[level])
            row = sel[int(i)]
            nb[base:base + len(row)] = row
    return {"assign_probas": probas, "cum_nneighbor_per_level": cum, "levels": (lev + 1).astype(np.int32),
            "offsets": offsets, "neighbors": nb, "entry_point": int(np.nonzero(lev == top)[0][0]) if n else -1,
            "max_level": top, "efConstruction": int(ef_construction), "efSearch": 16, "upper_beam": 1}


# ---------------------------------------------------------------------------------------------
# incremental build: faiss's insertion (IndexHNSWFlat.add of new rows), batched
# ---------------------------------------------------------------------------------------------
def draw_levels(n: int, probas, seed: int = 12345) -> np.ndarray:
    """0-based node levels as ``VectorStore._build_graph`` draws them (numpy's generator, seeded;
    faiss's ``random_level`` rule over ``assign_probas``).  The stream is prefix-consistent: the
    first n of a longer draw are these, so a graph extended row by row keeps every old level."""
    f = np.random.default_rng(seed).random(n)
    lev = np.full(n, len(probas) - 1, dtype=np.int64)
    open_ = np.ones(n, dtype=bool)
    for level, p in enumerate(probas):
        hit = open_ & (f < p)
        lev[hit] = level
        open_ &= ~hit
        f[open_] -= p
    return lev


def insert_batch(x_stored, graph: dict, n_old: int, ef_construction: int, metric="ip", seed: int = 12345,
                 cmax: int = HP_C_MAX) -> dict:
    """The graph ``hnsw.insert_rows`` makes of ``graph`` (nodes [0, n_old)) and the new rows
    [n_old, n) of ``x_stored``, restated.  faiss inserts one node at a time: on each of its levels
    it takes efConstruction candidates from a beam over the graph so far, keeps a shrunk list
    (``shrink_neighbor_list``) and links back (``add_link``).  The batch form: for a new node u and
    each level l <= level(u), its candidates are
      * level 0: the best C = max(efConstruction, width) of a beam search over the OLD graph
        (``_search_one``, ef = efConstruction, k = C), and
      * level >= 1: the exact best C old level-l members (the upper levels are small),
    together with the exact best C new nodes of level >= l (itself excluded); the union goes through
    the heuristic, forward lists first; then every node v named by a new forward list receives the
    new sources: a new v keeps its forward list followed by them (ascending, unlisted ones), an old
    v its old list followed by them -- unpruned while that fits the width, else shrunk over the
    union (cut at ``cmax`` first).  A new node above the old top level becomes the entry point
    (the first such of the highest level)."""
    x = np.asarray(x_stored, dtype=np.float32)
    n = x.shape[0]
    probas = np.asarray(graph["assign_probas"])
    cum = np.asarray(graph["cum_nneighbor_per_level"])
    old_lev = np.asarray(graph["levels"], dtype=np.int64)[:n_old] - 1
    lev = np.concatenate([old_lev, draw_levels(n, probas, seed)[n_old:]])  # new node i: entry i of the draw
    dist = _distances(x, x, metric)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(cum[lev + 1].astype(np.uint64))
    nb = np.full(int(offsets[-1]), -1, dtype=np.int32)
    old_off = np.asarray(graph["offsets"], dtype=np.uint64)
    nb[:int(old_off[n_old])] = np.asarray(graph["neighbors"], dtype=np.int32)[:int(old_off[n_old])]
    old = {"levels": old_lev + 1, "offsets": old_off[:n_old + 1], "neighbors": graph["neighbors"],
           "cum_nneighbor_per_level": cum, "entry_point": graph["entry_point"], "max_level": graph["max_level"]}
    new = np.arange(n_old, n)
    top_new = int(lev[new].max()) if new.size else -1
    for level in range(max(top_new, -1), -1, -1):
        width = int(cum[level + 1] - cum[level])
        C = min(max(int(ef_construction), width), cmax)
        nmem = new[lev[new] >= level]
        omem = np.nonzero(old_lev >= level)[0]
        cands = {}
        for u in nmem:
            u = int(u)
            if level == 0 and n_old > 0:
                # the beam over the old graph: its rows only (distance row restricted to [0, n_old))
                res = _search_one(old, dist[u, :n_old], C, int(ef_construction))
                oc = [v for _, v in res]
            else:
                oc = [int(v) for v in omem[np.lexsort((omem, dist[u, omem]))[:C]]] if omem.size else []
            others = nmem[nmem != u]
            bc = [int(v) for v in others[np.lexsort((others, dist[u, others]))[:C]]] if others.size else []
            cands[u] = sorted(set(oc) | set(bc))
        F = {int(u): shrink_neighbor_list(dist, int(u), cands[int(u)], width) for u in nmem}
        R = {}
        for u in sorted(F):
            for v in F[u]:
                R.setdefault(v, []).append(u)
        for v in sorted(set(F) | set(R)):
            base = int(offsets[v]) + int(cum[level])
            if v >= n_old:
                head = F[v]
            else:
                head = [int(t) for t in nb[base:base + width] if t >= 0]
            hs = set(head)
            U = (head + [u for u in sorted(R.get(v, [])) if u not in hs])[:cmax]
            row = U if len(U) <= width else shrink_neighbor_list(dist, v, U, width)
            nb[base:base + width] = -1
            nb[base:base + len(row)] = row
    entry, top = int(graph["entry_point"]), int(graph["max_level"])
    if top_new > top or entry < 0:
        top = top_new
        entry = int(new[lev[new] == top_new][0])
    out = dict(graph)
    out.update({"levels": (lev + 1).astype(np.int32), "offsets": offsets, "neighbors": nb, "entry_point": entry,
                "max_level": top, "efConstruction": int(ef_construction)})
    return out
