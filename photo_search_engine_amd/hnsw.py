"""``HNSWGraph``: faiss ``IndexHNSWFlat`` graph search over a :class:`FlatIndex`.

The reference builds ``faiss.IndexHNSWFlat(d, M, metric)`` for ``index_type="hnsw"`` and sets
``hnsw.efSearch`` (/root/reference/utils/vector_store.py:73-78), then searches it at ``:191``.
Here the graph -- the arrays of an IHNf file (:func:`faiss_format.read_hnsw_graph`) or one built
by :func:`faiss_format.single_level_graph` -- lives on the index's GPU next to its rows, and
``search`` runs faiss's ``HNSW::search`` there (include/vs.h "HNSW graph search"): one workgroup per
query, the flat path's exact canonical scores as distances, so the same inputs give the same ids
and scores as ``oracle/hnsw_oracle.py``.

Graph build: :func:`select_level` applies faiss's neighbour-selection heuristic
(``HNSW::shrink_neighbor_list``, which ``IndexHNSWFlat.add`` runs at /root/reference/utils/
vector_store.py:164) to one level's candidate lists on the GPU (``vs_hnsw_prune``), then adds the
reverse links the way faiss's ``add_link`` does: appended while a list has room, the list re-shrunk
over the union once it would overflow.  ``VectorStore._build_graph`` feeds it exact candidates.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class HNSWGraph:
    """A faiss-layout HNSW graph over the rows of ``index`` (node i = row i)."""

    def __init__(self, index, graph: dict, ef_search: Optional[int] = None) -> None:
        self._h = None
        from .index import FlatIndex
        if not isinstance(index, FlatIndex):  # (vs_hnsw_create reads a one-device vs_index)
            raise TypeError("HNSWGraph indexes the rows of a FlatIndex; a multi-device index searches its "
                            "graph through its own hnsw_search (a one-device copy of the rows)")
        L = _lib.load()
        levels = np.ascontiguousarray(graph["levels"], dtype=np.int32)
        n = int(levels.shape[0])
        offsets = np.ascontiguousarray(graph["offsets"], dtype=np.uint64)
        neighbors = np.ascontiguousarray(graph["neighbors"], dtype=np.int32)
        cum = np.ascontiguousarray(graph["cum_nneighbor_per_level"], dtype=np.int32)
        if offsets.shape[0] != n + 1:
            raise ValueError("offsets must hold n + 1 entries")
        if n and int(offsets[-1]) != neighbors.shape[0]:
            raise ValueError("offsets[n] must equal the neighbour array's length")
        h = ctypes.c_void_p()
        check(L.vs_hnsw_create(index._h, n, _ptr(levels), _ptr(offsets), _ptr(neighbors), _ptr(cum),
                               int(cum.shape[0]), int(graph["entry_point"]), int(graph["max_level"]),
                               ctypes.byref(h)))
        self._h = h
        self._L = L
        self.index = index  # the rows the graph indexes must outlive it
        self.d = index.d
        self.ntotal = n
        self.efSearch = int(ef_search if ef_search is not None else graph.get("efSearch", 16))

    def search(self, q, k: int, ef_search: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """faiss ``IndexHNSWFlat.search``: (D float32 nq x k, I int64 nq x k), best first, -1 padded."""
        q = np.ascontiguousarray(q, dtype=np.float32)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        if q.ndim != 2 or q.shape[1] != self.d:
            raise ValueError(f"queries must be (nq, {self.d})")
        k = int(k)
        if k <= 0:
            raise _lib.VsError(_lib.VS_ERR_ARG, "k must be > 0")
        nq = q.shape[0]
        D = np.empty((nq, k), dtype=np.float32)
        I = np.empty((nq, k), dtype=np.int64)
        check(self._L.vs_hnsw_search(self._h, _ptr(q), nq, k, int(ef_search or self.efSearch), _ptr(D), _ptr(I)))
        return D, I

    def patch(self, pos: np.ndarray, val: np.ndarray, entry_point: int, max_level: int) -> None:
        """Rewrite neighbour slots ``pos`` (indices into the neighbour array) with ``val`` and set the
        entry point / top level (include/vs.h ``vs_hnsw_patch``)."""
        pos = np.ascontiguousarray(pos, dtype=np.uint64)
        val = np.ascontiguousarray(val, dtype=np.int32)
        if pos.shape != val.shape:
            raise ValueError("pos and val must have the same length")
        check(self._L.vs_hnsw_patch(self._h, int(pos.shape[0]), _ptr(pos), _ptr(val), int(entry_point),
                                    int(max_level)))

    def close(self) -> None:
        if self._h is not None:
            self._L.vs_hnsw_destroy(self._h)
            self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass


HP_C_MAX = 2048  # largest candidate list of one node (include/vs.h vs_hnsw_prune)


def prune_neighbors(index, nodes, cand, W: int) -> np.ndarray:
    """faiss ``HNSW::shrink_neighbor_list`` for every node, by the index (``FlatIndex.hnsw_prune``:
    ``vs_hnsw_prune`` on the GPU): ``cand`` (m x C, distinct row ids, -1 padded at the end) ->
    (m x W) kept ids best first, -1 padded."""
    return index.hnsw_prune(nodes, cand, int(W))


def select_level(index, members, cand, W: int, cmax: int = HP_C_MAX) -> np.ndarray:
    """One level of the batch build (oracle/hnsw_oracle.py ``select_level``): ``members`` ascending
    row ids, ``cand`` (m x C) their candidate row ids best first (-1 padded).  Forward lists =
    shrink(candidates, W); each member then keeps its forward list followed by the members that
    linked to it (ascending id, those already listed skipped) -- unpruned while that fits W, shrunk
    to W over the union otherwise (a union longer than ``cmax`` is cut there first).  Returns
    (m x W) neighbour ids, -1 padded."""
    members = np.ascontiguousarray(members, dtype=np.int64)
    m = members.shape[0]
    W = int(W)
    F = prune_neighbors(index, members, cand, W)
    if m == 0:
        return F
    # (owner row, neighbour, group, key): forward entries keep their order, reverse ones ascend by source
    fr, fc = np.nonzero(F >= 0)
    fwd_owner, fwd_nb = fr, F[fr, fc].astype(np.int64)
    rev_owner = np.searchsorted(members, fwd_nb)
    rev_nb = members[fr]
    n_glob = int(members[-1]) + 1
    dup = np.isin(rev_owner * n_glob + rev_nb, fwd_owner * n_glob + fwd_nb)
    rev_owner, rev_nb = rev_owner[~dup], rev_nb[~dup]
    owner = np.concatenate([fwd_owner, rev_owner])
    nb = np.concatenate([fwd_nb, rev_nb])
    group = np.concatenate([np.zeros(fwd_owner.shape[0], np.int64), np.ones(rev_owner.shape[0], np.int64)])
    key = np.concatenate([fc.astype(np.int64), rev_nb])
    o = np.lexsort((key, group, owner))
    owner, nb = owner[o], nb[o]
    counts = np.bincount(owner, minlength=m)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    pos = np.arange(owner.shape[0]) - starts[owner]
    keep = pos < cmax
    owner, nb, pos = owner[keep], nb[keep], pos[keep]
    counts = np.minimum(counts, cmax)
    U = np.full((m, int(counts.max())), -1, dtype=np.int32)
    U[owner, pos] = nb
    out = np.full((m, W), -1, dtype=np.int32)
    small = counts <= W
    out[small] = U[small, :W] if U.shape[1] >= W else np.pad(U[small], ((0, 0), (0, W - U.shape[1])),
                                                             constant_values=-1)
    big = np.nonzero(~small)[0]
    if big.size:
        Ub = U[big, :int(counts[big].max())]
        out[big] = prune_neighbors(index, members[big], Ub, W)
    return out


# ---------------------------------------------------------------------------------------------
# incremental build (faiss IndexHNSWFlat.add of new rows, batched)
# ---------------------------------------------------------------------------------------------
def draw_levels(n: int, probas, seed: int = 12345) -> np.ndarray:
    """0-based node levels: faiss's ``random_level`` rule over ``assign_probas`` with numpy's
    generator (seeded; not faiss's).  Prefix-consistent: a longer draw starts with these, so a
    graph extended by insertions keeps every old node's level."""
    f = np.random.default_rng(seed).random(n)
    lev = np.full(n, len(probas) - 1, dtype=np.int64)
    open_ = np.ones(n, dtype=bool)
    for level, p in enumerate(probas):
        hit = open_ & (f < p)
        lev[hit] = level
        open_ &= ~hit
        f[open_] -= p
    return lev


def beam_search(index, graph: dict, q: np.ndarray, k: int, ef: int) -> np.ndarray:
    """Ids (nq x k, -1 padded) of faiss's HNSW search over ``graph`` (the GPU kernel, or the
    index's own ``hnsw_search`` where it has one)."""
    f = getattr(index, "hnsw_search", None)
    if f is not None:
        return f(graph, q, k, ef)
    g = HNSWGraph(index, graph, ef)
    try:
        return g.search(q, k, ef)[1]
    finally:
        g.close()


def _exact_candidates(make_index, index, members: np.ndarray, queries: np.ndarray, C: int,
                      exclude_self: bool) -> list:
    """Per query node (global id in ``queries``): its exact best C of ``members`` (ascending global
    ids), by a temporary flat index over their stored values (ties -> lower id), itself excluded."""
    out = [[] for _ in range(queries.shape[0])]
    m = int(members.shape[0])
    if m == 0 or queries.shape[0] == 0:
        return out
    tmp = make_index()
    try:
        for r0 in range(0, m, 65536):
            tmp.add(np.ascontiguousarray(_rows(index, members[r0:r0 + 65536])))
        kk = min(m, C + (1 if exclude_self else 0))
        for r0 in range(0, queries.shape[0], 4096):
            qs = queries[r0:r0 + 4096]
            _, I = tmp.search(np.ascontiguousarray(_rows(index, qs)), kk)
            for a in range(qs.shape[0]):
                row = [int(members[i]) for i in I[a] if i >= 0]
                if exclude_self:
                    row = [v for v in row if v != int(qs[a])]
                out[r0 + a] = row[:C]
    finally:
        close = getattr(tmp, "close", None)
        if close:
            close()
    return out


def _rows(index, ids: np.ndarray) -> np.ndarray:
    """Stored values of rows ``ids`` (ascending or not), by contiguous runs."""
    ids = np.asarray(ids, dtype=np.int64)
    out = np.empty((ids.shape[0], index.d), dtype=np.float32)
    if ids.size == 0:
        return out
    order = np.argsort(ids, kind="stable")
    s = ids[order]
    cuts = np.nonzero(np.diff(s) != 1)[0] + 1
    for seg in np.split(np.arange(s.shape[0]), cuts):
        lo, hi = int(s[seg[0]]), int(s[seg[-1]]) + 1
        out[order[seg]] = index.reconstruct_n(lo, hi - lo)
    return out


def insert_rows(index, graph: dict, n_old: int, n: int, ef_construction: int, make_index, seed: int = 12345,
                batch: int = 4096, cmax: int = HP_C_MAX) -> dict:
    """Extend ``graph`` (nodes [0, n_old) of ``index``'s rows) to nodes [0, n) the way faiss's
    ``IndexHNSWFlat.add`` inserts rows (/root/reference/utils/vector_store.py:164), in batches of
    ``batch`` rows: for a new node on each of its levels, the candidates are the best C =
    max(efConstruction, width) old nodes -- on level 0 from faiss's search over the old graph
    (beam efConstruction), above it exactly (the upper levels are small) -- together with the
    exact best C new nodes of that level; the heuristic keeps its forward list
    (``vs_hnsw_prune``); every node it names gets the new sources appended (faiss ``add_link``),
    the list re-shrunk over the union when it would overflow.  A new node above the old top level
    becomes the entry point.  Equal to ``oracle/hnsw_oracle.py insert_batch`` batch by batch.

    Cost: the node levels, offsets and the neighbour array are laid out ONCE for the final n (a
    node's slots never move), and ONE device graph over them serves every batch's beams -- nodes
    not inserted yet have empty lists and nothing links to them, so they are unreachable -- patched
    after each batch with the slots it wrote (``vs_hnsw_patch``).  Each batch costs its own rows
    and links, not the graph's size."""
    if n_old >= n:
        return graph
    probas = np.asarray(graph["assign_probas"])
    cum = np.asarray(graph["cum_nneighbor_per_level"]).astype(np.int64)
    # old nodes keep the graph's levels (a faiss-built graph's included); new node i gets entry i of
    # this build's draw
    old_lev = np.asarray(graph["levels"], dtype=np.int64)[:n_old] - 1
    lev = np.concatenate([old_lev, draw_levels(n, probas, seed)[n_old:]])
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(cum[lev + 1].astype(np.uint64))
    old_off = np.asarray(graph["offsets"], dtype=np.uint64)
    nb = np.full(int(offsets[-1]), -1, dtype=np.int32)
    nb[:int(old_off[n_old])] = np.asarray(graph["neighbors"], dtype=np.int32)[:int(old_off[n_old])]
    st = {"lev": lev, "offsets": offsets, "nb": nb, "cum": cum, "entry": int(graph["entry_point"]),
          "top": int(graph["max_level"])}
    full = dict(graph, levels=(lev + 1).astype(np.int32), offsets=offsets, neighbors=nb)
    dev = None
    try:
        while n_old < n:
            n1 = min(n, n_old + int(batch))
            if n_old > 0 and dev is None:  # the beams' graph (nodes >= n_old unreachable until patched)
                dev = _beam_graph(index, full, st, ef_construction)
            pos = _insert_batch(index, st, n_old, n1, int(ef_construction), make_index, cmax, dev)
            if dev is not None and n1 < n:
                dev.patch(pos, nb[pos.astype(np.int64)], st["entry"], st["top"])
            n_old = n1
    finally:
        if dev is not None:
            dev.close()
    out = dict(graph)
    out.update({"levels": (lev + 1).astype(np.int32), "offsets": offsets, "neighbors": nb, "entry_point": st["entry"],
                "max_level": st["top"], "efConstruction": int(ef_construction)})
    return out


class _IndexBeams:
    """The beams of an index that searches a graph dict itself (``hnsw_search``: the test checker):
    a snapshot of the in-place arrays, taken at creation and at every patch, as the device graph
    sees them (nothing a batch writes is visible to its own beams)."""

    def __init__(self, index, full: dict, st: dict) -> None:
        self.index, self.full, self.st = index, full, st
        self.patch(None, None, st["entry"], st["top"])

    def search(self, q, k: int, ef: int):
        return None, self.index.hnsw_search(self.g, q, k, ef)

    def patch(self, pos, val, entry_point: int, max_level: int) -> None:
        self.g = dict(self.full, neighbors=np.array(self.full["neighbors"], copy=True), entry_point=int(entry_point),
                      max_level=int(max_level))

    def close(self) -> None:
        pass


def _beam_graph(index, full: dict, st: dict, ef: int):
    if hasattr(index, "_one_device_copy"):  # multi-device rows: the HNSW kernels read one device's HBM
        return HNSWGraph(index._one_device_copy(), dict(full, entry_point=st["entry"], max_level=st["top"]), ef)
    if hasattr(index, "hnsw_search"):
        return _IndexBeams(index, full, st)
    return HNSWGraph(index, dict(full, entry_point=st["entry"], max_level=st["top"]), ef)


def _insert_batch(index, st: dict, n_old: int, n: int, ef_construction: int, make_index, cmax: int,
                  dev) -> np.ndarray:
    """Insert nodes [n_old, n) into the in-place arrays of ``st``; returns the neighbour slots it
    wrote (for the device graph's patch).  ``dev``: the device graph of nodes [0, n_old)."""
    lev, offsets, nb, cum = st["lev"], st["offsets"], st["nb"], st["cum"]
    old_lev = lev[:n_old]
    new = np.arange(n_old, n, dtype=np.int64)
    top_new = int(lev[new].max()) if new.size else -1
    written = []
    for level in range(top_new, -1, -1):
        width = int(cum[level + 1] - cum[level])
        C = min(max(ef_construction, width), cmax)
        nmem = new[lev[new] >= level]
        omem = np.nonzero(old_lev >= level)[0]
        if level == 0 and n_old > 0:
            I = dev.search(np.ascontiguousarray(_rows(index, nmem)), C, ef_construction)[1]
            oc = [[int(v) for v in row if v >= 0] for row in I]
        else:
            oc = _exact_candidates(make_index, index, omem, nmem, C, exclude_self=False)
        bc = _exact_candidates(make_index, index, nmem, nmem, C, exclude_self=True)
        union = [sorted(set(a) | set(b)) for a, b in zip(oc, bc)]
        U = np.full((nmem.shape[0], max(1, max((len(u) for u in union), default=1))), -1, dtype=np.int32)
        for i, u in enumerate(union):
            U[i, :len(u)] = u
        F = index.hnsw_prune(nmem, U, width) if nmem.size else np.zeros((0, width), dtype=np.int32)
        # reverse links: every node named by a new forward list gets the new sources
        src = {}
        for i, u in enumerate(nmem.tolist()):
            for v in F[i][F[i] >= 0].tolist():
                src.setdefault(v, []).append(u)
        fwd = {u: F[i][F[i] >= 0].tolist() for i, u in enumerate(nmem.tolist())}
        targets = sorted(set(fwd) | set(src))
        heads, lists = [], []
        for v in targets:
            base = int(offsets[v]) + int(cum[level])
            head = fwd[v] if v >= n_old else [int(t) for t in nb[base:base + width] if t >= 0]
            hs = set(head)
            lists.append((head + [u for u in sorted(src.get(v, [])) if u not in hs])[:cmax])
            heads.append(v)
        big = [i for i, L in enumerate(lists) if len(L) > width]
        if big:
            Ub = np.full((len(big), max(len(lists[i]) for i in big)), -1, dtype=np.int32)
            for r, i in enumerate(big):
                Ub[r, :len(lists[i])] = lists[i]
            shr = index.hnsw_prune(np.array([heads[i] for i in big], dtype=np.int64), Ub, width)
            for r, i in enumerate(big):
                lists[i] = shr[r][shr[r] >= 0].tolist()
        for v, L in zip(heads, lists):
            base = int(offsets[v]) + int(cum[level])
            nb[base:base + width] = -1
            nb[base:base + len(L)] = L
            written.append(np.arange(base, base + width, dtype=np.uint64))
    if new.size and (top_new > st["top"] or st["entry"] < 0):
        st["top"] = top_new
        st["entry"] = int(new[lev[new] == top_new][0])
    return np.concatenate(written) if written else np.zeros(0, dtype=np.uint64)
