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
