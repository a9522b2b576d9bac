"""``HNSWGraph``: faiss ``IndexHNSWFlat`` graph search over a :class:`FlatIndex`.

The reference builds ``faiss.IndexHNSWFlat(d, M, metric)`` for ``index_type="hnsw"`` and sets
``hnsw.efSearch`` (/root/reference/utils/vector_store.py:73-78), then searches it at ``:191``.
Here the graph -- the arrays of an IHNf file (:func:`faiss_format.read_hnsw_graph`) or one built
by :func:`faiss_format.single_level_graph` -- lives on the index's GPU next to its rows, and
``search`` runs faiss's ``HNSW::search`` there (include/vs.h "HNSW graph search"): one workgroup per
query, the flat path's exact canonical scores as distances, so the same inputs give the same ids
and scores as ``oracle/hnsw_oracle.py``.
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
