"""``IVFFlatIndex``: the faiss ``IndexIVFFlat``-shaped handle over libvs.

The reference's ``VectorStore`` offers flat and HNSW indexes only
(/root/reference/utils/vector_store.py:51-53, 72-81); IVF-Flat is the next index family its
faiss dependency (``faiss-cpu>=1.7.0``, requirements.txt:5) provides, rebuilt for MI355X:
``train`` (k-means; assignments on the GPU through the exact coarse quantizer, centroid means on
the host in fp64), ``add``, ``search`` with ``nprobe``, ``reconstruct``.  Searches are exact
*within the probed lists* (include/vs.h "IVF-Flat"): the same inputs give the same ids and fp64
scores as ``oracle/ivf_oracle.py``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import DTYPE_CODES, METRIC_IP, METRIC_L2, check


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class IVFFlatIndex:
    """Inverted-file index with exact per-list scans, resident in one GPU's HBM."""

    def __init__(self, d: int, nlist: int, metric: str = "ip", dtype: str = "f32", device: int = 0,
                 nprobe: int = 1) -> None:
        self._h = None
        L = _lib.load()
        m = metric.lower()
        if m in ("ip", "cosine", "inner_product"):
            code = METRIC_IP
        elif m in ("l2", "euclidean"):
            code = METRIC_L2
        else:
            raise ValueError(f"unknown metric {metric!r}")
        if dtype not in DTYPE_CODES:
            raise ValueError(f"unknown dtype {dtype!r}")
        h = ctypes.c_void_p()
        check(L.vs_ivf_create(int(d), int(nlist), code, DTYPE_CODES[dtype], int(device), ctypes.byref(h)))
        self._h = h
        self._L = L
        self.d = int(d)
        self.nlist = int(nlist)
        self.metric_type = code
        self.dtype = dtype
        self.device = int(device)
        self.nprobe = int(nprobe)

    # -- faiss-like surface ------------------------------------------------------------------
    @property
    def ntotal(self) -> int:
        return int(self._L.vs_ivf_ntotal(self._h))

    @property
    def is_trained(self) -> bool:
        return bool(self._L.vs_ivf_is_trained(self._h) == 1)

    def _rows(self, x, what: str) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 2 or x.shape[1] != self.d:
            raise ValueError(f"{what} expects an (n, {self.d}) array, got {x.shape}")
        return x

    def set_centroids(self, c) -> None:
        c = self._rows(c, "set_centroids")
        if c.shape[0] != self.nlist:
            raise ValueError(f"expected {self.nlist} centroids, got {c.shape[0]}")
        check(self._L.vs_ivf_set_centroids(self._h, _ptr(c)))

    def centroids(self) -> np.ndarray:
        out = np.empty((self.nlist, self.d), dtype=np.float32)
        check(self._L.vs_ivf_get_centroids(self._h, _ptr(out)))
        return out

    def assign(self, x) -> np.ndarray:
        """Exact list id of every row (the coarse quantizer's top-1 for the row rounded to the index
        dtype, i.e. as it would be stored; ties -> lower list id)."""
        x = self._rows(x, "assign")
        out = np.empty((x.shape[0],), dtype=np.int64)
        if x.shape[0]:
            check(self._L.vs_ivf_assign(self._h, _ptr(x), x.shape[0], _ptr(out)))
        return out

    def train(self, x, niter: int = 10, seed: int = 1234, max_points_per_centroid: int = 256) -> None:
        """k-means (faiss Clustering defaults: at most 256 training points per centroid, random
        initial centroids from the rows).  Empty clusters keep their previous centroid."""
        x = self._rows(x, "train")
        if self.ntotal:
            raise ValueError("train() needs an empty index (reset() first)")
        n = x.shape[0]
        if n < self.nlist:
            raise ValueError(f"need at least nlist={self.nlist} training rows, got {n}")
        rng = np.random.default_rng(seed)
        if n > self.nlist * max_points_per_centroid:
            x = x[np.sort(rng.permutation(n)[: self.nlist * max_points_per_centroid])]
            n = x.shape[0]
        c = np.ascontiguousarray(x[np.sort(rng.permutation(n)[: self.nlist])])
        for _ in range(int(niter)):
            self.set_centroids(c)
            a = self.assign(x)
            sums = np.zeros((self.nlist, self.d), dtype=np.float64)
            np.add.at(sums, a, x.astype(np.float64))
            cnt = np.bincount(a, minlength=self.nlist)
            nz = cnt > 0
            c = c.copy()
            c[nz] = (sums[nz] / cnt[nz, None]).astype(np.float32)
        self.set_centroids(c)

    def add(self, x) -> None:
        x = self._rows(x, "add")
        check(self._L.vs_ivf_add(self._h, _ptr(x), x.shape[0]))

    def add_device(self, x_ptr: int, n: int, stream: Optional[int] = None) -> None:
        """Append n fp32 rows (row-major n x d) from device memory; ``stream`` is synchronised first."""
        check(self._L.vs_ivf_add_device(self._h, x_ptr, int(n), stream or None))

    def reserve(self, n: int) -> None:
        """Size the page pool for ``n`` more rows in one allocation."""
        check(self._L.vs_ivf_reserve(self._h, int(n)))

    def add_synthetic(self, seed: int, global_row0: int, n: int, normalize: bool = True) -> None:
        check(self._L.vs_ivf_add_synthetic(self._h, int(seed), int(global_row0), int(n), int(bool(normalize))))

    def search(self, q, k: int, nprobe: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        q = self._rows(q, "search")
        k = int(k)
        if k <= 0:
            raise _lib.VsError(_lib.VS_ERR_ARG, "k must be > 0")
        nq = q.shape[0]
        D = np.empty((nq, k), dtype=np.float32)
        I = np.empty((nq, k), dtype=np.int64)
        check(self._L.vs_ivf_search(self._h, _ptr(q), nq, k, int(nprobe or self.nprobe), _ptr(D), _ptr(I)))
        return D, I

    def search_device(self, q_ptr: int, nq: int, k: int, D_ptr: Optional[int], I_ptr: int,
                      S64_ptr: Optional[int] = None, nprobe: Optional[int] = None, stream: Optional[int] = None) -> None:
        check(self._L.vs_ivf_search_device(self._h, q_ptr, int(nq), int(k), int(nprobe or self.nprobe), D_ptr or None,
                                           I_ptr, S64_ptr or None, stream or None))

    def reconstruct(self, i: int) -> np.ndarray:
        out = np.empty((self.d,), dtype=np.float32)
        check(self._L.vs_ivf_reconstruct(self._h, int(i), _ptr(out)))
        return out

    def list_sizes(self) -> np.ndarray:
        out = np.empty((self.nlist,), dtype=np.int64)
        check(self._L.vs_ivf_list_sizes(self._h, _ptr(out)))
        return out

    def reset(self) -> None:
        check(self._L.vs_ivf_reset(self._h))

    _SCANS = {"auto": 0, "gemv": 1, "mfma": 2}

    def set_scan(self, mode: str) -> None:
        """List-scan kernels: "auto" (cost model), "gemv" (never MFMA), "mfma" (every list probed by
        more than one query, bf16/f16).  Results are identical in every mode."""
        if mode not in self._SCANS:
            raise ValueError(f"scan mode must be one of {sorted(self._SCANS)}")
        check(self._L.vs_ivf_set_scan(self._h, self._SCANS[mode]))

    _QTILES = {"plain": 0, "split": 1}

    def set_query_tiles(self, mode: str) -> None:
        """Query tiles of the MFMA list scans' first pass: "split" (default: (hi, lo) parts, 128 a
        tile) or "plain" (each query rounded once, 256 a tile, the wider rounding margin certified
        by the refine).  Results are identical in both modes (include/vs.h vs_ivf_set_query_tiles)."""
        if mode not in self._QTILES:
            raise ValueError(f"query-tile mode must be one of {sorted(self._QTILES)}")
        check(self._L.vs_ivf_set_query_tiles(self._h, self._QTILES[mode]))

    def last_search_stats(self) -> Tuple[int, int]:
        """First pass of the last search: (MFMA list scans, queries re-searched for their certificate)."""
        return self.last_search_detail()[:2]

    def last_search_detail(self) -> Tuple[int, int, float, float]:
        """(MFMA list scans, re-searched queries, page bytes read by the MFMA scans, by the GEMV scan)."""
        m, u = ctypes.c_int(0), ctypes.c_int(0)
        by = (ctypes.c_double * 2)()
        check(self._L.vs_ivf_last_search_stats(self._h, ctypes.byref(m), ctypes.byref(u), by))
        return int(m.value), int(u.value), float(by[0]), float(by[1])

    @property
    def last_mfma_lists(self) -> int:
        """List scans the last search's first pass ran on the MFMA screen."""
        return self.last_search_stats()[0]

    # -- measurement ---------------------------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        check(self._L.vs_ivf_set_timing(self._h, int(bool(enable))))

    def timing_fetch(self, cap: int = 4096):
        ms = (ctypes.c_float * cap)()
        by = (ctypes.c_double * cap)()
        n = check(self._L.vs_ivf_timing_fetch(self._h, ms, by, cap))
        return [float(ms[i]) for i in range(n)], [float(by[i]) for i in range(n)]

    # -- lifecycle ----------------------------------------------------------------------------
    def close(self) -> None:
        if self._h is not None and self._h.value:
            self._L.vs_ivf_destroy(self._h)
        self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass
