"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the IVF-Flat path (BASELINE cfg5).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker.  The product (``photo_search_engine_amd.ivf``) never does.

The reference has no IVF index (``index_type`` is "flat" or "hnsw",
/root/reference/utils/vector_store.py:51-53).  IVF-Flat is the faiss ``IndexIVFFlat`` design
(third-party ``faiss-cpu>=1.7.0``, /root/reference/requirements.txt:5, neither vendored nor
installed), restated with the flat path's exact semantics, so a result is a deterministic
function of (stored rows, stored centroids, queries):

* coarse assignment of a row: its best centroid under the canonical fp64 score
  (``oracle.knn_exact`` with k=1; IP: max, L2: min; ties -> lower centroid id).  faiss assigns
  with its flat quantizer the same way (IndexFlatIP for METRIC_INNER_PRODUCT, else IndexFlatL2);
* probed lists of a query: its exact top-``nprobe`` centroids, same order and tie rule;
* result: the exact top-k (canonical fp64 score, ties -> lower row id) over the rows of the
  probed lists only; slots past the number of such rows get id -1 and the worst score.

k-means training is NOT in the parity loop: both sides get the same centroids (values as stored,
i.e. rounded to the index dtype).  parity is pinned by restatement (faiss is absent).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from . import oracle as O


def assign(x_stored: np.ndarray, c_stored: np.ndarray, metric="ip") -> np.ndarray:
    """List id of every row: the exact best centroid (ties -> lower centroid id)."""
    if x_stored.shape[0] == 0:
        return np.zeros((0,), dtype=np.int64)
    _, I = O.knn_exact(c_stored, x_stored, 1, metric)
    return I[:, 0].copy()


def assign_ip_fast(x_stored: np.ndarray, c_stored: np.ndarray, chunk: int = 32768) -> np.ndarray:
    """``assign`` for the IP metric at sizes where the canonical scan is too slow (BASELINE cfg5:
    4096 centroids x d=1536): an fp32 GEMM (numpy, any summation order) gives every row's fp32
    top-2 centroids; where their fp32 gap exceeds twice the fp32 error bound the fp32 winner IS the
    canonical winner, and every other row is resolved by the canonical fp64 scan (``assign``).

    Bound: any summation order of a d-term fp32 dot product errs by at most
    gamma_n * sum|x_i c_i| <= gamma_n * ||x|| * ||c||, gamma_n = n u / (1 - n u), n = d + 64
    (margin for blocked partial sums), u = 2^-24.  If fp32(c1) - fp32(c2) > 2 * bound, every
    centroid c != c1 has exact(c) <= fp32(c) + bound <= fp32(c2) + bound < fp32(c1) - bound
    <= exact(c1), so c1 is the unique canonical best.  Same result as ``assign``, by construction.
    """
    x_stored = np.ascontiguousarray(x_stored, dtype=np.float32)
    c_stored = np.ascontiguousarray(c_stored, dtype=np.float32)
    n, d = x_stored.shape
    if n == 0:
        return np.zeros((0,), dtype=np.int64)
    if c_stored.shape[0] < 2:
        return np.zeros((n,), dtype=np.int64)
    u = 2.0 ** -24
    g = (d + 64) * u / (1.0 - (d + 64) * u)
    cmax = float(np.max(np.linalg.norm(c_stored.astype(np.float64), axis=1)))
    out = np.empty((n,), dtype=np.int64)
    unsure = []
    ct = np.ascontiguousarray(c_stored.T)
    for r0 in range(0, n, chunk):
        xb = x_stored[r0:r0 + chunk]
        s = xb @ ct  # fp32
        top2 = np.argpartition(-s, 1, axis=1)[:, :2]
        s2 = np.take_along_axis(s, top2, axis=1).astype(np.float64)
        first = np.where(s2[:, 0] >= s2[:, 1], 0, 1)
        out[r0:r0 + xb.shape[0]] = top2[np.arange(xb.shape[0]), first]
        gap = np.abs(s2[:, 0] - s2[:, 1])
        bound = g * np.linalg.norm(xb.astype(np.float64), axis=1) * cmax * 1.01
        unsure.append(r0 + np.flatnonzero(gap <= 2.0 * bound))
    unsure = np.concatenate(unsure)
    if unsure.size:
        out[unsure] = assign(x_stored[unsure], c_stored, "ip")
    return out


def probe(q: np.ndarray, c_stored: np.ndarray, nprobe: int, metric="ip") -> np.ndarray:
    """Probed lists of every query: exact top-nprobe centroids, best first."""
    nprobe = min(int(nprobe), c_stored.shape[0])
    _, I = O.knn_exact(c_stored, q, nprobe, metric)
    return I


def search(x_stored: np.ndarray, ids: np.ndarray, lists: np.ndarray, c_stored: np.ndarray, q: np.ndarray,
           k: int, nprobe: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """IVF-Flat search restated: (S fp64 nq x k, I int64 nq x k), -1 / worst-score padding.

    ``x_stored`` rows (values as stored) carry user ids ``ids`` and list ids ``lists``.
    """
    q = np.ascontiguousarray(q, dtype=np.float32)
    ids = np.asarray(ids, dtype=np.int64)
    lists = np.asarray(lists, dtype=np.int64)
    nq = q.shape[0]
    ip = O._metric(metric) == O.METRIC_IP
    S = np.full((nq, k), -np.inf if ip else np.inf, dtype=np.float64)
    I = np.full((nq, k), -1, dtype=np.int64)
    P = probe(q, c_stored, nprobe, metric)
    # rows of each list, ascending (one sort instead of an isin over all rows per query)
    by_list = np.argsort(lists, kind="stable")
    bounds = np.searchsorted(lists[by_list], np.arange(c_stored.shape[0] + 1))
    for a in range(nq):
        sel = np.sort(np.concatenate([by_list[bounds[l]:bounds[l + 1]] for l in P[a]]))
        if sel.size == 0:
            continue
        sc = O.canon_scores(x_stored[sel], q[a:a + 1], metric)[0]
        uid = ids[sel]
        order = np.lexsort((uid, -sc if ip else sc))[:k]
        S[a, :order.size] = sc[order]
        I[a, :order.size] = uid[order]
    return S, I


def sample_centroids(x: np.ndarray, nlist: int, seed: int) -> np.ndarray:
    """Deterministic centroids for tests: ``nlist`` rows picked by a seeded permutation (faiss'
    k-means also starts from a random subset of the training rows)."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.permutation(x.shape[0])[:nlist])
    return np.ascontiguousarray(x[idx], dtype=np.float32)
