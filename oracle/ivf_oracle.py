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
    for a in range(nq):
        sel = np.flatnonzero(np.isin(lists, P[a]))
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
