"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the flat k-NN hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the reported CPU baseline.  The product package
(``photo_search_engine_amd``) never imports it: with its HIP library missing it fails loudly.

Two implementations of the same semantics:

* ``liborc.so`` (``oracle/vs_oracle.c``, built by ``oracle/Makefile``) -- the C restatement of
  faiss ``IndexFlatIP``/``IndexFlatL2`` search (called by the reference at
  ``/root/reference/utils/vector_store.py:191``), the canonical exact fp64 score, the synthetic
  data generator, and the per-shard merge.
* a numpy twin (``np_canon_scores``, ``np_knn_exact``, ``np_normalize_like_reference``) for small
  cases, so the C code is itself cross-checked.

faiss is third-party (``faiss-cpu>=1.7.0``, ``/root/reference/requirements.txt:5``), not vendored
under ``/root/reference`` and not installed in this image; its published algorithm is restated.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborc.so")

METRIC_IP = 0
METRIC_L2 = 1
DTYPE_F32 = 0
DTYPE_BF16 = 1
DTYPE_F16 = 2
DTYPES = {"f32": DTYPE_F32, "fp32": DTYPE_F32, "bf16": DTYPE_BF16, "f16": DTYPE_F16, "fp16": DTYPE_F16}

SEED_CORPUS = 20260417
SEED_QUERIES = 20260418

_lib = None


def build() -> str:
    """Compile liborc.so (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
        u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
        i64 = ctypes.c_int64
        L.orc_version.restype = ctypes.c_int
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_round_dtype.argtypes = [f32p, i64, ctypes.c_int, f32p]
        L.orc_to_bf16_bits.argtypes = [f32p, i64, u16p]
        L.orc_to_f16_bits.argtypes = [f32p, i64, u16p]
        L.orc_synth_rows.argtypes = [ctypes.c_uint64, i64, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p]
        L.orc_canon_scores.argtypes = [f32p, i64, ctypes.c_int, f32p, i64, ctypes.c_int, f64p]
        L.orc_knn_exact.argtypes = [f32p, i64, ctypes.c_int, f32p, i64, ctypes.c_int, ctypes.c_int, f64p, i64p]
        L.orc_merge_topk.argtypes = [f64p, i64p, ctypes.c_int, i64, ctypes.c_int, ctypes.c_int, f64p, i64p]
        L.orc_knn_faiss_fp32.argtypes = [f32p, i64, ctypes.c_int, f32p, i64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, f32p, i64p]
        _lib = L
    return _lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _metric(metric) -> int:
    if isinstance(metric, str):
        return METRIC_IP if metric.lower() in ("ip", "cosine", "inner_product") else METRIC_L2
    return int(metric)


# --------------------------------------------------------------------------------------------
# data
# --------------------------------------------------------------------------------------------
def synth_rows(seed: int, row0: int, n: int, d: int, normalize: bool = True, dtype="f32") -> np.ndarray:
    """Rows [row0, row0+n) of the synthetic matrix (bit-identical to the HIP generator)."""
    out = np.empty((n, d), dtype=np.float32)
    lib().orc_synth_rows(ctypes.c_uint64(seed), row0, n, d, int(normalize), DTYPES.get(dtype, dtype), out)
    return out


def round_dtype(x, dtype) -> np.ndarray:
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_round_dtype(x.reshape(-1), x.size, DTYPES.get(dtype, dtype), out.reshape(-1))
    return out


# --------------------------------------------------------------------------------------------
# search
# --------------------------------------------------------------------------------------------
def knn_exact(x, q, k: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """Exact top-k under the canonical fp64 score: (S float64 nq x k, I int64 nq x k)."""
    x = _f32(x)
    q = _f32(q)
    N, d = x.shape
    nq = q.shape[0]
    S = np.empty((nq, k), dtype=np.float64)
    I = np.empty((nq, k), dtype=np.int64)
    lib().orc_knn_exact(x.reshape(-1), N, d, q.reshape(-1), nq, k, _metric(metric), S.reshape(-1), I.reshape(-1))
    return S, I


def canon_scores(x, q, metric="ip") -> np.ndarray:
    x = _f32(x)
    q = _f32(q)
    S = np.empty((q.shape[0], x.shape[0]), dtype=np.float64)
    lib().orc_canon_scores(x.reshape(-1), x.shape[0], x.shape[1], q.reshape(-1), q.shape[0], _metric(metric),
                           S.reshape(-1))
    return S


def knn_faiss_fp32(x, q, k: int, metric="ip", nthreads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """faiss IndexFlat search restated in fp32 (score-noise reference + CPU baseline)."""
    x = _f32(x)
    q = _f32(q)
    D = np.empty((q.shape[0], k), dtype=np.float32)
    I = np.empty((q.shape[0], k), dtype=np.int64)
    lib().orc_knn_faiss_fp32(x.reshape(-1), x.shape[0], x.shape[1], q.reshape(-1), q.shape[0], k,
                             _metric(metric), nthreads, D.reshape(-1), I.reshape(-1))
    return D, I


def merge_topk(S_parts: np.ndarray, I_parts: np.ndarray, k: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """Merge G per-shard (S, I) lists shaped (G, nq, k) with global ids."""
    S_parts = np.ascontiguousarray(S_parts, dtype=np.float64)
    I_parts = np.ascontiguousarray(I_parts, dtype=np.int64)
    G, nq, kk = S_parts.shape
    assert kk == k
    S = np.empty((nq, k), dtype=np.float64)
    I = np.empty((nq, k), dtype=np.int64)
    lib().orc_merge_topk(S_parts.reshape(-1), I_parts.reshape(-1), G, nq, k, _metric(metric), S.reshape(-1),
                         I.reshape(-1))
    return S, I


# --------------------------------------------------------------------------------------------
# numpy twin (small sizes) -- same expression trees as vs_oracle.c
# --------------------------------------------------------------------------------------------
def np_canon_scores(x, q, metric="ip") -> np.ndarray:
    """Canonical fp64 scores: element i -> lane (i>>3)&63, sequential per lane, xor-butterfly."""
    x = _f32(x).astype(np.float64)
    q = _f32(q).astype(np.float64)
    N, d = x.shape
    nq = q.shape[0]
    acc = np.zeros((nq, N, 64), dtype=np.float64)
    for i in range(d):
        lane = (i >> 3) & 63
        if _metric(metric) == METRIC_IP:
            p = q[:, i][:, None] * x[:, i][None, :]
        else:
            dl = x[:, i][None, :] - q[:, i][:, None]
            p = dl * dl
        acc[:, :, lane] = acc[:, :, lane] + p
    lanes = np.arange(64)
    for s in (32, 16, 8, 4, 2, 1):
        acc = acc + acc[:, :, lanes ^ s]
    return acc[:, :, 0]


def np_topk(S: np.ndarray, k: int, metric="ip") -> Tuple[np.ndarray, np.ndarray]:
    """(score desc | asc, id asc) top-k of an (nq, N) score matrix."""
    nq, N = S.shape
    ids = np.arange(N)
    outS = np.empty((nq, k))
    outI = np.full((nq, k), -1, dtype=np.int64)
    for a in range(nq):
        key = -S[a] if _metric(metric) == METRIC_IP else S[a]
        order = np.lexsort((ids, key))[:k]
        outS[a, : len(order)] = S[a, order]
        outI[a, : len(order)] = order
    return outS, outI


def np_knn_exact(x, q, k: int, metric="ip"):
    return np_topk(np_canon_scores(x, q, metric), k, metric)


def np_normalize_like_reference(vector):
    """``VectorStore._normalize_vector`` (/root/reference/utils/vector_store.py:83-90) verbatim in
    behaviour: fp32 array, ``np.linalg.norm``, zero norm -> input unchanged."""
    array = np.array(vector, dtype="float32")
    norm = np.linalg.norm(array)
    if norm == 0:
        return vector
    return (array / norm).astype("float32").tolist()


# --------------------------------------------------------------------------------------------
# comparators
# --------------------------------------------------------------------------------------------
def compare_ids_tie_tolerant(I_got, I_ref, S_ref_full_fn, eps: float):
    """Tie-tolerant comparison against an fp32 faiss-like result: a position may differ only if
    the exact (fp64) scores of the two ids are within ``eps``.  Returns (exact_rate, tol_rate)."""
    I_got = np.asarray(I_got)
    I_ref = np.asarray(I_ref)
    exact = float(np.mean(I_got == I_ref))
    ok = 0
    total = I_got.size
    for a in range(I_got.shape[0]):
        for j in range(I_got.shape[1]):
            if I_got[a, j] == I_ref[a, j]:
                ok += 1
            else:
                s1 = S_ref_full_fn(a, I_got[a, j])
                s2 = S_ref_full_fn(a, I_ref[a, j])
                ok += int(abs(s1 - s2) <= eps)
    return exact, ok / total


def recall_at(I_got, I_ref, k: int) -> float:
    I_got = np.asarray(I_got)[:, :k]
    I_ref = np.asarray(I_ref)[:, :k]
    hit = 0
    for a in range(I_got.shape[0]):
        hit += len(set(I_got[a].tolist()) & set(I_ref[a].tolist()))
    return hit / float(I_ref.shape[0] * k)
