"""TEST INFRASTRUCTURE: a checker-backed stand-in with FlatIndex's surface.

Used only by CPU tests to exercise the host logic of ``VectorStore`` (validation, files, result
layout) without a GPU.  Its search is the oracle's exact canonical search -- the same definition
the HIP path is held to bit-for-bit in the GPU tests.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


class OracleFlatIndex:
    def __init__(self, d: int, metric: str = "ip") -> None:
        self.d = int(d)
        self.metric_type = 0 if metric in ("ip", "cosine") else 1
        self._x = np.zeros((0, self.d), dtype=np.float32)

    @property
    def ntotal(self) -> int:
        return int(self._x.shape[0])

    def add(self, x) -> None:
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.ndim == 2 and x.shape[1] == self.d
        self._x = np.concatenate([self._x, x], axis=0)

    def search(self, q, k: int):
        q = np.ascontiguousarray(q, dtype=np.float32)
        if k <= 0:
            raise RuntimeError("k must be > 0")
        S, I = O.knn_exact(self._x, q, int(k), "ip" if self.metric_type == 0 else "l2")
        D = S.astype(np.float32)
        D[I < 0] = -3.4028235e38 if self.metric_type == 0 else 3.4028235e38
        return D, I

    def hnsw_prune(self, nodes, cand, W: int) -> np.ndarray:
        from oracle import hnsw_oracle as H
        dist = H._distances(self._x, self._x, "ip" if self.metric_type == 0 else "l2")
        out = np.full((len(nodes), int(W)), -1, dtype=np.int32)
        for i, v in enumerate(nodes):
            kept = H.shrink_neighbor_list(dist, int(v), cand[i], int(W))
            out[i, :len(kept)] = kept
        return out

    def reconstruct(self, i: int) -> np.ndarray:
        return self._x[int(i)].copy()

    def reconstruct_n(self, i0: int, n: int) -> np.ndarray:
        return self._x[int(i0):int(i0) + int(n)].copy()

    def add_from_file(self, path: str, byte_offset: int, n: int) -> None:
        x = np.fromfile(path, dtype="<f4", count=int(n) * self.d, offset=int(byte_offset))
        assert x.size == int(n) * self.d, "file too short"
        self.add(x.reshape(int(n), self.d))

    def write_rows(self, path: str, byte_offset: int, i0: int, n: int) -> None:
        with open(path, "r+b") as f:
            f.seek(int(byte_offset))
            f.write(np.ascontiguousarray(self._x[int(i0):int(i0) + int(n)], dtype="<f4").tobytes())

    def reset(self) -> None:
        self._x = np.zeros((0, self.d), dtype=np.float32)


def oracle_factory(dimension: int, metric: str):
    return OracleFlatIndex(dimension, "ip" if metric == "cosine" else "l2")


def _hnsw_search(self, graph, q, k, ef):
    """ids of faiss's HNSW search over ``graph`` (the oracle's ordered-multiset statement, the
    kernel's): the checker-backed form of ``hnsw.beam_search``."""
    from oracle import hnsw_oracle as H
    n = int(np.asarray(graph["levels"]).shape[0])
    _, I = H.search(self._x[:n], graph, q, int(k), int(ef), "ip" if self.metric_type == 0 else "l2")
    return I


OracleFlatIndex.hnsw_search = _hnsw_search
