"""Drop-in ``VectorStore`` backed by the MI355X flat k-NN library.

Same class name, constructor keywords, methods, attributes, error types/messages and sidecar
files as /root/reference/utils/vector_store.py:15-280, so ``core/indexer.py`` and
``core/searcher.py`` run unchanged.  Integration: replace the reference's
``utils/vector_store.py`` body with ``from photo_search_engine_amd.vector_store import VectorStore``
(INTEGRATION.md).

What changes underneath:
  * ``self.index`` is a :class:`~photo_search_engine_amd.index.FlatIndex` (HBM-resident shard on
    one GPU) instead of a faiss CPU index; searches are exact (see include/vs.h).
  * ``index_type="hnsw"`` is accepted, validated and recorded in the sidecar exactly as before,
    and served by exact flat search by default (recall 1.0 >= HNSW); ``VECTOR_HNSW_SEARCH=graph``
    runs faiss's HNSW search instead, on the GPU (:class:`~photo_search_engine_amd.hnsw.HNSWGraph`)
    with ``efSearch = hnsw_ef_search`` as the reference sets it (utils/vector_store.py:77,135), over
    the graph of the loaded IHNf file or the one ``save()`` writes.  ``save()`` writes an IHNf file
    that the reference's faiss can load back: faiss's level draw, each node's neighbours chosen by
    faiss's selection heuristic (``HNSW::shrink_neighbor_list``, on the GPU) from exact candidates,
    reverse links as faiss's ``add_link`` adds them, + the flat storage (``_build_graph``).
    ``load()`` reads flat and HNSW files.
  * ``_embeddings`` caches only rows added in this process (a dict), not one Python list per row.
  * Bulk additions: :meth:`add` (n x d array) and :meth:`search_batch` (faiss (D, I) layout).

Normalisation stays on the host in numpy, bit-identical to the reference
(utils/vector_store.py:83-90), so stored vectors and query vectors are the same fp32 values.

Environment knobs (new, optional): ``VECTOR_DEVICE`` (GPU ordinal, default 0), ``VECTOR_DEVICES``
(e.g. ``0,1,2,3,4,5,6,7``: one index over those GPUs of this process, include/vs.h vs_multi_*),
``VECTOR_DTYPE`` (f32 | bf16 | f16 storage, default f32 = the reference's storage precision),
``VECTOR_SCREEN`` (int8 | native: the screen in front of the exact refine, either metric; default
int8 -- the certified int8 pre-screen, same exact results) and
``VECTOR_HNSW_SEARCH`` (exact | graph: how an ``index_type="hnsw"`` store searches).
"""
from __future__ import annotations

import json
import os
import struct
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import faiss_format
from . import hnsw as hnsw_mod
from .hnsw import HNSWGraph
from .index import FlatIndex, MultiDeviceFlatIndex

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1


def _default_index_factory(dimension: int, metric: str):
    dtype = (os.environ.get("VECTOR_DTYPE", "f32") or "f32").strip().lower()
    kind = "ip" if metric == "cosine" else "l2"
    devices = [d.strip() for d in (os.environ.get("VECTOR_DEVICES", "") or "").split(",") if d.strip()]
    if len(devices) > 1:  # one index over several GPUs of this process (rows dealt in 64k-id chunks)
        index = MultiDeviceFlatIndex(dimension, metric=kind, dtype=dtype, devices=[int(d) for d in devices])
    else:
        device = int(devices[0]) if devices else int(os.environ.get("VECTOR_DEVICE", "0") or 0)
        index = FlatIndex(dimension, metric=kind, dtype=dtype, device=device)
    # the certified int8 pre-screen unless VECTOR_SCREEN=native: results are exact either way (the
    # refine scores every candidate canonically and a certificate covers the rest), and the index
    # routes batches back to the native screen by itself on data denser than the int8 margins
    screen = (os.environ.get("VECTOR_SCREEN", "") or "").strip().lower() or "int8"
    index.set_screen(screen)
    return index


# Module-level hook: tests may substitute a checker-backed index with the same surface.
_index_factory = _default_index_factory


def _hnsw_graph_max_rows() -> int:
    """Rows of an ``index_type="hnsw"`` store whose graph is built at once from exact candidates
    (:meth:`VectorStore._build_graph`); rows beyond it are inserted into that graph in batches,
    faiss's way (:func:`hnsw.insert_rows`), so every save writes an IHNf file whatever the size."""
    return int(os.environ.get("VECTOR_HNSW_GRAPH_MAX_ROWS", "200000") or 200000)


_HNSW_EF_MAX = 2048  # largest max(efSearch, k) of the GPU graph search (include/vs.h)
# graph mode rebuilds the graph once the store holds this many times the rows the graph covers
_GRAPH_REBUILD_GROWTH = 1.25


def _merge_topk(D1: np.ndarray, I1: np.ndarray, D2: np.ndarray, I2: np.ndarray, k: int,
                higher_is_better: bool) -> Tuple[np.ndarray, np.ndarray]:
    """Per query, the best k of two (D, I) result lists (faiss layout, -1 padded): by score (IP:
    larger first; L2: smaller first), ties to the lower id, padding last.  The merge sees the fp32
    distances only, so two rows whose canonical fp64 scores differ but round to the same fp32 value
    are ordered by id here, where an exact search orders them by the fp64 score.  Only graph mode
    merges (its graph results with the exactly searched rows added behind the graph), and graph
    search is approximate to begin with."""
    D = np.concatenate([D1, D2], axis=1)
    I = np.concatenate([I1, I2], axis=1)
    key = -D if higher_is_better else D.copy()
    key = np.where(I >= 0, key, np.inf)
    order = np.lexsort((np.where(I >= 0, I, np.iinfo(np.int64).max), key), axis=1)[:, :k]
    Do = np.take_along_axis(D, order, axis=1)
    Io = np.take_along_axis(I, order, axis=1)
    if Do.shape[1] < k:  # fewer candidates than k: faiss padding
        pad = k - Do.shape[1]
        fill = np.float32(-np.finfo(np.float32).max if higher_is_better else np.finfo(np.float32).max)
        Do = np.concatenate([Do, np.full((Do.shape[0], pad), fill, dtype=Do.dtype)], axis=1)
        Io = np.concatenate([Io, np.full((Io.shape[0], pad), -1, dtype=Io.dtype)], axis=1)
    Do = np.where(Io >= 0, Do, np.float32(-np.finfo(np.float32).max if higher_is_better else np.finfo(np.float32).max))
    return Do.astype(np.float32), Io.astype(np.int64)


def _hnsw_graph_search() -> bool:
    return (os.environ.get("VECTOR_HNSW_SEARCH", "exact") or "exact").strip().lower() == "graph"


class VectorStore:
    """
    向量存储与检索封装 (vector storage and retrieval).

    Attributes:
        dimension (Optional[int]): 向量维度
        index_path (str): 索引文件路径
        metadata_path (str): 元数据文件路径
    """

    def __init__(
        self,
        dimension: Optional[int],
        index_path: str,
        metadata_path: str,
        metric: str = "cosine",
        index_type: str = "flat",
        hnsw_m: int = 32,
        hnsw_ef_construction: int = 200,
        hnsw_ef_search: int = 96,
    ) -> None:
        # utils/vector_store.py:44-62
        self.dimension = dimension
        self.index_path = index_path
        self.metadata_path = metadata_path
        self.meta_path = f"{self.index_path}.meta.json"
        self.metric = metric.lower().strip() if metric else "l2"
        if self.metric not in {"l2", "cosine"}:
            raise ValueError("metric仅支持l2或cosine")
        self.index_type = (index_type or "flat").strip().lower()
        if self.index_type not in {"flat", "hnsw"}:
            raise ValueError("index_type仅支持flat或hnsw")
        self.hnsw_m = max(4, int(hnsw_m))
        self.hnsw_ef_construction = max(8, int(hnsw_ef_construction))
        self.hnsw_ef_search = max(8, int(hnsw_ef_search))

        self.index = self._create_index(dimension) if dimension else None
        self.metadata: List[Dict] = []
        self._normalize = self.metric == "cosine"
        self._embeddings: Dict[int, List[float]] = {}
        self._path_to_index: Dict[str, int] = {}
        # what the index file on disk holds, when it is known to be a prefix of this index
        # (set by save() / load(); None after clear()): lets save() append instead of rewriting
        self._persisted: Optional[Dict[str, Any]] = None
        # VECTOR_HNSW_SEARCH=graph: the graph arrays last loaded or saved, and its GPU copy
        self._graph_arrays: Optional[Dict[str, Any]] = None
        self._hnsw: Optional[HNSWGraph] = None
        self._graph_tail: Optional[FlatIndex] = None  # rows added behind the graph, searched exactly
        # a flat-configured store loaded from an HNSW file: the reference's index object stays an
        # IndexHNSWFlat (utils/vector_store.py:249), so its save() writes an HNSW file again
        self._file_hnsw = False

    # ------------------------------------------------------------------ internals
    def _rebuild_path_index(self) -> None:
        path_to_index: Dict[str, int] = {}
        for index, metadata in enumerate(self.metadata):
            photo_path = metadata.get("photo_path")
            if isinstance(photo_path, str) and photo_path:
                path_to_index[photo_path] = index
        self._path_to_index = path_to_index

    def _create_index(self, dimension: int):
        return _index_factory(int(dimension), self.metric)

    def _normalize_vector(self, vector: List[float]) -> List[float]:
        # utils/vector_store.py:83-90, verbatim semantics (fp32, np.linalg.norm, zero passthrough)
        if not self._normalize:
            return vector
        array = np.array(vector, dtype="float32")
        norm = np.linalg.norm(array)
        if norm == 0:
            return vector
        return (array / norm).astype("float32").tolist()

    def _normalize_query(self, vector) -> np.ndarray:
        """``np.array([_normalize_vector(vector)], dtype="float32")`` without the Python-list round trip
        (~0.19 ms of a 0.5 ms call at d=4096): fp32 -> Python float -> fp32 is exact, so the bits
        are the same.  A list of Python numbers is converted by ``struct`` (the same C double ->
        float cast as numpy's, ~3x faster than ``np.array`` on a list: ~24 vs ~70 us at d=1536); a
        value beyond the fp32 range (numpy makes it inf) or anything else takes ``np.array``.
        Anything but a flat vector takes the reference's own expression (whose extra axes the index
        then rejects, as faiss does)."""
        array = None
        if type(vector) is list:
            try:
                array = np.frombuffer(struct.pack(f"{len(vector)}f", *vector), dtype=np.float32)
            except (struct.error, OverflowError, TypeError):
                array = None
        if array is None:
            array = np.array(vector, dtype="float32")
        if array.ndim != 1:
            return np.array([self._normalize_vector(vector)], dtype="float32")
        if self._normalize:
            norm = np.linalg.norm(array)
            if norm != 0:
                array = (array / norm).astype("float32")
        return array.reshape(1, -1)

    def _normalize_rows(self, rows: np.ndarray) -> np.ndarray:
        """Bulk form of ``_normalize_vector``: each row normalised exactly as the single-row path
        (same numpy calls per row, so the stored bits are identical)."""
        rows = np.array(rows, dtype="float32", copy=True)
        if not self._normalize:
            return rows
        for i in range(rows.shape[0]):
            norm = np.linalg.norm(rows[i])
            if norm != 0:
                rows[i] = (rows[i] / norm).astype("float32")
        return rows

    def _write_index_meta(self) -> None:
        payload = {
            "index_type": self.index_type,
            "metric": self.metric,
            "dimension": self.dimension,
            "hnsw_m": self.hnsw_m,
            "hnsw_ef_construction": self.hnsw_ef_construction,
            "hnsw_ef_search": self.hnsw_ef_search,
        }
        with open(self.meta_path, "w", encoding="utf-8") as file:
            json.dump(payload, file, ensure_ascii=False, indent=2)

    def _load_index_meta(self) -> Dict[str, Any]:
        if not os.path.exists(self.meta_path):
            raise ValueError("索引元信息缺失，请重新构建索引")
        with open(self.meta_path, "r", encoding="utf-8") as file:
            payload = json.load(file)
        if not isinstance(payload, dict):
            raise ValueError("索引元信息损坏，请重新构建索引")
        return payload

    def _validate_loaded_index(self, payload: Dict[str, Any], loaded: "faiss_format.FaissFile") -> None:
        # utils/vector_store.py:125-140, rule for rule: the sidecar's index_type and metric must match
        # the configuration; an HNSW configuration needs an HNSW file (IndexHNSWFlat, :137-138) and
        # never checks the file's metric; a flat configuration checks only the file's metric_type
        # (:139-143), so an HNSW file of the configured metric loads too.
        index_type = str(payload.get("index_type") or "").strip().lower()
        metric = str(payload.get("metric") or "").strip().lower()
        if index_type != self.index_type:
            raise ValueError("索引类型与配置不一致，请重新构建索引")
        if metric != self.metric:
            raise ValueError("索引度量与配置不一致，请重新构建索引")
        if self.index_type == "hnsw":
            if loaded.kind != "hnsw":
                raise ValueError("索引结构与配置不一致，请重新构建索引")
        elif self.index_type == "flat":
            want = METRIC_INNER_PRODUCT if self.metric == "cosine" else METRIC_L2
            if loaded.metric_type != want:
                raise ValueError("索引度量与配置不一致，请重新构建索引")

    # ------------------------------------------------------------------ reference API
    # 内部接口：仅允许indexer模块调用，禁止直接暴露给前端
    def add_item(self, embedding: List[float], metadata: Dict) -> None:
        """写入向量与元数据 (utils/vector_store.py:143-169)."""
        if embedding is None:
            raise ValueError("向量不能为空")
        if self.index is None:
            self.dimension = len(embedding)
            self.index = self._create_index(self.dimension)
        if len(embedding) != self.dimension:
            raise ValueError(f"向量维度不匹配: {len(embedding)} != {self.dimension}")

        normalized = self._normalize_vector(embedding)
        vector = np.array([normalized], dtype="float32")
        self.index.add(vector)
        self.metadata.append(metadata)
        self._embeddings[len(self.metadata) - 1] = normalized
        photo_path = metadata.get("photo_path")
        if isinstance(photo_path, str) and photo_path:
            self._path_to_index[photo_path] = len(self.metadata) - 1

    # 内部接口：仅允许searcher模块调用，禁止前端直接访问向量数据库
    def search(self, query_embedding: List[float], top_k: int) -> List[Dict]:
        """相似度检索 (utils/vector_store.py:172-198)."""
        if self.index is None or self.index.ntotal == 0:
            return []
        if len(query_embedding) != self.dimension:
            raise ValueError(f"向量维度不匹配: {len(query_embedding)} != {self.dimension}")

        k = min(top_k, self.index.ntotal)
        distances, indices = self._search_rows(self._normalize_query(query_embedding), k)

        results: List[Dict] = []
        for distance, index in zip(distances[0].tolist(), indices[0].tolist()):
            if index == -1:
                continue
            results.append({"metadata": self.metadata[index], "distance": float(distance)})
        return results

    def get_embedding_by_photo_path(self, photo_path: str) -> Optional[List[float]]:
        index = self._path_to_index.get(photo_path)
        if index is None:
            return None
        if index < len(self.metadata) and self.index is not None and index < self.index.ntotal:
            cached = self._embeddings.get(index)
            if cached is None:
                vector = self.index.reconstruct(index)
                cached = vector.astype("float32").tolist()
                self._embeddings[index] = cached
            if cached is not None:
                return list(cached)
        return None

    def has_photo_path(self, photo_path: str) -> bool:
        return photo_path in self._path_to_index

    def save(self) -> None:
        """索引持久化 (utils/vector_store.py:217-237)."""
        if self.index is None:
            raise ValueError("索引未初始化")

        index_dir = os.path.dirname(self.index_path)
        metadata_dir = os.path.dirname(self.metadata_path)
        if index_dir:
            os.makedirs(index_dir, exist_ok=True)
        if metadata_dir:
            os.makedirs(metadata_dir, exist_ok=True)

        # The reference rewrites the whole index per indexer batch (utils/vector_store.py:234,
        # core/indexer.py:945): O(N) per save.  Rows never change once added, so when the file on
        # disk is the one this store last wrote or loaded, only the new rows and the header are
        # written -- the bytes are identical to a full rewrite.  Payload bytes stream HBM -> file.
        n, d, mt = int(self.index.ntotal), int(self.index.d), int(self.index.metric_type)
        old = self._appendable_rows(d, mt)
        if self.index_type == "hnsw" or self._file_hnsw:
            # an IHNf file the reference's faiss can load (rollback), at every size; a graph loaded
            # from file is kept (rows added since are inserted into it), with efSearch as configured
            # (the reference sets hnsw.efSearch after every load of an HNSW configuration,
            # utils/vector_store.py:135, and faiss writes it back; a flat configuration keeps the
            # file's)
            ef = self.hnsw_ef_search if self.index_type == "hnsw" else None
            if self._graph_covers(n):
                graph = dict(self._graph_arrays)
                if ef is not None:
                    graph["efSearch"] = ef
            else:
                graph = self._build_graph(n)
            faiss_format.write_hnsw(self.index_path, graph, d, n, mt, lambda path, off: self.index.write_rows(path, off, 0, n))
            self._graph_arrays = graph
            self._persisted = None
            self._write_index_meta()
            with open(self.metadata_path, "w", encoding="utf-8") as file:
                json.dump(self.metadata, file, ensure_ascii=False, indent=2)
            return
        if old is not None and old <= n:
            faiss_format.append_flat_rows(self.index_path, d, old, n, mt,
                                          lambda path, off: self.index.write_rows(path, off, old, n - old))
        else:
            faiss_format.write_flat_rows(self.index_path, d, n, mt,
                                         lambda path, off: self.index.write_rows(path, off, 0, n))
        self._persisted = self._file_state(n, d, mt)
        self._write_index_meta()
        with open(self.metadata_path, "w", encoding="utf-8") as file:
            json.dump(self.metadata, file, ensure_ascii=False, indent=2)

    def load(self) -> bool:
        """加载索引与元数据 (utils/vector_store.py:239-260)."""
        if not os.path.exists(self.index_path) or not os.path.exists(self.metadata_path):
            return False

        loaded = faiss_format.read_index(self.index_path)
        index = self._create_index_with_metric(loaded.d, loaded.metric_type)
        if loaded.ntotal:  # payload streamed file -> pinned chunks -> HBM (no host copy of the matrix)
            index.add_from_file(self.index_path, loaded.payload_offset, loaded.ntotal)
        self._drop_graph()
        self.index = index
        self._persisted = (self._file_state(loaded.ntotal, loaded.d, loaded.metric_type)
                           if loaded.kind == "flat" else None)
        payload = self._load_index_meta()
        self._validate_loaded_index(payload, loaded)
        # a flat configuration keeps an HNSW file's graph: save() writes it back (extended by the
        # rows added since), as the reference's IndexHNSWFlat would be
        self._file_hnsw = loaded.kind == "hnsw" and self.index_type == "flat"
        if loaded.kind == "hnsw" and (self._file_hnsw or _hnsw_graph_search()):
            self._graph_arrays = faiss_format.read_hnsw_graph(self.index_path)

        with open(self.metadata_path, "r", encoding="utf-8") as file:
            self.metadata = json.load(file)
        if self.index.ntotal != len(self.metadata):
            raise ValueError("索引与元数据数量不一致，请重新构建索引")
        self.dimension = self.index.d
        self._embeddings = {}
        self._rebuild_path_index()
        return True

    def _create_index_with_metric(self, dimension: int, metric_type: int):
        metric = "cosine" if metric_type == METRIC_INNER_PRODUCT else "l2"
        return _index_factory(int(dimension), metric)

    def get_total_items(self) -> int:
        """获取当前向量数量."""
        if self.index is None:
            return 0
        return int(self.index.ntotal)

    def clear(self) -> None:
        """清空索引与元数据."""
        self._drop_graph()
        self._file_hnsw = False
        self.index = self._create_index(self.dimension) if self.dimension else None
        self.metadata = []
        self._embeddings = {}
        self._path_to_index = {}
        self._persisted = None

    # ------------------------------------------------------------------ HNSW graph search
    def _graph_covers(self, n: int) -> bool:
        g = self._graph_arrays
        return g is not None and int(np.asarray(g["levels"]).shape[0]) == n

    def _drop_graph(self) -> None:
        self._drop_graph_search()
        self._graph_arrays = None

    def _search_rows(self, q: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """``index.search``, or with ``VECTOR_HNSW_SEARCH=graph`` on an HNSW store, faiss's HNSW
        search on the GPU over the graph of the loaded file or the graph ``save()`` writes
        (:meth:`_build_graph`).  The graph is rebuilt only once the store has grown by
        ``_GRAPH_REBUILD_GROWTH`` since it was built; rows added behind it meanwhile are searched
        exactly (a flat index of those rows) and merged with the graph's results, so alternating
        ``add_item`` / ``search`` does not pay a whole-graph build per search.  Stores above
        ``VECTOR_HNSW_GRAPH_MAX_ROWS`` (their graph is still saved: :meth:`save`), beams wider than
        the GPU search takes (max(efSearch, k) > 2048) and multi-GPU indexes search exactly."""
        n = int(self.index.ntotal)
        if (self.index_type != "hnsw" or not _hnsw_graph_search() or not isinstance(self.index, FlatIndex)
                or max(k, self.hnsw_ef_search) > _HNSW_EF_MAX or n > _hnsw_graph_max_rows()):
            return self.index.search(q, k)
        if self._hnsw is not None and self._hnsw.index is not self.index:
            self._drop_graph_search()
        covered = self._hnsw.ntotal if self._hnsw is not None else 0
        if self._hnsw is None or n > covered * _GRAPH_REBUILD_GROWTH:
            self._drop_graph_search()
            g = self._graph_arrays
            if g is None or not 0 < int(np.asarray(g["levels"]).shape[0]) <= n or \
                    n > int(np.asarray(g["levels"]).shape[0]) * _GRAPH_REBUILD_GROWTH:
                self._graph_arrays = self._build_graph(n)
            self._hnsw = HNSWGraph(self.index, self._graph_arrays, self.hnsw_ef_search)
            covered = self._hnsw.ntotal
        D, I = self._hnsw.search(q, k, self.hnsw_ef_search)
        if covered == n:
            return D, I
        # rows [covered, n): exact search over a flat index of just those rows, then a merge
        tail = self._graph_tail
        if tail is None:
            tail = self._graph_tail = self._create_index(self.dimension)
        have = covered + int(tail.ntotal)
        if have < n:
            tail.add(np.ascontiguousarray(self.index.reconstruct_n(have, n - have)))
        Dt, It = tail.search(q, min(k, n - covered))
        It = np.where(It >= 0, It + covered, -1)
        return _merge_topk(D, I, Dt, It, k, int(self.index.metric_type) == METRIC_INNER_PRODUCT)

    def _drop_graph_search(self) -> None:
        """Release the GPU graph and the exactly-searched tail behind it (the arrays stay)."""
        if self._hnsw is not None:
            self._hnsw.close()
        self._hnsw = None
        if self._graph_tail is not None:
            self._graph_tail.close()
        self._graph_tail = None

    def _build_graph(self, n: int) -> Dict[str, Any]:
        """The faiss-layout HNSW graph over the n stored rows.  A graph already covering the first
        m < n rows (the one last saved or loaded, a faiss-built file's included) is extended by
        inserting rows [m, n) the way faiss's ``IndexHNSWFlat.add`` does, batched
        (:func:`hnsw.insert_rows`: an efConstruction beam over the existing graph + the batch's
        exact candidates, the selection heuristic, reverse links); otherwise the first
        ``VECTOR_HNSW_GRAPH_MAX_ROWS`` rows are built at once from exact candidates
        (:meth:`_build_graph_exact`) and the rest inserted.  Cost per save: the new rows only."""
        g = self._graph_arrays
        make = lambda: self._create_index(self.dimension)  # noqa: E731
        if g is not None and 0 < int(np.asarray(g["levels"]).shape[0]) < n:
            # (a flat configuration over an HNSW file inserts with the file's efConstruction, as the
            # reference's loaded IndexHNSWFlat would)
            efc = int(g["efConstruction"]) if self._file_hnsw else int(self.hnsw_ef_construction)
            return hnsw_mod.insert_rows(self.index, g, int(np.asarray(g["levels"]).shape[0]), n, efc, make)
        n0 = min(n, max(1, _hnsw_graph_max_rows()))
        g = self._build_graph_exact(n0)
        if n0 < n:
            g = hnsw_mod.insert_rows(self.index, g, n0, n, int(self.hnsw_ef_construction), make)
        return g

    def _build_graph_exact(self, n: int) -> Dict[str, Any]:
        """A faiss-layout HNSW graph over the first n stored rows built at once: node levels drawn
        as faiss's ``HNSW::random_level`` does (``set_default_probas(M, 1/ln M)``; numpy's
        generator, seed 12345, not faiss's: :func:`hnsw.draw_levels`); on every level each node's
        candidates are its exact max(efConstruction, width) nearest nodes of that level (the flat
        search, ties -> lower id) and its neighbours (2M on level 0, M above) are chosen from them
        by faiss's heuristic, reverse links included (:func:`hnsw.select_level`, on the GPU); the
        entry point is the first node of the top level (oracle/hnsw_oracle.py ``heuristic_graph``
        restates it)."""
        M = self.hnsw_m
        probas, cum = faiss_format.hnsw_default_probas(M)
        lev = hnsw_mod.draw_levels(n, probas)
        levels = (lev + 1).astype(np.int32)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        offsets[1:] = np.cumsum(cum[levels].astype(np.uint64))
        nb = np.full(int(offsets[-1]), -1, dtype=np.int32)
        top = int(lev.max()) if n else -1
        for level in range(top + 1):
            members = np.nonzero(lev >= level)[0]
            width = int(cum[level + 1] - cum[level])
            C = min(max(int(self.hnsw_ef_construction), width), hnsw_mod.HP_C_MAX)
            cand = self._knn_graph(C, None if level == 0 and n == int(self.index.ntotal) else members)
            sel = hnsw_mod.select_level(self.index, members, cand, width)
            base = offsets[members].astype(np.int64) + int(cum[level])
            for j in range(members.shape[0]):
                row = sel[j][sel[j] >= 0]
                nb[base[j]:base[j] + len(row)] = row
        return {"assign_probas": probas, "cum_nneighbor_per_level": cum, "levels": levels, "offsets": offsets,
                "neighbors": nb, "entry_point": int(np.nonzero(lev == top)[0][0]) if n else -1, "max_level": top,
                "efConstruction": int(self.hnsw_ef_construction), "efSearch": int(self.hnsw_ef_search),
                "upper_beam": 1}

    def _knn_graph(self, width: int, members: Optional[np.ndarray] = None) -> np.ndarray:
        """Exact top-``width`` neighbours (itself excluded, -1 padded) of every stored row, or of
        every row of ``members`` among ``members`` only (global ids; a temporary index over their
        stored values), by the GPU flat search."""
        n = int(self.index.ntotal)
        index, ids = self.index, None
        if members is not None:
            ids = np.asarray(members, dtype=np.int64)
            index = self._create_index(self.dimension)
            for r0 in range(0, n, 65536):
                rows = self.index.reconstruct_n(r0, min(65536, n - r0))
                sel = ids[(ids >= r0) & (ids < r0 + rows.shape[0])] - r0
                if sel.size:
                    index.add(np.ascontiguousarray(rows[sel]))
        m = int(index.ntotal)
        out = np.full((m, width), -1, dtype=np.int32)
        kk = min(m, width + 1)
        try:
            for r0 in range(0, m, 4096):
                rows = index.reconstruct_n(r0, min(4096, m - r0))
                _, I = index.search(rows, kk)
                own = np.arange(r0, r0 + I.shape[0])[:, None]
                ok = (I >= 0) & (I != own)
                pos = np.cumsum(ok, axis=1) - 1  # order kept, itself dropped
                ok &= pos < width
                r, c = np.nonzero(ok)
                nbr = I[r, c] if ids is None else ids[I[r, c]]
                out[r0 + r, pos[r, c]] = nbr
        finally:
            if ids is not None and hasattr(index, "close"):
                index.close()
        return out

    # ------------------------------------------------------------------ persistence state
    def _file_state(self, rows: int, d: int, metric_type: int) -> Optional[Dict[str, Any]]:
        try:
            st = os.stat(self.index_path)
        except OSError:
            return None
        return {"path": os.path.abspath(self.index_path), "rows": int(rows), "d": int(d), "metric_type": int(metric_type),
                "stat": (st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns)}

    def _appendable_rows(self, d: int, metric_type: int) -> Optional[int]:
        """Rows of the index file if it is still exactly what this store last wrote or loaded."""
        p = self._persisted
        if not p or p["path"] != os.path.abspath(self.index_path) or p["d"] != d or p["metric_type"] != metric_type:
            return None
        try:
            st = os.stat(self.index_path)
        except OSError:
            return None
        if (st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns) != p["stat"]:
            return None
        if st.st_size != faiss_format.FLAT_HEADER_BYTES + p["rows"] * d * 4:
            return None
        return p["rows"]

    # ------------------------------------------------------------------ batched additions
    def add(self, embeddings: np.ndarray, metadatas: Sequence[Dict]) -> None:
        """Bulk ``add_item``: n x d rows + n metadata dicts in one device transfer."""
        rows = np.asarray(embeddings, dtype="float32")
        if rows.ndim != 2:
            raise ValueError("embeddings must be an (n, d) array")
        if len(metadatas) != rows.shape[0]:
            raise ValueError("metadatas must have one entry per row")
        if rows.shape[0] == 0:
            return
        if self.index is None:
            self.dimension = rows.shape[1]
            self.index = self._create_index(self.dimension)
        if rows.shape[1] != self.dimension:
            raise ValueError(f"向量维度不匹配: {rows.shape[1]} != {self.dimension}")
        self.index.add(self._normalize_rows(rows))
        base = len(self.metadata)
        self.metadata.extend(metadatas)
        for i, md in enumerate(metadatas):
            photo_path = md.get("photo_path") if isinstance(md, dict) else None
            if isinstance(photo_path, str) and photo_path:
                self._path_to_index[photo_path] = base + i

    def search_batch(self, queries: np.ndarray, top_k: int) -> Tuple[np.ndarray, np.ndarray]:
        """Batched search in faiss layout: (D nq x k float32, I nq x k int64), rows normalised
        exactly like ``search``; k is clamped to ntotal as ``search`` does."""
        q = np.asarray(queries, dtype="float32")
        if q.ndim != 2:
            raise ValueError("queries must be an (nq, d) array")
        if self.index is None or self.index.ntotal == 0:
            return np.zeros((q.shape[0], 0), dtype=np.float32), np.zeros((q.shape[0], 0), dtype=np.int64)
        if q.shape[1] != self.dimension:
            raise ValueError(f"向量维度不匹配: {q.shape[1]} != {self.dimension}")
        k = min(top_k, self.index.ntotal)
        return self._search_rows(self._normalize_rows(q), k)
