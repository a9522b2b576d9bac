"""Byte-compatible reader/writer of faiss' flat index files (the persistence half of the path).

The reference persists its index with ``faiss.write_index`` / ``faiss.read_index``
(/root/reference/utils/vector_store.py:234, :249).  Those files are what the indexer worker
hands to the server process (core/indexer.py:945,970 -> core/searcher.py:368), so existing
``data/`` directories must load unchanged.

Formats (faiss' ``index_write.cpp`` layout, little endian), decoded from the reference's own
fixtures ``pytest-tmp/build-smoke/data/idx`` (IxFI, d=8, 77 bytes) and
``data/photo_search.index`` (IHNf over IxFI, d=4096, 77 rows):

  header  = fourcc[4] | int32 d | int64 ntotal | int64 dummy (1<<20) | int64 dummy (1<<20)
            | uint8 is_trained | int32 metric_type [| float32 metric_arg if metric_type > 1]
  IxFI/IxF2 (IndexFlatIP / IndexFlatL2): header | uint64 n_floats | float32[n_floats]
  IHNf (IndexHNSWFlat): header | vec<double> assign_probas | vec<int32> cum_nneighbor_per_level
            | vec<int32> levels | vec<uint64> offsets | vec<int32> neighbors
            | int32 entry_point, max_level, efConstruction, efSearch, upper_beam
            | storage index (IxFI / IxF2), recursively
  vec<T>  = uint64 count | T[count]

Flat files are written for flat indexes; an HNSW-configured store writes an ``IHNf`` file whose
graph is the exact k-NN graph of the rows on one level (:func:`single_level_graph`), so the
reference's faiss can still load it.  Searches here are exact flat searches either way.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

FOURCC_FLAT_IP = b"IxFI"
FOURCC_FLAT_L2 = b"IxF2"
FOURCC_HNSW_FLAT = b"IHNf"
METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
_DUMMY = 1 << 20


@dataclass
class FaissFile:
    kind: str            # "flat" or "hnsw"
    fourcc: bytes
    d: int
    ntotal: int
    metric_type: int
    vectors: np.ndarray  # (ntotal, d) float32 (memory-mapped for large files)
    hnsw_params: dict
    payload_offset: int = 0  # byte offset of the row-major float32 payload in the file


class FaissFormatError(ValueError):
    pass


def _header(buf: memoryview, off: int):
    # fourcc(4) | d(4) | ntotal(8) | dummy(8) | dummy(8) | is_trained(1) | metric_type(4)
    if len(buf) - off < 37:
        raise FaissFormatError("truncated faiss index header")
    fourcc = bytes(buf[off:off + 4])
    d, ntotal = struct.unpack_from("<iq", buf, off + 4)
    is_trained = buf[off + 32]
    (metric_type,) = struct.unpack_from("<i", buf, off + 33)
    off += 37
    if metric_type > 1:
        off += 4  # metric_arg
    return fourcc, d, ntotal, is_trained, metric_type, off


def _read_at(path: str, buf: memoryview, off: int) -> FaissFile:
    fourcc, d, ntotal, _trained, metric_type, off = _header(buf, off)
    if fourcc in (FOURCC_FLAT_IP, FOURCC_FLAT_L2):
        (nf,) = struct.unpack_from("<Q", buf, off)
        off += 8
        if nf != d * ntotal:
            raise FaissFormatError(f"flat payload has {nf} floats, expected {d} x {ntotal}")
        if len(buf) < off + 4 * nf:
            raise FaissFormatError("truncated flat payload")
        if nf * 4 >= (64 << 20):
            vec = np.memmap(path, dtype="<f4", mode="r", offset=off, shape=(ntotal, d))
        else:
            vec = np.frombuffer(buf, dtype="<f4", count=nf, offset=off).reshape(ntotal, d).copy()
        mt = METRIC_INNER_PRODUCT if fourcc == FOURCC_FLAT_IP else METRIC_L2
        return FaissFile("flat", fourcc, d, ntotal, mt if metric_type in (0, 1) else metric_type,
                         np.asarray(vec, dtype=np.float32), {}, off)
    if fourcc == FOURCC_HNSW_FLAT:
        for es in (8, 4, 4, 8, 4):  # assign_probas, cum_nneighbor_per_level, levels, offsets, neighbors
            (n,) = struct.unpack_from("<Q", buf, off)
            off += 8 + n * es
        entry_point, max_level, ef_c, ef_s, _upper = struct.unpack_from("<5i", buf, off)
        off += 20
        storage = _read_at(path, buf, off)
        if storage.d != d or storage.ntotal != ntotal:
            raise FaissFormatError("HNSW storage does not match its header")
        return FaissFile("hnsw", fourcc, d, ntotal, metric_type, storage.vectors,
                         {"entry_point": entry_point, "max_level": max_level, "efConstruction": ef_c,
                          "efSearch": ef_s}, storage.payload_offset)
    raise FaissFormatError(f"unsupported faiss index type {fourcc!r}")


def hnsw_default_probas(M: int):
    """faiss ``HNSW::set_default_probas(M, 1 / log(M))``: level probabilities (computed with a
    float level multiplier, stored as float, widened to double) and cumulative neighbour counts
    (2M on level 0, M above).  Pinned bit for bit by the reference's HNSW fixture (M = 48)."""
    lm = np.float32(1.0 / np.log(M))
    probas, cum, nn, level = [], [0], 0, 0
    while True:
        p = np.float32(np.exp(np.float64(np.float32(-level) / lm)) * (1.0 - np.exp(np.float64(np.float32(-1) / lm))))
        if p < 1e-9:
            break
        probas.append(float(p))
        nn += 2 * M if level == 0 else M
        cum.append(nn)
        level += 1
    return np.array(probas, dtype="<f8"), np.array(cum, dtype="<i4")


def read_hnsw_graph(path: str) -> dict:
    """The graph arrays of an ``IHNf`` file (faiss ``write_index`` of an IndexHNSWFlat)."""
    # reads the header and the graph arrays only (they precede the storage's row payload)
    with open(path, "rb") as f:
        head = f.read(41)
        fourcc, d, ntotal, _trained, metric_type, off = _header(memoryview(head), 0)
        if fourcc != FOURCC_HNSW_FLAT:
            raise FaissFormatError(f"not an HNSW file: {fourcc!r}")
        f.seek(off)
        g = {"d": d, "ntotal": ntotal, "metric_type": metric_type}
        for name, dt in (("assign_probas", "<f8"), ("cum_nneighbor_per_level", "<i4"), ("levels", "<i4"),
                         ("offsets", "<u8"), ("neighbors", "<i4")):
            raw = f.read(8)
            if len(raw) != 8:
                raise FaissFormatError("truncated HNSW graph")
            (n,) = struct.unpack("<Q", raw)
            nbytes = n * np.dtype(dt).itemsize
            body = f.read(nbytes)
            if len(body) != nbytes:
                raise FaissFormatError("truncated HNSW graph")
            g[name] = np.frombuffer(body, dtype=dt, count=n).copy()
            off += 8 + nbytes
        raw = f.read(20)
        if len(raw) != 20:
            raise FaissFormatError("truncated HNSW graph")
        (g["entry_point"], g["max_level"], g["efConstruction"], g["efSearch"],
         g["upper_beam"]) = struct.unpack("<5i", raw)
    g["storage_offset"] = off + 20
    return g


def write_hnsw(path: str, graph: dict, d: int, ntotal: int, metric_type: int, write_rows) -> None:
    """Write an ``IHNf`` file: the HNSW header and graph arrays (faiss ``write_index`` layout) and
    the flat storage, whose fp32 payload comes from ``write_rows(path, offset)``.  Temporary name +
    rename, like :func:`write_flat_rows`."""
    parts = [FOURCC_HNSW_FLAT + struct.pack("<iqqqBi", d, ntotal, _DUMMY, _DUMMY, 1, metric_type)]
    for name, dt in (("assign_probas", "<f8"), ("cum_nneighbor_per_level", "<i4"), ("levels", "<i4"),
                     ("offsets", "<u8"), ("neighbors", "<i4")):
        a = np.ascontiguousarray(graph[name], dtype=dt)
        parts.append(struct.pack("<Q", a.size) + a.tobytes())
    parts.append(struct.pack("<5i", graph["entry_point"], graph["max_level"], graph["efConstruction"],
                             graph["efSearch"], graph["upper_beam"]))
    parts.append(flat_bytes_header(d, ntotal, metric_type))
    head = b"".join(parts)
    tmp = f"{path}.tmp-{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(head)
    if ntotal:
        write_rows(tmp, len(head))
    os.replace(tmp, path)


def single_level_graph(knn: np.ndarray, M: int, ef_construction: int, ef_search: int) -> dict:
    """HNSW graph arrays for a one-level graph: every node on level 0 with the given neighbour
    lists (n x <=2M ids, -1 padded).  A valid faiss IndexHNSWFlat graph (its search starts at the
    entry point and walks level 0)."""
    probas, cum = hnsw_default_probas(M)
    n = knn.shape[0]
    nb = np.full((n, 2 * M), -1, dtype="<i4")
    w = min(knn.shape[1], 2 * M)
    nb[:, :w] = knn[:, :w]
    return {"assign_probas": probas, "cum_nneighbor_per_level": cum, "levels": np.ones(n, dtype="<i4"),
            "offsets": np.arange(n + 1, dtype="<u8") * np.uint64(2 * M), "neighbors": nb.reshape(-1),
            "entry_point": 0 if n else -1, "max_level": 0 if n else -1, "efConstruction": int(ef_construction),
            "efSearch": int(ef_search), "upper_beam": 1}


def read_index(path: str) -> FaissFile:
    with open(path, "rb") as f:
        data = f.read() if os.path.getsize(path) < (64 << 20) else None
    if data is None:
        mm = np.memmap(path, dtype=np.uint8, mode="r")
        return _read_at(path, memoryview(mm), 0)
    return _read_at(path, memoryview(data), 0)


def flat_bytes_header(d: int, ntotal: int, metric_type: int) -> bytes:
    fourcc = FOURCC_FLAT_IP if metric_type == METRIC_INNER_PRODUCT else FOURCC_FLAT_L2
    return (fourcc + struct.pack("<iqqqBi", d, ntotal, _DUMMY, _DUMMY, 1, metric_type)
            + struct.pack("<Q", d * ntotal))


FLAT_HEADER_BYTES = 45  # fourcc .. metric_type (37) + uint64 n_floats (8)


def write_flat_rows(path: str, d: int, ntotal: int, metric_type: int, write_rows) -> None:
    """Full rewrite of an IxFI / IxF2 file whose payload is produced by ``write_rows(path, offset)``
    (the device-to-file stream of ``FlatIndex.write_rows``).  Temporary name + rename, so a crash
    never leaves a torn index."""
    tmp = f"{path}.tmp-{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(flat_bytes_header(d, ntotal, metric_type))
    if ntotal:
        write_rows(tmp, FLAT_HEADER_BYTES)
    os.replace(tmp, path)


def append_flat_rows(path: str, d: int, old_ntotal: int, new_ntotal: int, metric_type: int, write_rows) -> None:
    """Grow an existing flat file from ``old_ntotal`` to ``new_ntotal`` rows in place: the new rows
    go after the old payload (``write_rows(path, offset)``), then the header is rewritten in one
    write.  The result is byte-identical to a full rewrite; until the header write lands, readers
    see the old index (faiss and :func:`read_index` ignore trailing bytes)."""
    if new_ntotal > old_ntotal:
        write_rows(path, FLAT_HEADER_BYTES + old_ntotal * d * 4)
    with open(path, "r+b") as f:
        f.write(flat_bytes_header(d, new_ntotal, metric_type))


def write_flat(path: str, vectors: np.ndarray, metric_type: int) -> None:
    """Write an IxFI / IxF2 file byte-identical to faiss.write_index of an IndexFlat.
    Written to a temporary name and renamed, so a crash never leaves a torn index."""
    v = np.ascontiguousarray(vectors, dtype="<f4")
    if v.ndim != 2:
        raise ValueError("vectors must be 2-D")
    tmp = f"{path}.tmp-{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(flat_bytes_header(v.shape[1], v.shape[0], metric_type))
        if v.size:
            f.write(memoryview(v).cast("B"))
    os.replace(tmp, path)
