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

Writing always produces a flat file (IxFI for inner product, IxF2 for L2): the drop-in serves
every index exactly, so there is no graph to persist (DESIGN.md "HNSW").
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
