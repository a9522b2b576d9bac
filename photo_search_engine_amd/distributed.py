"""Row-sharded exact search across GPUs: one process per GPU over ``torch.distributed``.

SURVEY.md §8(e): rows are independent, so the global top-k is the merge of per-shard top-k
lists.  Each rank holds a contiguous row range ``[row0, row0 + n_local)`` of the corpus in its
own :class:`~photo_search_engine_amd.index.FlatIndex` (HBM-resident); a search is

  1. local exact search on the rank's shard (MFMA/GEMV screen + exact refine), returning the
     per-shard top-k as (exact fp64 score, GLOBAL id) -- ids offset on the device;
  2. one all-gather of those lists as interleaved (score bits, id) pairs (``nq * k * 16`` bytes
     per rank; RCCL over xGMI with the ``nccl`` backend) -- the only collective, and the path's
     only exchange step;
  3. a merge of the G sorted lists on the device (``vs_merge_shards_device``) on every rank, so
     all ranks hold the same final (D, I) without a second collective.

Ordering is total (score, then lower id), so the result is identical to a single-GPU search of
the whole corpus.  The reference has no multi-device path (faiss CPU index, utils/vector_store.py
:72-81); this module is the MI355X scale-out of the same ``index.search`` contract (:191).

The local search and the merge are injectable so the collective logic can be exercised on the
CPU with ``gloo`` (tests/test_distributed.py drives it with the oracle as the checker); the
defaults are the HIP library, with no CPU fallback.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

METRIC_CODES = {"ip": 0, "cosine": 0, "l2": 1}


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced row range of ``rank``: (row0, n_local)."""
    row0 = n_total * rank // world
    return row0, n_total * (rank + 1) // world - row0


def _worst(metric: int) -> float:
    return -1.7976931348623157e308 if metric == 0 else 1.7976931348623157e308


def _device_merge(metric: int, Sg: torch.Tensor, Ig: torch.Tensor, k: int):
    """HIP merge of [G][nq][k] sorted lists (vs_merge_shards_device) on the tensors' device."""
    from .index import merge_shards_device
    G, nq, _ = Sg.shape
    S = torch.empty((nq, k), dtype=torch.float64, device=Sg.device)
    I = torch.empty((nq, k), dtype=torch.int64, device=Sg.device)
    D = torch.empty((nq, k), dtype=torch.float32, device=Sg.device)
    stream = torch.cuda.current_stream(Sg.device).cuda_stream
    merge_shards_device(metric, Sg.data_ptr(), Ig.data_ptr(), G, nq, k, S.data_ptr(), I.data_ptr(), D.data_ptr(),
                        stream)
    return S, I, D


def _device_local_search(index, q: torch.Tensor, k: int, row0: int):
    """Exact top-k of the local shard as (S fp64, global I int64, D fp32) device tensors."""
    nq = q.shape[0]
    S = torch.empty((nq, k), dtype=torch.float64, device=q.device)
    I = torch.empty((nq, k), dtype=torch.int64, device=q.device)
    D = torch.empty((nq, k), dtype=torch.float32, device=q.device)
    stream = torch.cuda.current_stream(q.device).cuda_stream
    # exact for every query: uncertified screens are re-searched by a fallback round queued on the
    # device behind the first pass (bf16/f16; no host sync before the exchange)
    index.search_device_exact(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), row0, stream)
    return S, I, D


class ShardedFlatIndex:
    """One shard of a row-partitioned exact flat index per rank of ``group``.

    Build the shard with :meth:`add_shard` (rows this rank owns, e.g. a slice of a memory-mapped
    faiss file) or :meth:`add_synthetic` (each rank generates its own rows); then every rank
    calls :meth:`search` with the same query batch (or passes ``src`` to broadcast it).
    """

    def __init__(self, d: int, metric: str = "ip", dtype: str = "f32", device: Optional[int] = None,
                 group=None, index=None,
                 local_search: Optional[Callable] = None, merge: Optional[Callable] = None) -> None:
        # without an initialised process group this process is the only shard (1 GPU)
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.d = int(d)
        self.metric = METRIC_CODES[metric]
        if index is None:
            from .index import FlatIndex
            dev = torch.cuda.current_device() if device is None else int(device)
            index = FlatIndex(d, metric="ip" if self.metric == 0 else "l2", dtype=dtype, device=dev)
        self.index = index
        self._local_search = local_search or _device_local_search
        self._merge = merge or _device_merge
        self.row0 = 0
        self.n_total = 0

    # -- build ---------------------------------------------------------------------------------
    def add_shard(self, x_local, row0: int, n_total: int) -> None:
        """Add this rank's rows ``[row0, row0 + len(x_local))`` of an ``n_total``-row corpus."""
        self.row0, self.n_total = int(row0), int(n_total)
        if len(x_local):
            self.index.add(x_local)

    def add_shard_from_file(self, path: str) -> None:
        """Load this rank's contiguous row range of a faiss flat (or HNSW-wrapped flat) index file:
        only the shard's bytes are read, streamed file -> pinned chunks -> this rank's HBM."""
        from . import faiss_format
        ff = faiss_format.read_index(path)
        if ff.d != self.d:
            raise ValueError(f"index file dimension {ff.d} != {self.d}")
        row0, n = shard_range(ff.ntotal, self.rank, self.world)
        self.row0, self.n_total = row0, int(ff.ntotal)
        if n:
            self.index.add_from_file(path, ff.payload_offset + row0 * self.d * 4, n)

    def add_synthetic(self, seed: int, n_total: int, normalize: bool = True) -> None:
        """Each rank generates its own contiguous shard of the synthetic corpus in HBM."""
        row0, n = shard_range(int(n_total), self.rank, self.world)
        self.row0, self.n_total = row0, int(n_total)
        if n:
            self.index.add_synthetic(seed, row0, n, normalize)

    @property
    def n_local(self) -> int:
        return int(self.index.ntotal)

    def unresolved_count(self) -> int:
        """Queries this rank's device fallback could not certify so far (synchronising; 0 unless
        more than KP_MAX rows tie within the screen's error margin -- see vs_unresolved_count)."""
        f = getattr(self.index, "unresolved_count", None)
        return int(f()) if f else 0

    # -- search --------------------------------------------------------------------------------
    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        else:
            dist.all_gather(list(out.unbind(0)), t.contiguous(), group=self.group)
        return out

    def search(self, q: torch.Tensor, k: int, src: Optional[int] = None):
        """Exact global top-k for the batch ``q`` (nq x d fp32, on this rank's device).

        Returns (D fp32, I int64, S fp64) tensors [nq][k] -- identical on every rank.  Rows past
        the corpus size are padded with id -1 and the worst score (faiss layout).
        """
        if k <= 0:
            raise ValueError("k must be > 0")
        if q.dim() != 2 or q.shape[1] != self.d:
            raise ValueError(f"query shape {tuple(q.shape)} does not match dimension {self.d}")
        if src is not None and self.world > 1:
            dist.broadcast(q, src=src, group=self.group)
        nq = q.shape[0]
        if self.n_local > 0:
            S, I, D = self._local_search(self.index, q, k, self.row0)
        else:  # empty shard (n_total < world): contributes only padding
            S = torch.full((nq, k), _worst(self.metric), dtype=torch.float64, device=q.device)
            I = torch.full((nq, k), -1, dtype=torch.int64, device=q.device)
            D = torch.full((nq, k), -3.4028234663852886e38 if self.metric == 0 else 3.4028234663852886e38,
                           dtype=torch.float32, device=q.device)
        if self.world == 1:
            return D, I, S
        # ONE all-gather of interleaved (fp64 score bits, id) pairs: a second collective would add
        # its full latency to every step (the payload is only nq * k * 16 B per rank)
        SI = torch.stack([S.contiguous().view(torch.int64), I.contiguous()], dim=-1)
        g = self._gather(SI)
        S, I, D = self._merge(self.metric, g[..., 0].contiguous().view(torch.float64), g[..., 1].contiguous(), k)
        return D, I, S

    def close(self) -> None:
        close = getattr(self.index, "close", None)
        if close:
            close()
