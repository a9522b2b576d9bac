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

With the int8 screen on bf16/f16 shards (``vs_two_phase_ok``: one int8 MFMA batch), step 1 runs in
two phases around one more exchange of the same shape: phase A scores each query's best few keys
per shard and the shards all-gather + merge those lists; the merged k-th score is a lower bound of
the global k-th best, so in phase B each shard exactly scores only the rows whose screen bound
reaches it (its share of the global refine window, not a whole window of its own) and certifies
against it.  The final exchange and merge are unchanged, and so is the result.

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


def _device_merge_packed(metric: int, g: torch.Tensor, k: int):
    """The HIP merge reading an all-gather of interleaved (score bits, id) pairs [G][nq][k][2] in
    place (in_stride 2): no unpacking copies."""
    from .index import merge_shards_device
    G, nq = g.shape[0], g.shape[1]
    S = torch.empty((nq, k), dtype=torch.float64, device=g.device)
    I = torch.empty((nq, k), dtype=torch.int64, device=g.device)
    D = torch.empty((nq, k), dtype=torch.float32, device=g.device)
    stream = torch.cuda.current_stream(g.device).cuda_stream
    merge_shards_device(metric, g.data_ptr(), g.data_ptr() + 8, G, nq, k, S.data_ptr(), I.data_ptr(), D.data_ptr(),
                        stream, in_stride=2)
    return S, I, D


def _pack(S: torch.Tensor, I: torch.Tensor) -> torch.Tensor:
    """(S fp64, I int64) [nq][k] -> interleaved (score bits, id) pairs [nq][k][2] (int64)."""
    return torch.stack([S.contiguous().view(torch.int64), I.contiguous()], dim=-1)


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


def _device_phase_a(index, q: torch.Tensor, k: int, row0: int, world: int):
    """Two-phase local search, phase A: the shard's best-so-far lists as interleaved (score bits, id)
    pairs [nq][k][2] (written in that layout by the library, ready for the all-gather) + the
    pending search."""
    nq = q.shape[0]
    SI = torch.empty((nq, k, 2), dtype=torch.int64, device=q.device)
    stream = torch.cuda.current_stream(q.device).cuda_stream
    pend = index.search_phase_a(q.data_ptr(), nq, k, world, SI.data_ptr(), SI.data_ptr() + 8, row0, stream, stride=2)
    return SI, pend


def _device_phase_b(index, pend, floor_S: torch.Tensor, q: torch.Tensor, k: int):
    """Phase B with the merged phase-A lists as the floor: the shard's exact top-k as interleaved
    (score bits, id) pairs [nq][k][2].  Consumes ``pend`` whatever happens (a pending search holds
    the index's read lock and a workspace lease until it is freed)."""
    try:  # nothing may fail between here and the C call without freeing the pending search
        nq = q.shape[0]
        SI = torch.empty((nq, k, 2), dtype=torch.int64, device=q.device)
        stream = torch.cuda.current_stream(q.device).cuda_stream
        floor_ptr = floor_S.data_ptr()
    except BaseException:
        index.search_pending_free(pend)
        raise
    # (the library frees the pending search itself, on success and on every error)
    index.search_phase_b(pend, floor_ptr, None, SI.data_ptr() + 8, SI.data_ptr(), stream, stride=2)
    return SI


def _device_two_phase_ok(index, nq: int, k: int) -> bool:
    f = getattr(index, "two_phase_ok", None)
    return bool(f(nq, k)) if f else False


class ShardedFlatIndex:
    """One shard of a row-partitioned exact flat index per rank of ``group``.

    Build the shard with :meth:`add_shard` (rows this rank owns, e.g. a slice of a memory-mapped
    faiss file) or :meth:`add_synthetic` (each rank generates its own rows); then every rank
    calls :meth:`search` with the same query batch (or passes ``src`` to broadcast it).
    """

    def __init__(self, d: int, metric: str = "ip", dtype: str = "f32", device: Optional[int] = None,
                 group=None, index=None,
                 local_search: Optional[Callable] = None, merge: Optional[Callable] = None,
                 phase_a: Optional[Callable] = None, phase_b: Optional[Callable] = None,
                 two_phase_ok: Optional[Callable] = None) -> None:
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
        self._phase_a = phase_a or _device_phase_a
        self._phase_b = phase_b or _device_phase_b
        # (injected local searches without phase functions keep the one-phase protocol)
        self._two_phase_ok = two_phase_ok or (_device_two_phase_ok if local_search is None else (lambda *a: False))
        self.row0 = 0
        self.n_total = 0
        # measurement only (bench.py --shard-of G): a single rank runs the G-shard step on its shard,
        # the exchanges included (over its one-rank process group)
        self.shards_hint: Optional[int] = None
        # ... and the floor the other shards would have contributed (the G shards' merged phase-A
        # lists, computed beforehand), used in place of its one-rank exchange's merge
        self.floor_override: Optional[torch.Tensor] = None
        # measurement only: HIP events around every all-gather on the calling stream
        self.exchange_timing = False
        self._xevents: list = []

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

    def full_scan_count(self) -> int:
        """Queries this rank's shard answered by the exact full scan so far (synchronising; 0 unless
        more than KP_MAX rows tie within the screen's error margin -- see vs_full_scan_count).  Their
        shard lists are exact like every other's: nothing uncertified is ever merged."""
        f = getattr(self.index, "full_scan_count", None)
        return int(f()) if f else 0

    # -- search --------------------------------------------------------------------------------
    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:  # a one-rank group has nothing to exchange (bench --shard-of G: the
            return t.unsqueeze(0)  # measured rank's own lists; the G-rank run adds RCCL's latency)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        ev = None
        if self.exchange_timing and t.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        else:
            dist.all_gather(list(out.unbind(0)), t.contiguous(), group=self.group)
        if ev is not None:
            ev[1].record()
            self._xevents.append(ev)
        return out

    def exchange_times_fetch(self) -> list:
        """ms of every all-gather timed since the last fetch (synchronising; exchange_timing)."""
        out = [a.elapsed_time(b) for a, b in self._xevents]
        self._xevents = []
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
        # (every rank takes the same branch: the test depends only on the index configuration)
        shards = self.shards_hint or self.world
        if shards > 1 and self._two_phase_ok(self.index, nq, k):
            # ONE more all-gather of the same shape first (the phase-A lists -> the floor)
            return self._exchange_packed(self._two_phase_local(q, k, shards), k)
        if self.n_local > 0:
            S, I, D = self._local_search(self.index, q, k, self.row0)
        else:  # empty shard (n_total < world): contributes only padding
            S, I, D = self._padding(nq, k, q.device)
        if shards == 1:
            return D, I, S
        # ONE all-gather of interleaved (fp64 score bits, id) pairs: a second collective would add
        # its full latency to every step (the payload is only nq * k * 16 B per rank)
        return self._exchange_packed(_pack(S, I), k)

    def _padding(self, nq: int, k: int, device):
        S = torch.full((nq, k), _worst(self.metric), dtype=torch.float64, device=device)
        I = torch.full((nq, k), -1, dtype=torch.int64, device=device)
        D = torch.full((nq, k), -3.4028234663852886e38 if self.metric == 0 else 3.4028234663852886e38,
                       dtype=torch.float32, device=device)
        return S, I, D

    def _exchange_packed(self, SI: torch.Tensor, k: int):
        """all-gather of the packed (score bits, id) lists + the device merge: (D, I, S), identical on
        every rank."""
        g = self._gather(SI)
        if self._merge is _device_merge:  # the HIP merge reads the gathered pairs in place
            S, I, D = _device_merge_packed(self.metric, g, k)
        else:
            S, I, D = self._merge(self.metric, g[..., 0].contiguous().view(torch.float64), g[..., 1].contiguous(), k)
        return D, I, S

    def _two_phase_local(self, q: torch.Tensor, k: int, shards: int) -> torch.Tensor:
        """The shard's exact top-k (packed pairs) by the two-phase search: phase A, the exchange of
        the phase-A lists (their merge = the floor), phase B."""
        nq = q.shape[0]
        pend = None
        if self.n_local > 0:
            SIa, pend = self._phase_a(self.index, q, k, self.row0, shards)
        else:
            SIa = _pack(*self._padding(nq, k, q.device)[:2])
        try:
            _, _, floor_S = self._exchange_packed(SIa, k)
            if self.floor_override is not None:
                floor_S = self.floor_override
        except BaseException:
            if pend is not None:
                free = getattr(self.index, "search_pending_free", None)
                if free:
                    free(pend)
            raise
        if pend is None:
            return _pack(*self._padding(nq, k, q.device)[:2])
        return self._phase_b(self.index, pend, floor_S, q, k)  # consumes pend on every path

    def close(self) -> None:
        close = getattr(self.index, "close", None)
        if close:
            close()
