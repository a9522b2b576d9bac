"""``FlatIndex``: the faiss-IndexFlat-shaped handle over libvs (one GPU shard).

It is what ``VectorStore`` holds in ``.index`` where the reference holds a
``faiss.IndexFlatIP`` / ``faiss.IndexFlatL2`` (/root/reference/utils/vector_store.py:72-81):
``ntotal``, ``d``, ``metric_type``, ``add``, ``search``, ``reconstruct``, ``reset``.  Host
methods take numpy arrays; ``*_device`` methods take raw device pointers (ints) so callers may
hand in torch tensors' ``data_ptr()`` without torch types crossing the C ABI.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import DTYPE_CODES, METRIC_IP, METRIC_L2, check

METRIC_INNER_PRODUCT = METRIC_IP  # faiss.METRIC_INNER_PRODUCT == 0
METRIC_L2_ = METRIC_L2            # faiss.METRIC_L2 == 1


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class FlatIndex:
    """Exact flat inner-product / squared-L2 index resident in one GPU's HBM."""

    def __init__(self, d: int, metric: str = "ip", dtype: str = "f32", device: int = 0) -> None:
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
        check(L.vs_create(int(d), code, DTYPE_CODES[dtype], int(device), ctypes.byref(h)))
        self._h = h
        self._L = L
        self.d = int(d)
        self.metric_type = code
        self.dtype = dtype
        self.device = int(device)

    # -- faiss-like surface ------------------------------------------------------------------
    @property
    def ntotal(self) -> int:
        return int(self._L.vs_ntotal(self._h))

    def add(self, x) -> None:
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 2 or x.shape[1] != self.d:
            raise ValueError(f"add expects an (n, {self.d}) array, got {x.shape}")
        check(self._L.vs_add(self._h, _ptr(x), x.shape[0]))

    def search(self, q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(q, dtype=np.float32)
        if q.ndim != 2 or q.shape[1] != self.d:
            raise ValueError(f"search expects an (nq, {self.d}) array, got {q.shape}")
        nq = q.shape[0]
        k = int(k)
        if k <= 0:
            raise _lib.VsError(_lib.VS_ERR_ARG, "k must be > 0")
        D = np.empty((nq, k), dtype=np.float32)
        I = np.empty((nq, k), dtype=np.int64)
        check(self._L.vs_search(self._h, _ptr(q), nq, k, _ptr(D), _ptr(I)))
        return D, I

    def reconstruct(self, i: int) -> np.ndarray:
        out = np.empty((self.d,), dtype=np.float32)
        check(self._L.vs_reconstruct(self._h, int(i), _ptr(out)))
        return out

    def reconstruct_n(self, i0: int, n: int) -> np.ndarray:
        out = np.empty((int(n), self.d), dtype=np.float32)
        if n:
            check(self._L.vs_reconstruct_n(self._h, int(i0), int(n), _ptr(out)))
        return out

    def hnsw_prune(self, nodes, cand, W: int) -> np.ndarray:
        """faiss's HNSW neighbour selection per node on the GPU (include/vs.h ``vs_hnsw_prune``):
        ``cand`` (m x C distinct row ids, -1 padded at the end) -> (m x W) kept ids, -1 padded."""
        nodes = np.ascontiguousarray(nodes, dtype=np.int64)
        cand = np.ascontiguousarray(cand, dtype=np.int32)
        if cand.ndim != 2 or cand.shape[0] != nodes.shape[0]:
            raise ValueError("cand must be (len(nodes), C)")
        m, C = cand.shape
        out = np.full((m, int(W)), -1, dtype=np.int32)
        if m:
            check(self._L.vs_hnsw_prune(self._h, m, _ptr(nodes), _ptr(cand), int(C), int(W), _ptr(out)))
        return out

    def reset(self) -> None:
        check(self._L.vs_reset(self._h))

    # -- screen selection ----------------------------------------------------------------------
    SCREENS = {"native": 0, "int8": 1}

    def set_screen(self, screen: str) -> None:
        """``"int8"``: keep an int8 copy of the rows and screen query batches with int8 MFMAs under
        a proven error bound (exact results, include/vs.h); ``"native"``: screen the stored rows."""
        if screen not in self.SCREENS:
            raise ValueError(f"unknown screen {screen!r}")
        check(self._L.vs_set_screen(self._h, self.SCREENS[screen]))

    @property
    def screen(self) -> str:
        v = int(self._L.vs_screen(self._h))
        return {0: "native", 1: "int8"}.get(v, "unknown")

    # -- persistence (faiss read_index / write_index payloads, streamed file <-> HBM) ---------------
    def add_from_file(self, path: str, byte_offset: int, n: int) -> None:
        """Append rows [0, n) of the row-major fp32 payload at ``byte_offset`` of ``path``."""
        check(self._L.vs_add_from_file(self._h, os.fsencode(path), int(byte_offset), int(n)))

    def write_rows(self, path: str, byte_offset: int, i0: int, n: int) -> None:
        """Write stored rows [i0, i0+n) as fp32 at ``byte_offset`` of ``path`` (no truncation)."""
        check(self._L.vs_write_rows_to_file(self._h, os.fsencode(path), int(byte_offset), int(i0), int(n)))

    # -- device-resident surface (bench / multi-GPU) -----------------------------------------
    def add_device(self, x_ptr: int, n: int, stream: Optional[int] = None) -> None:
        check(self._L.vs_add_device(self._h, x_ptr, int(n), stream or None))

    def add_synthetic(self, seed: int, global_row0: int, n: int, normalize: bool = True) -> None:
        check(self._L.vs_add_synthetic(self._h, int(seed), int(global_row0), int(n), int(bool(normalize))))

    def reserve(self, n: int) -> None:
        """Size the HBM row storage for ``n`` more rows in one allocation (no regrowth up to it)."""
        check(self._L.vs_reserve(self._h, int(n)))

    @property
    def capacity(self) -> int:
        return int(self._L.vs_capacity(self._h))

    def search_device(self, q_ptr: int, nq: int, k: int, D_ptr: Optional[int], I_ptr: int,
                      S64_ptr: Optional[int] = None, id_offset: int = 0, stream: Optional[int] = None) -> None:
        check(self._L.vs_search_device(self._h, q_ptr, int(nq), int(k), D_ptr or None, I_ptr, S64_ptr or None,
                                       int(id_offset), stream or None))

    def search_device_exact(self, q_ptr: int, nq: int, k: int, D_ptr: Optional[int], I_ptr: int,
                            S64_ptr: Optional[int] = None, id_offset: int = 0, stream: Optional[int] = None) -> None:
        """``search_device`` exact for every query: a failed certificate is re-searched by a fallback
        round queued on the device (no host sync), and a query even that round cannot certify (more
        near-tied rows than the deepest screen lists) by the exact full scan of the shard, counted in
        :meth:`full_scan_count`."""
        check(self._L.vs_search_device_exact(self._h, q_ptr, int(nq), int(k), D_ptr or None, I_ptr, S64_ptr or None,
                                             int(id_offset), stream or None))

    # -- two-phase search (the sharded step with a global T' exchange, include/vs.h) -------------
    def two_phase_ok(self, nq: int, k: int) -> bool:
        """Whether :meth:`search_phase_a` applies to a batch of ``nq`` queries at ``k`` (depends only
        on the index configuration, so every shard of a collective answers the same)."""
        return int(check(self._L.vs_two_phase_ok(self._h, int(nq), int(k)))) == 1

    def search_phase_a(self, q_ptr: int, nq: int, k: int, world: int, S_ptr: int, I_ptr: int, id_offset: int = 0,
                       stream: Optional[int] = None, stride: int = 1) -> int:
        """Phase A: this shard's best-so-far (S, I) lists for the exchange (``stride=2``: interleaved
        (score bits, id) pairs); returns the pending search for :meth:`search_phase_b` (or
        :meth:`search_pending_free`)."""
        out = ctypes.c_void_p(0)
        check(self._L.vs_search_device_phase_a(self._h, q_ptr, int(nq), int(k), int(world), int(id_offset), S_ptr,
                                               I_ptr, int(stride), stream or None, ctypes.byref(out)))
        return int(out.value)

    def search_phase_b(self, pending: int, floor_S_ptr: int, D_ptr: Optional[int], I_ptr: int,
                       S64_ptr: Optional[int] = None, stream: Optional[int] = None, stride: int = 1) -> None:
        """Phase B with the merged phase-A lists as the floor; frees the pending search."""
        check(self._L.vs_search_device_phase_b(ctypes.c_void_p(pending), floor_S_ptr, D_ptr or None, I_ptr,
                                               S64_ptr or None, int(stride), stream or None))

    def search_pending_free(self, pending: int) -> None:
        self._L.vs_search_pending_free(ctypes.c_void_p(pending))

    def set_timing(self, enable: bool) -> None:
        check(self._L.vs_set_timing(self._h, int(bool(enable))))

    def timing_fetch(self, cap: int = 4096):
        buf = (ctypes.c_float * cap)()
        kind = ctypes.c_int(0)
        n = check(self._L.vs_timing_fetch(self._h, buf, cap, ctypes.byref(kind)))
        return [float(buf[i]) for i in range(n)], {1: "mfma", 2: "gemv", 3: "mfma_i8", 4: "gemv_i8", 5: "full_scan"}.get(kind.value, "none")

    def uncertified_count(self) -> int:
        """First-pass certificate failures so far (each one was re-searched)."""
        return int(check(self._L.vs_uncertified_count(self._h)))

    def screen_state(self) -> dict:
        """The screen's state (include/vs.h ``vs_screen_state``): group residuals, the int8 margins'
        maxima and the screen-health feedback (int8 union depth, native routing, native seed depth)."""
        buf = (ctypes.c_double * 9)()
        check(self._L.vs_screen_state(self._h, buf, 9))
        keys = ("screen", "group_residuals", "groups_with_mean", "max_mean_norm", "max_code_norm",
                "max_row_error", "i8_union_log2", "i8_routed_searches", "native_seed_log2")
        return {k: (float(buf[i]) if "max" in k else int(buf[i])) for i, k in enumerate(keys)}

    def screen_probe(self, q_ptr: int, nq: int, screen: str, zero_queries: bool, stream: Optional[int] = None) -> float:
        """ms of one main-screen launch over the index with every threshold at +inf (no survivors),
        the query tile zeroed when ``zero_queries`` (include/vs.h ``vs_screen_probe``)."""
        ms = ctypes.c_float(0.0)
        check(self._L.vs_screen_probe(self._h, q_ptr, int(nq), FlatIndex.SCREENS[screen], int(bool(zero_queries)),
                                      stream or None, ctypes.byref(ms)))
        return float(ms.value)

    K1_PROBES = {"loads": 0, "lds": 1, "mfma": 2, "full": 3, "full_ms": 4, "full_prio": 5, "full_ms_prio": 6}

    def k1_probe(self, q_ptr: int, nq: int, screen: str, variant: str, zero_queries: bool, reps: int = 5,
                 stream: Optional[int] = None):
        """Diagnostic forms of the direct screen's loop (include/vs.h ``vs_k1_probe``): ``reps`` launches
        back to back -> (ms per launch, stamps [reps][G][4] uint64: s_memtime at the loop's start and
        end, s_memrealtime at the same points)."""
        import numpy as np
        ms = (ctypes.c_float * reps)()
        st = np.zeros((reps, 256, 4), dtype=np.uint64)
        G = ctypes.c_int32(0)
        check(self._L.vs_k1_probe(self._h, q_ptr, int(nq), FlatIndex.SCREENS[screen], FlatIndex.K1_PROBES[variant],
                                  int(bool(zero_queries)), int(reps), stream or None, ms, st.ctypes.data,
                                  ctypes.byref(G)))
        g = int(G.value)
        flat = st.reshape(-1)[: reps * g * 4].reshape(reps, g, 4)
        return [float(x) for x in ms], flat

    def set_scan_limit(self, nbytes: int) -> None:
        """Single-query calls over at most ``nbytes`` of stored rows use the exact full scan instead of
        a screen (include/vs.h ``vs_set_scan_limit``; 0 = always screen)."""
        check(self._L.vs_set_scan_limit(self._h, int(nbytes)))

    def full_scan_count(self) -> int:
        """Queries answered by the exact full scan so far: no bounded screen could certify them (more
        rows than KP_MAX tied within its margin).  Synchronises."""
        return int(check(self._L.vs_full_scan_count(self._h)))

    def host_staging_bytes(self) -> int:
        """Pinned host bytes held for ``search``'s query / result staging (bounded per context)."""
        return int(check(self._L.vs_host_staging_bytes(self._h)))

    def screen_copy_bytes(self) -> int:
        """HBM bytes of the int8 screen's copy (codes, per-row scale | error norm) on top of the
        stored rows; 0 on the native screen."""
        return int(check(self._L.vs_screen_copy_bytes(self._h)))

    # -- lifecycle ----------------------------------------------------------------------------
    def close(self) -> None:
        if self._h is not None and self._h.value:
            self._L.vs_destroy(self._h)
        self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass


def merge_shards_device(metric_type: int, S_ptr: int, I_ptr: int, G: int, nq: int, k: int, S_out: int, I_out: int,
                        D_out: Optional[int] = None, stream: Optional[int] = None, in_stride: int = 1) -> None:
    """Merge G per-shard sorted (S64, id) lists [G][nq][k] on the device (after an all-gather);
    ``in_stride=2``: one interleaved array of (score bits, id) pairs (``I_ptr = S_ptr + 8``)."""
    L = _lib.load()
    check(L.vs_merge_shards_device(int(metric_type), S_ptr, I_ptr, int(in_stride), int(G), int(nq), int(k), S_out,
                                   I_out, D_out or None, stream or None))


def set_k1_schedule(schedule: int) -> None:
    """The K-step schedule of the int8 inner-product direct screen, process-wide (include/vs.h
    ``vs_set_k1_schedule``): 0 = a barrier at the head of every K-step, 1 (default) = the mid-step
    barrier.  Results are identical."""
    check(_lib.load().vs_set_k1_schedule(int(schedule)))


def k1_schedule() -> int:
    return int(_lib.load().vs_k1_schedule())


def synthesize_device(device: int, seed: int, global_row0: int, n: int, d: int, out_ptr: int, normalize: bool = True,
                      dtype: str = "f32", stream: Optional[int] = None) -> None:
    """Write synthetic rows [global_row0, +n) as row-major fp32 (rounded to ``dtype``) to device
    memory -- the same counter-hash generator as ``FlatIndex.add_synthetic``."""
    L = _lib.load()
    check(L.vs_synthesize(int(device), int(seed), int(global_row0), int(n), int(d), int(bool(normalize)),
                          DTYPE_CODES[dtype], out_ptr, stream or None))


class MultiDeviceFlatIndex:
    """One exact flat index over several GPUs of this process (``vs_multi_*``, include/vs.h).

    The same faiss-IndexFlat-shaped surface as :class:`FlatIndex` (``ntotal``, ``d``,
    ``metric_type``, ``add``, ``search``, ``reconstruct``, ``reconstruct_n``, ``reset`` and the
    persistence hooks), so ``VectorStore`` holds it in ``.index`` unchanged; rows are dealt over the
    devices in chunks of 65,536 ids and every search merges the per-device exact top-k on
    ``devices[0]`` (the result equals one index over all rows).  A device may be listed more than
    once (several shards on one GPU).
    """

    def __init__(self, d: int, metric: str = "ip", dtype: str = "f32", devices=(0,)) -> None:
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
        devs = [int(x) for x in devices]
        if not devs:
            raise ValueError("devices must name at least one GPU")
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_void_p()
        check(L.vs_multi_create(int(d), code, DTYPE_CODES[dtype], len(devs), arr, ctypes.byref(h)))
        self._h = h
        self._L = L
        self.d = int(d)
        self.metric_type = code
        self.dtype = dtype
        self.devices = devs
        self._prune_copy = None  # (ntotal, FlatIndex on devices[0]) for hnsw_prune

    @property
    def ntotal(self) -> int:
        return int(self._L.vs_multi_ntotal(self._h))

    def shard_rows(self):
        return [int(self._L.vs_multi_shard_rows(self._h, g)) for g in range(len(self.devices))]

    def add(self, x) -> None:
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 2 or x.shape[1] != self.d:
            raise ValueError(f"add expects an (n, {self.d}) array, got {x.shape}")
        self._drop_prune_copy()
        check(self._L.vs_multi_add(self._h, _ptr(x), x.shape[0]))

    def search(self, q, k: int) -> Tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(q, dtype=np.float32)
        if q.ndim != 2 or q.shape[1] != self.d:
            raise ValueError(f"search expects an (nq, {self.d}) array, got {q.shape}")
        k = int(k)
        if k <= 0:
            raise _lib.VsError(_lib.VS_ERR_ARG, "k must be > 0")
        D = np.empty((q.shape[0], k), dtype=np.float32)
        I = np.empty((q.shape[0], k), dtype=np.int64)
        check(self._L.vs_multi_search(self._h, _ptr(q), q.shape[0], k, _ptr(D), _ptr(I)))
        return D, I

    def reconstruct_n(self, i0: int, n: int) -> np.ndarray:
        out = np.empty((int(n), self.d), dtype=np.float32)
        if n:
            check(self._L.vs_multi_reconstruct_n(self._h, int(i0), int(n), _ptr(out)))
        return out

    def reconstruct(self, i: int) -> np.ndarray:
        return self.reconstruct_n(int(i), 1)[0]

    def _one_device_copy(self) -> "FlatIndex":
        """A one-device copy of the rows on ``devices[0]`` for the HNSW kernels (they gather rows by
        id from one device's HBM).  Made once and kept until the rows change (a graph build calls
        the kernels several times per level)."""
        n = self.ntotal
        if self._prune_copy is None or self._prune_copy[0] != n:
            self._drop_prune_copy()
            tmp = FlatIndex(self.d, "ip" if self.metric_type == METRIC_IP else "l2", self.dtype, self.devices[0])
            try:
                tmp.reserve(n)
                for r0 in range(0, n, 65536):
                    tmp.add(self.reconstruct_n(r0, min(65536, n - r0)))
            except BaseException:
                tmp.close()
                raise
            self._prune_copy = (n, tmp)
        return self._prune_copy[1]

    def hnsw_prune(self, nodes, cand, W: int) -> np.ndarray:
        """:meth:`FlatIndex.hnsw_prune` on the one-device copy of the rows."""
        if len(nodes) == 0:
            return np.full((0, int(W)), -1, dtype=np.int32)
        return self._one_device_copy().hnsw_prune(nodes, cand, W)

    def hnsw_search(self, graph: dict, q: np.ndarray, k: int, ef: int) -> np.ndarray:
        """Ids (nq x k, -1 padded) of faiss's HNSW search over ``graph`` on the one-device copy of
        the rows (``hnsw.beam_search``: the insertion beam of a graph save)."""
        from .hnsw import HNSWGraph
        g = HNSWGraph(self._one_device_copy(), graph, ef)
        try:
            return g.search(q, k, ef)[1]
        finally:
            g.close()

    def _drop_prune_copy(self) -> None:
        pc, self._prune_copy = getattr(self, "_prune_copy", None), None
        if pc is not None:
            pc[1].close()

    def reset(self) -> None:
        self._drop_prune_copy()
        check(self._L.vs_multi_reset(self._h))

    def set_screen(self, screen: str) -> None:
        if screen not in FlatIndex.SCREENS:
            raise ValueError(f"unknown screen {screen!r}")
        check(self._L.vs_multi_set_screen(self._h, FlatIndex.SCREENS[screen]))

    def add_from_file(self, path: str, byte_offset: int, n: int) -> None:
        self._drop_prune_copy()
        check(self._L.vs_multi_add_from_file(self._h, os.fsencode(path), int(byte_offset), int(n)))

    def write_rows(self, path: str, byte_offset: int, i0: int, n: int) -> None:
        check(self._L.vs_multi_write_rows_to_file(self._h, os.fsencode(path), int(byte_offset), int(i0), int(n)))

    def close(self) -> None:
        self._drop_prune_copy()
        if self._h is not None and self._h.value:
            self._L.vs_multi_destroy(self._h)
        self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass
