"""ctypes binding of libvs.so (include/vs.h).

The library is the product path: if it is missing or cannot be loaded this module raises, loudly.
There is no CPU fallback anywhere in ``photo_search_engine_amd``.
"""
from __future__ import annotations

import ctypes
from typing import Optional
import os
import re
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvs.so")  # the in-tree build (python -m photo_search_engine_amd.build)
HEADER_PATH = os.path.join(HERE, "..", "include", "vs.h")

METRIC_IP = 0
METRIC_L2 = 1
DTYPE_F32 = 0
DTYPE_BF16 = 1
DTYPE_F16 = 2
DTYPE_CODES = {"f32": DTYPE_F32, "fp32": DTYPE_F32, "float32": DTYPE_F32,
               "bf16": DTYPE_BF16, "bfloat16": DTYPE_BF16,
               "f16": DTYPE_F16, "fp16": DTYPE_F16, "float16": DTYPE_F16}

VS_OK = 0
VS_ERR_ARG = -1
VS_ERR_DEVICE = -2
VS_ERR_OOM = -3
VS_ERR_UNCERTIFIED = -4
VS_ERR_INTERNAL = -5


class VsError(RuntimeError):
    """A libvs call failed (device, allocation, argument or certification error)."""

    def __init__(self, code: int, message: str) -> None:
        super().__init__(f"libvs error {code}: {message}")
        self.code = code


_lock = threading.Lock()
_lib = None

_c_i64 = ctypes.c_int64
_vp = ctypes.c_void_p
_SIGS = {
    # name: (restype, argtypes)
    "vs_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "vs_destroy": (None, [_vp]),
    "vs_reset": (ctypes.c_int, [_vp]),
    "vs_add": (ctypes.c_int, [_vp, _vp, _c_i64]),
    "vs_add_device": (ctypes.c_int, [_vp, _vp, _c_i64, _vp]),
    "vs_add_synthetic": (ctypes.c_int, [_vp, ctypes.c_uint64, _c_i64, _c_i64, ctypes.c_int]),
    "vs_reserve": (ctypes.c_int, [_vp, _c_i64]),
    "vs_capacity": (_c_i64, [_vp]),
    "vs_synthesize": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, _c_i64, _c_i64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, _vp, _vp]),
    "vs_search": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, _vp, _vp]),
    "vs_search_device": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, _vp, _vp, _vp, _c_i64, _vp]),
    "vs_search_device_exact": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, _vp, _vp, _vp, _c_i64, _vp]),
    "vs_two_phase_ok": (ctypes.c_int, [_vp, _c_i64, ctypes.c_int32]),
    "vs_search_device_phase_a": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, _c_i64, _vp, _vp,
                                                ctypes.c_int32, _vp, ctypes.POINTER(ctypes.c_void_p)]),
    "vs_search_device_phase_b": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_int32, _vp]),
    "vs_search_pending_free": (None, [_vp]),
    "vs_merge_shards_device": (ctypes.c_int, [ctypes.c_int, _vp, _vp, ctypes.c_int32, ctypes.c_int, _c_i64,
                                              ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "vs_seed_select_device": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int32, _c_i64, ctypes.c_int32, _vp, _vp]),
    "vs_add_from_file": (ctypes.c_int, [_vp, ctypes.c_char_p, _c_i64, _c_i64]),
    "vs_write_rows_to_file": (ctypes.c_int, [_vp, ctypes.c_char_p, _c_i64, _c_i64, _c_i64]),
    "vs_reconstruct": (ctypes.c_int, [_vp, _c_i64, _vp]),
    "vs_reconstruct_n": (ctypes.c_int, [_vp, _c_i64, _c_i64, _vp]),
    "vs_ntotal": (_c_i64, [_vp]),
    "vs_dim": (ctypes.c_int, [_vp]),
    "vs_metric": (ctypes.c_int, [_vp]),
    "vs_dtype": (ctypes.c_int, [_vp]),
    "vs_device": (ctypes.c_int, [_vp]),
    "vs_last_error": (ctypes.c_char_p, []),
    "vs_version": (ctypes.c_char_p, []),
    "vs_set_screen": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_screen": (ctypes.c_int, [_vp]),
    "vs_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_timing_fetch": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "vs_uncertified_count": (_c_i64, [_vp]),
    "vs_full_scan_count": (_c_i64, [_vp]),
    "vs_set_scan_limit": (ctypes.c_int, [_vp, _c_i64]),
    "vs_screen_probe": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "vs_k1_probe": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   _vp, _vp, _vp, _vp]),
    "vs_set_k1_schedule": (ctypes.c_int, [ctypes.c_int32]),
    "vs_k1_schedule": (ctypes.c_int, []),
    "vs_host_staging_bytes": (_c_i64, [_vp]),
    "vs_screen_copy_bytes": (_c_i64, [_vp]),
    "vs_screen_state": (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    # multi-device flat index
    "vs_multi_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                       ctypes.POINTER(_vp)]),
    "vs_multi_destroy": (None, [_vp]),
    "vs_multi_add": (ctypes.c_int, [_vp, _vp, _c_i64]),
    "vs_multi_add_from_file": (ctypes.c_int, [_vp, ctypes.c_char_p, _c_i64, _c_i64]),
    "vs_multi_write_rows_to_file": (ctypes.c_int, [_vp, ctypes.c_char_p, _c_i64, _c_i64, _c_i64]),
    "vs_multi_search": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, _vp, _vp]),
    "vs_multi_reconstruct_n": (ctypes.c_int, [_vp, _c_i64, _c_i64, _vp]),
    "vs_multi_reset": (ctypes.c_int, [_vp]),
    "vs_multi_set_screen": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_multi_ntotal": (_c_i64, [_vp]),
    "vs_multi_ndev": (ctypes.c_int, [_vp]),
    "vs_multi_shard_rows": (_c_i64, [_vp, ctypes.c_int]),
    # IVF-Flat
    "vs_ivf_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_vp)]),
    "vs_ivf_destroy": (None, [_vp]),
    "vs_ivf_set_centroids": (ctypes.c_int, [_vp, _vp]),
    "vs_ivf_get_centroids": (ctypes.c_int, [_vp, _vp]),
    "vs_ivf_is_trained": (ctypes.c_int, [_vp]),
    "vs_ivf_assign": (ctypes.c_int, [_vp, _vp, _c_i64, _vp]),
    "vs_ivf_add": (ctypes.c_int, [_vp, _vp, _c_i64]),
    "vs_ivf_add_device": (ctypes.c_int, [_vp, _vp, _c_i64, _vp]),
    "vs_ivf_add_synthetic": (ctypes.c_int, [_vp, ctypes.c_uint64, _c_i64, _c_i64, ctypes.c_int]),
    "vs_ivf_reserve": (ctypes.c_int, [_vp, _c_i64]),
    "vs_ivf_search": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "vs_ivf_search_device": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "vs_ivf_reconstruct": (ctypes.c_int, [_vp, _c_i64, _vp]),
    "vs_ivf_list_sizes": (ctypes.c_int, [_vp, _vp]),
    "vs_ivf_reset": (ctypes.c_int, [_vp]),
    "vs_ivf_ntotal": (_c_i64, [_vp]),
    "vs_ivf_nlist": (ctypes.c_int, [_vp]),
    "vs_ivf_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_ivf_timing_fetch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int]),
    "vs_ivf_set_scan": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_ivf_set_query_tiles": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vs_ivf_last_search_stats": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    # HNSW graph search
    "vs_hnsw_create": (ctypes.c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.POINTER(_vp)]),
    "vs_hnsw_destroy": (None, [_vp]),
    "vs_hnsw_search": (ctypes.c_int, [_vp, _vp, _c_i64, ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    "vs_hnsw_ntotal": (_c_i64, [_vp]),
    "vs_hnsw_patch": (ctypes.c_int, [_vp, _c_i64, _vp, _vp, ctypes.c_int32, ctypes.c_int32]),
    "vs_hnsw_prune": (ctypes.c_int, [_vp, _c_i64, _vp, _vp, ctypes.c_int32, ctypes.c_int32, _vp]),
}


def header_functions(path: str = HEADER_PATH):
    """Names of every function include/vs.h declares (used by the symbol-export test)."""
    text = open(path, encoding="utf-8").read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vs_[a-z0-9_]+)\s*\(", text)))


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libvs.so and bind every entry point; raises if the library is absent.  (VS_LIB_PATH:
    another build of the same library, for A/B measurements.)"""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = path or os.environ.get("VS_LIB_PATH") or LIB_PATH
        # One HIP runtime per process: torch wheels bundle their own libamdhip64.so.7 /
        # libhsa-runtime64.so.1.  If torch is importable, load it first so libvs binds to the
        # SAME runtime (same SONAME) instead of /opt/rocm's copy; two HSA runtimes in one process
        # leave the second one without devices.  VS_NO_TORCH=1 skips this (pure C-ABI users).
        if os.environ.get("VS_NO_TORCH", "0") != "1" and "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(path):
            raise ImportError(
                f"libvs.so not found at {path}: the HIP library is the only implementation of this path; "
                "build it with `python -m photo_search_engine_amd.build` (hipcc, gfx950)")
        L = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            if path != LIB_PATH and not hasattr(L, name):
                continue  # (an A/B build from before an entry point was added)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L


def last_error() -> str:
    msg = load().vs_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int) -> int:
    if rc < 0:
        raise VsError(rc, last_error())
    return rc
