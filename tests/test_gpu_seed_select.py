"""The screens' threshold seed (k_seed_select through vs_seed_select_device) against numpy: the
rank-th largest of each query's sampled maxima, as an ordered-fp32 key << 32, bit-exact."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
from photo_search_engine_amd import _lib  # noqa: E402


def _ord(x: np.ndarray) -> np.ndarray:
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000)


def _expected(m: np.ndarray, rank: int) -> np.ndarray:
    nq, M = m.shape
    if M < rank:
        return np.zeros(nq, dtype=np.uint64)
    o = np.sort(_ord(m), axis=1)[:, M - rank]
    neg_inf = _ord(np.array([-np.inf], dtype=np.float32))[0]
    return np.where(o == neg_inf, 0, o << 32).astype(np.uint64)


def _run(m: np.ndarray, rank: int) -> np.ndarray:
    L = _lib.load()
    dev = torch.device("cuda", 0)
    md = torch.from_numpy(np.ascontiguousarray(m, dtype=np.float32)).to(dev)
    out = torch.full((m.shape[0],), -1, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = L.vs_seed_select_device(0, ctypes.c_void_p(md.data_ptr()), m.shape[1], m.shape[0], rank,
                                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st))
    assert rc == 0, _lib.last_error()
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("M,rank", [(4096, 1), (4096, 1300), (4096, 4096), (1000, 37), (8192, 655),
                                    (256, 200), (5000, 4999)])
def test_seed_select_matches_sort(M, rank):
    rng = np.random.default_rng(M * 7 + rank)
    nq = 64
    # maxima of 16 Gaussian scores (one float exponent or two: the screens' real distribution),
    # a few wide-range rows, negative rows, and rows with heavy ties
    m = rng.standard_normal((nq, M, 16)).max(axis=2).astype(np.float32) * 0.03
    m[1] = rng.standard_normal(M).astype(np.float32) * 1e3
    m[2] = -np.abs(m[2]) - 1.0
    m[3] = np.float32(0.125)
    m[4] = np.round(m[4] * 50) / 50
    m[5, : M // 2] = -np.inf
    assert np.array_equal(_run(m, rank), _expected(m, rank))


@pytest.mark.gpu
def test_seed_select_fewer_values_than_rank():
    m = np.random.default_rng(1).standard_normal((8, 100)).astype(np.float32)
    assert np.array_equal(_run(m, 101), np.zeros(8, dtype=np.uint64))
    assert np.array_equal(_run(m, 100), _expected(m, 100))


@pytest.mark.gpu
def test_seed_select_all_minus_inf_gives_no_threshold():
    m = np.full((4, 512), -np.inf, dtype=np.float32)
    assert np.array_equal(_run(m, 10), np.zeros(4, dtype=np.uint64))
