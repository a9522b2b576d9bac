"""The int8 pre-screen (``FlatIndex.set_screen("int8")``, include/vs.h VS_SCREEN_I8) on the GPU.

The screen streams an int8 copy of the rows (per-row scale) and keeps every row whose proven
upper bound can still reach the k-th best; the exact refine scores them, so results must be the
SAME ids and canonical scores as the native path and as ``oracle.knn_exact`` on the stored
values -- bit-exact, for every storage dtype.  Cases: unseeded small corpora and seeded ones
(>= 4 tiles per CU), d not a multiple of 64, partial tiles, k near the int8 limit, exact
duplicates (ties -> lower id), zero rows, incremental adds after switching, an adversarial corpus
whose seed sample lies (certificate rejects, native re-search), and the argument errors.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def FlatIndex():
    # the screen kernels under test: single-query calls on small corpora would otherwise take the
    # exact full scan (vs_set_scan_limit), which tests/test_gpu_parity.py covers on its own
    from photo_search_engine_amd.index import FlatIndex as FI

    class Screened(FI):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            self.set_scan_limit(0)
    return Screened


def _num_cu():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


def _exact(ix, q, k, metric="ip"):
    x = ix.reconstruct_n(0, ix.ntotal)
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(x, q, k, metric)
    np.testing.assert_array_equal(I, Ie)
    Dexp = S.astype(np.float32)
    Dexp[Ie < 0] = -3.4028235e38 if metric == "ip" else 3.4028235e38
    np.testing.assert_array_equal(D, Dexp)
    return D, I


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("nq,k,N,d", [(40, 10, 9000, 128), (256, 100, 20000, 192), (300, 7, 3001, 72),
                                     (64, 1000, 150000, 96), (17, 1, 5000, 40)])
def test_int8_screen_exact(FlatIndex, dtype, nq, k, N, d):
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    ix.set_screen("int8")
    assert ix.screen == "int8"
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    _exact(ix, q, k)
    assert ix.uncertified_count() == 0
    ix.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("nq,k,N,d", [(40, 10, 9000, 512), (256, 100, 20000, 768), (300, 7, 3001, 1024),
                                     (64, 1000, 150000, 512), (17, 1, 5000, 512), (200, 50, 70000, 1536)])
def test_int8_direct_screen_exact(FlatIndex, dtype, nq, k, N, d):
    """d a multiple of 256 (K-steps per tile a multiple of 4): the main pass is the direct form
    k_screen_i8d (corpus fragments straight to registers).  Unseeded and seeded corpora, a partial
    last tile, k = 1000 (candidate compaction in the K loop), two query blocks."""
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS + 5, 0, N, True)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES + 5, 0, nq, d, True, "f32")
    _exact(ix, q, k)
    assert ix.uncertified_count() == 0
    ix.close()


@pytest.mark.parametrize("k", [10, 100])
def test_int8_screen_seeded_matches_native(FlatIndex, k):
    # >= 4 tiles per CU: the int8 seed pass, optimistic union and adaptive refine depth
    N, d, nq = 256 * 4 * _num_cu() + 777, 1536, 64
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    Dn, In = ix.search(q, k)
    ix.set_screen("int8")
    D8, I8 = _exact(ix, q, k)
    np.testing.assert_array_equal(I8, In)
    np.testing.assert_array_equal(D8, Dn)
    assert ix.uncertified_count() == 0
    ix.close()


@pytest.mark.parametrize("d", [64, 512])
def test_int8_screen_ties_zero_rows_and_incremental_adds(FlatIndex, d):
    rng = np.random.default_rng(5)
    base = rng.standard_normal((60, d)).astype(np.float32)
    x = np.concatenate([base, np.repeat(base[7:8], 300, axis=0), np.zeros((40, d), np.float32), base], axis=0)
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x[:100])
    ix.set_screen("int8")
    ix.add(x[100:])  # the int8 copy follows later adds
    q = np.concatenate([np.repeat(base[7:8], 12, axis=0), -base[:8]], axis=0)
    D, I = _exact(ix, O.round_dtype(q, "bf16"), 40)
    assert I[0, 0] == 7  # the earliest copy wins the tie
    ix.set_screen("native")
    assert ix.screen == "native"
    _exact(ix, O.round_dtype(q, "bf16"), 40)
    ix.close()


def test_int8_screen_adversarial_seed_falls_back_exactly(FlatIndex):
    # near-copies of the queries only in the sampled tiles (each workgroup's first): 4 per tile, 64
    # per query, more than the int8 seed rank (ceil(1024 * sampled / N) = 32 here), so the seeded
    # threshold sits among them and too few rows are listed; the certificate rejects and the native
    # path re-searches exactly
    d, k = 64, 10
    cu = _num_cu()
    tiles = 32 * cu + 3
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 16, d, True, "f32")
    rng = np.random.default_rng(11)
    for j in range(cu):
        for t in range(4):
            x[(tiles * j // cu) * 256 + 5 + t] = q[(4 * j + t) % 16] + 0.01 * rng.standard_normal(d).astype(np.float32)
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    ix.set_screen("int8")
    _exact(ix, O.round_dtype(q, "bf16"), k)
    assert ix.uncertified_count() > 0


def test_int8_screen_device_api_with_offset(FlatIndex):
    import torch
    N, d, nq, k = 120_000, 256, 48, 25
    ix = FlatIndex(d, "ip", "f16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    qd = torch.from_numpy(q).cuda()
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    ix.search_device_exact(qd.data_ptr(), nq, k, None, I.data_ptr(), S.data_ptr(), 1000, 0)
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, N), q, k, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie + 1000)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)


def test_int8_screen_argument_errors(FlatIndex):
    with pytest.raises(ValueError):
        FlatIndex(32, "ip", "bf16").set_screen("fp4")


# ---- L2 indexes: keys 2 (upper bound of <x, q>) - ||x||^2 in the int8 screens, the canonical
# distance in the refine; same ids and distances as the native path and knn_exact ----

def _l2_rows(N, d, seed, unit):
    x = O.synth_rows(O.SEED_CORPUS + seed, 0, N, d, True, "f32")
    if not unit:  # row norms spread over [0.25, 4): ||x||^2 decides as much as the angle
        rng = np.random.default_rng(seed)
        x *= rng.uniform(0.25, 4.0, size=(N, 1)).astype(np.float32)
    return x


@pytest.mark.parametrize("unit", [True, False])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("nq,k,N,d", [(40, 10, 9000, 128), (256, 100, 20000, 192), (300, 7, 3001, 72),
                                     (200, 50, 70000, 1536), (64, 1000, 150000, 512)])
def test_int8_screen_l2_exact(FlatIndex, dtype, unit, nq, k, N, d):
    """Both K1 forms (tiled: d % 256 != 0; direct k_screen_i8d: d % 256 == 0), unseeded and seeded
    corpora, partial tiles, k = 1000, unit and spread row norms."""
    x = _l2_rows(N, d, 21, unit)
    ix = FlatIndex(d, "l2", dtype)
    ix.add(x)
    ix.set_screen("int8")
    assert ix.screen == "int8"
    q = O.synth_rows(O.SEED_QUERIES + 21, 0, nq, d, True, "f32") * (1.0 if unit else 1.7)
    _exact(ix, q.astype(np.float32), k, "l2")
    assert ix.uncertified_count() == 0
    ix.close()


@pytest.mark.parametrize("k", [10, 100])
@pytest.mark.parametrize("d", [1536, 320])
def test_int8_screen_l2_seeded_matches_native(FlatIndex, k, d):
    # >= 4 tiles per CU: the int8 seed pass and union target on L2 keys
    N, nq = 256 * 4 * _num_cu() + 777, 64
    ix = FlatIndex(d, "l2", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    Dn, In = ix.search(q, k)
    ix.set_screen("int8")
    ix.set_timing(True)
    D8, I8 = _exact(ix, q, k, "l2")
    ix.set_timing(False)
    assert ix.timing_fetch()[1] == "mfma_i8"
    np.testing.assert_array_equal(I8, In)
    np.testing.assert_array_equal(D8, Dn)
    assert ix.uncertified_count() == 0
    ix.close()


@pytest.mark.parametrize("d", [64, 512])
def test_int8_screen_l2_ties_zero_rows_and_adds(FlatIndex, d):
    rng = np.random.default_rng(7)
    base = rng.standard_normal((60, d)).astype(np.float32)
    x = np.concatenate([base, np.repeat(base[7:8], 300, axis=0), np.zeros((40, d), np.float32), base], axis=0)
    ix = FlatIndex(d, "l2", "bf16")
    ix.add(x[:100])
    ix.set_screen("int8")
    ix.add(x[100:])
    q = np.concatenate([np.repeat(base[7:8], 12, axis=0), -base[:8], np.zeros((4, d), np.float32)], axis=0)
    D, I = _exact(ix, O.round_dtype(q, "bf16"), 40, "l2")
    assert I[0, 0] == 7 and D[0, 0] == 0.0  # the earliest copy wins the tie
    ix.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("nq,k", [(1, 1), (1, 10), (3, 37), (8, 100)])
def test_int8_gemv_screen_l2_exact(FlatIndex, dtype, nq, k):
    N, d = 120_000, 200
    x = _l2_rows(N, d, 5, False)
    ix = FlatIndex(d, "l2", dtype)
    ix.add(x)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES, 40 + nq, nq, d, True, "f32")
    ix.set_timing(True)
    _exact(ix, q, k, "l2")
    ix.set_timing(False)
    assert ix.timing_fetch()[1] in ("gemv_i8", "gemv")
    assert ix.uncertified_count() == 0
    ix.close()


def test_int8_screen_l2_adversarial_seed_falls_back_exactly(FlatIndex):
    d, k = 64, 10
    cu = _num_cu()
    tiles = 32 * cu + 3
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 16, d, True, "f32")
    rng = np.random.default_rng(11)
    for j in range(cu):
        for t in range(4):
            x[(tiles * j // cu) * 256 + 5 + t] = q[(4 * j + t) % 16] + 0.01 * rng.standard_normal(d).astype(np.float32)
    ix = FlatIndex(d, "l2", "bf16")
    ix.add(x)
    ix.set_screen("int8")
    _exact(ix, O.round_dtype(q, "bf16"), k, "l2")
    assert ix.uncertified_count() > 0


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("nq,k", [(1, 1), (1, 10), (1, 500), (3, 37), (8, 100)])
def test_int8_gemv_screen_exact(FlatIndex, dtype, nq, k):
    # few queries (the product's single-query call): the GEMV streams the int8 copy with the fp32
    # query (k <= 128); ids and scores bit-exact, and the timed screen is the int8 GEMV
    N, d = 120_000, 200
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES, 40 + nq, nq, d, True, "f32")
    ix.set_timing(True)
    _exact(ix, q, k)
    ix.set_timing(False)
    assert ix.timing_fetch()[1] == ("gemv_i8" if k <= 128 else "gemv")  # deep single queries: native
    assert ix.uncertified_count() == 0
    ix.close()


def test_int8_gemv_cfg2_shape_matches_native(FlatIndex):
    # BASELINE cfg2 (N=1M d=1536 fp32, batch 1, top-10) through the int8 GEMV screen
    N, d = 1_000_000, 1536
    ix = FlatIndex(d, "ip", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    qs = [O.synth_rows(O.SEED_QUERIES, i, 1, d, True, "f32") for i in range(4)]
    native = [ix.search(q, 10) for q in qs]
    ix.set_screen("int8")
    x = ix.reconstruct_n(0, N)
    for q, (Dn, In) in zip(qs, native):
        D, I = ix.search(q, 10)
        S, Ie = O.knn_exact(x, q, 10, "ip")
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(I, In)
        np.testing.assert_array_equal(D, Dn)
    assert ix.uncertified_count() == 0
    ix.close()


def test_int8_screen_copy_bytes(FlatIndex):
    # vs_screen_copy_bytes: 0 on the native screen; with the int8 screen at least the codes and the
    # per-row (scale | error norm) word of every row (allocated capacity, tiles of 256 rows); back to
    # 0 when the screen is switched off again; grows with incremental adds
    N, d = 5000, 200
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    assert ix.screen_copy_bytes() == 0
    ix.set_screen("int8")
    b = ix.screen_copy_bytes()
    assert b >= N * (d + 4)
    assert b % 4 == 0
    ix.add_synthetic(O.SEED_CORPUS, N, 4 * N, True)
    b2 = ix.screen_copy_bytes()
    assert b2 >= 5 * N * (d + 4) and b2 >= b
    q = O.synth_rows(O.SEED_QUERIES, 3, 40, d, True, "f32")
    _exact(ix, q, 17)
    ix.set_screen("native")
    assert ix.screen_copy_bytes() == 0
