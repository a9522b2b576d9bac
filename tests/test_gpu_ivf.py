"""IVF-Flat on the GPU (libvs vs_ivf_* through the C ABI) against oracle/ivf_oracle.py (MI355X only).

Bar: ids bit-exact and D = fp32 of the oracle's canonical fp64 score, on the same stored rows and
centroids.  Covers both metrics, f32/bf16/f16 storage, every scan query class (1/2/4/8 queries per
list item), lists spanning several scan items, coarse probing over the MFMA path (nq > 8, bf16),
nprobe = nlist (= exact flat search), k beyond the probed rows (-1 padding), exact duplicate rows
(ties -> lower id), incremental adds, reconstruct and k-means training.
"""
import numpy as np
import pytest

from oracle import ivf_oracle as IO
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def IVF():
    from photo_search_engine_amd.ivf import IVFFlatIndex
    return IVFFlatIndex


def _check(ix, x_st, c_st, q, k, nprobe, metric, ids=None):
    lists = IO.assign(x_st, c_st, metric)
    ids = np.arange(x_st.shape[0]) if ids is None else ids
    D, I = ix.search(q, k, nprobe)
    S, Ie = IO.search(x_st, ids, lists, c_st, q, k, nprobe, metric)
    np.testing.assert_array_equal(I, Ie)
    Dexp = S.astype(np.float32)
    Dexp[Ie < 0] = -3.4028235e38 if metric == "ip" else 3.4028235e38
    np.testing.assert_array_equal(D, Dexp)
    return D, I, lists


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_ivf_matches_oracle(IVF, metric, dtype):
    d, N, nlist, nq, k, nprobe = 64, 20000, 64, 40, 10, 8
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)  # = the stored values
    ix = IVF(d, nlist, metric, dtype)
    ix.set_centroids(IO.sample_centroids(x, nlist, 5))
    c = ix.centroids()
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    assert ix.ntotal == N
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    _, _, lists = _check(ix, x, c, q, k, nprobe, metric)
    np.testing.assert_array_equal(ix.list_sizes(), np.bincount(lists, minlength=nlist))
    np.testing.assert_array_equal(ix.assign(x[:500]), lists[:500])
    np.testing.assert_array_equal(ix.reconstruct(12345), x[12345])
    ix.close()


def test_ivf_query_classes_and_multi_item_lists(IVF):
    # few lists and many queries: lists are probed by 1..40 queries (every scan class, several
    # query groups per list) and hold > 16 pages (several page-range items per list)
    d, N, nlist = 48, 90000, 8
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    ix = IVF(d, nlist, "ip", "bf16")
    ix.set_centroids(IO.sample_centroids(x, nlist, 9))
    ix.add(x)
    assert (ix.list_sizes() > 16 * 256).any()
    for nq, nprobe in ((1, 1), (2, 2), (5, 3), (40, 2)):
        q = O.synth_rows(O.SEED_QUERIES, 100, nq, d, True, "f32")
        _check(ix, x, ix.centroids(), q, 25, nprobe, "ip")


def test_ivf_mfma_probe_batch(IVF):
    # nq > 8 with bf16 centroids: the coarse probe runs on the MFMA screen path
    d, N, nlist, nq = 128, 60000, 512, 300
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    ix = IVF(d, nlist, "ip", "bf16")
    ix.set_centroids(IO.sample_centroids(x, nlist, 3))
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    _check(ix, x, ix.centroids(), q, 20, 16, "ip")


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_ivf_nprobe_all_lists_is_flat_search(IVF, metric):
    d, N, nlist = 32, 7000, 16
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    ix = IVF(d, nlist, metric, "f32")
    ix.set_centroids(IO.sample_centroids(x, nlist, 1))
    ix.add(x)
    q = O.synth_rows(O.SEED_QUERIES, 0, 9, d, True, "f32")
    D, I = ix.search(q, 30, nlist)
    S, Ie = O.knn_exact(x, q, 30, metric)
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))


def test_ivf_padding_incremental_adds_and_ties(IVF):
    rng = np.random.default_rng(21)
    d, nlist = 16, 32
    base = rng.standard_normal((100, d)).astype(np.float32)
    base /= np.linalg.norm(base, axis=1, keepdims=True)  # unit rows: a row's best IP match is itself
    x = np.concatenate([base, np.repeat(base[3:4], 40, axis=0), base[:60]], axis=0)  # duplicates
    ix = IVF(d, nlist, "ip", "f32")
    c = IO.sample_centroids(base, nlist, 2)
    ix.set_centroids(c)
    for a, b in ((0, 50), (50, 120), (120, x.shape[0])):
        ix.add(x[a:b])
    assert ix.ntotal == x.shape[0]
    q = np.concatenate([base[3:4], base[:5]], axis=0)
    D, I, _ = _check(ix, x, ix.centroids(), q, 64, 1, "ip")  # k beyond one list's rows -> -1
    assert (I == -1).any()
    assert I[0, 0] == 3  # the earliest copy wins the tie
    np.testing.assert_array_equal(ix.reconstruct(130), x[130])


def test_ivf_empty_and_errors(IVF):
    from photo_search_engine_amd._lib import VsError
    ix = IVF(8, 4, "ip", "f32")
    with pytest.raises(VsError):
        ix.add(np.ones((2, 8), np.float32))  # untrained
    ix.set_centroids(np.eye(4, 8, dtype=np.float32))
    D, I = ix.search(np.ones((2, 8), np.float32), 3, 2)
    assert (I == -1).all() and (D == -3.4028235e38).all()
    ix.add(np.eye(8, dtype=np.float32))
    with pytest.raises(VsError):
        ix.set_centroids(np.eye(4, 8, dtype=np.float32))  # not empty
    ix.reset()
    assert ix.ntotal == 0 and ix.list_sizes().sum() == 0


def test_ivf_train_kmeans_then_exact(IVF):
    d, N, nlist = 32, 12000, 24
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    ix = IVF(d, nlist, "l2", "f32")
    ix.train(x, niter=4)
    c = ix.centroids()
    assert np.isfinite(c).all() and len({tuple(r) for r in c.tolist()}) == nlist
    ix.add(x)
    q = O.synth_rows(O.SEED_QUERIES, 0, 17, d, True, "f32")
    _check(ix, x, c, q, 12, 4, "l2")


@pytest.mark.parametrize("metric,dtype", [("ip", "bf16"), ("l2", "bf16"), ("ip", "f16")])
def test_ivf_mfma_list_scan_matches_oracle(IVF, metric, dtype):
    # lists probed by many queries scanned by the MFMA screen over their pages: 2 lists of ~100k
    # rows (~390 pages: > 1 page per workgroup, a partial last page), 300 queries probing both
    # (split query tiles of 128 + 128 + 44); identical to the oracle and to the GEMV scan, and no
    # query needs a re-search (the (hi, lo) query split keeps the screen near fp32 precision)
    d, N, nlist, nq, k = 64, 200_000, 2, 300, 10
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    ix = IVF(d, nlist, metric, dtype)
    ix.set_centroids(IO.sample_centroids(x, nlist, 4))
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    ix.set_scan("mfma")
    D, I, _ = _check(ix, x, ix.centroids(), q, k, 2, metric)
    assert ix.last_search_stats() == (6, 0)  # 2 lists x 3 query blocks, every query certified
    ix.set_scan("gemv")
    D2, I2 = ix.search(q, k, 2)
    assert ix.last_mfma_lists == 0
    np.testing.assert_array_equal(I2, I)
    np.testing.assert_array_equal(D2, D)
    ix.close()


def test_ivf_mfma_skewed_lists_mixed_scans(IVF):
    # Zipf-like list sizes: the head lists take the MFMA scan, the tail the GEMV items, in one
    # search; single queries (nql = 1) always stay on the GEMV scan
    rng = np.random.default_rng(5)
    d, nlist = 96, 24
    c = rng.standard_normal((nlist, d)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    w = 1.0 / np.arange(1, nlist + 1) ** 1.3
    cid = rng.choice(nlist, size=150_000, p=w / w.sum())
    x = c[cid] + 0.6 * rng.standard_normal((cid.size, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    ix = IVF(d, nlist, "ip", "bf16")
    ix.set_centroids(c)
    ix.add(x)
    x_st = O.round_dtype(x, "bf16")
    qc = rng.choice(nlist, size=120, p=w / w.sum())
    q = c[qc] + 0.6 * rng.standard_normal((qc.size, d)).astype(np.float32)
    ix.set_scan("mfma")
    _check(ix, x_st, ix.centroids(), q, 20, 3, "ip")
    assert ix.last_mfma_lists > 0
    _check(ix, x_st, ix.centroids(), q[:1], 20, 3, "ip")
    assert ix.last_mfma_lists == 0
    ix.close()


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_ivf_mfma_plain_query_tiles(IVF, metric):
    # the direct mapped form (padded dim a multiple of 128): plain query tiles (256 queries a tile,
    # lists probed by <= 64 queries on the narrow 64-column form) and split (hi, lo) tiles (128 a
    # tile, narrow up to 32) return the same exact answer as the oracle; 300 queries probing both
    # lists: 2 x 2 plain tiles vs 2 x 3 split tiles; 50 queries: the narrow plain form
    d, N, nlist, k = 256, 60_000, 2, 10
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    ix = IVF(d, nlist, metric, "bf16")
    ix.set_centroids(IO.sample_centroids(x, nlist, 4))
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 300, d, True, "f32")
    ix.set_scan("mfma")
    out = {}
    for mode, nq, scans in (("plain", 300, 4), ("split", 300, 6), ("plain", 50, 2), ("split", 50, 2)):
        ix.set_query_tiles(mode)
        D, I, _ = _check(ix, x, ix.centroids(), q[:nq], k, 2, metric)
        assert ix.last_search_stats()[0] == scans
        out[(mode, nq)] = (D, I)
    for nq in (300, 50):
        np.testing.assert_array_equal(out[("plain", nq)][1], out[("split", nq)][1])
        np.testing.assert_array_equal(out[("plain", nq)][0], out[("split", nq)][0])
    with pytest.raises(ValueError):
        ix.set_query_tiles("hi-lo")
    ix.close()


def test_ivf_plain_query_tiles_tight_clusters_researched(IVF):
    # rows within ~1e-3 of their centroid: the 10th and 32nd best scores of a query differ by less
    # than the plain tile's query-rounding margin (~2^-9 ||q|| ||x||), so the first pass leaves
    # queries uncertified; their re-search packs split tiles (margin ~2^-17) and certifies them --
    # the answer is the oracle's either way
    rng = np.random.default_rng(11)
    d, nlist, N, nq, k = 256, 4, 40_000, 96, 10
    c = rng.standard_normal((nlist, d)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    cid = rng.integers(0, nlist, N)
    x = c[cid] + 1e-3 * rng.standard_normal((N, d)).astype(np.float32)
    ix = IVF(d, nlist, "ip", "bf16")
    ix.set_centroids(c)
    ix.add(x)
    x_st = O.round_dtype(x, "bf16")
    q = c[rng.integers(0, nlist, nq)] + 0.05 * rng.standard_normal((nq, d)).astype(np.float32)
    ix.set_scan("mfma")
    ix.set_query_tiles("plain")
    D, I, _ = _check(ix, x_st, ix.centroids(), q, k, 2, "ip")
    assert ix.last_search_stats()[1] > 0  # re-searched on split tiles
    ix.set_query_tiles("split")
    D2, I2, _ = _check(ix, x_st, ix.centroids(), q, k, 2, "ip")
    assert ix.last_search_stats()[1] == 0
    np.testing.assert_array_equal(I2, I)
    np.testing.assert_array_equal(D2, D)
    ix.close()
