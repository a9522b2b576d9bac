"""The int8 pre-screen on non-isotropic data: clustered rows in random and in
cluster-sorted insertion order, tight and loose clusters, and the reference's own 77 x 4096 photo
vectors.  The screen's seed is a sample (each workgroup's first tile): on sorted clusters it is
biased, so the certificate may reject queries -- they are re-searched -- but the answer must stay
bit-exact against ``oracle.knn_exact`` and identical to the native screen's."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from photo_search_engine_amd import faiss_format

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _mixture(n, d, n_clusters, sigma, seed, sort):
    """normalise(c[cid] + sigma * g): the bench's cfg5 data model (bench.py `_mixture_rows`) on the
    host; `sort` inserts the rows cluster by cluster (a corpus indexed folder by folder)."""
    c = O.synth_rows(O.SEED_CORPUS + 900, 0, n_clusters, d, True)
    g = O.synth_rows(seed, 0, n, d, True)
    cid = np.random.default_rng(seed).integers(0, n_clusters, n)
    if sort:
        cid = np.sort(cid)
    x = c[cid] + np.float32(sigma) * g
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("sigma,sort", [(1.0, False), (1.0, True), (0.3, False), (0.3, True)])
@pytest.mark.parametrize("k", [10, 100])
def test_int8_screen_clustered_rows_exact(sigma, sort, k):
    from photo_search_engine_amd.index import FlatIndex

    N, d, nq, C = 300_000, 1536, 64, 64  # 1172 tiles: the seeded int8 path (>= 4 tiles per CU)
    x = _mixture(N, d, C, sigma, O.SEED_CORPUS + 71, sort)
    q = _mixture(nq, d, C, sigma, O.SEED_QUERIES + 71, False)
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    Dn, In = ix.search(q, k)
    ix.set_screen("int8")
    xs = ix.reconstruct_n(0, N)
    S, Ie = O.knn_exact(xs, q, k, "ip")
    # the first int8 batch may fail its certificates on dense clusters (re-searched exactly); its
    # failure count, read back behind it, routes the following batches to the native screen, whose
    # failing batches deepen its seed (include/vs.h "screen health")
    for rep in range(6):
        u0 = ix.uncertified_count()
        D8, I8 = ix.search(q, k)
        np.testing.assert_array_equal(I8, Ie)
        np.testing.assert_array_equal(D8, S.astype(np.float32))
        np.testing.assert_array_equal(I8, In)
        np.testing.assert_array_equal(D8, Dn)
        if rep == 5:  # by then the index has adapted: re-searches are rare
            assert ix.uncertified_count() - u0 <= nq // 8
    ix.close()


def test_int8_screen_reference_photo_vectors():
    """The reference's own index (77 real 4096-d photo embeddings, tests/golden): every row as a
    query, int8 screen == native == oracle."""
    from photo_search_engine_amd.index import FlatIndex

    x = np.ascontiguousarray(faiss_format.read_index(os.path.join(GOLDEN, "ref_photo_search.index")).vectors,
                             dtype=np.float32)
    assert x.shape == (77, 4096)
    for dtype in ("f32", "bf16"):
        ix = FlatIndex(4096, "ip", dtype)
        ix.add(x)
        Dn, In = ix.search(x, 10)
        ix.set_screen("int8")
        D8, I8 = ix.search(x, 10)
        S, Ie = O.knn_exact(ix.reconstruct_n(0, 77), x, 10, "ip")
        np.testing.assert_array_equal(I8, Ie)
        np.testing.assert_array_equal(D8, S.astype(np.float32))
        np.testing.assert_array_equal(I8, In)
        if dtype == "f32":
            assert (I8[:, 0] == np.arange(77)).all()  # every (unit) photo vector finds itself first
        ix.close()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_int8_group_residuals_incremental_adds(dtype):
    """Cluster-sorted rows with the int8 screen switched on first and rows added in chunks that end
    mid-group: each add re-derives the means of the groups it touches and re-quantises their rows
    against them (group residuals).  Batches through the seeded direct pass add
    <mu_g, q> to every key; smaller batches and shards without that pass take the native screen.
    Every answer bit-exact against the oracle; the sorted clusters certify (no collapse)."""
    from photo_search_engine_amd.index import FlatIndex

    N, d, C = 300_000, 512, 32
    x = _mixture(N, d, C, 0.3, O.SEED_CORPUS + 81, True)
    q = _mixture(96, d, C, 0.3, O.SEED_QUERIES + 81, False)
    ix = FlatIndex(d, "ip", dtype)
    ix.set_screen("int8")
    for a in range(0, N, 70_001):
        ix.add(x[a:a + 70_001])
    xs = ix.reconstruct_n(0, N)
    for nq, k in ((96, 50), (64, 10), (4, 10), (1, 100)):
        S, Ie = O.knn_exact(xs, q[:nq], k, "ip")
        for _ in range(3):
            D, I = ix.search(q[:nq], k)
            np.testing.assert_array_equal(I, Ie)
            np.testing.assert_array_equal(D, S.astype(np.float32))
    u0 = ix.uncertified_count()
    for _ in range(4):
        ix.search(q, 50)
    assert ix.uncertified_count() - u0 <= 96 // 16  # group residuals keep the int8 screen certifying
    st = ix.screen_state()
    assert st["screen"] == 1 and st["group_residuals"] == 1 and st["groups_with_mean"] >= N // 4096 - 1
    assert 0.0 < st["max_mean_norm"] <= 1.0 and st["i8_routed_searches"] == 0
    ix.close()
