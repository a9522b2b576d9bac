"""The int8 direct main pass (k_screen_i8d, inner product, d a multiple of 256) behind its seed
pass (>= 4 tiles per workgroup: one sample tile per workgroup, 16-row-group maxima, the rank-r
maximum per query as the starting threshold).  Results must be bit-exact against
``oracle.knn_exact`` on the stored values whatever the seed does: a seed that lies only fails the
certificate (the device fallback round re-searches), it never changes an answer.

Cases: every storage dtype, k 1 / 10 / 100 / 1000, one and two query blocks, a partial last
tile, near-copies of the queries planted in exactly the sampled tiles (the selected seed sits
among them), a sampled tile holding a query's whole top-k, exact duplicates across the corpus
(ties -> lower id), the device API with an id offset, and the two-phase sharded step's phase A / B.
(Round 4 also ran these cases against a form that seeded inside the main pass; it measured slower
and was removed, profiles/r04_seed_ab.txt.)
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


def _exact(ix, q, k):
    x = ix.reconstruct_n(0, ix.ntotal)
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(x, q, k, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    return D, I


def _sample_tiles(tiles, G):
    """The seed pass's tiles (vs_api.hip search_block_i8): workgroup b of min(G, 512) screens tile
    b * (tiles // that)."""
    g = min(G, 512)
    return [b * (tiles // g) for b in range(g)]


@pytest.mark.parametrize("dtype,d,nq,k,tpc", [
    ("bf16", 512, 256, 10, 4.5),
    ("f16", 512, 64, 100, 5.25),
    ("f32", 768, 100, 1, 4.0),
    ("bf16", 1536, 256, 100, 4.8),
    ("bf16", 512, 300, 25, 6.1),   # two query blocks (256 + 44)
    ("bf16", 512, 32, 1000, 4.2),  # deep screens: compaction inside the K loop
])
def test_direct_direct_exact(FlatIndex, dtype, d, nq, k, tpc):
    G = _num_cu()
    N = int(256 * G * tpc) + 77  # a partial last tile
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS + 9, 0, N, True)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES + 9, 0, nq, d, True, "f32")
    _exact(ix, q, k)
    assert ix.uncertified_count() == 0
    assert ix.full_scan_count() == 0
    st = ix.screen_state()  # isotropic rows: no group has a mean worth coding against
    assert st["group_residuals"] == 0 and st["groups_with_mean"] == 0 and st["i8_union_log2"] == 0
    ix.close()


def test_direct_native_and_int8_identical_at_cfg3_width(FlatIndex):
    G = _num_cu()
    N, d, nq, k = 256 * G * 5 + 1, 1536, 128, 100
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    Dn, In = ix.search(q, k)
    ix.set_screen("int8")
    for _ in range(3):  # repeated launches: the counters and thresholds are per launch
        D8, I8 = ix.search(q, k)
        np.testing.assert_array_equal(I8, In)
        np.testing.assert_array_equal(D8, Dn)
    assert ix.uncertified_count() == 0
    ix.close()


def test_direct_planted_sample_tiles_exact(FlatIndex):
    # near-copies of 16 queries in exactly the sample tiles (4 rows per tile, ~64 per query, in one
    # 16-row group each): the selected seed lands among them, far above the rest of the corpus, so
    # the main pass lists almost nothing but the planted rows -- still enough for the certificate
    # (a seed is a group maximum of real rows: it never exceeds the k-th score by more than its
    # key slack), and the answer is the planted rows, exactly
    G = _num_cu()
    d, k, nq = 512, 10, 16
    tiles = 6 * G + 5
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    rng = np.random.default_rng(17)
    for j, t in enumerate(_sample_tiles(tiles, G)):
        for r in range(4):
            x[t * 256 + 3 + r] = q[(4 * j + r) % nq] + 0.01 * rng.standard_normal(d).astype(np.float32)
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    ix.set_screen("int8")
    qb = O.round_dtype(q, "bf16")
    _, I = _exact(ix, np.concatenate([qb, qb]), k)  # 32 queries: the MFMA path
    planted = {t * 256 + 3 + r for t in _sample_tiles(tiles, G) for r in range(4)}
    assert all(int(i) in planted for i in I.ravel())
    assert ix.full_scan_count() == 0
    ix.close()


def test_direct_sample_tile_holding_the_top_k(FlatIndex):
    # one sampled tile holds 200 near-copies of query 0 spread over all 16 of its groups: the
    # seed sits among them (the sample is not representative of the corpus), and the answer must
    # stay exact (a lying seed fails the certificate; the fallback round re-searches)
    G = _num_cu()
    d, k, nq = 512, 100, 24
    tiles = 5 * G + 1
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS + 1, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES + 1, 0, nq, d, True, "f32")
    t = _sample_tiles(tiles, G)[G // 3]
    rng = np.random.default_rng(5)
    x[t * 256:t * 256 + 200] = q[0] + 0.05 * rng.standard_normal((200, d)).astype(np.float32)
    ix = FlatIndex(d, "ip", "f16")
    ix.add(x)
    ix.set_screen("int8")
    _exact(ix, q, k)
    assert ix.full_scan_count() == 0
    ix.close()


def test_direct_exact_duplicates_tie_to_lower_id(FlatIndex):
    G = _num_cu()
    d, k, nq = 512, 20, 40
    N = 256 * G * 4 + 300
    x = O.synth_rows(O.SEED_CORPUS + 2, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES + 2, 0, nq, d, True, "f32")
    # each query's best-matching row copied 12 times across the corpus (exact score ties)
    S, I = O.knn_exact(O.round_dtype(x, "bf16"), O.round_dtype(q, "bf16"), 1, "ip")
    rng = np.random.default_rng(3)
    for qi in range(nq):
        for pos in rng.choice(N, 12, replace=False):
            x[pos] = x[I[qi, 0]]
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    ix.set_screen("int8")
    _exact(ix, O.round_dtype(q, "bf16"), k)
    ix.close()


def test_direct_device_api_with_offset_and_phases(FlatIndex):
    import torch
    G = _num_cu()
    d, nq, k = 512, 64, 30
    N = 256 * G * 4 + 999
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS + 3, 0, N, True)
    ix.set_screen("int8")
    x = ix.reconstruct_n(0, N)
    q = O.synth_rows(O.SEED_QUERIES + 3, 0, nq, d, True, "f32")
    Se, Ie = O.knn_exact(x, q, k, "ip")
    qd = torch.from_numpy(q).cuda()
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ix.search_device_exact(qd.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), 1000, stream)
    np.testing.assert_array_equal(I.cpu().numpy(), Ie + 1000)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    # the two-phase step on this one index (its own phase-A lists as the floor) equals the search
    assert ix.two_phase_ok(nq, k)
    Sa = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    Ia = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    p = ix.search_phase_a(qd.data_ptr(), nq, k, 1, Sa.data_ptr(), Ia.data_ptr(), 0, stream)
    ix.search_phase_b(p, Sa.data_ptr(), D.data_ptr(), I.data_ptr(), S.data_ptr(), stream)
    np.testing.assert_array_equal(I.cpu().numpy(), Ie)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    assert ix.full_scan_count() == 0
    ix.close()
