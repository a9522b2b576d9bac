"""Parity of the HIP path (libvs.so through the C ABI) against the CPU oracle (MI355X only).

Bar: returned ids bit-exact and distances bit-exact (D = fp32 rounding of the canonical fp64
score, oracle/vs_oracle.c) against ``oracle.knn_exact`` on the SAME stored values (rows read back
through vs_reconstruct_n, i.e. after the dtype rounding the index applies), and within 1e-5 of
the faiss fp32 restatement.  Shapes cover both screen kernels (GEMV: nq <= 8 or f32 storage;
MFMA: bf16/f16 with nq > 8), both metrics, padding of d and N, k > ntotal, exact duplicates
(ties -> lower id), zero vectors, multi-block query batches, and the synthetic generator.
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


def _check_exact(ix, q, k, metric):
    x = ix.reconstruct_n(0, ix.ntotal)
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(x, q, k, metric)
    np.testing.assert_array_equal(I, Ie)
    Dexp = np.where(Ie < 0, 0.0, S).astype(np.float32)
    Dexp[Ie < 0] = -3.4028235e38 if metric == "ip" else 3.4028235e38
    np.testing.assert_array_equal(D, Dexp)
    Df, _ = O.knn_faiss_fp32(x, q, min(k, x.shape[0]), metric)
    assert np.max(np.abs(D[:, :Df.shape[1]].astype(np.float64) - Df)) <= 1e-5
    return D, I


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_synthetic_generator_bit_identical(FlatIndex, dtype):
    ix = FlatIndex(200, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 1000, 777, True)
    got = ix.reconstruct_n(0, 777)
    want = O.synth_rows(O.SEED_CORPUS, 1000, 777, 200, True, dtype)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_add_roundtrip_rounding(FlatIndex, dtype):
    rng = np.random.default_rng(3)
    x = rng.standard_normal((300, 70)).astype(np.float32)
    ix = FlatIndex(70, "ip", dtype)
    ix.add(x[:100])
    ix.add(x[100:])
    np.testing.assert_array_equal(ix.reconstruct_n(0, 300), O.round_dtype(x, dtype))
    np.testing.assert_array_equal(ix.reconstruct(123), O.round_dtype(x[123], dtype))


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("nq,k", [(1, 10), (3, 5), (8, 37)])
def test_gemv_path_exact(FlatIndex, metric, dtype, nq, k):
    d, N = 96, 5000
    ix = FlatIndex(d, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    _check_exact(ix, q, k, metric)


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["bf16", "f16", "f32"])
@pytest.mark.parametrize("nq,k,N,d", [(40, 10, 9000, 128), (256, 100, 20000, 192), (300, 7, 3001, 72),
                                     (64, 400, 150000, 96)])  # Kp 512: the largest MFMA screening depth
def test_mfma_path_exact(FlatIndex, metric, dtype, nq, k, N, d):
    # (fp32 rows: the fp32 MFMA screen from 64 queries on, four 16x16x4 MFMAs per fragment)
    ix = FlatIndex(d, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, dtype)  # queries in the corpus dtype (cfg3)
    _check_exact(ix, q, k, metric)


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("nq,k,N,d", [(256, 100, None, 512), (64, 1000, 150_000, 256), (300, 10, 50_000, 384),
                                     (20, 50, 3000, 1536)])
def test_direct_16bit_screen_exact(FlatIndex, metric, dtype, nq, k, N, d):
    """bf16 / f16 rows with 32-element K-steps per tile a multiple of 4: the main pass is the
    direct form k_screen_d16 (corpus fragments HBM -> VGPRs, both halves of each 128 B line in
    consecutive K-steps).  Seeded (>= 4 tiles per CU) and unseeded corpora, partial last tiles, k =
    1000 (compaction in the K loop), two query blocks, fp32 queries."""
    if N is None:
        N = 256 * 4 * _num_cu() + 777
    ix = FlatIndex(d, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS + 3, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES + 3, 0, nq, d, True, "f32")
    _check_exact(ix, q, k, metric)
    ix.close()


def test_mfma_fp32_queries_over_bf16_corpus(FlatIndex):
    # queries NOT representable in bf16: screen uses rounded queries, refine uses the exact ones
    ix = FlatIndex(256, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, 30000, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 64, 256, True, "f32")
    _check_exact(ix, q, 50, "ip")


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("nq,kind", [(63, "gemv"), (64, "mfma"), (256, "mfma")])
def test_f32_batches_choose_mfma_from_64_queries(FlatIndex, metric, nq, kind):
    # fp32 native batches: GEMV passes of 8 queries below 64, the fp32 MFMA screen from 64 on (d
    # not a multiple of the 16-element K-step's chunk: padding), seeded (>= 4 tiles per CU)
    d, N = 200, 256 * 4 * _num_cu() + 999
    ix = FlatIndex(d, metric, "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    ix.set_timing(True)
    _check_exact(ix, q, 25, metric)
    ix.set_timing(False)
    assert ix.timing_fetch()[1] == kind
    ix.close()


def test_f32_batch_over_gemv_blocks(FlatIndex):
    ix = FlatIndex(1536, "ip", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, 12000, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 21, 1536, True, "f32")
    _check_exact(ix, q, 10, "ip")


def test_edge_small_and_k_beyond_ntotal(FlatIndex):
    for metric in ("ip", "l2"):
        ix = FlatIndex(8, metric, "f32")
        x = np.array([[1.0] * 8, [0.5] * 8, [0.0] * 8], np.float32)
        ix.add(x)
        D, I = ix.search(x[:1], 5)
        assert list(I[0, 3:]) == [-1, -1]
        _check_exact(ix, x, 5, metric)


def test_edge_duplicates_ties_lower_id(FlatIndex):
    rng = np.random.default_rng(4)
    base = rng.standard_normal((50, 64)).astype(np.float32)
    x = np.concatenate([base, np.repeat(base[7:8], 300, axis=0), base], axis=0)  # 300 exact copies
    for dtype in ("f32", "bf16"):
        ix = FlatIndex(64, "ip", dtype)
        ix.add(x)
        q = np.repeat(base[7:8], 20, axis=0) if dtype == "bf16" else base[7:8]
        D, I = _check_exact(ix, q, 40, "ip")
        assert I[0, 0] == 7  # the earliest copy wins the tie


def test_edge_zero_vectors_and_constant_rows(FlatIndex):
    x = np.zeros((600, 40), np.float32)
    x[::3] = 1.0 / np.sqrt(40)
    ix = FlatIndex(40, "ip", "f32")
    ix.add(x)
    q = np.full((2, 40), 1.0 / np.sqrt(40), np.float32)
    _check_exact(ix, q, 250, "ip")


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_mfma_partial_tile_all_negative_scores(FlatIndex, dtype):
    # a corpus smaller than one tile whose scores are all negative for every query: the zero
    # padding rows of the tile (exact score 0) must never become candidates (regression: they
    # did on the MFMA path with an unseeded threshold)
    rng = np.random.default_rng(8)
    x = np.abs(rng.standard_normal((8, 48))).astype(np.float32)
    q = -np.abs(rng.standard_normal((40, 48))).astype(np.float32)
    ix = FlatIndex(48, "ip", dtype)
    ix.add(x)
    D, I = _check_exact(ix, O.round_dtype(q, dtype), 5, "ip")
    assert (D < 0).all() and (I < 8).all()


def test_large_k(FlatIndex):
    ix = FlatIndex(64, "ip", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, 50000, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 2, 64, True, "f32")
    _check_exact(ix, q, 1500, "ip")


def test_device_api_and_uncertified_counter(FlatIndex):
    import torch
    ix = FlatIndex(128, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, 40000, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 100, 128, True, "bf16")
    qd = torch.from_numpy(q).cuda()
    D = torch.empty((100, 10), dtype=torch.float32, device="cuda")
    I = torch.empty((100, 10), dtype=torch.int64, device="cuda")
    S = torch.empty((100, 10), dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ix.search_device(qd.data_ptr(), 100, 10, D.data_ptr(), I.data_ptr(), S.data_ptr(), 5, st)
    torch.cuda.synchronize()
    x = ix.reconstruct_n(0, ix.ntotal)
    Se, Ie = O.knn_exact(x, q, 10, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie + 5)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    assert ix.uncertified_count() == 0


def test_reset_and_reuse(FlatIndex):
    ix = FlatIndex(32, "l2", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, 1000, True)
    ix.reset()
    assert ix.ntotal == 0
    x = O.synth_rows(7, 0, 500, 32, True, "f32")
    ix.add(x)
    _check_exact(ix, x[:4], 9, "l2")


def test_real_reference_index_self_queries(FlatIndex):
    import os
    from photo_search_engine_amd import faiss_format
    ff = faiss_format.read_index(os.path.join(os.path.dirname(__file__), "golden", "ref_photo_search.index"))
    ix = FlatIndex(ff.d, "ip", "f32")
    ix.add(np.ascontiguousarray(ff.vectors))
    D, I = _check_exact(ix, np.ascontiguousarray(ff.vectors), 10, "ip")
    np.testing.assert_array_equal(I[:, 0], np.arange(77))


@pytest.mark.parametrize("d", [16, 32])
def test_mfma_tiny_dim_many_tiles_per_workgroup(FlatIndex, d):
    # d <= 32 is one 32-element chunk; the layout pads it to two K-steps so the screen's
    # per-tile compaction check runs.  ~3.8 tiles per workgroup, unseeded threshold: without
    # compaction a workgroup's candidate buffer (768 keys per query) would overflow.
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, 250_000, False)
    q = O.synth_rows(O.SEED_QUERIES, 0, 40, d, False, "bf16")
    _check_exact(ix, q, 100, "ip")


def _num_cu():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("k", [10, 100])
def test_seeded_threshold_search_exact(FlatIndex, metric, k):
    # >= 4 tiles per CU: the MFMA path seeds every workgroup's threshold from a strided tile
    # sample (optimistic rank), so this covers the seed pass + certificate on real sizes
    N = 256 * 4 * _num_cu() + 777
    ix = FlatIndex(64, metric, "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 48, 64, True, "bf16")
    _check_exact(ix, q, k, metric)
    assert ix.uncertified_count() == 0


def test_optimistic_seed_failure_falls_back_exactly(FlatIndex):
    # Adversarial corpus: one near-copy of the query in every SAMPLED tile (each workgroup's first) and
    # nowhere else, so the optimistic seed threshold (16th best sample maximum) lets fewer than Kp
    # rows through; the certificate must reject it and vs_search must re-search exactly.
    # 32 tiles per CU: the optimistic rank is ceil(8 * Kp / 32) = 8 < the 16 planted rows/query
    d, k = 64, 10
    cu = _num_cu()
    tiles = 32 * cu + 3
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 16, d, True, "f32")
    rng = np.random.default_rng(11)
    for j in range(cu):  # the sampled tile of workgroup j: the first of its range
        r = (tiles * j // cu) * 256 + 5
        x[r] = q[j % 16] + 0.01 * rng.standard_normal(d).astype(np.float32)
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    _check_exact(ix, O.round_dtype(q, "bf16"), k, "ip")
    assert ix.uncertified_count() > 0  # the optimistic pass was rejected (and then redone exactly)


@pytest.mark.parametrize("nq,dtype", [(16, "bf16"), (300, "bf16"), (64, "f32"), (300, "f32")])
def test_device_exact_search_re_searches_uncertified_queries(FlatIndex, nq, dtype):
    # the adversarial corpus above through the device API used by the multi-GPU layers: the
    # optimistic pass is rejected on the device and the failed queries are re-searched by the
    # fallback round queued behind it (no host round trip).  nq = 300: two query blocks, only the
    # first holds adversarial queries, so the second block's fallback kernels are gated off.
    import torch
    d, k = 64, 10
    cu = _num_cu()
    tiles = 32 * cu + 3
    N = tiles * 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    rng = np.random.default_rng(11)
    for j in range(cu):  # the sampled tile of workgroup j: the first of its range
        x[(tiles * j // cu) * 256 + 5] = q[j % 16] + 0.01 * rng.standard_normal(d).astype(np.float32)
    # (fp32 rows: batches of >= 64 queries take the seeded fp32 MFMA screen, and the fallback round
    # is the fp32 MFMA screen too, also queued without a host sync)
    ix = FlatIndex(d, "ip", dtype)
    ix.add(x)
    qb = O.round_dtype(q, dtype)
    qd = torch.from_numpy(qb).cuda()
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    ix.search_device_exact(qd.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), 1000, 0)
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, N), qb, k, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie + 1000)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    np.testing.assert_array_equal(D.cpu().numpy(), Se.astype(np.float32))
    assert ix.uncertified_count() > 0
    assert ix.full_scan_count() == 0


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("nq,copies", [(1, 5000), (20, 12000), (3, 20000)])
def test_ties_beyond_max_depth_full_scan(FlatIndex, nq, copies, dtype, metric):
    # `copies` identical rows tie with the query's best score: more than the deepest bounded screen
    # (KP_MAX = 4096 rows, the adaptive refine's 8192) can certify.  faiss answers with the k lowest
    # ids of the tie (/root/reference/utils/vector_store.py:191); so must every entry point: the
    # host API (escalation, then the exact full scan), the device API (fallback round, then the gated
    # full scan, no host sync) and the multi-device handle whose shards run the device path.
    import torch
    from photo_search_engine_amd.index import MultiDeviceFlatIndex
    d, k, N = 64, 10, 25_000
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    v = x[123].copy()
    pos = np.random.default_rng(3).choice(N, copies, replace=False)
    x[pos] = v
    q = np.repeat(v[None], nq, axis=0)
    ix = FlatIndex(d, metric, dtype)
    ix.add(x)
    xs = ix.reconstruct_n(0, N)
    Se, Ie = O.knn_exact(xs, q, k, metric)
    tie = np.unique(np.concatenate([pos, [123]]))
    np.testing.assert_array_equal(Ie, np.repeat(tie[None, :k], nq, axis=0))  # (the checker itself)
    D, I = ix.search(q, k)
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, Se.astype(np.float32))
    fs0 = ix.full_scan_count()
    assert fs0 >= 1  # the bounded screens could not certify it
    qd = torch.from_numpy(q).cuda()
    I2 = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    S2 = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    D2 = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    ix.search_device_exact(qd.data_ptr(), nq, k, D2.data_ptr(), I2.data_ptr(), S2.data_ptr(), 7, 0)
    np.testing.assert_array_equal(I2.cpu().numpy(), Ie + 7)
    np.testing.assert_array_equal(S2.cpu().numpy(), Se)
    np.testing.assert_array_equal(D2.cpu().numpy(), Se.astype(np.float32))
    assert ix.full_scan_count() >= fs0 + (nq if copies > 8192 else 0)
    m = MultiDeviceFlatIndex(d, metric, dtype, devices=[0, 0])  # (its shards run the device path)
    m.add(x)
    Dm, Im = m.search(q, k)
    np.testing.assert_array_equal(Im, Ie)
    np.testing.assert_array_equal(Dm, Se.astype(np.float32))
    m.close()
    ix.close()


@pytest.mark.parametrize("dtype,screen", [("f32", "native"), ("bf16", "native"), ("bf16", "int8")])
def test_single_query_duplicate_burst_certified_by_research(FlatIndex, dtype, screen):
    # a single query's GEMV first pass keeps only Kb keys per block; a burst of a few
    # hundred contiguous duplicates (photos imported one after another) sits in one block and fails
    # that pass.  The host API's deeper re-search keeps whole lists, so it certifies the query
    # without the full scan (a truncated re-search would fail the same way at every depth).
    d, k, N, copies = 128, 10, 120_000, 300
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    x[60_000:60_000 + copies] = x[60_000]
    q = x[60_000:60_001].copy()
    ix = FlatIndex(d, "ip", dtype)
    ix.set_scan_limit(0)
    ix.add(x)
    ix.set_screen(screen)
    xs = ix.reconstruct_n(0, N)
    Se, Ie = O.knn_exact(xs, q, k, "ip")
    np.testing.assert_array_equal(Ie[0], np.arange(60_000, 60_000 + k))
    D, I = ix.search(q, k)
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, Se.astype(np.float32))
    assert ix.uncertified_count() >= 1  # the truncated first pass could not certify it
    assert ix.full_scan_count() == 0    # the re-search did
    ix.close()


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_full_scan_near_ties_and_k_beyond_rows(FlatIndex, metric):
    # The full scan's own ordering: rows tied to the last bit mixed with rows one ulp apart (bf16),
    # every row scanned by a workgroup whose range starts mid-tie, and k larger than the index
    # (padding).  Forced through the host API on a tie the screens cannot list.
    d, N = 64, 9000
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    v = x[7].copy()
    rng = np.random.default_rng(11)
    pos = rng.choice(N, 6000, replace=False)
    x[pos] = v
    near = rng.choice(pos, 300, replace=False)
    x[near, 0] = v[0] + np.float32(2.0 ** -8) * np.sign(v[0] if v[0] != 0 else 1.0)  # near-ties
    ix = FlatIndex(d, metric, "bf16")
    ix.add(x)
    xs = ix.reconstruct_n(0, N)
    for k in (1, 64, 1000):
        D, I = ix.search(v[None], k)
        Se, Ie = O.knn_exact(xs, v[None].astype(np.float32), k, metric)
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, Se.astype(np.float32))
    # k beyond the rows present: faiss pads (host API searches min(k, ntotal) and pads)
    small = FlatIndex(d, metric, "bf16")
    small.add(np.repeat(v[None], 50, axis=0))
    D, I = small.search(v[None], 60)
    assert I[0, :50].tolist() == list(range(50)) and (I[0, 50:] == -1).all()
    small.close()
    ix.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_gemv_block_failure_goes_to_full_scan(FlatIndex, dtype):
    # a GEMV first pass (1-8 queries) whose certificate fails -- 300 copies of the query's best row
    # tie beyond its Kp-deep lists -- is answered on the device by the gated full scan alone (no
    # MFMA fallback round for GEMV blocks); exact, and counted in full_scan_count
    import torch
    d, k, N, nq = 64, 10, 30_000, 4
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    v = x[4242].copy()
    x[np.random.default_rng(2).choice(N, 300, replace=False)] = v
    ix = FlatIndex(d, "ip", dtype)  # (screened fixture: no small scan)
    ix.add(x)
    q = np.concatenate([np.repeat(v[None], 2, axis=0), O.synth_rows(O.SEED_QUERIES, 0, nq - 2, d, True, dtype)])
    qd = torch.from_numpy(q).cuda()
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    ix.search_device_exact(qd.data_ptr(), nq, k, None, I.data_ptr(), S.data_ptr(), 0, 0)
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, N), q, k, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    assert ix.uncertified_count() >= 2 and ix.full_scan_count() >= 2
    ix.close()


@pytest.mark.parametrize("d", [64, 512])
def test_batch_refine_certifies_ties_within_its_depth(FlatIndex, d):
    """5000 exact ties (beyond KP_MAX = 4096) in a 20-query batch: the adaptive refine lists and
    scores every copy (<= 8192 rows), so the batch certifies with the exact answer -- the lowest-id
    copies, faiss' tie order -- where a fixed-depth screen could only report the query.  d = 512:
    the direct 16-bit screen, seeded from one tile per workgroup at this size."""
    k, nq = 10, 20
    x = O.synth_rows(O.SEED_CORPUS, 0, 25_000, d, True, "bf16")
    v = x[123].copy()
    dup = np.random.default_rng(3).choice(25_000, 5000, replace=False)
    x[dup] = v
    ix = FlatIndex(d, "ip", "bf16")
    ix.add(x)
    q = np.repeat(v[None], nq, axis=0)
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(ix.reconstruct_n(0, 25_000), q, k, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    assert set(I[0].tolist()) <= set(dup.tolist()) | {123}
    assert ix.full_scan_count() == 0
    ix.close()


def test_device_exact_search_k_beyond_shard_rows(FlatIndex):
    # a row shard smaller than k (many GPUs, small corpus): padded like faiss, no error
    import torch
    ix = FlatIndex(32, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, 5, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 12, 32, True, "bf16")
    qd = torch.from_numpy(q).cuda()
    S = torch.empty((12, 10), dtype=torch.float64, device="cuda")
    I = torch.empty((12, 10), dtype=torch.int64, device="cuda")
    ix.search_device_exact(qd.data_ptr(), 12, 10, None, I.data_ptr(), S.data_ptr(), 7, 0)
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, 5), q, 10, "ip")
    Ih = I.cpu().numpy()
    np.testing.assert_array_equal(Ih[:, :5], Ie[:, :5] + 7)
    assert (Ih[:, 5:] == -1).all()
    np.testing.assert_array_equal(S.cpu().numpy()[:, :5], Se[:, :5])


def test_device_shard_merge_matches_oracle(FlatIndex):
    # 4 row shards searched separately (one shorter than k -> id -1 padding), merged on the device
    import torch
    from photo_search_engine_amd.index import merge_shards_device
    d, k, nq = 48, 17, 33
    bounds = [0, 5000, 5010, 9000, 12000]
    x = O.synth_rows(O.SEED_CORPUS, 0, bounds[-1], d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    Sg = np.empty((4, nq, k), dtype=np.float64)
    Ig = np.empty((4, nq, k), dtype=np.int64)
    for g in range(4):
        ix = FlatIndex(d, "ip", "f32")
        ix.add(x[bounds[g]:bounds[g + 1]])
        Sd = torch.empty((nq, k), dtype=torch.float64, device="cuda")
        Id = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        qd = torch.from_numpy(q).cuda()
        ix.search_device(qd.data_ptr(), nq, k, None, Id.data_ptr(), Sd.data_ptr(), bounds[g],
                         torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        Sg[g], Ig[g] = Sd.cpu().numpy(), Id.cpu().numpy()
        ix.close()
    assert (Ig[1][:, 10:] == -1).all()  # the 10-row shard pads
    St, It = torch.from_numpy(Sg).cuda(), torch.from_numpy(Ig).cuda()
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    merge_shards_device(0, St.data_ptr(), It.data_ptr(), 4, nq, k, S.data_ptr(), I.data_ptr(), D.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    Sm, Im = O.merge_topk(Sg, Ig, k, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Im)
    np.testing.assert_array_equal(S.cpu().numpy(), Sm)
    Se, Ie = O.knn_exact(x, q, k, "ip")  # = one index over all rows
    np.testing.assert_array_equal(I.cpu().numpy(), Ie)
    np.testing.assert_array_equal(D.cpu().numpy(), Se.astype(np.float32))


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("G,k", [(1, 100), (3, 17), (8, 100), (8, 512), (16, 300), (5, 1000)])
def test_device_shard_merge_ties_and_padding(metric, G, k):
    # synthetic sorted lists with many equal scores (ties -> lower id), ragged padding; G * k <=
    # 4096 takes the rank merge, larger ones the wave-per-query merge: both equal the oracle's merge
    import torch
    from photo_search_engine_amd.index import merge_shards_device
    rng = np.random.default_rng(G * 1000 + k)
    nq = 37
    Sg = np.empty((G, nq, k), dtype=np.float64)
    Ig = np.empty((G, nq, k), dtype=np.int64)
    worst = -1.7976931348623157e308 if metric == "ip" else 1.7976931348623157e308
    for g in range(G):
        for qi in range(nq):
            nv = int(rng.integers(0, k + 1)) if rng.random() < 0.3 else k
            sc = rng.integers(0, 40, size=nv).astype(np.float64) / 8.0  # few distinct values
            ids = rng.choice(1 << 40, size=nv, replace=False) + g  # globally distinct ids
            order = np.lexsort((ids, -sc if metric == "ip" else sc))
            Sg[g, qi, :nv], Ig[g, qi, :nv] = sc[order], ids[order]
            Sg[g, qi, nv:], Ig[g, qi, nv:] = worst, -1
    St, It = torch.from_numpy(Sg).cuda(), torch.from_numpy(Ig).cuda()
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    merge_shards_device(0 if metric == "ip" else 1, St.data_ptr(), It.data_ptr(), G, nq, k, S.data_ptr(),
                        I.data_ptr(), D.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    Sm, Im = O.merge_topk(Sg, Ig, k, metric)
    np.testing.assert_array_equal(I.cpu().numpy(), Im)
    np.testing.assert_array_equal(S.cpu().numpy()[Im >= 0], Sm[Im >= 0])
    assert (S.cpu().numpy()[Im < 0] == worst).all()


def test_sharded_index_single_process_matches_oracle():
    import torch
    from photo_search_engine_amd.distributed import ShardedFlatIndex
    sh = ShardedFlatIndex(96, "l2", "bf16", device=0)
    sh.add_synthetic(O.SEED_CORPUS, 30000, True)
    q = torch.from_numpy(O.synth_rows(O.SEED_QUERIES, 0, 20, 96, True, "bf16")).cuda()
    D, I, S = sh.search(q, 25)
    x = sh.index.reconstruct_n(0, 30000)
    Se, Ie = O.knn_exact(x, q.cpu().numpy(), 25, "l2")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    sh.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("N,k", [(20, 16), (5000, 10), (70_000, 1), (70_000, 100), (300_000, 10), (300_000, 400)])
def test_single_query_merge_stop_exact(FlatIndex, metric, N, k, dtype):
    # one query: the GEMV path stops its merge tree once <= 2048 keys remain and the refine selects
    # the best Kp from them (shards of >= Kp rows), else merges to one list; both must be exact,
    # for every storage dtype (single queries always take the GEMV path)
    ix = FlatIndex(48, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    for i in range(3):
        q = O.synth_rows(O.SEED_QUERIES, 100 + i, 1, 48, True, "f32")
        _check_exact(ix, q, k, metric)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_single_query_device_api_s64(FlatIndex, dtype):
    # the sharded layer's call: one query through vs_search_device with id offset and fp64 outputs
    import torch
    N, d, k = 300_000, 48, 37
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 7, 1, d, True, "f32")
    qd = torch.from_numpy(q).cuda()
    I = torch.empty((1, k), dtype=torch.int64, device="cuda")
    S = torch.empty((1, k), dtype=torch.float64, device="cuda")
    D = torch.empty((1, k), dtype=torch.float32, device="cuda")
    ix.search_device(qd.data_ptr(), 1, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), 11, 0)
    torch.cuda.synchronize()
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, N), q, k, "ip")
    np.testing.assert_array_equal(I.cpu().numpy(), Ie + 11)
    np.testing.assert_array_equal(S.cpu().numpy(), Se)
    np.testing.assert_array_equal(D.cpu().numpy(), Se.astype(np.float32))


@pytest.mark.parametrize("k", [1000, 2048])
def test_mfma_large_k_batches_stay_on_mfma(FlatIndex, k):
    # the product's relaxed candidate_k (core/searcher.py:807-817) batched: k up to 2048 at nq > 8
    # stays on the MFMA screen (512 per workgroup, drop-bounded certificate), bit-exact
    N, d, nq = 150_000, 1536, 64
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    ix.set_timing(True)
    D, I = ix.search(q, k)
    ix.set_timing(False)
    ms, kind = ix.timing_fetch()
    assert kind == "mfma" and len(ms) == 1  # one MFMA launch for the whole batch, no GEMV passes
    S, Ie = O.knn_exact(ix.reconstruct_n(0, N), q, k, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    assert ix.uncertified_count() == 0
    ix.close()


def test_k_3000_single_query_and_batch(FlatIndex):
    # depths above 2048 (k up to 3276): the wide merge on the GEMV path, the 4096-key refine
    ix = FlatIndex(64, "ip", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, 200_000, True)
    for nq in (1, 12):
        q = O.synth_rows(O.SEED_QUERIES, 3, nq, 64, True, "f32")
        _check_exact(ix, q, 3000, "ip")


def test_reserve_sizes_storage_once(FlatIndex):
    # vs_reserve: one allocation for the rows to come; chunked adds up to it never regrow, and the
    # search over them is exact
    d, N = 80, 7000
    ix = FlatIndex(d, "ip", "bf16")
    ix.reserve(N)
    cap = ix.capacity
    assert cap >= N and cap < N + 256
    for r0 in range(0, N, 1000):
        ix.add_synthetic(O.SEED_CORPUS, r0, min(1000, N - r0), True)
        assert ix.capacity == cap
    ix.add_synthetic(O.SEED_CORPUS, N, 300, True)  # past the reservation: regrows
    assert ix.capacity > cap
    x = O.synth_rows(O.SEED_CORPUS, 0, N + 300, d, True, "bf16")
    q = O.synth_rows(O.SEED_QUERIES, 0, 30, d, True, "f32")
    D, I = ix.search(q, 9)
    S, Ie = O.knn_exact(x, q, 9, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("nq,k,N", [(1, 400, 60_000), (3, 257, 40_000), (8, 700, 30_000), (1, 300, 350)])
def test_few_query_deep_refine_split_exact(FlatIndex, dtype, metric, nq, k, N):
    # few queries (GEMV screen) with deep lists: k_refine spreads each query's kept rows over
    # several workgroups, the last one to finish sorts and certifies (refine_split); repeated
    # calls check that the per-query completion counters come back to zero; N=350 leaves most
    # slices empty (k close to the shard size)
    ix = FlatIndex(96, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    for i in range(3):
        q = O.synth_rows(O.SEED_QUERIES, 500 + 10 * i, nq, 96, True, "f32")
        _check_exact(ix, q, k, metric)


@pytest.fixture(scope="module")
def PlainFlatIndex():
    from photo_search_engine_amd.index import FlatIndex as FI
    return FI


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("N,nq,k", [(10_000, 1, 10), (777, 2, 1), (4_099, 1, 64), (50, 1, 60), (65_536, 2, 33)])
def test_small_scan_exact(PlainFlatIndex, metric, dtype, N, nq, k):
    # calls of 1-2 queries (k <= 64) over a corpus under the scan limits (<= 65536 rows, default 192 MiB) skip
    # the screen: one launch scores every row canonically and selects the top-k (k_full_scan, the
    # timed kernel); ids and scores bit-exact, k beyond the rows padded, nothing counted as a
    # fallback full scan
    d = 136
    ix = PlainFlatIndex(d, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 5, nq, d, True, "f32")
    ix.set_timing(True)
    _check_exact(ix, q, k, metric)
    ix.set_timing(False)
    assert ix.timing_fetch()[1] == "full_scan"
    assert ix.full_scan_count() == 0 and ix.uncertified_count() == 0
    # the device API (exact path), with an id offset: the same answer
    import torch
    qd = torch.from_numpy(q).cuda()
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    ix.search_device_exact(qd.data_ptr(), nq, k, None, I.data_ptr(), S.data_ptr(), 11, 0)
    Se, Ie = O.knn_exact(ix.reconstruct_n(0, N), q, k, metric)
    np.testing.assert_array_equal(I.cpu().numpy(), np.where(Ie >= 0, Ie + 11, -1))
    valid = Ie >= 0
    np.testing.assert_array_equal(S.cpu().numpy()[valid], Se[valid])
    # a limit of 0: the screen path, same bits
    D1, I1 = ix.search(q, k)
    ix.set_scan_limit(0)
    D2, I2 = ix.search(q, k)
    np.testing.assert_array_equal(I1, I2)
    np.testing.assert_array_equal(D1, D2)
    ix.close()


def test_small_scan_ties_and_zero_rows(PlainFlatIndex):
    # 20000 identical rows and zero vectors in a small corpus: the single-query call's full scan
    # returns faiss's lowest ids of the tie directly
    d, N, k = 64, 25_000, 10
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    v = x[77].copy()
    pos = np.random.default_rng(1).choice(N, 20_000, replace=False)
    x[pos] = v
    x[:5] = 0.0
    ix = PlainFlatIndex(d, "ip", "bf16")
    ix.add(x)
    for qv in (v, np.zeros(d, np.float32)):
        D, I = ix.search(qv[None], k)
        S, Ie = O.knn_exact(ix.reconstruct_n(0, N), qv[None].astype(np.float32), k, "ip")
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


@pytest.mark.parametrize("screen", ["native", "int8"])
@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_zero_query_in_batch_ties_to_lowest_ids(FlatIndex, screen, metric):
    # zero queries inside an MFMA batch: every inner-product score is exactly 0 (all rows tie), so
    # the refines' selections and rank sorts must return the lowest ids in order; half the rows
    # are all-negative (their products with 0 are -0.0) and a few rows are zero vectors
    rng = np.random.default_rng(11)
    d, N, nq, k = 96, 20_000, 256, 50
    x = rng.standard_normal((N, d)).astype(np.float32)
    x[::2] = -np.abs(x[::2])
    x /= np.linalg.norm(x, axis=1, keepdims=True)  # (unit rows: distances ~2, the fp32 check's scale)
    x[5:9] = 0.0
    q = rng.standard_normal((nq, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    q[[0, 100, 255]] = 0.0
    ix = FlatIndex(d, metric, "bf16")
    ix.add(x)
    if screen == "int8":
        ix.set_screen("int8")
    D, I = _check_exact(ix, O.round_dtype(q, "bf16"), k, metric)
    if metric == "ip":
        for r in (0, 100, 255):
            np.testing.assert_array_equal(I[r], np.arange(k))
            assert (D[r] == 0.0).all()
    ix.close()
