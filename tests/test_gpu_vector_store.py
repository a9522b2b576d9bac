"""The drop-in VectorStore over the REAL HIP index (libvs.so), MI355X only.

* The reference-wrapper golden scenarios (tests/golden/wrapper_golden.json.gz, recorded from
  /root/reference/utils/vector_store.py) replayed through the default index factory: results,
  distances, normalised embeddings, errors and written files must equal the recording.
* Persistence: the streamed file <-> HBM payload path (vs_add_from_file,
  vs_write_rows_to_file) over several pinned chunks, append-saves byte-identical to full rewrites,
  and every storage dtype.
"""
import os

import numpy as np
import pytest

import wrapper_replay
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SCENARIOS = wrapper_replay.load_golden()["scenarios"]


@pytest.fixture(scope="module")
def VS():
    from photo_search_engine_amd import vector_store as vsmod
    assert vsmod._index_factory is vsmod._default_index_factory  # the HIP index, no substitute
    return vsmod.VectorStore


@pytest.mark.parametrize("scenario", SCENARIOS, ids=[s["script"]["name"] for s in SCENARIOS])
def test_reference_wrapper_replay_on_gpu(VS, scenario):
    wrapper_replay.replay(VS, scenario)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_streamed_save_load_multi_chunk(tmp_path, dtype):
    from photo_search_engine_amd import faiss_format as F
    from photo_search_engine_amd.index import FlatIndex
    d, n = 256, 100_003  # 32 MiB chunks of 32768 rows: 4 chunks, the last one partial
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, n, True)
    want = O.synth_rows(O.SEED_CORPUS, 0, n, d, True, dtype)
    p = str(tmp_path / "big.index")
    F.write_flat_rows(p, d, n, 0, lambda path, off: ix.write_rows(path, off, 0, n))
    F.write_flat(str(tmp_path / "ref.index"), want, 0)
    assert open(p, "rb").read() == open(str(tmp_path / "ref.index"), "rb").read()
    ff = F.read_index(p)
    iy = FlatIndex(d, "ip", dtype)
    iy.add_from_file(p, ff.payload_offset, ff.ntotal)
    np.testing.assert_array_equal(iy.reconstruct_n(0, n), want)
    q = want[[5, 70_000, 99_999]]
    D, I = iy.search(q, 3)
    assert I[:, 0].tolist() == [5, 70_000, 99_999]
    # a range in the middle, at an unaligned offset
    iz = FlatIndex(d, "ip", dtype)
    iz.add_from_file(p, ff.payload_offset + 12_345 * d * 4, 40_000)
    np.testing.assert_array_equal(iz.reconstruct_n(0, 40_000), want[12_345:52_345])
    for x in (ix, iy, iz):
        x.close()


def test_add_from_file_errors(tmp_path):
    from photo_search_engine_amd import _lib
    from photo_search_engine_amd.index import FlatIndex
    ix = FlatIndex(8, "ip", "f32")
    p = tmp_path / "short.bin"
    p.write_bytes(b"\0" * 100)
    with pytest.raises(_lib.VsError, match="too short"):
        ix.add_from_file(str(p), 0, 4)
    with pytest.raises(_lib.VsError, match="open"):
        ix.add_from_file(str(tmp_path / "missing.bin"), 0, 1)
    assert ix.ntotal == 0
    ix.add_from_file(str(p), 4, 3)  # 96 bytes of zeros
    assert ix.ntotal == 3 and not ix.reconstruct_n(0, 3).any()
    ix.close()


def test_vector_store_append_saves_on_gpu(VS, tmp_path):
    from photo_search_engine_amd import faiss_format as F
    rng = np.random.default_rng(21)
    X = rng.standard_normal((3000, 96)).astype(np.float32)
    store = VS(dimension=96, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "m.json"))
    for b in range(0, 3000, 1000):  # the indexer's batch loop: add, then save
        store.add(X[b:b + 1000], [{"photo_path": f"/{i}"} for i in range(b, b + 1000)])
        store.save()
        full = str(tmp_path / "full")
        F.write_flat(full, store.index.reconstruct_n(0, store.index.ntotal), 0)
        assert open(str(tmp_path / "idx"), "rb").read() == open(full, "rb").read()
    s2 = VS(dimension=96, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "m.json"))
    assert s2.load() and s2.get_total_items() == 3000
    np.testing.assert_array_equal(s2.index.reconstruct_n(0, 3000), store.index.reconstruct_n(0, 3000))
    r = s2.search(X[1234].tolist(), 2)
    assert r[0]["metadata"]["photo_path"] == "/1234"


def test_device_calls_are_ordered_with_torch_default_stream():
    # regression: a NULL stream used to mean the index's private non-blocking stream, so a pack
    # could read a torch-produced buffer before the producing kernels (default stream) finished
    import torch
    from photo_search_engine_amd.index import FlatIndex
    from photo_search_engine_amd.ivf import IVFFlatIndex
    stream = torch.cuda.current_stream().cuda_stream
    assert stream == 0  # torch's default stream: the NULL handle
    d, n = 512, 200_000
    a = torch.randn((n, 64), device="cuda")
    b = torch.randn((64, d), device="cuda")
    ix = FlatIndex(d, "ip", "f32")
    buf = torch.empty((n, d), device="cuda")
    for rep in range(3):  # the same buffer refilled by slow producers, handed over without a sync
        torch.matmul(a * (rep + 1), b, out=buf)
        ix.add_device(buf.data_ptr(), n, stream)
    got = ix.reconstruct_n(2 * n, n)
    np.testing.assert_array_equal(got, torch.matmul(a * 3, b).cpu().numpy())
    # search outputs consumed by torch right away
    q = buf[:16].clone()
    S = torch.empty((16, 5), dtype=torch.float64, device="cuda")
    I = torch.empty((16, 5), dtype=torch.int64, device="cuda")
    ix.search_device(q.data_ptr(), 16, 5, None, I.data_ptr(), S.data_ptr(), 0, stream)
    first = I[:, 0].clone()  # a torch kernel on the default stream, no explicit sync
    assert first.cpu().tolist() == [2 * n + i for i in range(16)]
    ix.close()
    iv = IVFFlatIndex(64, 8, "ip", "f32")
    iv.set_centroids(np.eye(8, 64, dtype=np.float32))
    x = torch.empty((50_000, 64), device="cuda")
    for rep in range(2):
        torch.matmul(torch.randn((50_000, 256), device="cuda"), torch.randn((256, 64), device="cuda"), out=x)
        want = x.cpu().numpy() if rep == 1 else None
        iv.add_device(x.data_ptr(), 50_000, stream)
    np.testing.assert_array_equal(np.stack([iv.reconstruct(50_000 + i) for i in (0, 777, 49_999)]),
                                  want[[0, 777, 49_999]])
    iv.close()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_product_shapes_d4096_candidate_k(monkeypatch, tmp_path, dtype):
    # the product's own ranges: EMBEDDING_DIMENSION 4096 (config.py:142), one query per call with
    # candidate_k up to ~1.5k (core/searcher.py:807-817), image search k = 5 top_k (:1774-1777),
    # and batched rounds (search_batch) with large k through the GEMV screen in blocks of 8
    from photo_search_engine_amd import vector_store as vsmod
    monkeypatch.setenv("VECTOR_DTYPE", dtype)
    d, N = 4096, 12_000
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, False, "f32")  # unnormalised: VectorStore normalises
    store = vsmod.VectorStore(dimension=d, index_path=str(tmp_path / "i"), metadata_path=str(tmp_path / "m"))
    store.add(x, [{"photo_path": f"/{i}"} for i in range(N)])
    xs = store.index.reconstruct_n(0, N)
    q = O.synth_rows(O.SEED_QUERIES, 0, 40, d, False, "f32")
    qn = store._normalize_rows(q)
    for k in (250, 1500):
        res = store.search(q[0].tolist(), k)
        S, I = O.knn_exact(xs, qn[:1], k, "ip")
        assert [r["metadata"]["photo_path"] for r in res] == [f"/{i}" for i in I[0]]
        assert [r["distance"] for r in res] == S[0].astype(np.float32).tolist()
    for nq, k in ((5, 1500), (40, 300)):
        D, I = store.search_batch(q[:nq], k)
        S, Ie = O.knn_exact(xs, qn[:nq], k, "ip")
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, S.astype(np.float32))


def test_concurrent_searches_from_many_threads():
    # Flask's threaded server can call VectorStore.search concurrently (SURVEY §5, §8 b): each
    # call leases its own stream + workspace; the corpus is shared read-only
    from concurrent.futures import ThreadPoolExecutor
    from photo_search_engine_amd.index import FlatIndex
    d, N = 256, 60_000
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    qs = [O.synth_rows(O.SEED_QUERIES, 100 * t, nq, d, True, "f32") for t, nq in enumerate([1, 3, 9, 40, 1, 8, 64, 2])]
    ref = [ix.search(q, 20) for q in qs]

    def run(t):
        out = []
        for _ in range(6):
            out.append(ix.search(qs[t], 20))
            ix.reconstruct(t * 1000)
        return out

    with ThreadPoolExecutor(8) as ex:
        results = list(ex.map(run, range(8)))
    for t, outs in enumerate(results):
        for D, I in outs:
            np.testing.assert_array_equal(I, ref[t][1])
            np.testing.assert_array_equal(D, ref[t][0])
    ix.close()


def test_write_rows_to_file_errors(tmp_path):
    from photo_search_engine_amd import _lib
    from photo_search_engine_amd.index import FlatIndex
    ix = FlatIndex(8, "ip", "f32")
    ix.add(np.eye(8, dtype=np.float32))
    with pytest.raises(_lib.VsError, match="out of bounds"):
        ix.write_rows(str(tmp_path / "a.bin"), 0, 4, 8)
    with pytest.raises(_lib.VsError, match="open"):
        ix.write_rows(str(tmp_path / "no_such_dir" / "a.bin"), 0, 0, 1)
    ix.write_rows(str(tmp_path / "b.bin"), 16, 2, 3)  # at an offset, file created
    raw = (tmp_path / "b.bin").read_bytes()
    assert len(raw) == 16 + 3 * 32
    np.testing.assert_array_equal(np.frombuffer(raw[16:], dtype="<f4").reshape(3, 8), np.eye(8, dtype=np.float32)[2:5])
    ix.close()


def test_host_search_stages_large_batches_in_bounded_chunks():
    # a batch whose queries (16 MiB at d=4096) exceed the 8 MiB pinned staging cap runs in chunks:
    # exact results, and a later small search leaves the pinned footprint bounded
    from photo_search_engine_amd.index import FlatIndex
    d, N = 4096, 3000
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, 1100, d, True, "bf16")
    D, I = ix.search(q, 12)
    x = ix.reconstruct_n(0, N)
    S, Ie = O.knn_exact(x, q, 12, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    D1, I1 = ix.search(q[:1], 5)
    np.testing.assert_array_equal(I1, Ie[:1, :5])
    assert 0 < ix.host_staging_bytes() <= 2 * (8 << 20) + (1 << 20)
    ix.close()


def test_device_search_context_reuse_across_streams_is_ordered():
    # a device-API search returns with its kernels queued on stream A; the next search on stream B
    # leases the same pooled context and must not overwrite its workspace before A's kernels ran
    import torch
    from photo_search_engine_amd.index import FlatIndex
    d, N, nq, k = 256, 200_000, 64, 20
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    qa = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    qb = O.synth_rows(O.SEED_QUERIES, 500, nq, d, True, "bf16")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for q, s in ((qa, sa), (qb, sb)):
        with torch.cuda.stream(s):
            qd = torch.from_numpy(q).cuda()
            I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
            S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
            ix.search_device(qd.data_ptr(), nq, k, None, I.data_ptr(), S.data_ptr(), 0, s.cuda_stream)
            outs.append((qd, I, S))
    torch.cuda.synchronize()
    x = ix.reconstruct_n(0, N)
    for q, (_, I, S) in zip((qa, qb), outs):
        Se, Ie = O.knn_exact(x, q, k, "ip")
        np.testing.assert_array_equal(I.cpu().numpy(), Ie)
        np.testing.assert_array_equal(S.cpu().numpy(), Se)
    ix.close()


@pytest.mark.parametrize("metric", ["cosine", "l2"])
@pytest.mark.parametrize("copies", [5000, 20000])
def test_store_search_thousands_of_identical_embeddings(VS, tmp_path, metric, copies):
    # A photo library with thousands of identical embeddings (the same picture imported many
    # times): faiss returns the k lowest ids of the tie (/root/reference/utils/vector_store.py:191,
    # tie order pinned by /root/reference/tests/test_searcher.py:323-350); so does the drop-in, for
    # any tie count -- beyond the deepest bounded screen the exact full scan answers.
    d, n, k = 64, 25_000, 10
    x = O.synth_rows(O.SEED_CORPUS, 0, n, d, True, "f32")
    v = x[4321].copy()
    pos = np.random.default_rng(9).choice(n, copies, replace=False)
    x[pos] = v
    store = VS(dimension=d, index_path=str(tmp_path / "t.index"), metadata_path=str(tmp_path / "t.json"),
               metric=metric)
    store.add(x, [{"photo_path": f"p{i}.jpg"} for i in range(n)])
    xs = store._normalize_rows(x)
    qn = store._normalize_query(v.tolist())
    Se, Ie = O.knn_exact(xs, np.asarray(qn, dtype=np.float32), k, "ip" if metric == "cosine" else "l2")
    tie = np.unique(np.concatenate([pos, [4321]]))
    assert Ie[0].tolist() == tie[:k].tolist()
    res = store.search(v.tolist(), k)
    assert [r["metadata"]["photo_path"] for r in res] == [f"p{i}.jpg" for i in tie[:k]]
    assert [r["distance"] for r in res] == [float(np.float32(s)) for s in Se[0]]
    store.index.close()
