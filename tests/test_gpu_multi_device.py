"""One index over several devices of one process (``MultiDeviceFlatIndex`` / include/vs.h
``vs_multi_*``) on the box's GPU: shards are separate libvs handles (two or three on device 0),
rows dealt in 65,536-id chunks, per-shard exact searches merged on devices[0].  Results must equal
the oracle's exact answer over all rows (ids and fp32 scores bit-exact), for both screens, both
metrics, batches and single queries, empty shards and k beyond the rows; the VectorStore
``VECTOR_DEVICES`` path must save byte-identical files and load them back."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Multi():
    from photo_search_engine_amd.index import MultiDeviceFlatIndex
    return MultiDeviceFlatIndex


def _exact(ix, x, q, k, metric):
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(x, q, k, metric)
    np.testing.assert_array_equal(I, Ie)
    Dexp = S.astype(np.float32)
    Dexp[Ie < 0] = -3.4028235e38 if metric == "ip" else 3.4028235e38
    np.testing.assert_array_equal(D, Dexp)


@pytest.mark.parametrize("dtype,metric", [("bf16", "ip"), ("f32", "l2"), ("f16", "ip")])
def test_two_shards_match_one_index(Multi, dtype, metric):
    N, d = 200_000, 64  # 4 chunks of 65,536 ids: shard 0 holds chunks 0 and 2, shard 1 chunks 1 and 3
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    ix = Multi(d, metric, dtype, devices=[0, 0])
    for a, b in ((0, 70_000), (70_000, 70_001), (70_001, N)):  # adds crossing chunk boundaries
        ix.add(x[a:b])
    assert ix.ntotal == N
    assert ix.shard_rows() == [2 * 65536, 65536 + (N - 3 * 65536)]
    np.testing.assert_array_equal(ix.reconstruct_n(65_000, 1_000), x[65_000:66_000])
    for nq, k in ((40, 25), (1, 10), (9, 100)):
        q = O.synth_rows(O.SEED_QUERIES, nq, nq, d, True, "f32")
        _exact(ix, x, q, k, metric)
    ix.close()


def test_empty_shard_k_beyond_rows_and_int8_screen(Multi):
    d = 48
    x = O.synth_rows(O.SEED_CORPUS, 0, 5000, d, True, "bf16")  # one chunk: shards 1 and 2 stay empty
    ix = Multi(d, "ip", "bf16", devices=[0, 0, 0])
    ix.add(x)
    assert ix.shard_rows() == [5000, 0, 0]
    q = O.synth_rows(O.SEED_QUERIES, 0, 12, d, True, "f32")
    _exact(ix, x, q, 20, "ip")
    small = Multi(d, "ip", "bf16", devices=[0, 0])
    small.add(x[:700])
    D, I = small.search(q[:2], 800)  # k beyond the rows: faiss padding
    assert (I[:, 700:] == -1).all() and (D[:, 700:] == -3.4028235e38).all()
    _exact(small, x[:700], q, 700, "ip")
    small.close()
    y = O.synth_rows(O.SEED_CORPUS, 5000, 150_000, d, True, "bf16")
    ix.add(y)
    ix.set_screen("int8")
    _exact(ix, np.concatenate([x, y]), O.synth_rows(O.SEED_QUERIES, 50, 64, d, True, "f32"), 50, "ip")
    ix.reset()
    assert ix.ntotal == 0 and ix.shard_rows() == [0, 0, 0]
    ix.close()


def test_vector_store_over_devices_saves_and_loads_identically(tmp_path, monkeypatch):
    from photo_search_engine_amd import vector_store as vsmod
    rng = np.random.default_rng(9)
    rows = rng.standard_normal((140_000, 32)).astype(np.float32)
    metas = [{"photo_path": f"p{i}.jpg"} for i in range(rows.shape[0])]

    def build(tag, devices):
        if devices:
            monkeypatch.setenv("VECTOR_DEVICES", devices)
        else:
            monkeypatch.delenv("VECTOR_DEVICES", raising=False)
        st = vsmod.VectorStore(dimension=32, index_path=str(tmp_path / f"{tag}.index"),
                               metadata_path=str(tmp_path / f"{tag}.json"))
        st.add(rows[:100_000], metas[:100_000])
        for i in range(100_000, 100_005):
            st.add_item(rows[i].tolist(), metas[i])
        st.save()
        st.add(rows[100_005:], metas[100_005:])
        st.save()  # an append-save across the chunk boundary
        return st

    one = build("one", "")
    two = build("two", "0,0")
    assert type(two.index).__name__ == "MultiDeviceFlatIndex"
    assert open(tmp_path / "one.index", "rb").read() == open(tmp_path / "two.index", "rb").read()
    for i in (3, 77_777, 139_999):
        assert one.search(rows[i].tolist(), 7) == two.search(rows[i].tolist(), 7)
    assert two.get_embedding_by_photo_path("p131072.jpg") == one.get_embedding_by_photo_path("p131072.jpg")
    back = vsmod.VectorStore(dimension=32, index_path=str(tmp_path / "two.index"),
                             metadata_path=str(tmp_path / "two.json"))
    assert back.load() and back.get_total_items() == rows.shape[0]
    assert back.search(rows[5].tolist(), 5) == one.search(rows[5].tolist(), 5)


def test_concurrent_searches_run_concurrently_and_exactly(Multi):
    """vs_multi_search from 8 threads (the reference serves from Flask's threaded server,
    /root/reference/main.py:353): every result exact, and calls overlap in wall-clock time (each
    call leases its own streams / buffers / workers; the handle's lock is shared)."""
    import threading
    import time

    N, d = 300_000, 128
    x = O.synth_rows(O.SEED_CORPUS + 61, 0, N, d, True, "bf16")
    ix = Multi(d, "ip", "bf16", devices=[0, 0])
    ix.add(x)
    qs = [O.synth_rows(O.SEED_QUERIES + 61, 64 * t, 64, d, True, "f32") for t in range(8)]
    ref = [O.knn_exact(x, q, 20, "ip") for q in qs]
    spans, errs = [], []

    def worker(t):
        try:
            for _ in range(6):
                t0 = time.perf_counter()
                D, I = ix.search(qs[t], 20)
                spans.append((t0, time.perf_counter()))
                np.testing.assert_array_equal(I, ref[t][1])
                np.testing.assert_array_equal(D, ref[t][0].astype(np.float32))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[0]
    spans.sort()
    overlapping = sum(1 for i in range(1, len(spans)) if spans[i][0] < max(e for _, e in spans[:i]))
    assert overlapping >= len(spans) // 2, f"only {overlapping} of {len(spans)} calls overlapped another"
    ix.close()


def test_failed_add_rolls_back_every_shard(Multi, tmp_path):
    """A multi-device add that fails on one shard (its rows lie beyond the end of the file) leaves
    no shard with extra rows: ids stay arithmetic and later adds and searches stay exact."""
    d = 32
    x = O.synth_rows(O.SEED_CORPUS + 62, 0, 65536 + 100, d, True, "f32")
    path = tmp_path / "rows.f32"
    x.tofile(path)
    ix = Multi(d, "ip", "f32", devices=[0, 0])
    with pytest.raises(Exception):
        ix.add_from_file(str(path), 0, 2 * 65536)  # shard 0's chunk reads, shard 1's runs past EOF
    assert ix.ntotal == 0 and ix.shard_rows() == [0, 0]
    ix.add(x)
    assert ix.shard_rows() == [65536, 100]
    q = O.synth_rows(O.SEED_QUERIES + 62, 0, 12, d, True, "f32")
    _exact(ix, x, q, 10, "ip")
    ix.close()


@pytest.mark.parametrize("metric,dtype,nq,k,N,d", [
    ("ip", "bf16", 64, 25, 400_000, 512),    # three shards of ~133k rows: the direct int8 screen
    ("ip", "f16", 256, 100, 300_000, 256),
    ("l2", "bf16", 40, 10, 250_000, 512),
    ("ip", "bf16", 9, 1, 200_000, 768),      # the smallest two-phase batch
])
def test_int8_two_phase_step_matches_one_index(Multi, metric, dtype, nq, k, N, d):
    # int8 screen on bf16 / f16 shards: vs_multi_search takes the two-phase step (phase A on every
    # device, the merged phase-A lists as every shard's floor, phase B, the final merge) -- the
    # answer must equal one index over all rows, bit for bit
    x = O.synth_rows(O.SEED_CORPUS + 7, 0, N, d, True, dtype)
    ix = Multi(d, metric, dtype, devices=[0, 0, 0])
    ix.add(x)
    ix.set_screen("int8")
    q = O.synth_rows(O.SEED_QUERIES + 7, 0, nq, d, True, "f32")
    for _ in range(2):  # (leased contexts reused)
        _exact(ix, x, q, k, metric)
    ix.close()


def test_int8_two_phase_concurrent_searches(Multi):
    from concurrent.futures import ThreadPoolExecutor
    N, d, k = 300_000, 512, 20
    x = O.synth_rows(O.SEED_CORPUS + 8, 0, N, d, True, "bf16")
    ix = Multi(d, "ip", "bf16", devices=[0, 0, 0])
    ix.add(x)
    ix.set_screen("int8")
    qs = [O.synth_rows(O.SEED_QUERIES + 8, 100 * t, 16 + 8 * t, d, True, "f32") for t in range(6)]
    want = [O.knn_exact(x, q, k, "ip") for q in qs]
    with ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda t: ix.search(qs[t], k), range(6)))
    for (D, I), (S, Ie) in zip(got, want):
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


def test_int8_two_phase_group_residual_small_shards(Multi):
    # cluster-sorted rows: every shard's int8 copy is coded against its group means, and each shard
    # (100k rows: under 4 tiles per workgroup) is too small for the seeded direct pass those codes
    # need -- phase A must run the native search on such a shard instead of the int8 one (a
    # per-shard choice: the exchanges stay the same), and the answer stays exact
    N, d, C, k = 300_000, 512, 32, 20
    c = O.synth_rows(O.SEED_CORPUS + 900, 0, C, d, True)
    g = O.synth_rows(O.SEED_CORPUS + 91, 0, N, d, True)
    cid = np.sort(np.random.default_rng(91).integers(0, C, N))
    x = c[cid] + np.float32(0.3) * g
    x = (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)
    qc = np.random.default_rng(92).integers(0, C, 64)
    q = c[qc] + np.float32(0.3) * O.synth_rows(O.SEED_QUERIES + 91, 0, 64, d, True)
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    ix = Multi(d, "ip", "bf16", devices=[0, 0, 0])
    ix.add(x)
    ix.set_screen("int8")
    xs = ix.reconstruct_n(0, N)
    S, Ie = O.knn_exact(xs, q, k, "ip")
    for _ in range(2):
        D, I = ix.search(q, k)
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


@pytest.mark.skipif(__import__("torch").cuda.device_count() < 2,
                    reason="needs >= 2 GPUs; the one-GPU box runs the same path with every shard on device 0")
@pytest.mark.parametrize("dtype,metric,screen", [("bf16", "ip", "int8"), ("bf16", "l2", "int8"),
                                                 ("f32", "ip", "native")])
def test_shards_on_distinct_gpus(Multi, dtype, metric, screen):
    # peer copies across physical devices both ways: the lists device g -> devices[0], the two-phase
    # floor devices[0] -> device g (int8 screen on bf16 shards)
    import torch
    G = min(torch.cuda.device_count(), 4)
    N, d = 300_000, 256
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    ix = Multi(d, metric, dtype, devices=list(range(G)))
    ix.add(x)
    ix.set_screen(screen)
    for nq, k in ((64, 20), (1, 10), (256, 100)):
        q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
        _exact(ix, x, q, k, metric)
    ix.close()
