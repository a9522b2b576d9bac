"""Host logic of the drop-in VectorStore, replayed against the REFERENCE wrapper's recorded
behaviour (tests/golden/wrapper_golden.json.gz) over a checker-backed index (CPU only).
The same replay runs over the real HIP index in tests/test_gpu_vector_store.py."""
import os

import numpy as np
import pytest

import wrapper_replay
from oracle_index import oracle_factory
from photo_search_engine_amd import vector_store as vsmod

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SCENARIOS = wrapper_replay.load_golden()["scenarios"]


@pytest.fixture
def VS(monkeypatch):
    monkeypatch.setattr(vsmod, "_index_factory", oracle_factory)
    return vsmod.VectorStore


@pytest.mark.parametrize("scenario", SCENARIOS, ids=[s["script"]["name"] for s in SCENARIOS])
def test_reference_wrapper_replay(VS, scenario):
    wrapper_replay.replay(VS, scenario)


def test_constructor_keywords_as_main_passes_them(VS, tmp_path):
    # /root/reference/main.py:59-68 and tests/test_main.py:129-138
    store = VS(dimension=4096, index_path=str(tmp_path / "photo_search.index"),
               metadata_path=str(tmp_path / "metadata.json"), metric="cosine", index_type="flat",
               hnsw_m=32, hnsw_ef_construction=200, hnsw_ef_search=96)
    assert store.dimension == 4096 and store.meta_path.endswith("photo_search.index.meta.json")
    assert (store.metric, store.index_type, store.hnsw_m) == ("cosine", "flat", 32)
    assert store.get_total_items() == 0 and store.metadata == []


def test_loads_reference_hnsw_data_dir(VS, tmp_path):
    import shutil
    idx = tmp_path / "photo_search.index"
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index"), idx)
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index.meta.json"), str(idx) + ".meta.json")
    meta = [{"photo_path": f"/photos/{i}.jpg"} for i in range(77)]
    import json
    (tmp_path / "metadata.json").write_text(json.dumps(meta))
    store = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"),
               index_type="hnsw", hnsw_m=48, hnsw_ef_construction=320, hnsw_ef_search=192)
    assert store.load() and store.get_total_items() == 77 and store.dimension == 4096
    emb = store.get_embedding_by_photo_path("/photos/5.jpg")
    res = store.search(emb, 3)
    assert res[0]["metadata"]["photo_path"] == "/photos/5.jpg"
    # the flat config refuses the HNSW payload, like the reference's structural check
    store2 = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"))
    with pytest.raises(ValueError):
        store2.load()


def test_bulk_add_and_search_batch_match_single_item_path(VS, tmp_path):
    rng = np.random.default_rng(5)
    X = rng.standard_normal((200, 24)).astype(np.float32)
    X[3] = 0.0
    Q = rng.standard_normal((9, 24)).astype(np.float32)
    a = VS(dimension=24, index_path=str(tmp_path / "a"), metadata_path=str(tmp_path / "am"))
    b = VS(dimension=24, index_path=str(tmp_path / "b"), metadata_path=str(tmp_path / "bm"))
    for i in range(200):
        a.add_item(X[i].tolist(), {"photo_path": f"/{i}"})
    b.add(X, [{"photo_path": f"/{i}"} for i in range(200)])
    assert np.array_equal(a.index.reconstruct_n(0, 200), b.index.reconstruct_n(0, 200))
    D, I = b.search_batch(Q, 7)
    for qi in range(9):
        r = a.search(Q[qi].tolist(), 7)
        assert [x["metadata"]["photo_path"] for x in r] == [f"/{i}" for i in I[qi]]
        assert [x["distance"] for x in r] == D[qi].tolist()
    assert b.has_photo_path("/199") and b.get_embedding_by_photo_path("/3") == [0.0] * 24


def test_save_writes_reference_byte_format(VS, tmp_path):
    store = VS(dimension=8, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "meta.json"))
    store.add_item([11.0 + i for i in range(8)], {"photo_path": "/sample.jpg"})
    store.save()
    assert (tmp_path / "idx").read_bytes() == open(os.path.join(GOLDEN, "ref_build_smoke.idx"), "rb").read()
    assert (tmp_path / "idx.meta.json").read_text() == open(os.path.join(GOLDEN, "ref_build_smoke.idx.meta.json")).read()


def _full_write_bytes(tmp_path, store):
    from photo_search_engine_amd import faiss_format as F
    p = str(tmp_path / "full.bin")
    F.write_flat(p, store.index.reconstruct_n(0, store.index.ntotal), store.index.metric_type)
    return open(p, "rb").read()


def test_save_appends_new_rows_byte_identical_to_full_rewrite(VS, tmp_path, monkeypatch):
    # the indexer saves after every batch (core/indexer.py:945); rows are immutable,
    # so the second save only writes the new rows + header -- same bytes as a full rewrite
    from photo_search_engine_amd import faiss_format as F
    rng = np.random.default_rng(11)
    X = rng.standard_normal((50, 16)).astype(np.float32)
    store = VS(dimension=16, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "m.json"))
    store.add(X[:30], [{"photo_path": f"/{i}"} for i in range(30)])
    store.save()
    ino = os.stat(tmp_path / "idx").st_ino
    full_calls = []
    real_full = F.write_flat_rows
    monkeypatch.setattr(F, "write_flat_rows", lambda *a, **k: (full_calls.append(1), real_full(*a, **k)))
    for i in range(30, 50):
        store.add_item(X[i].tolist(), {"photo_path": f"/{i}"})
    store.save()
    assert full_calls == [] and os.stat(tmp_path / "idx").st_ino == ino  # appended in place
    assert (tmp_path / "idx").read_bytes() == _full_write_bytes(tmp_path, store)
    store.save()  # nothing new: header rewrite only
    assert (tmp_path / "idx").read_bytes() == _full_write_bytes(tmp_path, store)
    # reload appends too
    s2 = VS(dimension=16, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "m.json"))
    assert s2.load() and s2.get_total_items() == 50
    s2.add_item(X[0].tolist(), {"photo_path": "/again"})
    s2.save()
    assert full_calls == []
    assert (tmp_path / "idx").read_bytes() == _full_write_bytes(tmp_path, s2)


def test_save_rewrites_when_file_changed_or_cleared(VS, tmp_path, monkeypatch):
    from photo_search_engine_amd import faiss_format as F
    rng = np.random.default_rng(12)
    X = rng.standard_normal((20, 8)).astype(np.float32)
    store = VS(dimension=8, index_path=str(tmp_path / "idx"), metadata_path=str(tmp_path / "m.json"))
    store.add(X[:10], [{} for _ in range(10)])
    store.save()
    full_calls = []
    real_full = F.write_flat_rows
    monkeypatch.setattr(F, "write_flat_rows", lambda *a, **k: (full_calls.append(1), real_full(*a, **k)))
    # another writer replaced the file: full rewrite
    F.write_flat(str(tmp_path / "idx"), X[10:13], 0)
    store.add(X[10:12], [{} for _ in range(2)])
    store.save()
    assert full_calls == [1]
    assert (tmp_path / "idx").read_bytes() == _full_write_bytes(tmp_path, store)
    # clear() then re-add as many rows: the old payload must not be reused
    store.clear()
    store.add(X[5:20], [{} for _ in range(15)])
    store.save()
    assert full_calls == [1, 1]
    assert (tmp_path / "idx").read_bytes() == _full_write_bytes(tmp_path, store)
    ff = F.read_index(str(tmp_path / "idx"))
    assert np.array_equal(ff.vectors, store.index.reconstruct_n(0, 15))


def test_hnsw_store_saves_ihnf_with_heuristic_graph(VS, tmp_path):
    # index_type="hnsw" (the env templates' setting, .env.example:82-83): save() writes an IHNf file
    # the reference's faiss can read back -- same header/array layout as the reference's own
    # fixture, storage = the stored rows, graph = faiss's level draw and neighbour-selection
    # heuristic over every level's exact candidates (2M on level 0, M above)
    import json
    import shutil
    from oracle import oracle as O
    from photo_search_engine_amd import faiss_format as F
    idx = tmp_path / "photo_search.index"
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index"), idx)
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index.meta.json"), str(idx) + ".meta.json")
    (tmp_path / "metadata.json").write_text(json.dumps([{"photo_path": f"/p/{i}"} for i in range(77)]))
    store = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"),
               index_type="hnsw", hnsw_m=4, hnsw_ef_construction=320, hnsw_ef_search=192)
    assert store.load()
    ref = F.read_index(str(idx)).vectors.copy()
    store.save()
    ff = F.read_index(str(idx))
    assert ff.kind == "hnsw" and np.array_equal(ff.vectors, ref)
    g = F.read_hnsw_graph(str(idx))
    probas, cum = F.hnsw_default_probas(4)
    assert np.array_equal(g["assign_probas"], probas) and np.array_equal(g["cum_nneighbor_per_level"], cum)
    assert (g["efConstruction"], g["efSearch"], g["upper_beam"]) == (320, 192, 1)
    lev = g["levels"].astype(np.int64) - 1
    assert g["max_level"] == lev.max() >= 1 and lev[g["entry_point"]] == g["max_level"]
    assert g["entry_point"] == int(np.nonzero(lev == lev.max())[0][0])
    assert np.array_equal(np.diff(g["offsets"].astype(np.int64)), cum[g["levels"]])
    # the neighbours: faiss's heuristic over each node's exact candidates, reverse links included
    from oracle import hnsw_oracle as H
    want = H.heuristic_graph(ref, 4, 320, "ip", levels=g["levels"])
    assert np.array_equal(g["neighbors"], want["neighbors"])
    assert (g["neighbors"] >= 0).sum() > 0
    # and it loads back (graph kept on disk, exact search by default)
    s2 = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"),
            index_type="hnsw", hnsw_m=4, hnsw_ef_construction=320, hnsw_ef_search=192)
    assert s2.load() and s2.get_total_items() == 77


def test_reference_hnsw_fixture_rewrites_byte_identical(tmp_path):
    from photo_search_engine_amd import faiss_format as F
    src = os.path.join(GOLDEN, "ref_photo_search.index")
    g = F.read_hnsw_graph(src)
    ff = F.read_index(src)
    probas, cum = F.hnsw_default_probas(48)  # faiss set_default_probas, pinned by the fixture
    assert np.array_equal(g["assign_probas"], probas) and np.array_equal(g["cum_nneighbor_per_level"], cum)
    out = str(tmp_path / "rt.index")

    def rows(path, off):
        with open(path, "r+b") as f:
            f.seek(off)
            f.write(np.ascontiguousarray(ff.vectors, dtype="<f4").tobytes())

    F.write_hnsw(out, g, ff.d, ff.ntotal, ff.metric_type, rows)
    assert open(out, "rb").read() == open(src, "rb").read()


def test_flat_config_over_reference_hnsw_file_loads_and_saves_hnsw(VS, tmp_path):
    # utils/vector_store.py:125-143: a flat configuration checks only the file's metric_type, so the
    # reference's own IP HNSW file loads under a "flat" sidecar; its faiss index object stays an
    # IndexHNSWFlat, so save() writes the HNSW file back: unchanged rows -> the same bytes
    import json
    import shutil
    from photo_search_engine_amd import faiss_format as F
    idx = tmp_path / "photo_search.index"
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index"), idx)
    meta = json.load(open(os.path.join(GOLDEN, "ref_photo_search.index.meta.json")))
    meta["index_type"] = "flat"
    (tmp_path / "photo_search.index.meta.json").write_text(json.dumps(meta))
    (tmp_path / "metadata.json").write_text(json.dumps([{"photo_path": f"/p/{i}"} for i in range(77)]))
    store = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"))
    assert store.load() and store.get_total_items() == 77
    ref = F.read_index(str(idx)).vectors.copy()
    res = store.search(ref[5].tolist(), 3)  # exact search: a stored row finds itself first
    assert res[0]["metadata"] == {"photo_path": "/p/5"}
    before = open(idx, "rb").read()
    store.save()
    assert open(idx, "rb").read() == before
    assert json.load(open(str(idx) + ".meta.json"))["index_type"] == "flat"
    # a row added after the load is inserted into the file's graph (its M = 48, its efConstruction)
    store.add_item([float(v) for v in ref[3]], {"photo_path": "/p/new"})
    store.save()
    ff = F.read_index(str(idx))
    g = F.read_hnsw_graph(str(idx))
    assert ff.kind == "hnsw" and ff.ntotal == 78 and g["levels"].shape[0] == 78
    probas, cum = F.hnsw_default_probas(48)
    assert np.array_equal(g["cum_nneighbor_per_level"], cum) and g["efConstruction"] == 320
    s2 = VS(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"))
    assert s2.load() and s2.get_total_items() == 78
    # clear() starts a flat index again (the reference's clear() creates a fresh flat index)
    s2.clear()
    s2.add_item([float(v) for v in ref[0]], {"photo_path": "/p/0"})
    s2.save()
    assert F.read_index(str(idx)).kind == "flat"


def test_hnsw_store_beyond_exact_build_inserts_and_saves_ihnf(VS, tmp_path, monkeypatch):
    # every size saves an IHNf file (rollback to the reference's faiss): the first
    # VECTOR_HNSW_GRAPH_MAX_ROWS rows get the exact-candidate build, the rest are inserted the way
    # faiss's IndexHNSWFlat.add does (batched), and each later save inserts only the new rows
    from oracle import hnsw_oracle as H
    from photo_search_engine_amd import faiss_format as F
    monkeypatch.setenv("VECTOR_HNSW_GRAPH_MAX_ROWS", "50")
    rng = np.random.default_rng(3)
    X = rng.standard_normal((170, 12)).astype(np.float32)
    kw = dict(index_path=str(tmp_path / "i"), metadata_path=str(tmp_path / "m"), index_type="hnsw", hnsw_m=4,
              hnsw_ef_construction=24, hnsw_ef_search=16)
    store = VS(dimension=12, **kw)
    store.add(X[:130], [{"photo_path": f"/{i}"} for i in range(130)])
    store.save()
    assert F.read_index(str(tmp_path / "i")).kind == "hnsw"
    g = F.read_hnsw_graph(str(tmp_path / "i"))
    xs = store.index.reconstruct_n(0, 130)
    want = H.insert_batch(xs, H.heuristic_graph(xs[:50], 4, 24, "ip"), 50, 24, "ip")
    for key in ("levels", "offsets", "neighbors"):
        assert np.array_equal(np.asarray(g[key]), np.asarray(want[key])), key
    assert (g["entry_point"], g["max_level"]) == (want["entry_point"], want["max_level"])
    # the next batch of the indexer: only the new rows are inserted
    store.add(X[130:], [{"photo_path": f"/{i}"} for i in range(130, 170)])
    store.save()
    g2 = F.read_hnsw_graph(str(tmp_path / "i"))
    want2 = H.insert_batch(store.index.reconstruct_n(0, 170), want, 130, 24, "ip")
    assert np.array_equal(g2["neighbors"], want2["neighbors"]) and np.array_equal(g2["levels"], want2["levels"])
    # reload (graph mode keeps the file's graph) and grow again: the loaded graph is extended
    monkeypatch.setenv("VECTOR_HNSW_SEARCH", "graph")
    s2 = VS(dimension=12, **kw)
    assert s2.load() and s2.get_total_items() == 170
    s2.add(X[:5] * 2.0, [{"photo_path": f"/x{i}"} for i in range(5)])
    s2.save()
    g3 = F.read_hnsw_graph(str(tmp_path / "i"))
    want3 = H.insert_batch(s2.index.reconstruct_n(0, 175), want2, 170, 24, "ip")
    assert np.array_equal(g3["neighbors"], want3["neighbors"])


@pytest.mark.parametrize("d", [8, 1536, 4096])
def test_query_normalisation_skips_list_round_trip_bit_identically(d):
    # search() normalises its query as an array; the bits must equal the reference's
    # np.array([_normalize_vector(v)], dtype="float32") (utils/vector_store.py:83-90,189-191)
    store = vsmod.VectorStore.__new__(vsmod.VectorStore)
    store._normalize = True
    rng = np.random.default_rng(d)
    cases = [(rng.standard_normal(d) * s).astype(np.float32).tolist() for s in (1e-3, 1.0, 7.5, 1e3)]
    cases.append([0.0] * d)
    for v in cases:
        want = np.array([store._normalize_vector(v)], dtype="float32")
        got = store._normalize_query(v)
        assert got.shape == want.shape and got.tobytes() == want.tobytes()


@pytest.mark.parametrize("normalize", [True, False])
@pytest.mark.parametrize("d", [8, 1536])
def test_query_normalisation_float64_and_l2_bit_identical(d, normalize):
    # float64 lists / arrays and the l2 store (no normalisation) take the same fp32 bits as the
    # reference's np.array([_normalize_vector(v)], dtype="float32")
    store = vsmod.VectorStore.__new__(vsmod.VectorStore)
    store._normalize = normalize
    rng = np.random.default_rng(d + 1)
    for s in (1e-3, 1.0, 3e2):
        v64 = rng.standard_normal(d) * s
        for v in (v64.tolist(), v64, v64.astype(np.float32)):
            want = np.array([store._normalize_vector(v)], dtype="float32")
            got = store._normalize_query(v)
            assert got.shape == want.shape and got.tobytes() == want.tobytes()


@pytest.mark.parametrize("normalize", [True, False])
def test_query_list_conversion_edge_values_bit_identical(normalize):
    # the struct fast path of a list query: subnormals, fp64 values between fp32 neighbours (round
    # to nearest even), values beyond the fp32 range (numpy: inf -- the fallback), ints, bools,
    # numpy scalars and strings of numbers (numpy parses them -- the fallback) give the reference's bits
    store = vsmod.VectorStore.__new__(vsmod.VectorStore)
    store._normalize = normalize
    rng = np.random.default_rng(9)
    base = (rng.standard_normal(64) * 1e-3).tolist()
    cases = [
        base,
        [1e-45, 3e-41, -2e-40] + base[3:],
        [1.0 + 2.0 ** -24, 1.0 + 3 * 2.0 ** -25, -(1.0 + 2.0 ** -24)] + base[3:],
        [3.5e38, -1e39] + base[2:],
        [1, 2, True] + base[3:],
        [np.float32(0.5), np.float64(0.25), np.int64(3)] + base[3:],
        ["1.5", "-2"] + base[2:],
    ]
    for v in cases:
        with np.errstate(all="ignore"):
            want = np.array([store._normalize_vector(v)], dtype="float32")
            got = store._normalize_query(v)
        assert got.shape == want.shape and got.tobytes() == want.tobytes(), v[:3]


def test_query_with_extra_axis_is_rejected_like_the_reference():
    # a (d, 1) array passes the reference's len() check but its np.array([...]) is 3-D, which the
    # index rejects; it must not be silently flattened into a valid (1, d) query
    store = vsmod.VectorStore.__new__(vsmod.VectorStore)
    for normalize in (True, False):
        store._normalize = normalize
        q = store._normalize_query(np.ones((8, 1), dtype=np.float32))
        assert q.ndim != 2 or q.shape[0] != 1


def test_graph_tail_merge_matches_oracle_merge():
    """graph mode's merge of the graph's results with the exactly searched tail (rows added behind
    the graph): the same top-k as the oracle's shard merge, ties to the lower id, padding last."""
    from oracle import oracle as O
    from photo_search_engine_amd.vector_store import _merge_topk

    rng = np.random.default_rng(5)
    nq, k = 7, 6
    for metric in ("ip", "l2"):
        S1 = np.sort(rng.integers(0, 9, (nq, k)).astype(np.float64), axis=1)
        S2 = np.sort(rng.integers(0, 9, (nq, k)).astype(np.float64), axis=1)
        if metric == "ip":
            S1, S2 = S1[:, ::-1].copy(), S2[:, ::-1].copy()
        I1 = rng.permutation(50)[: nq * k].reshape(nq, k).astype(np.int64)
        I2 = 50 + rng.permutation(50)[: nq * k].reshape(nq, k).astype(np.int64)
        # keep each list sorted by (score, id) as both searches return it
        for S, I in ((S1, I1), (S2, I2)):
            for r in range(nq):
                o = np.lexsort((I[r], -S[r] if metric == "ip" else S[r]))
                S[r], I[r] = S[r][o], I[r][o]
        Sr, Ir = O.merge_topk(np.stack([S1, S2]), np.stack([I1, I2]), k, metric)
        D, I = _merge_topk(S1.astype(np.float32), I1, S2.astype(np.float32), I2, k, metric == "ip")
        assert np.array_equal(I, Ir) and np.array_equal(D, Sr.astype(np.float32))
    # a short tail (fewer rows than k) and faiss padding
    D, I = _merge_topk(np.array([[3.0, 1.0]], np.float32), np.array([[4, -1]]), np.array([[2.0]], np.float32),
                       np.array([[9]]), 3, True)
    assert I.tolist() == [[4, 9, -1]] and D[0, :2].tolist() == [3.0, 2.0]
