"""HNSW graph build on the GPU: ``vs_hnsw_prune`` (faiss's neighbour-selection
heuristic, k_hnsw_prune) equals oracle/hnsw_oracle.py ``shrink_neighbor_list`` id for id, and the
graph ``VectorStore`` builds equals ``heuristic_graph``; graph-mode recall on clustered rows."""
import numpy as np
import pytest

from oracle import hnsw_oracle as H
from oracle import oracle as O
from photo_search_engine_amd import _lib
from photo_search_engine_amd import hnsw as hnsw_mod
from photo_search_engine_amd.index import FlatIndex
from photo_search_engine_amd.vector_store import VectorStore

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("d", [72, 100])
def test_prune_matches_oracle(dtype, metric, d):
    n = 700
    ix = FlatIndex(d, metric, dtype, device=0)
    ix.add_synthetic(O.SEED_CORPUS + 61, 0, n, True)
    x = ix.reconstruct_n(0, n)
    dist = H._distances(x, x, metric)
    rng = np.random.default_rng(d)
    m, C = 160, 48
    nodes = rng.choice(n, m, replace=False).astype(np.int64)
    cand = np.full((m, C), -1, dtype=np.int32)
    for i, v in enumerate(nodes):
        L = C if i % 5 else int(rng.integers(1, C))  # some short lists (fewer than W for a few)
        pool = np.setdiff1d(np.arange(n), [v])
        cand[i, :L] = rng.choice(pool, L, replace=False)
    for W in (1, 8, 32):
        out = hnsw_mod.prune_neighbors(ix, nodes, cand, W)
        for i, v in enumerate(nodes):
            ref = H.shrink_neighbor_list(dist, int(v), cand[i], W)
            assert out[i][out[i] >= 0].tolist() == ref, (W, i)
            assert (out[i][len(ref):] == -1).all()
    ix.close()


def test_prune_argument_checks():
    ix = FlatIndex(16, "ip", "f32", device=0)
    ix.add(O.synth_rows(O.SEED_CORPUS, 0, 10, 16, True))
    with pytest.raises(_lib.VsError):  # candidate id out of range
        hnsw_mod.prune_neighbors(ix, np.array([0]), np.array([[1, 10]]), 2)
    with pytest.raises(_lib.VsError):  # padding in the middle
        hnsw_mod.prune_neighbors(ix, np.array([0]), np.array([[1, -1, 2]]), 2)
    with pytest.raises(_lib.VsError):  # node out of range
        hnsw_mod.prune_neighbors(ix, np.array([12]), np.array([[1, 2]]), 2)
    assert hnsw_mod.prune_neighbors(ix, np.zeros(0, np.int64), np.zeros((0, 3), np.int32), 2).shape == (0, 2)
    ix.close()


def _mixture(n, d, seed, ncl=16, sigma=0.35):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((ncl, d)).astype(np.float32)
    x = centers[rng.integers(0, ncl, n)] + sigma * rng.standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_store_graph_equals_oracle_build(tmp_path, metric, monkeypatch):
    monkeypatch.setenv("VECTOR_HNSW_SEARCH", "graph")
    n, d, M, efc = 1400, 48, 6, 40
    allx = _mixture(n + 64, d, 7)
    rows, qrows = allx[:n], allx[n:]
    store = VectorStore(dimension=d, index_path=str(tmp_path / "i.index"), metadata_path=str(tmp_path / "m.json"),
                        metric=metric, index_type="hnsw", hnsw_m=M, hnsw_ef_construction=efc, hnsw_ef_search=32)
    store.add(rows, [{"photo_path": f"/p/{i}.jpg"} for i in range(n)])
    g = store._build_graph(n)
    x = store.index.reconstruct_n(0, n)
    om = "ip" if metric == "cosine" else "l2"
    ref = H.heuristic_graph(x, M, efc, om, levels=g["levels"])
    assert g["entry_point"] == ref["entry_point"] and g["max_level"] == ref["max_level"]
    assert np.array_equal(g["offsets"], ref["offsets"])
    assert np.array_equal(g["neighbors"], ref["neighbors"])
    # graph-mode recall for queries from the same mixture, efSearch 32: 0.95 in the oracle (the
    # exact per-level k-NN graph it replaces: 0.66 on the same rows)
    q = store._normalize_rows(qrows) if metric == "cosine" else qrows
    D, I = store.search_batch(q, 10)
    _, I_e = O.knn_exact(x, q, 10, om)
    assert O.recall_at(I, I_e, 10) >= 0.9


@pytest.mark.parametrize("dtype,metric,d", [("bf16", "ip", 128), ("f32", "l2", 64)])
def test_insert_rows_matches_oracle(dtype, metric, d):
    # faiss's insertion, batched (hnsw.insert_rows): the GPU graph search's efConstruction beam over
    # the old graph, the batch's exact candidates (flat search), the prune kernel and the host's
    # reverse links equal oracle/hnsw_oracle.py insert_batch batch by batch (bf16 at d=128: at d=64
    # its inner products of 2600 rows hold exact ties)
    n, n0 = 2600, 800
    ix = FlatIndex(d, metric, dtype, device=0)
    ix.add_synthetic(O.SEED_CORPUS + 71, 0, n, True)
    x = ix.reconstruct_n(0, n)
    assert not H.has_exact_ties(x, x[:50], metric)
    g0 = H.heuristic_graph(x[:n0], 8, 48, metric)
    got = hnsw_mod.insert_rows(ix, g0, n0, n, 48, lambda: FlatIndex(d, metric, dtype, device=0), batch=700)
    want = g0
    for a in range(n0, n, 700):
        want = H.insert_batch(x[:min(n, a + 700)], want, a, 48, metric)
    for key in ("levels", "offsets", "neighbors"):
        assert np.array_equal(np.asarray(got[key]), np.asarray(want[key])), key
    assert (got["entry_point"], got["max_level"]) == (want["entry_point"], want["max_level"])
    # the grown graph searches like the at-once one
    q = O.synth_rows(O.SEED_QUERIES + 71, 0, 40, d, True, "f32")
    _, I_e = O.knn_exact(x, q, 10, metric)
    g = hnsw_mod.HNSWGraph(ix, got, 128)
    _, I_g = g.search(q, 10, 128)
    assert O.recall_at(I_g, I_e, 10) >= 0.9  # oracle's own search on this graph: 0.9225 / 0.9725
    g.close()
    ix.close()


def test_store_beyond_exact_build_size_saves_ihnf(tmp_path, monkeypatch):
    from photo_search_engine_amd import faiss_format as F
    monkeypatch.setenv("VECTOR_HNSW_GRAPH_MAX_ROWS", "1000")
    n, d = 3000, 96
    ix = FlatIndex(d, "ip", "f32", device=0)
    ix.add_synthetic(O.SEED_CORPUS + 72, 0, n, False)
    X = ix.reconstruct_n(0, n)
    ix.close()
    store = VectorStore(dimension=d, index_path=str(tmp_path / "i"), metadata_path=str(tmp_path / "m"),
                        index_type="hnsw", hnsw_m=8, hnsw_ef_construction=40, hnsw_ef_search=32)
    store.add(X, [{"photo_path": f"/{i}"} for i in range(n)])
    store.save()
    assert F.read_index(str(tmp_path / "i")).kind == "hnsw"
    g = F.read_hnsw_graph(str(tmp_path / "i"))
    xs = store.index.reconstruct_n(0, n)
    want = H.insert_batch(xs, H.heuristic_graph(xs[:1000], 8, 40, "ip"), 1000, 40, "ip")
    assert np.array_equal(g["neighbors"], want["neighbors"]) and np.array_equal(g["levels"], want["levels"])
