"""HNSW graph build: the oracle's restatement of faiss's neighbour-selection
heuristic (oracle/hnsw_oracle.py ``shrink_neighbor_list`` / ``select_level``), and the host-side
bookkeeping of photo_search_engine_amd/hnsw.py ``select_level`` (reverse links, union, cut) checked
against the oracle with the GPU prune replaced by the oracle's shrink (no GPU here)."""
import numpy as np
import pytest

from oracle import hnsw_oracle as H
from oracle import oracle as O
from photo_search_engine_amd import hnsw as hnsw_mod


def test_shrink_keeps_diverse_neighbours():
    # node 0 at the origin; 1 and 2 close together on one side, 3 farther on the other side
    x = np.array([[0, 0], [1.0, 0], [1.1, 0.05], [-1.5, 0]], dtype=np.float32)
    dist = H._distances(x, x, "l2")
    assert H.shrink_neighbor_list(dist, 0, [1, 2, 3], 3) == [1, 3]  # 2 is closer to 1 than to 0
    assert H.shrink_neighbor_list(dist, 0, [1, 2, 3], 1) == [1]
    assert H.shrink_neighbor_list(dist, 0, [3, 2, 1], 4) == [1, 2, 3]  # fewer than W: all, sorted
    assert H.shrink_neighbor_list(dist, 0, [2, -1], 4) == [2]


def test_heuristic_graph_recall_beats_plain_knn_graph():
    """On clustered rows the diversified graph reaches far more of the true neighbours than the
    per-level exact k-NN graph at the same M and ef (the point of faiss's heuristic)."""
    rng = np.random.default_rng(3)
    d, n = 24, 1200
    centers = rng.standard_normal((12, d)).astype(np.float32)
    x = centers[rng.integers(0, 12, n)] + 0.35 * rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = x[rng.choice(n, 40, replace=False)] + 0.05 * rng.standard_normal((40, d)).astype(np.float32)
    _, I_e = O.knn_exact(x, q, 10, "ip")
    g_h = H.heuristic_graph(x, 4, 40, "ip")
    g_k = H.layered_knn_graph(x, 4, "ip", seed=1)
    _, I_h = H.search(x, g_h, q, 10, 24, "ip")
    _, I_k = H.search(x, g_k, q, 10, 24, "ip")
    r_h, r_k = O.recall_at(I_h, I_e, 10), O.recall_at(I_k, I_e, 10)
    assert r_h >= 0.9 and r_h > r_k + 0.1, (r_h, r_k)


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_host_select_level_matches_oracle(metric, monkeypatch):
    rng = np.random.default_rng(5)
    n, d = 300, 16
    x = rng.standard_normal((n, d)).astype(np.float32)
    dist = H._distances(x, x, metric)

    def fake_prune(index, nodes, cand, W):
        out = np.full((len(nodes), W), -1, dtype=np.int32)
        for i, v in enumerate(nodes):
            kept = H.shrink_neighbor_list(dist, int(v), cand[i], W)
            out[i, :len(kept)] = kept
        return out

    monkeypatch.setattr(hnsw_mod, "prune_neighbors", fake_prune)
    members = np.sort(rng.choice(n, 180, replace=False))
    C, W = 20, 6
    cands = []
    for i in members:
        others = members[members != i]
        cands.append(others[np.lexsort((others, dist[i, others]))[:C]])
    cand = np.array(cands, dtype=np.int32)
    cand[::7, 15:] = -1  # some short lists
    ref = H.select_level(dist, members, [c[c >= 0] for c in cand], W)
    got = hnsw_mod.select_level(None, members, cand, W)
    for j, v in enumerate(members):
        row = got[j][got[j] >= 0].tolist()
        assert row == ref[int(v)], (v, row, ref[int(v)])
    # a union cut at cmax
    ref_c = H.select_level(dist, members, [c[c >= 0] for c in cand], W, cmax=8)
    got_c = hnsw_mod.select_level(None, members, cand, W, cmax=8)
    for j, v in enumerate(members):
        assert got_c[j][got_c[j] >= 0].tolist() == ref_c[int(v)]


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_oracle_insertion_from_empty_is_the_batch_build(metric):
    # inserting every row into an empty graph (one batch: exact candidates among the batch) is the
    # at-once build
    rng = np.random.default_rng(8)
    x = rng.standard_normal((150, 10)).astype(np.float32)
    probas, cum = H._default_probas(4)
    empty = {"assign_probas": probas, "cum_nneighbor_per_level": cum, "levels": np.zeros(0, np.int32),
             "offsets": np.zeros(1, np.uint64), "neighbors": np.zeros(0, np.int32), "entry_point": -1,
             "max_level": -1, "efConstruction": 20, "efSearch": 16, "upper_beam": 1}
    a = H.insert_batch(x, empty, 0, 20, metric)
    b = H.heuristic_graph(x, 4, 20, metric)
    for key in ("levels", "offsets", "neighbors"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key
    assert (a["entry_point"], a["max_level"]) == (b["entry_point"], b["max_level"])


def test_oracle_insertion_keeps_recall():
    # a graph grown by insertions (several batches) searches as well as one built at once
    rng = np.random.default_rng(9)
    d, n = 24, 1500
    centers = rng.standard_normal((15, d)).astype(np.float32)
    x = centers[rng.integers(0, 15, n)] + 0.35 * rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    q = x[rng.choice(n, 40, replace=False)] + 0.05 * rng.standard_normal((40, d)).astype(np.float32)
    _, I_e = O.knn_exact(x, q, 10, "ip")
    g = H.heuristic_graph(x[:300], 4, 40, "ip")
    for a, b in ((300, 700), (700, 1100), (1100, n)):
        g = H.insert_batch(x[:b], g, a, 40, "ip")
    _, I_g = H.search(x, g, q, 10, 24, "ip")
    assert O.recall_at(I_g, I_e, 10) >= 0.9


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_host_insert_rows_matches_oracle(metric):
    # photo_search_engine_amd/hnsw.py insert_rows over the checker-backed index (its prune and beam
    # are the oracle's) equals the oracle's insert_batch, batch by batch
    from oracle_index import OracleFlatIndex
    rng = np.random.default_rng(10)
    x = rng.standard_normal((400, 14)).astype(np.float32)
    ix = OracleFlatIndex(14, metric)
    ix.add(x)
    g0 = H.heuristic_graph(x[:100], 6, 30, metric)
    got = hnsw_mod.insert_rows(ix, g0, 100, 400, 30, lambda: OracleFlatIndex(14, metric), batch=120)
    want = g0
    for a in (100, 220, 340):
        want = H.insert_batch(x[:min(400, a + 120)], want, a, 30, metric)
    for key in ("levels", "offsets", "neighbors"):
        assert np.array_equal(np.asarray(got[key]), np.asarray(want[key])), key
    assert (got["entry_point"], got["max_level"]) == (want["entry_point"], want["max_level"])
