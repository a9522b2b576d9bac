"""HNSW graph search on the GPU against oracle/hnsw_oracle.py: ids bit-exact,
scores equal to the oracle's canonical fp64 score rounded to fp32."""
import os

import numpy as np
import pytest

from oracle import hnsw_oracle as H
from oracle import oracle as O
from photo_search_engine_amd import _lib, faiss_format
from photo_search_engine_amd.hnsw import HNSWGraph
from photo_search_engine_amd.index import FlatIndex

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _index(n, d, dtype, metric, seed=11):
    ix = FlatIndex(d, metric, dtype, device=0)
    ix.add_synthetic(O.SEED_CORPUS + seed, 0, n, True)
    return ix, ix.reconstruct_n(0, n)


def _check(D, I, S_ref, I_ref):
    assert np.array_equal(I, I_ref)
    assert np.array_equal(D, S_ref.astype(np.float32))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_hnsw_search_matches_oracle(dtype, metric):
    n, d = 2500, 96
    ix, x = _index(n, d, dtype, metric)
    q = O.synth_rows(O.SEED_QUERIES + 5, 0, 24, d, True)
    assert not H.has_exact_ties(x, q, metric)
    g = H.layered_knn_graph(x, 6, metric, seed=4)
    assert g["max_level"] >= 1
    hg = HNSWGraph(ix, g)
    for k, ef in ((1, 16), (10, 16), (10, 64), (64, 40)):
        D, I = hg.search(q, k, ef)
        S_ref, I_ref = H.search(x, g, q, k, ef, metric)
        _check(D, I, S_ref, I_ref)
    hg.close()
    ix.close()


def test_hnsw_single_level_graph_and_padding():
    n, d = 300, 40
    ix, x = _index(n, d, "f32", "ip", seed=3)
    q = O.synth_rows(O.SEED_QUERIES + 9, 0, 8, d, True)
    g = H.layered_knn_graph(x, 2, "ip", seed=1, level_mult=0.0)  # 4 neighbours, one level
    hg = HNSWGraph(ix, g)
    D, I = hg.search(q, 400, 400)  # more slots than rows: the unreached ones are padded
    S_ref, I_ref = H.search(x, g, q, 400, 400, "ip")
    _check(D, I, S_ref, I_ref)
    assert (I[:, n:] == -1).all()
    # a wide beam on a connected graph is exact
    g2 = H.layered_knn_graph(x, 16, "ip", seed=2)
    hg2 = HNSWGraph(ix, g2)
    D, I = hg2.search(q, 10, 300)
    S_e, I_e = O.knn_exact(x, q, 10, "ip")
    _check(D, I, S_e, I_e)


def test_hnsw_reference_file_graph():
    """The reference's own IndexHNSWFlat file (77 rows, d=4096, M=48): GPU = oracle, and every
    stored row finds itself first (/root/reference/tests/test_vector_store.py:35-51)."""
    path = os.path.join(GOLDEN, "ref_photo_search.index")
    ff = faiss_format.read_index(path)
    g = faiss_format.read_hnsw_graph(path)
    x = np.asarray(ff.vectors, dtype=np.float32)
    ix = FlatIndex(ff.d, "ip", "f32", device=0)
    ix.add(x)
    hg = HNSWGraph(ix, g)
    D, I = hg.search(x, 5)
    S_ref, I_ref = H.search(x, g, x, 5, g["efSearch"], "ip")
    _check(D, I, S_ref, I_ref)
    assert np.array_equal(I[:, 0], np.arange(x.shape[0]))


def test_hnsw_recall_at_scale():
    n, d = 6000, 128
    ix, x = _index(n, d, "bf16", "ip", seed=21)
    q = O.synth_rows(O.SEED_QUERIES + 21, 0, 64, d, True)
    g = H.layered_knn_graph(x, 12, "ip", seed=7)
    hg = HNSWGraph(ix, g)
    _, I_e = O.knn_exact(x, q, 10, "ip")
    rec = {}
    for ef in (96, 400):
        D, I = hg.search(q, 10, ef)
        S_ref, I_ref = H.search(x, g, q, 10, ef, "ip")
        _check(D, I, S_ref, I_ref)
        rec[ef] = O.recall_at(I, I_e, 10)
    # this plain per-level k-NN graph (no neighbour diversification) on random d=128 data:
    # recall@10 0.82 at ef 96, 0.997 at ef 400 (the oracle's own numbers)
    assert rec[400] >= 0.99 and rec[96] < rec[400]


def test_hnsw_graph_validation_and_staleness():
    n, d = 200, 16
    ix, x = _index(n, d, "f32", "l2", seed=8)
    g = H.layered_knn_graph(x, 4, "l2", seed=3)
    bad = dict(g)
    bad["neighbors"] = g["neighbors"].copy()
    bad["neighbors"][0] = n + 5
    with pytest.raises(_lib.VsError):
        HNSWGraph(ix, bad)
    bad = dict(g)
    bad["max_level"] = g["max_level"] + 1
    with pytest.raises(_lib.VsError):
        HNSWGraph(ix, bad)
    # a later duplicate in a list changes no search
    dup = dict(g)
    dup["neighbors"] = g["neighbors"].copy()
    base = int(g["offsets"][5])
    dup["neighbors"][base + 1] = dup["neighbors"][base]
    hg = HNSWGraph(ix, dup)
    q = O.synth_rows(O.SEED_QUERIES + 8, 0, 6, d, True)
    D, I = hg.search(q, 5, 20)
    S_ref, I_ref = H.search(x, dup, q, 5, 20, "l2")
    _check(D, I, S_ref, I_ref)
    # rows are append-only: the graph keeps searching its own first n rows after adds (the store
    # searches the newer rows exactly and merges, test_gpu_hnsw_store.py)
    ix.add(O.synth_rows(O.SEED_CORPUS + 99, 0, 3, d, True))
    D, I = hg.search(q, 5, 20)
    _check(D, I, S_ref, I_ref)
    ix.reset()  # fewer rows than the graph covers: refused
    with pytest.raises(_lib.VsError):
        hg.search(q, 5, 20)


def test_hnsw_patch_validates_whole_lists():
    # vs_hnsw_patch takes whole (node, level) lists, each as vs_hnsw_create leaves them
    # (distinct ids, then -1s); partial lists, duplicates and ids after the terminator are refused
    # and leave the graph unchanged
    n, d = 200, 16
    ix, x = _index(n, d, "f32", "l2", seed=8)
    g = H.layered_knn_graph(x, 4, "l2", seed=3)
    hg = HNSWGraph(ix, g)
    cum = np.asarray(g["cum_nneighbor_per_level"]).astype(np.int64)
    lo = int(g["offsets"][7])
    width = int(cum[1] - cum[0])
    pos = np.arange(lo, lo + width, dtype=np.uint64)
    cur = g["neighbors"][lo:lo + width].copy()
    ep, top = int(g["entry_point"]), int(g["max_level"])
    q = O.synth_rows(O.SEED_QUERIES + 8, 0, 6, d, True)
    D0, I0 = hg.search(q, 5, 20)
    bad_dup = cur.copy()
    bad_dup[1] = bad_dup[0]
    bad_after = cur.copy()
    bad_after[1] = -1  # (ids 2.. follow the terminator)
    for p_, v_ in ((pos[:-1], cur[:-1]), (pos, bad_dup), (pos, bad_after),
                   (np.concatenate([pos, pos[:1]]), np.concatenate([cur, cur[1:2]]))):
        with pytest.raises(_lib.VsError):
            hg.patch(p_, v_, ep, top)
    D1, I1 = hg.search(q, 5, 20)
    assert np.array_equal(I0, I1) and np.array_equal(D0, D1)
    # a whole list, rewritten compacted (its last id dropped, -1 padded): accepted, and the search
    # equals the oracle's over the patched graph
    new = np.full(width, -1, dtype=np.int32)
    kept = cur[cur >= 0][:-1]
    new[:kept.shape[0]] = kept
    hg.patch(np.concatenate([pos, pos[:2]]), np.concatenate([new, new[:2]]), ep, top)  # (repeats agree)
    g2 = dict(g)
    g2["neighbors"] = g["neighbors"].copy()
    g2["neighbors"][lo:lo + width] = new
    D2, I2 = hg.search(q, 5, 20)
    S_ref, I_ref = H.search(x, g2, q, 5, 20, "l2")
    _check(D2, I2, S_ref, I_ref)
    hg.close()
    ix.close()
