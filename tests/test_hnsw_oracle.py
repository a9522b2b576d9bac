"""HNSW graph-search oracle: the literal faiss array-heap restatement against
the ordered-multiset statement the HIP kernel implements, plus the reference's own HNSW file.
CPU only."""
import os

import numpy as np
import pytest

from oracle import hnsw_oracle as H
from oracle import oracle as O
from photo_search_engine_amd import faiss_format

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _data(n, d, nq, seed=3):
    x = O.synth_rows(O.SEED_CORPUS + seed, 0, n, d, True)
    q = O.synth_rows(O.SEED_QUERIES + seed, 0, nq, d, True)
    return x, q


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("M,lm", [(4, None), (8, None), (6, 0.0)])
def test_multiset_statement_equals_faiss_heaps(metric, M, lm):
    x, q = _data(500, 24, 12)
    assert not H.has_exact_ties(x, q, metric)
    g = H.layered_knn_graph(x, M, metric, seed=M, level_mult=lm)
    if lm is None:
        assert g["max_level"] >= 1  # the greedy upper-level descent is exercised
    for k, ef in ((1, 8), (10, 16), (10, 40), (50, 24)):
        S1, I1 = H.search_faiss(x, g, q, k, ef, metric)
        S2, I2 = H.search(x, g, q, k, ef, metric)
        assert np.array_equal(I1, I2), (k, ef)
        assert np.array_equal(S1, S2), (k, ef)


def test_large_ef_on_a_connected_graph_is_exact():
    x, q = _data(300, 16, 8, seed=5)
    g = H.layered_knn_graph(x, 16, "ip", seed=2)
    S, I = H.search(x, g, q, 10, 300, "ip")
    Se, Ie = O.knn_exact(x, q, 10, "ip")
    assert np.array_equal(I, Ie)
    assert np.array_equal(S, Se)


def test_fewer_reachable_rows_than_k_are_padded():
    x, q = _data(40, 8, 3, seed=7)
    g = H.layered_knn_graph(x, 2, "l2", seed=1, level_mult=0.0)
    S, I = H.search(x, g, q, 64, 64, "l2")
    S1, I1 = H.search_faiss(x, g, q, 64, 64, "l2")
    assert np.array_equal(I, I1) and np.array_equal(S, S1)
    assert (I[:, 40:] == -1).all() and (S[:, 40:] == float(np.finfo(np.float32).max)).all()


def test_reference_hnsw_file_self_queries():
    """The reference's own IndexHNSWFlat file (77 rows, d=4096, M=48, IP): every stored row finds
    itself first (the reference test's top-1 self-query, /root/reference/tests/test_vector_store.py
    :35-51), and both statements agree on the file's graph."""
    path = os.path.join(GOLDEN, "ref_photo_search.index")
    ff = faiss_format.read_index(path)
    g = faiss_format.read_hnsw_graph(path)
    x = np.asarray(ff.vectors, dtype=np.float32)
    assert g["upper_beam"] == 1 and g["entry_point"] >= 0
    S1, I1 = H.search_faiss(x, g, x, 5, g["efSearch"], "ip")
    S2, I2 = H.search(x, g, x, 5, g["efSearch"], "ip")
    assert np.array_equal(I1, I2) and np.array_equal(S1, S2)
    assert np.array_equal(I2[:, 0], np.arange(x.shape[0]))
