"""The IVF-Flat oracle (oracle/ivf_oracle.py) on the CPU: it reduces to the flat oracle when every
list is probed, probes only the chosen lists otherwise, and keeps the flat tie rule."""
import numpy as np

from oracle import ivf_oracle as IO
from oracle import oracle as O


def _setup(N=3000, d=24, nlist=12, metric="ip"):
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    c = IO.sample_centroids(x, nlist, 4)
    return x, c, IO.assign(x, c, metric)


def test_assign_is_the_exact_best_centroid():
    x, c, lists = _setup()
    S = O.np_canon_scores(c, x[:50], "ip")
    np.testing.assert_array_equal(lists[:50], np.argmax(S, axis=1))
    # every centroid is one of the rows: that row lands in its own list
    assert set(lists.tolist()) == set(range(12))


def test_all_lists_probed_equals_flat():
    for metric in ("ip", "l2"):
        x, c, lists = _setup(metric=metric)
        q = O.synth_rows(O.SEED_QUERIES, 0, 7, x.shape[1], True, "f32")
        S, I = IO.search(x, np.arange(x.shape[0]), lists, c, q, 15, c.shape[0], metric)
        Se, Ie = O.knn_exact(x, q, 15, metric)
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(S, Se)


def test_one_probe_returns_rows_of_that_list_only_and_pads():
    x, c, lists = _setup()
    q = O.synth_rows(O.SEED_QUERIES, 3, 5, x.shape[1], True, "f32")
    P = IO.probe(q, c, 1)
    S, I = IO.search(x, np.arange(x.shape[0]), lists, c, q, 2000, 1)
    for a in range(q.shape[0]):
        got = I[a][I[a] >= 0]
        assert (lists[got] == P[a, 0]).all()
        assert got.size == (lists == P[a, 0]).sum()
        assert (S[a][I[a] < 0] == -np.inf).all()


def test_ties_go_to_lower_id():
    rng = np.random.default_rng(0)
    base = rng.standard_normal((20, 8)).astype(np.float32)
    x = np.concatenate([base, base[4:5], base[4:5]], axis=0)
    c = base[:4].copy()
    lists = IO.assign(x, c, "l2")
    S, I = IO.search(x, np.arange(x.shape[0]), lists, c, base[4:5], 3, 4, "l2")
    assert list(I[0]) == [4, 20, 21]


def test_assign_ip_fast_equals_canonical_assign():
    # the fp32-GEMM shortcut with its rigorous gap test must reproduce the canonical assignment,
    # including rows exactly or nearly tied between two centroids (resolved canonically)
    x = O.synth_rows(O.SEED_CORPUS, 0, 4000, 64, True, "f32")
    c = IO.sample_centroids(x, 40, 6)
    c[1] = c[0]  # an exact centroid tie: ties -> lower list id
    c[3] = c[2] + np.float32(1e-7)
    mid = (c[5] + c[6]) / 2
    x[:50] = mid / np.linalg.norm(mid)  # rows equidistant from two centroids
    np.testing.assert_array_equal(IO.assign_ip_fast(x, c, chunk=1000), IO.assign(x, c, "ip"))
