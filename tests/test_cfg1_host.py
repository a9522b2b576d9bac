"""BASELINE cfg1 (N=10k, d=1536, nq=1, top-10) on the CPU: the oracle and this repo's VectorStore
host logic (over the checker-backed index) against the reference-wrapper recording
tests/golden/cfg1_wrapper_golden.npz.  The same case runs over the HIP index in
tests/test_gpu_cfg1.py."""
import numpy as np
import pytest

import cfg1_case as C
from oracle import oracle as O
from oracle_index import oracle_factory
from photo_search_engine_amd import vector_store as vsmod


@pytest.fixture(scope="module")
def data():
    return C.load_golden(), C.corpus()


def test_oracle_pinned_by_reference_wrapper_at_cfg1(data):
    # the reference wrapper normalises in numpy (utils/vector_store.py:83-90) and faiss-semantics
    # exact search follows; the oracle on the same normalised rows reproduces every recorded slice
    g, (x, q) = data
    xn = np.array([O.np_normalize_like_reference(r) for r in x], dtype=np.float32)
    qn = np.array([O.np_normalize_like_reference(r) for r in q], dtype=np.float32)
    for metric, xs, qs, nq in (("cosine", xn, qn, C.NQ), ("l2", x, q, C.NQ_L2)):
        for top_k in C.TOPKS:
            S, I = O.knn_exact(xs, qs[:nq], top_k, "ip" if metric == "cosine" else "l2")
            assert np.array_equal(I, g[f"{metric}_top{top_k}_I"])
            assert np.array_equal(S.astype(np.float32), g[f"{metric}_top{top_k}_D"])
    # the faiss fp32 restatement agrees within 1e-5 on the scores
    Df, _ = O.knn_faiss_fp32(xn, qn, 10, "ip")
    assert np.max(np.abs(Df - g["cosine_top10_D"])) < 1e-5
    np.testing.assert_array_equal(g["cosine_probe_emb"], xn[g["cosine_probe_rows"]])


@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_vector_store_host_logic_at_cfg1(data, monkeypatch, tmp_path, metric):
    monkeypatch.setattr(vsmod, "_index_factory", oracle_factory)
    g, (x, q) = data
    store = C.build_store(vsmod.VectorStore, tmp_path, metric, x)
    C.check_store(store, g, metric, q, topks=(10,))
