"""BASELINE cfg1 through the drop-in ``VectorStore`` over the HIP index (libvs.so), MI355X only.

* cfg1_wrapper_golden.npz (the reference wrapper run on the same raw rows, tests/golden/
  make_goldens.py): 10k x 1536 rows (bulk ``add`` + ``add_item``), one query per ``search`` call,
  top_k 10 / 1 / 50: ids and distances equal to the recording, both metrics, every screen; the
  probe embeddings; the saved index file's sha256; VECTOR_DTYPE=bf16 against the oracle slice.
* oracle_golden.npz (the canonical oracle at the cfg1 shape, 64 queries, top-100): the index layer
  bit-exact on its ip / bf16 / l2 slices, one query per call and batched.
"""
import os

import numpy as np
import pytest

import cfg1_case as C
from photo_search_engine_amd import vector_store as vsmod

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    return C.load_golden(), C.corpus()


@pytest.fixture(autouse=True)
def hip_factory():
    assert vsmod._index_factory is vsmod._default_index_factory  # the HIP index, no substitute


@pytest.mark.parametrize("screen", ["native", "int8"])
@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_vector_store_cfg1_matches_reference_wrapper(data, monkeypatch, tmp_path, metric, screen):
    monkeypatch.setenv("VECTOR_SCREEN", screen)
    g, (x, q) = data
    store = C.build_store(vsmod.VectorStore, tmp_path, metric, x)
    C.check_store(store, g, metric, q)
    # reload from the saved file (streamed file -> HBM) and search again
    s2 = vsmod.VectorStore(dimension=C.D, index_path=store.index_path, metadata_path=store.metadata_path,
                           metric=metric)
    assert s2.load() and s2.get_total_items() == C.N
    C.check_store(s2, g, metric, q, topks=(10,), files=False)
    store.index.close()
    s2.index.close()


@pytest.mark.parametrize("screen", ["native", "int8"])
def test_vector_store_cfg1_bf16_rows(data, monkeypatch, tmp_path, screen):
    monkeypatch.setenv("VECTOR_DTYPE", "bf16")
    monkeypatch.setenv("VECTOR_SCREEN", screen)
    g, (x, q) = data
    store = C.build_store(vsmod.VectorStore, tmp_path, "cosine", x)
    C.check_store(store, g, "cosine", q, prefix="cosine_bf16", topks=(10,), files=False)
    store.index.close()


@pytest.mark.parametrize("dtype,slice_,metric", [("f32", "ip", "ip"), ("bf16", "bf16", "ip"), ("f32", "l2", "l2")])
def test_index_layer_oracle_golden_cfg1_shape(golden_dir, dtype, slice_, metric):
    from oracle import oracle as O
    from photo_search_engine_amd.index import FlatIndex
    g = np.load(os.path.join(golden_dir, "oracle_golden.npz"))
    N, d = int(g["N"]), int(g["d"])
    S, I = g[f"{slice_}_S"], g[f"{slice_}_I"].astype(np.int64)
    nq, k = I.shape
    ix = FlatIndex(d, metric, dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)  # the golden's rows, generated on the device
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    for screen in ("native", "int8"):
        ix.set_screen(screen)
        Db, Ib = ix.search(q, k)  # batched
        np.testing.assert_array_equal(Ib, I)
        np.testing.assert_array_equal(Db, S.astype(np.float32))
        for a in range(0, nq, 7):  # one query per call (the product's nq = 1)
            D1, I1 = ix.search(q[a:a + 1], k)
            np.testing.assert_array_equal(I1[0], I[a])
            np.testing.assert_array_equal(D1[0], S[a].astype(np.float32))
    ix.close()
