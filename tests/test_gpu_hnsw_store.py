"""VectorStore with index_type="hnsw" and VECTOR_HNSW_SEARCH=graph: faiss's HNSW
search on the GPU over the store's graph, checked against oracle/hnsw_oracle.py."""
import json
import os
import shutil

import numpy as np
import pytest

from oracle import hnsw_oracle as H
from oracle import oracle as O
from photo_search_engine_amd import faiss_format
from photo_search_engine_amd.vector_store import VectorStore

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _store(tmp_path, d, ef=32, m=8):
    return VectorStore(dimension=d, index_path=str(tmp_path / "photo_search.index"),
                       metadata_path=str(tmp_path / "metadata.json"), metric="cosine", index_type="hnsw",
                       hnsw_m=m, hnsw_ef_construction=64, hnsw_ef_search=ef)


def test_store_graph_mode_search_save_load_add(tmp_path, monkeypatch):
    monkeypatch.setenv("VECTOR_HNSW_SEARCH", "graph")
    n, d = 1500, 64
    rows = O.synth_rows(O.SEED_CORPUS + 31, 0, n, d, False)
    store = _store(tmp_path, d)
    store.add(rows, [{"photo_path": f"/p/{i}.jpg"} for i in range(n)])
    q = O.synth_rows(O.SEED_QUERIES + 31, 0, 16, d, False)
    D, I = store.search_batch(q, 10)
    x = store.index.reconstruct_n(0, n)
    qn = store._normalize_rows(q)
    S_ref, I_ref = H.search(x, store._graph_arrays, qn, 10, 32, "ip")
    assert np.array_equal(I, I_ref) and np.array_equal(D, S_ref.astype(np.float32))
    # the reference-shaped single search takes the same path
    res = store.search(q[3].tolist(), 10)
    assert [r["metadata"]["photo_path"] for r in res] == [f"/p/{i}.jpg" for i in I[3]]
    assert [r["distance"] for r in res] == D[3].tolist()
    # save writes the graph it searched; a fresh store loads and searches it
    store.save()
    g = faiss_format.read_hnsw_graph(store.index_path)
    assert np.array_equal(g["neighbors"], store._graph_arrays["neighbors"])
    s2 = _store(tmp_path, d)
    assert s2.load()
    D2, I2 = s2.search_batch(q, 10)
    assert np.array_equal(I2, I) and np.array_equal(D2, D)
    # rows added after: the graph is rebuilt over every row
    extra = O.synth_rows(O.SEED_CORPUS + 32, 0, 200, d, False)
    s2.add(extra, [{"photo_path": f"/e/{i}.jpg"} for i in range(200)])
    D3, I3 = s2.search_batch(q, 10)
    x3 = s2.index.reconstruct_n(0, n + 200)
    assert int(np.asarray(s2._graph_arrays["levels"]).shape[0]) == n + 200
    S3, I3r = H.search(x3, s2._graph_arrays, qn, 10, 32, "ip")
    assert np.array_equal(I3, I3r) and np.array_equal(D3, S3.astype(np.float32))


def test_store_graph_mode_on_the_reference_file(tmp_path, monkeypatch):
    """The reference's own data dir (HNSW, M=48, 77 rows): graph search over the file's graph
    with the configured efSearch."""
    monkeypatch.setenv("VECTOR_HNSW_SEARCH", "graph")
    idx = tmp_path / "photo_search.index"
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index"), idx)
    shutil.copy(os.path.join(GOLDEN, "ref_photo_search.index.meta.json"), str(idx) + ".meta.json")
    (tmp_path / "metadata.json").write_text(json.dumps([{"photo_path": f"/photos/{i}.jpg"} for i in range(77)]))
    store = VectorStore(dimension=4096, index_path=str(idx), metadata_path=str(tmp_path / "metadata.json"),
                        index_type="hnsw", hnsw_m=48, hnsw_ef_construction=320, hnsw_ef_search=192)
    assert store.load()
    x = store.index.reconstruct_n(0, 77)
    g = faiss_format.read_hnsw_graph(str(idx))
    D, I = store.search_batch(x, 5)
    S_ref, I_ref = H.search(x, g, store._normalize_rows(x), 5, 192, "ip")
    assert np.array_equal(I, I_ref) and np.array_equal(D, S_ref.astype(np.float32))
    res = store.search(x[7].tolist(), 3)
    assert res[0]["metadata"]["photo_path"] == "/photos/7.jpg"
