"""Generate the committed golden fixtures under tests/golden/ (run in the dev container only).

  python tests/golden/make_goldens.py

1. wrapper_golden.json -- behaviour of the REFERENCE ``VectorStore``
   (/root/reference/utils/vector_store.py, imported from its file) on scripted scenarios taken
   from the reference's own tests (tests/test_vector_store.py, tests/test_searcher.py:293-406,
   tests/helpers.py FakeEmbeddingService) plus seeded random cases.  faiss is not installed in
   this image, so a stand-in ``faiss`` module is placed on sys.path for the import; its search is
   the oracle's exact canonical search (oracle/oracle.py) and its file I/O writes faiss' flat
   format.  What the fixture pins is the reference WRAPPER's behaviour around the arithmetic:
   normalisation bits, k clamping, -1 filtering, result layout, error types and messages,
   sidecar JSON and the index file bytes.
3. cfg1_wrapper_golden.npz -- BASELINE cfg1 (N=10k, d=1536, one query per call, top-10) through the
   reference wrapper imported the same way (``make_cfg1_golden``).
2. oracle_golden.npz -- exact top-k (ids + fp64 scores + fp64 rank gaps) of the canonical oracle on
   cfg1-shaped synthetic data (N=10k, d=1536), cross-checked against the numpy twin and the faiss
   fp32 restatement at generation time.  Pins the oracle against regressions; the corpus itself
   is regenerated from the counter hash, not committed.

The reference's source is read here only to import it; nothing of it is copied into the fixtures.
"""
from __future__ import annotations

import gzip
import importlib.util
import json
import os
import shutil
import sys
import tempfile
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402
from photo_search_engine_amd import faiss_format  # noqa: E402

STANDIN = r'''
"""Stand-in for faiss (NOT faiss): exact canonical search from the repo oracle, faiss flat file
format.  Exists only so /root/reference/utils/vector_store.py can be imported to record goldens."""
import numpy as np
from oracle import oracle as _O
from photo_search_engine_amd import faiss_format as _F

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1


class _Flat:
    def __init__(self, d, metric_type):
        self.d = int(d)
        self.metric_type = metric_type
        self._parts = []
        self._cat = np.zeros((0, self.d), dtype=np.float32)
        self.is_trained = True

    @property
    def _x(self):
        if self._parts:  # appends are amortised: one concatenation per search / reconstruct
            self._cat = np.concatenate([self._cat] + self._parts, axis=0)
            self._parts = []
        return self._cat

    @property
    def ntotal(self):
        return int(self._cat.shape[0]) + sum(int(p.shape[0]) for p in self._parts)

    def add(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.ndim == 2 and x.shape[1] == self.d
        self._parts.append(x.copy())

    def search(self, q, k):
        q = np.ascontiguousarray(q, dtype=np.float32)
        if k <= 0:
            raise RuntimeError("Error in search: k > 0 failed")
        x = self._x
        # the C oracle and its numpy twin are the same canonical expression tree (tests/test_oracle.py);
        # the twin is kept for the small scenarios, the C form for cfg1-sized corpora
        knn = _O.knn_exact if x.shape[0] * q.shape[0] > 200000 else _O.np_knn_exact
        S, I = knn(x, q, int(k), "ip" if self.metric_type == 0 else "l2")
        D = S.astype(np.float32)
        D[I < 0] = -3.4028235e38 if self.metric_type == 0 else 3.4028235e38
        return D, I

    def reconstruct(self, i):
        return self._x[int(i)].copy()


class IndexFlatIP(_Flat):
    def __init__(self, d):
        super().__init__(d, METRIC_INNER_PRODUCT)


class IndexFlatL2(_Flat):
    def __init__(self, d):
        super().__init__(d, METRIC_L2)


class _HNSWParams:
    efConstruction = 40
    efSearch = 16


class IndexHNSWFlat(_Flat):
    def __init__(self, d, m, metric_type=METRIC_L2):
        super().__init__(d, metric_type)
        self.hnsw = _HNSWParams()


def write_index(index, path):
    _F.write_flat(path, index._x, index.metric_type)
    if isinstance(index, IndexHNSWFlat):
        with open(path + ".standin-hnsw", "w") as f:
            f.write("1")


def read_index(path):
    import os
    ff = _F.read_index(path)
    if os.path.exists(path + ".standin-hnsw"):
        idx = IndexHNSWFlat(ff.d, 16, ff.metric_type)
    elif ff.metric_type == 0:
        idx = IndexFlatIP(ff.d)
    else:
        idx = IndexFlatL2(ff.d)
    if ff.ntotal:
        idx.add(np.asarray(ff.vectors))
    return idx
'''


def fake_embedding(text: str, dimension: int = 8):
    """tests/helpers.py:10-12 behaviour: seed = sum(ord) % 13, vector = [seed + i]."""
    seed = float(sum(ord(char) for char in (text or "")) % 13)
    return [seed + float(index) for index in range(dimension)]


def import_reference_vector_store(tmp: str):
    pkg = os.path.join(tmp, "faiss")
    os.makedirs(pkg, exist_ok=True)
    with open(os.path.join(pkg, "__init__.py"), "w") as f:
        f.write(STANDIN)
    sys.path.insert(0, tmp)
    spec = importlib.util.spec_from_file_location("ref_vector_store", os.path.join(REF, "utils", "vector_store.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def rec_results(results):
    return [{"metadata": r["metadata"], "distance": r["distance"]} for r in results]


def run_op(store, op):
    """Execute one scripted op on a store; return a JSON-able record of what happened."""
    kind = op["op"]
    try:
        if kind == "add_item":
            store.add_item(op["embedding"], op["metadata"])
            out = None
        elif kind == "search":
            out = rec_results(store.search(op["query"], op["top_k"]))
        elif kind == "get_embedding":
            out = store.get_embedding_by_photo_path(op["photo_path"])
        elif kind == "has_photo_path":
            out = store.has_photo_path(op["photo_path"])
        elif kind == "total":
            out = store.get_total_items()
        elif kind == "save":
            store.save()
            out = None
        elif kind == "load":
            out = store.load()
        elif kind == "clear":
            store.clear()
            out = None
        elif kind == "dimension":
            out = store.dimension
        elif kind == "write_file":
            with open(os.path.join(op["dir"], op["name"]), "w", encoding="utf-8") as f:
                f.write(op["text"])
            out = None
        else:
            raise AssertionError(kind)
        return {"ok": True, "out": out}
    except Exception as e:  # record error type + message
        return {"ok": False, "error": type(e).__name__, "message": str(e)}


def scenarios():
    """Scripted scenarios; {dir} in paths is substituted per run."""
    sc = []
    # --- reference tests/test_vector_store.py behaviours at several dimensions
    for d in (8, 768, 1536, 4096):
        sc.append({"name": f"add_search_self_d{d}", "ctor": {"dimension": d}, "ops": [
            {"op": "add_item", "embedding": [0.1] * d, "metadata": {"id": 1, "photo": "test1.jpg"}},
            {"op": "add_item", "embedding": [0.5] * d, "metadata": {"id": 2, "photo": "test2.jpg"}},
            {"op": "search", "query": [0.1] * d, "top_k": 1},
            {"op": "search", "query": [0.5] * d, "top_k": 2},
        ]})
        ops = [{"op": "add_item", "embedding": [i * 0.1] * d, "metadata": {"id": i}} for i in range(10)]
        ops += [{"op": "search", "query": [0.1] * d, "top_k": 5}, {"op": "search", "query": [0.1] * d, "top_k": 50},
                {"op": "total"}]
        sc.append({"name": f"topk_clamp_zero_vector_d{d}", "ctor": {"dimension": d}, "ops": ops})
        sc.append({"name": f"embedding_by_path_d{d}", "ctor": {"dimension": d}, "ops": [
            {"op": "add_item", "embedding": [0.1] * d, "metadata": {"photo_path": "/a.jpg"}},
            {"op": "add_item", "embedding": [0.2] * d, "metadata": {"photo_path": "/b.jpg"}},
            {"op": "get_embedding", "photo_path": "/b.jpg"},
            {"op": "get_embedding", "photo_path": "/missing.jpg"},
            {"op": "has_photo_path", "photo_path": "/a.jpg"},
        ]})
    # --- errors
    sc.append({"name": "errors", "ctor": {"dimension": 8}, "ops": [
        {"op": "search", "query": [0.1] * 8, "top_k": 10},
        {"op": "add_item", "embedding": [0.1] * 8, "metadata": {"id": 1}},
        {"op": "add_item", "embedding": [0.1] * 9, "metadata": {"id": 2}},
        {"op": "search", "query": [0.1] * 9, "top_k": 1},
        {"op": "add_item", "embedding": None, "metadata": {"id": 3}},
        {"op": "search", "query": [0.3] * 8, "top_k": 0},
        {"op": "total"},
    ]})
    sc.append({"name": "bad_metric", "ctor": {"dimension": 8, "metric": "dot"}, "ops": []})
    sc.append({"name": "bad_index_type", "ctor": {"dimension": 8, "index_type": "ivf"}, "ops": []})
    sc.append({"name": "lazy_dimension", "ctor": {"dimension": None}, "ops": [
        {"op": "search", "query": [1.0] * 6, "top_k": 3},
        {"op": "total"},
        {"op": "add_item", "embedding": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0], "metadata": {"id": 0}},
        {"op": "dimension"},
        {"op": "search", "query": [1.0] * 6, "top_k": 3},
    ]})
    # --- FakeEmbeddingService corpora (tests/test_searcher.py:293-406 shapes)
    texts = [f"图片 {i}" for i in range(12)] + ["雪后松树", "上传图片", "photo 图片 1"]
    ops = []
    for i, t in enumerate(texts):
        ops.append({"op": "add_item", "embedding": fake_embedding(t), "metadata": {"photo_path": f"/p{i}.jpg", "t": t}})
    for qt in ("图片 1", "上传图片 photo", "雪", "xyz", "photo 图片 1 上传图片"):
        for k in (1, 3, 5, 20):
            ops.append({"op": "search", "query": fake_embedding(qt), "top_k": k})
    ops.append({"op": "get_embedding", "photo_path": "/p3.jpg"})
    sc.append({"name": "fake_embedding_corpus", "ctor": {"dimension": 8}, "ops": ops})
    sc.append({"name": "exact_ties_dup", "ctor": {"dimension": 8}, "ops": [
        {"op": "add_item", "embedding": [1.0] * 8, "metadata": {"photo_path": "/q.jpg"}},
        {"op": "add_item", "embedding": [0.9] * 8, "metadata": {"photo_path": "/dup.jpg", "v": "a"}},
        {"op": "add_item", "embedding": [0.9] * 8, "metadata": {"photo_path": "/dup.jpg", "v": "b"}},
        {"op": "add_item", "embedding": [0.8] * 8, "metadata": {"photo_path": "/other.jpg"}},
        {"op": "search", "query": [1.0] * 8, "top_k": 4},
        {"op": "search", "query": [1.0] * 8, "top_k": 2},
        {"op": "get_embedding", "photo_path": "/dup.jpg"},
    ]})
    sc.append({"name": "self_exclusion_shape", "ctor": {"dimension": 8}, "ops": [
        {"op": "add_item", "embedding": [float(i + o) for o in range(8)], "metadata": {"photo_path": f"/photo_{i}.jpg"}}
        for i in range(3)] + [{"op": "search", "query": [float(o) for o in range(8)], "top_k": 3}]})
    # --- seeded random corpora, both metrics
    rng = np.random.default_rng(20260417)
    for metric in ("cosine", "l2"):
        for d in (16, 100):
            X = rng.standard_normal((300, d)).astype(np.float32)
            Q = rng.standard_normal((12, d)).astype(np.float32)
            ops = [{"op": "add_item", "embedding": [float(v) for v in X[i]], "metadata": {"row": i}}
                   for i in range(X.shape[0])]
            for qi in range(Q.shape[0]):
                ops.append({"op": "search", "query": [float(v) for v in Q[qi]], "top_k": 10})
            ops.append({"op": "search", "query": [float(v) for v in X[7]], "top_k": 3})
            sc.append({"name": f"random_{metric}_d{d}", "ctor": {"dimension": d, "metric": metric}, "ops": ops})
    # --- persistence
    d = 8
    ops = [{"op": "add_item", "embedding": fake_embedding(f"photo {i}"), "metadata": {"photo_path": f"/x{i}.jpg", "i": i}}
           for i in range(5)]
    ops += [{"op": "save"}, {"op": "search", "query": fake_embedding("photo 2"), "top_k": 3}]
    sc.append({"name": "save_load", "ctor": {"dimension": d}, "ops": ops, "reload": [
        {"op": "load"}, {"op": "total"}, {"op": "dimension"}, {"op": "has_photo_path", "photo_path": "/x3.jpg"},
        {"op": "search", "query": fake_embedding("photo 2"), "top_k": 3},
        {"op": "get_embedding", "photo_path": "/x4.jpg"},
    ]})
    sc.append({"name": "save_load_hnsw", "ctor": {"dimension": d, "index_type": "hnsw", "hnsw_m": 16,
                                                  "hnsw_ef_construction": 80, "hnsw_ef_search": 48},
               "ops": [{"op": "add_item", "embedding": [0.1] * d, "metadata": {"photo_path": "/a.jpg", "id": 1}},
                       {"op": "add_item", "embedding": [0.2] * d, "metadata": {"photo_path": "/b.jpg", "id": 2}},
                       {"op": "save"}],
               "reload": [{"op": "load"}, {"op": "total"}, {"op": "has_photo_path", "photo_path": "/b.jpg"}]})
    sc.append({"name": "load_missing", "ctor": {"dimension": d}, "ops": [{"op": "load"}]})
    sc.append({"name": "load_metadata_mismatch", "ctor": {"dimension": d},
               "ops": [{"op": "add_item", "embedding": [0.1] * d, "metadata": {"id": 1}}, {"op": "save"},
                       {"op": "write_file", "dir": "{dir}", "name": "metadata.json", "text": "[]"}],
               "reload": [{"op": "load"}]})
    sc.append({"name": "load_meta_missing", "ctor": {"dimension": d},
               "ops": [{"op": "add_item", "embedding": [0.1] * d, "metadata": {"id": 1}}, {"op": "save"},
                       {"op": "write_file", "dir": "{dir}", "name": "index.bin.meta.json", "text": "[1, 2]"}],
               "reload": [{"op": "load"}]})
    sc.append({"name": "load_metric_mismatch", "ctor": {"dimension": d},
               "ops": [{"op": "add_item", "embedding": [0.1] * d, "metadata": {"id": 1}}, {"op": "save"}],
               "reload_ctor": {"dimension": d, "metric": "l2"}, "reload": [{"op": "load"}]})
    sc.append({"name": "load_type_mismatch", "ctor": {"dimension": d},
               "ops": [{"op": "add_item", "embedding": [0.1] * d, "metadata": {"id": 1}}, {"op": "save"}],
               "reload_ctor": {"dimension": d, "index_type": "hnsw"}, "reload": [{"op": "load"}]})
    # --- the file's structure and metric against the configuration (utils/vector_store.py:125-143):
    # a sidecar rewritten so it matches the configuration while the file does not
    meta = lambda it, m: json.dumps({"index_type": it, "metric": m, "dimension": d, "hnsw_m": 32,  # noqa: E731
                                     "hnsw_ef_construction": 200, "hnsw_ef_search": 96})
    two = [{"op": "add_item", "embedding": fake_embedding("photo a"), "metadata": {"photo_path": "/a.jpg"}},
           {"op": "add_item", "embedding": fake_embedding("photo bb"), "metadata": {"photo_path": "/b.jpg"}},
           {"op": "add_item", "embedding": fake_embedding("photo ccc"), "metadata": {"photo_path": "/c.jpg"}}]
    probe = [{"op": "total"}, {"op": "search", "query": fake_embedding("photo bb"), "top_k": 3},
             {"op": "has_photo_path", "photo_path": "/c.jpg"}]
    sc.append({"name": "load_hnsw_sidecar_over_flat_file", "ctor": {"dimension": d},
               "ops": two + [{"op": "save"}, {"op": "write_file", "dir": "{dir}", "name": "index.bin.meta.json",
                                              "text": meta("hnsw", "cosine")}],
               "reload_ctor": {"dimension": d, "index_type": "hnsw"}, "reload": [{"op": "load"}] + probe})
    sc.append({"name": "load_flat_sidecar_over_hnsw_file_ip", "ctor": {"dimension": d, "index_type": "hnsw"},
               "ops": two + [{"op": "save"}, {"op": "write_file", "dir": "{dir}", "name": "index.bin.meta.json",
                                              "text": meta("flat", "cosine")}],
               "reload_ctor": {"dimension": d}, "reload": [{"op": "load"}] + probe})
    sc.append({"name": "load_flat_sidecar_over_hnsw_file_l2_mismatch", "ctor": {"dimension": d, "index_type": "hnsw",
                                                                                "metric": "l2"},
               "ops": two + [{"op": "save"}, {"op": "write_file", "dir": "{dir}", "name": "index.bin.meta.json",
                                              "text": meta("flat", "cosine")}],
               "reload_ctor": {"dimension": d}, "reload": [{"op": "load"}]})
    sc.append({"name": "load_hnsw_config_file_metric_unchecked", "ctor": {"dimension": d, "index_type": "hnsw",
                                                                          "metric": "l2"},
               "ops": two + [{"op": "save"}, {"op": "write_file", "dir": "{dir}", "name": "index.bin.meta.json",
                                              "text": meta("hnsw", "cosine")}],
               "reload_ctor": {"dimension": d, "index_type": "hnsw"}, "reload": [{"op": "load"}] + probe})
    sc.append({"name": "clear", "ctor": {"dimension": d}, "ops": [
        {"op": "add_item", "embedding": [0.1] * d, "metadata": {"photo_path": "/a.jpg"}}, {"op": "clear"},
        {"op": "total"}, {"op": "has_photo_path", "photo_path": "/a.jpg"},
        {"op": "search", "query": [0.1] * d, "top_k": 1}]})
    return sc


def subst(op, tmp):
    return {k: (v.replace("{dir}", tmp) if isinstance(v, str) else v) for k, v in op.items()}


def run_scenario(VS, s):
    tmp = tempfile.mkdtemp(prefix="vsgold-")
    try:
        ctor = dict(s["ctor"])
        kw = dict(index_path=os.path.join(tmp, "index.bin"), metadata_path=os.path.join(tmp, "metadata.json"))
        rec = {"name": s["name"], "steps": []}
        try:
            store = VS(**ctor, **kw)
        except Exception as e:
            rec["ctor_error"] = {"error": type(e).__name__, "message": str(e)}
            return rec
        for op in s["ops"]:
            rec["steps"].append(run_op(store, subst(op, tmp)))
        if "reload" in s:
            store2 = VS(**dict(s.get("reload_ctor", ctor)), **kw)
            rec["reload_steps"] = [run_op(store2, subst(op, tmp)) for op in s["reload"]]
        files = {}
        for name in ("index.bin", "metadata.json", "index.bin.meta.json"):
            p = os.path.join(tmp, name)
            if os.path.exists(p) and name != "index.bin":
                files[name] = open(p, encoding="utf-8").read()
            elif os.path.exists(p):
                files[name + ".hex"] = open(p, "rb").read().hex() if os.path.getsize(p) < 4096 else None
        rec["files"] = files
        return rec
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def make_wrapper_golden():
    tmp = tempfile.mkdtemp(prefix="vsfaiss-")
    try:
        mod = import_reference_vector_store(tmp)
        out = {"source": "reference utils/vector_store.py over a stand-in faiss (oracle exact search)",
               "scenarios": []}
        for s in scenarios():
            out["scenarios"].append({"script": s, "result": run_scenario(mod.VectorStore, s)})
        path = os.path.join(HERE, "wrapper_golden.json.gz")
        with gzip.open(path, "wt", encoding="utf-8", compresslevel=9) as f:
            json.dump(out, f, ensure_ascii=False)
        print("wrote", path, os.path.getsize(path), "bytes")
    finally:
        sys.path.remove(tmp)
        shutil.rmtree(tmp, ignore_errors=True)


def make_oracle_golden():
    N, d = 10000, 1536
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 64, d, True, "f32")
    S, I = O.knn_exact(x, q, 100, "ip")
    # cross-checks at generation time
    Sn, In = O.np_knn_exact(x[:2000], q[:4], 20, "ip")
    Sc, Ic = O.knn_exact(x[:2000], q[:4], 20, "ip")
    assert np.array_equal(In, Ic) and np.array_equal(Sn, Sc)
    Df, If = O.knn_faiss_fp32(x, q, 100, "ip")
    assert np.max(np.abs(Df - S)) < 1e-5
    S2, I2 = O.knn_exact(x, q[:16], 10, "l2")
    xb = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    Sb, Ib = O.knn_exact(xb, q[:16], 10, "ip")
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"),
                        N=N, d=d, ip_S=S, ip_I=I.astype(np.int32), l2_S=S2, l2_I=I2.astype(np.int32),
                        bf16_S=Sb, bf16_I=Ib.astype(np.int32),
                        x_probe=x[[0, 1, 9999]], q_probe=q[[0, 63]], xb_probe=xb[[0, 5]])
    print("wrote oracle_golden.npz; faiss32 id agreement", float(np.mean(If == I)))


CFG1_N, CFG1_D, CFG1_NQ, CFG1_NQ_L2 = 10000, 1536, 32, 8
CFG1_TOPKS = (10, 1, 50)


def cfg1_corpus():
    """The cfg1 workload's raw embeddings: un-normalised counter-hash Gaussian rows and queries
    (the wrapper normalises them, as it does the embedding service's vectors)."""
    x = O.synth_rows(O.SEED_CORPUS, 0, CFG1_N, CFG1_D, False, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, CFG1_NQ, CFG1_D, False, "f32")
    return x, q


def make_cfg1_golden():
    """BASELINE cfg1 through the REFERENCE wrapper: ``VectorStore(dimension=1536)`` fed the 10k raw
    rows one ``add_item`` at a time (/root/reference/utils/vector_store.py:143-169), then
    ``search(query, top_k)`` one query per call (:172-198) for top_k 10 (the config), 1 and 50;
    an ``metric="l2"`` store over the same rows (no normalisation) for the L2 slice; the
    normalised embeddings of three rows (:200-212) and the sha256 of the saved index file
    (:217-237).  The stand-in faiss searches with the oracle's canonical exact search, so what is
    pinned is the wrapper around it at the product's plumbing scale; the corpus is regenerated from
    the counter hash, only results are stored."""
    import hashlib
    tmp = tempfile.mkdtemp(prefix="vsfaiss-")
    try:
        mod = import_reference_vector_store(tmp)
        x, q = cfg1_corpus()
        out = {"N": CFG1_N, "d": CFG1_D}
        for metric, nq in (("cosine", CFG1_NQ), ("l2", CFG1_NQ_L2)):
            work = tempfile.mkdtemp(prefix="vscfg1-")
            store = mod.VectorStore(dimension=CFG1_D, index_path=os.path.join(work, "index.bin"),
                                    metadata_path=os.path.join(work, "metadata.json"), metric=metric)
            for i in range(CFG1_N):
                store.add_item(x[i].tolist(), {"photo_path": f"/photos/{i:05d}.jpg", "row": i})
            for top_k in CFG1_TOPKS:
                ids = np.full((nq, top_k), -1, dtype=np.int32)
                dist = np.zeros((nq, top_k), dtype=np.float32)
                for a in range(nq):
                    res = store.search(q[a].tolist(), top_k)
                    assert len(res) == top_k
                    ids[a] = [r["metadata"]["row"] for r in res]
                    dist[a] = [r["distance"] for r in res]
                out[f"{metric}_top{top_k}_I"] = ids
                out[f"{metric}_top{top_k}_D"] = dist
            probe = [0, 4321, CFG1_N - 1]
            out[f"{metric}_probe_rows"] = np.array(probe, dtype=np.int32)
            out[f"{metric}_probe_emb"] = np.array(
                [store.get_embedding_by_photo_path(f"/photos/{i:05d}.jpg") for i in probe], dtype=np.float32)
            store.save()
            with open(os.path.join(work, "index.bin"), "rb") as f:
                out[f"{metric}_index_sha256"] = np.array(hashlib.sha256(f.read()).hexdigest())
            shutil.rmtree(work, ignore_errors=True)
        # cross-check at generation time: the same top-10 from the oracle on numpy-normalised rows
        xn = np.array([O.np_normalize_like_reference(r) for r in x], dtype=np.float32)
        qn = np.array([O.np_normalize_like_reference(r) for r in q], dtype=np.float32)
        S, I = O.knn_exact(xn, qn, 10, "ip")
        assert np.array_equal(I, out["cosine_top10_I"]) and np.array_equal(S.astype(np.float32), out["cosine_top10_D"])
        # VECTOR_DTYPE=bf16 (not a reference option): the oracle on the bf16-rounded normalised rows
        Sb, Ib = O.knn_exact(O.round_dtype(xn, "bf16"), qn, 10, "ip")
        out["cosine_bf16_top10_I"] = Ib.astype(np.int32)
        out["cosine_bf16_top10_D"] = Sb.astype(np.float32)
        path = os.path.join(HERE, "cfg1_wrapper_golden.npz")
        np.savez_compressed(path, **out)
        print("wrote", path, os.path.getsize(path), "bytes")
    finally:
        sys.path.remove(tmp)
        sys.modules.pop("faiss", None)
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["wrapper", "oracle", "cfg1"]
    if "wrapper" in which:
        make_wrapper_golden()
    if "oracle" in which:
        make_oracle_golden()
    if "cfg1" in which:
        make_cfg1_golden()
