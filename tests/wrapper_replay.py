"""Replay the reference-wrapper golden scenarios (tests/golden/wrapper_golden.json.gz) against a
VectorStore class and compare every recorded observable: results (metadata + distance, exact),
normalised embeddings (exact), totals, error types and messages, and written files."""
from __future__ import annotations

import gzip
import json
import os
import shutil
import tempfile

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wrapper_golden.json.gz")


def load_golden():
    with gzip.open(GOLDEN, "rt", encoding="utf-8") as f:
        return json.load(f)


def _run_op(store, op):
    kind = op["op"]
    try:
        if kind == "add_item":
            store.add_item(op["embedding"], op["metadata"])
            out = None
        elif kind == "search":
            out = [{"metadata": r["metadata"], "distance": r["distance"]} for r in store.search(op["query"], op["top_k"])]
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
    except Exception as e:
        return {"ok": False, "error": type(e).__name__, "mro": [c.__name__ for c in type(e).__mro__],
                "message": str(e)}


def _subst(op, tmp):
    return {k: (v.replace("{dir}", tmp) if isinstance(v, str) else v) for k, v in op.items()}


def _same_step(got, want, where):
    assert got["ok"] == want["ok"], f"{where}: ok {got} vs golden {want}"
    if want["ok"]:
        assert got["out"] == want["out"], f"{where}: output differs\n got  {str(got['out'])[:400]}\n want {str(want['out'])[:400]}"
    else:
        if want["error"] == "RuntimeError":  # faiss' own exception type; ours subclasses it
            assert "RuntimeError" in got.get("mro", [got["error"]]), f"{where}: {got}"
        else:
            assert got["error"] == want["error"], f"{where}: {got} vs {want}"
            assert got["message"] == want["message"], f"{where}: {got} vs {want}"


def replay(VS, scenario):
    s, want = scenario["script"], scenario["result"]
    tmp = tempfile.mkdtemp(prefix="vsreplay-")
    try:
        kw = dict(index_path=os.path.join(tmp, "index.bin"), metadata_path=os.path.join(tmp, "metadata.json"))
        try:
            store = VS(**dict(s["ctor"]), **kw)
        except Exception as e:
            assert "ctor_error" in want, f"{s['name']}: unexpected ctor error {e!r}"
            assert type(e).__name__ == want["ctor_error"]["error"]
            assert str(e) == want["ctor_error"]["message"]
            return
        assert "ctor_error" not in want, f"{s['name']}: ctor should have failed"
        for i, op in enumerate(s["ops"]):
            _same_step(_run_op(store, _subst(op, tmp)), want["steps"][i], f"{s['name']} step {i} {op['op']}")
        if "reload" in s:
            store2 = VS(**dict(s.get("reload_ctor", s["ctor"])), **kw)
            for i, op in enumerate(s["reload"]):
                _same_step(_run_op(store2, _subst(op, tmp)), want["reload_steps"][i], f"{s['name']} reload {i} {op['op']}")
        for name, text in want.get("files", {}).items():
            if name.endswith(".hex"):
                if text is None:
                    continue
                p = os.path.join(tmp, name[:-4])
                if "hnsw" in s["name"]:
                    continue  # an HNSW structure: the stand-in writes flat rows + a marker, we an IHNf graph
                assert open(p, "rb").read().hex() == text, f"{s['name']}: {name} bytes differ"
            else:
                assert open(os.path.join(tmp, name), encoding="utf-8").read() == text, f"{s['name']}: {name} differs"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
