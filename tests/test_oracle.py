"""The CPU oracle, pinned before it is trusted (CPU only).

Pins: (1) the C restatement agrees bit-for-bit with its numpy twin; (2) the committed oracle
goldens; (3) the reference's own known answers (tests/test_vector_store.py:35-51, :150-175,
tests/test_searcher.py:323-350, the build-smoke index fixture, the 77 x 4096 real index);
(4) the faiss fp32 restatement agrees with the exact search within the fp32 noise bound.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_c_matches_numpy_twin_ip_l2():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((700, 77)).astype(np.float32)
    x[5] = x[3]  # exact duplicate -> exact score tie
    q = rng.standard_normal((6, 77)).astype(np.float32)
    q[2] = x[3]
    for metric in ("ip", "l2"):
        Sc = O.canon_scores(x, q, metric)
        Sn = O.np_canon_scores(x, q, metric)
        assert np.array_equal(Sc, Sn)
        S1, I1 = O.knn_exact(x, q, 17, metric)
        S2, I2 = O.np_knn_exact(x, q, 17, metric)
        assert np.array_equal(I1, I2) and np.array_equal(S1, S2)
    # tie resolves to the lower id
    S, I = O.knn_exact(x, q[2:3], 2, "ip")
    assert list(I[0]) == [3, 5]


def test_synth_is_deterministic_normalised_and_range_consistent():
    a = O.synth_rows(O.SEED_CORPUS, 0, 300, 130, True, "f32")
    b = O.synth_rows(O.SEED_CORPUS, 100, 50, 130, True, "f32")
    assert np.array_equal(a[100:150], b)
    n = np.linalg.norm(a.astype(np.float64), axis=1)
    assert np.all(np.abs(n - 1.0) < 1e-6)
    raw = O.synth_rows(O.SEED_CORPUS, 0, 2000, 64, False, "f32")
    assert abs(raw.mean()) < 0.01 and abs(raw.std() - 1.0) < 0.02
    bf = O.synth_rows(O.SEED_CORPUS, 0, 300, 130, True, "bf16")
    u = bf.view(np.uint32)
    assert np.all((u & 0xFFFF) == 0)
    assert np.max(np.abs(bf - a)) < 2 ** -8


def test_dtype_rounding_matches_numpy():
    rng = np.random.default_rng(2)
    v = np.concatenate([rng.standard_normal(5000).astype(np.float32) * 10,
                        np.array([65504, 65519, 1e-8, -3e-5, 6.1e-5, 0.0, -0.0], np.float32)])
    assert np.array_equal(O.round_dtype(v, "f16"), v.astype(np.float16).astype(np.float32))
    u = v.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16).astype(np.uint32).view(np.float32)
    assert np.array_equal(O.round_dtype(v, "bf16"), r)


def test_oracle_golden_fixture():
    g = np.load(os.path.join(GOLDEN, "oracle_golden.npz"))
    N, d = int(g["N"]), int(g["d"])
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 64, d, True, "f32")
    assert np.array_equal(x[[0, 1, 9999]], g["x_probe"]) and np.array_equal(q[[0, 63]], g["q_probe"])
    S, I = O.knn_exact(x, q, 100, "ip")
    assert np.array_equal(I, g["ip_I"]) and np.array_equal(S, g["ip_S"])
    S2, I2 = O.knn_exact(x, q[:16], 10, "l2")
    assert np.array_equal(I2, g["l2_I"]) and np.array_equal(S2, g["l2_S"])
    xb = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    assert np.array_equal(xb[[0, 5]], g["xb_probe"])
    Sb, Ib = O.knn_exact(xb, q[:16], 10, "ip")
    assert np.array_equal(Ib, g["bf16_I"]) and np.array_equal(Sb, g["bf16_S"])


@pytest.mark.parametrize("nq", [1, 5, 40])  # nq < 20: faiss sequential path; >= 20: BLAS path
@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_faiss_fp32_restatement_vs_exact(nq, metric):
    x = O.synth_rows(O.SEED_CORPUS, 0, 20000, 256, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, 256, True, "f32")
    k = 20
    D, I = O.knn_faiss_fp32(x, q, k, metric)
    S, Ie = O.knn_exact(x, q, k, metric)
    assert np.max(np.abs(D.astype(np.float64) - S)) < 1e-5
    Sfull = O.canon_scores(x, q, metric)
    exact, tol = O.compare_ids_tie_tolerant(I, Ie, lambda a, i: Sfull[a, i], eps=1e-6)
    assert tol == 1.0 and exact > 0.99
    assert O.recall_at(I, Ie, 10) >= 0.99


def _normalize(v):
    return O.np_normalize_like_reference(v)


@pytest.mark.parametrize("d", [8, 768, 1536, 4096])
def test_reference_known_answers(d):
    # tests/test_vector_store.py:35-51: [0.1]*d and [0.5]*d, self-query.  At d = 8 / 768 the two
    # normalise to the SAME fp32 vector (exact tie -> lower id 0); at d = 4096 (the reference's
    # configured EMBEDDING_DIMENSION, config.py:142) [0.5]*d normalises 2 ulp smaller -> id 0.
    # At d = 1536 it normalises 1 ulp LARGER, so the exact top-1 is id 1; fp32 implementations
    # disagree there (faiss AVX2-order restatement: id 1; numpy sdot: tie -> id 0), i.e. the
    # reference test's expectation is build-dependent at 1536, and the two scores are within
    # the fp32 noise bound -- the tie-tolerant comparator's case.
    x = np.array([_normalize([0.1] * d), _normalize([0.5] * d)], np.float32)
    S, I = O.knn_exact(x, x[:1], 2, "ip")
    assert I[0, 0] == (1 if d == 1536 else 0)
    assert abs(S[0, 0] - S[0, 1]) < 1e-6
    D, If = O.knn_faiss_fp32(x, x[:1], 2, "ip")
    assert np.max(np.abs(D - S)) < 1e-5
    # tests/test_vector_store.py:150-161: row 0 is the zero vector (normalisation passthrough)
    rows = [_normalize([i * 0.1] * d) for i in range(10)]
    assert rows[0] == [0.0] * d
    x = np.array(rows, np.float32)
    S, I = O.knn_exact(x, np.array([_normalize([0.1] * d)], np.float32), 5, "ip")
    assert 0 not in I[0] and len(set(I[0].tolist())) == 5
    # tests/test_vector_store.py:163-175: stored vector is 1/sqrt(d) to 6 places
    assert abs(_normalize([0.2] * d)[0] - 1.0 / d ** 0.5) < 5e-7


def test_reference_duplicates_known_answer():
    # tests/test_searcher.py:323-350: [1.0]*8, [0.9]*8 (twice), [0.8]*8 normalise to ONE vector
    rows = [_normalize([1.0] * 8), _normalize([0.9] * 8), _normalize([0.9] * 8), _normalize([0.8] * 8)]
    assert rows[0] == rows[1] == rows[2] == rows[3]
    S, I = O.knn_exact(np.array(rows, np.float32), np.array(rows[:1], np.float32), 4, "ip")
    assert list(I[0]) == [0, 1, 2, 3] and len(set(S[0].tolist())) == 1


def test_build_smoke_fixture_is_reference_normalisation():
    # pytest-tmp/build-smoke/data/idx holds the normalised FakeEmbeddingService vector [11+i]
    from photo_search_engine_amd import faiss_format
    ff = faiss_format.read_index(os.path.join(GOLDEN, "ref_build_smoke.idx"))
    want = np.array([_normalize([11.0 + i for i in range(8)])], np.float32)
    assert np.array_equal(ff.vectors, want)


def test_real_index_self_queries():
    from photo_search_engine_amd import faiss_format
    ff = faiss_format.read_index(os.path.join(GOLDEN, "ref_photo_search.index"))
    x = np.ascontiguousarray(ff.vectors)
    S, I = O.knn_exact(x, x, 5, "ip")
    assert np.array_equal(I[:, 0], np.arange(77))
    D, If = O.knn_faiss_fp32(x, x, 5, "ip")
    assert np.array_equal(If[:, 0], np.arange(77))
    assert np.max(np.abs(D - S)) < 1e-5


def test_merge_of_shards_equals_global():
    x = O.synth_rows(O.SEED_CORPUS, 0, 3000, 96, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, 7, 96, True, "f32")
    k = 13
    for metric in ("ip", "l2"):
        Sg, Ig = O.knn_exact(x, q, k, metric)
        bounds = [0, 700, 1900, 3000]
        Sp, Ip = [], []
        for g in range(3):
            s, i = O.knn_exact(x[bounds[g]:bounds[g + 1]], q, k, metric)
            Sp.append(s)
            Ip.append(np.where(i >= 0, i + bounds[g], -1))
        Sm, Im = O.merge_topk(np.stack(Sp), np.stack(Ip), k, metric)
        assert np.array_equal(Im, Ig) and np.array_equal(Sm, Sg)
