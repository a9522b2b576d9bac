"""Parity at the BASELINE.json shapes (MI355X only): every config the bench quotes is also run here
through the C ABI and checked against the oracle at its own (N, d, dtype, batch, k).

* cfg2  N=1M  d=1536 fp32, batch 1, top-10 (GEMV path): ids and scores bit-exact against
  ``oracle.knn_exact`` over the whole corpus.
* cfg3  N=10M d=1536 bf16, batch 256, top-100 (MFMA path, seeded threshold): the full corpus
  against the faiss fp32 restatement (``knn_faiss_fp32``; the canonical fp64 scan is minutes at this
  size) with the tie-tolerant rule below, plus a d=1536 case with >= 4 tiles per CU bit-exact
  against ``knn_exact``.
* cfg4  d=768 fp16, batch 256, top-10, row-sharded: ``ShardedFlatIndex`` over 4 ranks (gloo, all on
  the box's one GPU) at a reduced N of 4M rows; the merged answer checked like cfg3, the first
  16 queries bit-exact against ``knn_exact``, and the int8 screen's answer identical.
* cfg5  IVF-Flat nlist=4096 nprobe=32 d=1536 bf16, batch 256, top-10, at a reduced N of 500k rows
  of a Gaussian mixture with Zipf-sized clusters: bit-exact against ``oracle/ivf_oracle.py``.

Tie-tolerant rule (large shapes, ``_check_against_faiss32``): the GPU's scores must be the
canonical fp64 scores of the ids it returns (recomputed here), sorted (score desc, id asc); no id
of the faiss fp32 top-k may beat the GPU's k-th result under that order (exactness against every
candidate faiss found); and the fp32 distances agree within 1e-5 (north_star).
"""
import os
import socket

import numpy as np
import pytest

from oracle import ivf_oracle as IO
from oracle import oracle as O

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)


@pytest.fixture(scope="module")
def FlatIndex():
    from photo_search_engine_amd.index import FlatIndex as FI
    return FI


def _num_cu():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


def _returned_scores(x, q, I, metric="ip"):
    """Canonical fp64 scores of the returned ids (-1 slots: nan)."""
    S = np.full(I.shape, np.nan)
    for a in range(I.shape[0]):
        ok = I[a] >= 0
        if ok.any():
            S[a, ok] = O.canon_scores(x[I[a, ok]], q[a:a + 1], metric)[0]
    return S


def _check_against_faiss32(x, q, D, I, k, metric="ip"):
    """The tie-tolerant rule of the module docstring; returns the exact id-match rate."""
    Sg = _returned_scores(x, q, I, metric)
    np.testing.assert_array_equal(D, Sg.astype(np.float32))  # scores = fp32 of the canonical scores
    ip = metric == "ip"
    for a in range(I.shape[0]):  # sorted (score desc | asc, id asc)
        key = list(zip((-Sg[a] if ip else Sg[a]).tolist(), I[a].tolist()))
        assert key == sorted(key), f"query {a}: result not in (score, id) order"
    Dc, Ic = O.knn_faiss_fp32(x, q, k, metric, THREADS)
    assert np.max(np.abs(D.astype(np.float64) - Dc)) <= 1e-5
    for a in np.flatnonzero((I != Ic).any(axis=1)):
        miss = np.setdiff1d(Ic[a], I[a])
        if miss.size == 0:
            continue  # same set, near-tied order inside fp32 noise
        sm = O.canon_scores(x[miss], q[a:a + 1], metric)[0]
        tk, ik = Sg[a, k - 1], I[a, k - 1]
        for s, i in zip(sm.tolist(), miss.tolist()):
            better = (s > tk if ip else s < tk) or (s == tk and i < ik)
            assert not better, f"query {a}: faiss candidate {i} (exact {s!r}) beats the k-th result {ik} ({tk!r})"
    return float(np.mean(I == Ic))


# ------------------------------------------------------------------------------------------------
# cfg2: N=1M d=1536 fp32, batch 1, top-10
# ------------------------------------------------------------------------------------------------
def test_cfg2_full_shape_exact(FlatIndex):
    N, d, k = 1_000_000, 1536, 10
    ix = FlatIndex(d, "ip", "f32")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    for i in range(4):  # the product's call shape: one query per call
        q = O.synth_rows(O.SEED_QUERIES, i, 1, d, True, "f32")
        D, I = ix.search(q, k)
        S, Ie = O.knn_exact(x, q, k, "ip")
        np.testing.assert_array_equal(I, Ie)
        np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


# ------------------------------------------------------------------------------------------------
# cfg3: N=10M d=1536 bf16, batch 256, top-100
# ------------------------------------------------------------------------------------------------
def test_cfg3_d1536_seeded_mfma_exact(FlatIndex):
    # >= 4 tiles per CU: the seeded MFMA screen at the headline d (48 K-steps per tile)
    N, d, nq, k = 256 * 4 * _num_cu() + 777, 1536, 64, 100
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    D, I = ix.search(q, k)
    S, Ie = O.knn_exact(x, q, k, "ip")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    ix.close()


def test_cfg3_full_shape_vs_faiss32(FlatIndex):
    N, d, nq, k = 10_000_000, 1536, 256, 100
    ix = FlatIndex(d, "ip", "bf16")
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    D, I = ix.search(q, k)
    ix.set_screen("int8")  # the bench's default screen at this shape: the same exact answer
    D8, I8 = ix.search(q, k)
    np.testing.assert_array_equal(I8, I)
    np.testing.assert_array_equal(D8, D)
    assert ix.uncertified_count() == 0
    ix.close()
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")  # the stored values, upcast (61 GB)
    match = _check_against_faiss32(x, q, D, I, k)
    assert match >= 0.999, match
    del x


# ------------------------------------------------------------------------------------------------
# cfg4: d=768 fp16, batch 256, top-10, row-sharded over ranks (4 ranks on the one GPU, gloo)
# ------------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg4_worker(rank, world, port, N, d, nq, k, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from photo_search_engine_amd.distributed import ShardedFlatIndex
        from photo_search_engine_amd.index import synthesize_device
        sh = ShardedFlatIndex(d, "ip", "f16", device=0)
        sh.add_synthetic(O.SEED_CORPUS, N, True)
        q = torch.empty((nq, d), dtype=torch.float32, device="cuda")
        synthesize_device(0, O.SEED_QUERIES, 0, nq, d, q.data_ptr(), True, "f16",
                          torch.cuda.current_stream().cuda_stream)
        D, I, S = sh.search(q, k)
        sh.index.set_screen("int8")  # the bench's default screen for cfg4: the same exact answer
        D8, I8, S8 = sh.search(q, k)
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), D=D.cpu().numpy(), I=I.cpu().numpy(), S=S.cpu().numpy(),
                 I8=I8.cpu().numpy(), S8=S8.cpu().numpy(), n=sh.n_local, full_scan=sh.full_scan_count())
        sh.close()
    finally:
        dist.destroy_process_group()


def test_cfg4_shape_sharded_four_ranks(tmp_path):
    import torch.multiprocessing as mp
    N, d, nq, k, G = 4_000_000, 768, 256, 10, 4
    mp.spawn(_cfg4_worker, args=(G, _free_port(), N, d, nq, k, str(tmp_path)), nprocs=G, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(G)]
    assert sum(int(o["n"]) for o in outs) == N
    for o in outs[1:]:  # every rank holds the same merged answer
        np.testing.assert_array_equal(o["I"], outs[0]["I"])
        np.testing.assert_array_equal(o["S"], outs[0]["S"])
    D, I, S = outs[0]["D"], outs[0]["I"], outs[0]["S"]
    for o in outs:  # int8 screen on every shard: identical merged answer, no full scan
        np.testing.assert_array_equal(o["I8"], I)
        np.testing.assert_array_equal(o["S8"], S)
        assert int(o["full_scan"]) == 0
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f16")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f16")
    np.testing.assert_array_equal(D, S.astype(np.float32))
    match = _check_against_faiss32(x, q, D, I, k)
    assert match >= 0.999, match
    Se, Ie = O.knn_exact(x, q[:16], k, "ip")  # a bit-exact slice (the canonical scan over 4M rows)
    np.testing.assert_array_equal(I[:16], Ie)
    np.testing.assert_array_equal(S[:16], Se)


def test_cfg4_full_shape_eight_shards_one_gpu(FlatIndex):
    # cfg4 at its own size: 100M x 768 fp16 rows as the 8-GPU run shards them (8 contiguous shards of
    # 12.5M rows, each searched with its global id offset, the lists merged by the sharded step's
    # device merge), all 8 shards on the box's one GPU (230 GB of rows + int8 copies in 288 GB).
    # Checked: native == int8 screen bit for bit, no full scan; every query's returned scores are
    # the canonical scores of its ids, sorted; and on a 32-query slice the tie-tolerant rule against
    # the faiss fp32 restatement over all 100M rows (streamed in chunks: 307 GB of fp32 rows does
    # not fit the host)
    import torch
    from photo_search_engine_amd.distributed import shard_range, _device_merge
    from photo_search_engine_amd.index import synthesize_device
    N, d, nq, k, G, nslice = 100_000_000, 768, 256, 10, 8, 32
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    q = torch.empty((nq, d), dtype=torch.float32, device=dev)
    synthesize_device(0, O.SEED_QUERIES, 0, nq, d, q.data_ptr(), True, "f16", stream)
    shards = []
    for g in range(G):
        r0, n = shard_range(N, g, G)
        ix = FlatIndex(d, "ip", "f16")
        ix.reserve(n)
        ix.add_synthetic(O.SEED_CORPUS, r0, n, True)
        shards.append((ix, r0))
    out = {}
    for screen in ("native", "int8"):
        Sg = torch.empty((G, nq, k), dtype=torch.float64, device=dev)
        Ig = torch.empty((G, nq, k), dtype=torch.int64, device=dev)
        for g, (ix, r0) in enumerate(shards):
            ix.set_screen(screen)
            ix.search_device_exact(q.data_ptr(), nq, k, None, Ig[g].data_ptr(), Sg[g].data_ptr(), r0, stream)
        S, I, D = _device_merge(0, Sg, Ig, k)
        torch.cuda.synchronize()
        out[screen] = (S.cpu().numpy(), I.cpu().numpy(), D.cpu().numpy())
    assert sum(ix.full_scan_count() for ix, _ in shards) == 0
    for ix, _ in shards:
        ix.close()
    del shards
    S, I, D = out["native"]
    np.testing.assert_array_equal(out["int8"][1], I)
    np.testing.assert_array_equal(out["int8"][0], S)
    np.testing.assert_array_equal(D, S.astype(np.float32))
    qh = q.cpu().numpy()
    # every query: the returned scores are the canonical scores of the returned ids, in order
    for a in range(nq):
        rows = np.concatenate([O.synth_rows(O.SEED_CORPUS, int(i), 1, d, True, "f16") for i in I[a]])
        np.testing.assert_array_equal(O.canon_scores(rows, qh[a:a + 1], "ip")[0], S[a])
        key = list(zip((-S[a]).tolist(), I[a].tolist()))
        assert key == sorted(key)
    # the slice: faiss fp32 over every row, streamed in chunks generated on the device (the same
    # counter-hash generator as the oracle's, bit-identical) and merged by (fp32 score desc, id asc)
    Dc = np.full((nslice, k), -np.inf, dtype=np.float32)
    Ic = np.full((nslice, k), -1, dtype=np.int64)
    chunk = 5_000_000
    buf = torch.empty((chunk, d), dtype=torch.float32, device=dev)
    for r0 in range(0, N, chunk):
        n = min(chunk, N - r0)
        synthesize_device(0, O.SEED_CORPUS, r0, n, d, buf.data_ptr(), True, "f16", stream)
        torch.cuda.synchronize()
        Dp, Ip = O.knn_faiss_fp32(buf[:n].cpu().numpy(), qh[:nslice], k, "ip", THREADS)
        Dm = np.concatenate([Dc, Dp], axis=1)
        Im = np.concatenate([Ic, np.where(Ip >= 0, Ip + r0, -1)], axis=1)
        order = np.lexsort((Im, -Dm.astype(np.float64)), axis=1)[:, :k]
        Dc, Ic = np.take_along_axis(Dm, order, 1), np.take_along_axis(Im, order, 1)
    del buf
    assert np.max(np.abs(D[:nslice].astype(np.float64) - Dc)) <= 1e-5
    for a in range(nslice):
        miss = np.setdiff1d(Ic[a], I[a])
        if miss.size == 0:
            continue
        rows = np.concatenate([O.synth_rows(O.SEED_CORPUS, int(i), 1, d, True, "f16") for i in miss])
        sm = O.canon_scores(rows, qh[a:a + 1], "ip")[0]
        for s_, i in zip(sm.tolist(), miss.tolist()):
            assert not (s_ > S[a, k - 1] or (s_ == S[a, k - 1] and i < I[a, k - 1])), \
                f"query {a}: faiss candidate {i} beats the k-th result"
    assert float(np.mean(I[:nslice] == Ic)) >= 0.99


# ------------------------------------------------------------------------------------------------
# cfg5: IVF-Flat nlist=4096 nprobe=32 d=1536 bf16, batch 256, top-10 (reduced N, skewed lists)
# ------------------------------------------------------------------------------------------------
def zipf_mixture(N, d, centroids, sigma, zipf_s, seed):
    """normalise(c[cid(i)] + sigma * g_i), cid drawn with Zipf(s) weights over the centroids (a
    seeded permutation of ranks), g_i the unit counter-hash Gaussian row i (oracle generator)."""
    rng = np.random.default_rng(seed)
    nl = centroids.shape[0]
    w = 1.0 / np.arange(1, nl + 1) ** zipf_s
    w = w[rng.permutation(nl)]
    cid = rng.choice(nl, size=N, p=w / w.sum())
    g = O.synth_rows(seed, 0, N, centroids.shape[1], True, "f32")
    x = centroids[cid] + np.float32(sigma) * g
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return np.ascontiguousarray(x, dtype=np.float32)


def test_cfg5_shape_ivf_skewed_lists_exact():
    from photo_search_engine_amd.ivf import IVFFlatIndex
    N, d, nlist, nprobe, nq, k = 500_000, 1536, 4096, 32, 256, 10
    c0 = O.synth_rows(20260419, 0, nlist, d, True, "bf16")
    ix = IVFFlatIndex(d, nlist, "ip", "bf16", nprobe=nprobe)
    ix.set_centroids(c0)
    c = ix.centroids()
    x = zipf_mixture(N, d, c, 1.0, 1.1, O.SEED_CORPUS)
    ix.reserve(N)
    for r0 in range(0, N, 131072):
        ix.add(x[r0:r0 + 131072])
    xs = O.round_dtype(x, "bf16")
    del x
    lists = IO.assign_ip_fast(xs, c)
    sizes = ix.list_sizes()
    np.testing.assert_array_equal(sizes, np.bincount(lists, minlength=nlist))
    nz = sizes[sizes > 0]
    assert nz.max() >= 20 * max(int(np.median(nz)), 1)  # skewed: a heavy head of lists
    q = zipf_mixture(nq, d, c, 1.0, 1.1, O.SEED_QUERIES)
    D, I = ix.search(q, k, nprobe)
    S, Ie = IO.search(xs, np.arange(N), lists, c, q, k, nprobe, "ip")
    np.testing.assert_array_equal(I, Ie)
    Dexp = S.astype(np.float32)
    Dexp[Ie < 0] = -3.4028235e38
    np.testing.assert_array_equal(D, Dexp)
    ix.close()
