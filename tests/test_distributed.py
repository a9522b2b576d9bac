"""Multi-process (gloo, world_size 2, CPU) tests of the row-sharded search layer
(photo_search_engine_amd/distributed.py): shard ranges, the all-gather, query broadcast, empty
shards and k beyond a shard's rows.  The per-shard search and the merge are the CPU oracle here
(checker only); on GPUs they are the HIP library (same ShardedFlatIndex code)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from photo_search_engine_amd.distributed import ShardedFlatIndex, _pack, shard_range
from tests.oracle_index import OracleFlatIndex


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_local_search(index, q, k, row0):
    metric = "ip" if index.metric_type == 0 else "l2"
    S, I = O.knn_exact(index._x, q.numpy(), k, metric)
    worst = -1.7976931348623157e308 if metric == "ip" else 1.7976931348623157e308
    S = np.where(I >= 0, S, worst)
    D = S.astype(np.float32)
    D[I < 0] = -3.4028235e38 if metric == "ip" else 3.4028235e38
    I = np.where(I >= 0, I + row0, -1)
    return torch.from_numpy(S), torch.from_numpy(I), torch.from_numpy(D)


def _oracle_merge(metric, Sg, Ig, k):
    S, I = O.merge_topk(Sg.numpy(), Ig.numpy(), k, "ip" if metric == 0 else "l2")
    D = S.astype(np.float32)
    D[I < 0] = -3.4028235e38 if metric == 0 else 3.4028235e38
    return torch.from_numpy(S), torch.from_numpy(I), torch.from_numpy(D)


def _pad(S, I, k, metric):
    nq, m = S.shape
    worst = -1.7976931348623157e308 if metric == "ip" else 1.7976931348623157e308
    So = np.full((nq, k), worst)
    Io = np.full((nq, k), -1, dtype=np.int64)
    So[:, :min(m, k)] = S[:, :k]
    Io[:, :min(m, k)] = I[:, :k]
    So = np.where(Io >= 0, So, worst)
    return So, Io


def _oracle_phase_a(index, q, k, row0, world):
    """CPU restatement of vs_search_device_phase_a's contract: the shard's best KA rows (exact),
    their top-k for the exchange (packed pairs, as the device phase writes them); KA as the library
    picks it."""
    metric = "ip" if index.metric_type == 0 else "l2"
    ka = min(-(-(2 * k + 32) // 32) * 32, -(-(2 * -(-k // world) + 32) // 32) * 32)
    S, I = O.knn_exact(index._x, q.numpy(), ka, metric)
    I = np.where(I >= 0, I + row0, -1)
    Sa, Ia = _pad(S, I, k, metric)
    return _pack(torch.from_numpy(Sa), torch.from_numpy(Ia)), {"S": S, "I": I, "metric": metric, "row0": row0}


def _oracle_phase_b(index, pend, floor_S, q, k):
    """Phase B's contract: the shard's top-k among its phase-A rows and every row at least as good
    as the floor (the merged phase-A lists' k-th score) -- nothing below the floor is scored."""
    metric, row0 = pend["metric"], pend["row0"]
    n = index._x.shape[0]
    Sall, Iall = O.knn_exact(index._x, q.numpy(), n, metric)
    fl = floor_S.numpy()[:, k - 1]
    outS, outI = [], []
    for qi in range(q.shape[0]):
        keep = (Sall[qi] >= fl[qi]) if metric == "ip" else (Sall[qi] <= fl[qi])
        cand = {int(i): s for s, i in zip(Sall[qi][keep], Iall[qi][keep] + row0)}
        cand.update({int(i): s for s, i in zip(pend["S"][qi], pend["I"][qi]) if i >= 0})
        items = sorted(cand.items(), key=(lambda t: (-t[1], t[0])) if metric == "ip" else (lambda t: (t[1], t[0])))[:k]
        outS.append([s for _, s in items])
        outI.append([i for i, _ in items])
    m = max([len(r) for r in outS] + [0])
    worst = -1.7976931348623157e308 if metric == "ip" else 1.7976931348623157e308
    S = np.array([r + [worst] * (m - len(r)) for r in outS], dtype=np.float64).reshape(len(outS), m)
    I = np.array([r + [-1] * (m - len(r)) for r in outI], dtype=np.int64).reshape(len(outI), m)
    S, I = _pad(S, I, k, metric)
    return _pack(torch.from_numpy(S), torch.from_numpy(I))


def _worker(rank, world, port, N, d, nq, k, metric, use_broadcast, outdir, from_file=None, two_phase=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
        extra = {}
        if two_phase:
            extra = dict(phase_a=_oracle_phase_a, phase_b=_oracle_phase_b, two_phase_ok=lambda ix, nq_, k_: True)
        sh = ShardedFlatIndex(d, metric, index=OracleFlatIndex(d, metric),
                              local_search=_oracle_local_search, merge=_oracle_merge, **extra)
        row0, n = shard_range(N, rank, world)
        if from_file:  # each rank streams only its own row range of the faiss file
            sh.add_shard_from_file(from_file)
            assert (sh.row0, sh.n_local, sh.n_total) == (row0, n, N)
        else:
            sh.add_shard(x[row0:row0 + n], row0, N)
        q = torch.from_numpy(O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32"))
        if use_broadcast and rank != 0:
            q = torch.zeros_like(q)  # rank 0's batch must arrive by broadcast
        D, I, S = sh.search(q, k, src=0 if use_broadcast else None)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), D=D.numpy(), I=I.numpy(), S=S.numpy(), n=n)
    finally:
        dist.destroy_process_group()


def _run(tmp_path, N, d, nq, k, metric="ip", use_broadcast=False, world=2, from_file=None, two_phase=False):
    mp.spawn(_worker, args=(world, _free_port(), N, d, nq, k, metric, use_broadcast, str(tmp_path), from_file,
                            two_phase), nprocs=world, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")
    Se, Ie = O.knn_exact(x, q, k, metric)
    for o in outs:  # every rank holds the same, globally exact answer
        np.testing.assert_array_equal(o["I"], Ie)
        valid = Ie >= 0
        np.testing.assert_array_equal(o["S"][valid], Se[valid])
        np.testing.assert_array_equal(o["D"][valid], Se[valid].astype(np.float32))
    return outs


def test_shard_range_partitions_rows():
    for N in (0, 1, 7, 1000, 10_000_001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(N, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(n for _, n in spans) == N
            for (a0, an), (b0, _) in zip(spans, spans[1:]):
                assert a0 + an == b0
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_two_rank_search_matches_single_index(tmp_path, metric):
    outs = _run(tmp_path, N=1001, d=24, nq=5, k=12, metric=metric)
    assert int(outs[0]["n"]) + int(outs[1]["n"]) == 1001


def test_two_rank_query_broadcast(tmp_path):
    _run(tmp_path, N=300, d=16, nq=3, k=7, use_broadcast=True)


def test_two_rank_empty_shard_and_k_beyond_rows(tmp_path):
    # N = 1: rank 0 owns no rows, rank 1 one row; k = 4 pads with id -1
    outs = _run(tmp_path, N=1, d=8, nq=2, k=4)
    assert (outs[0]["I"][:, 1:] == -1).all()
    assert (outs[1]["I"][:, 0] == 0).all()


def test_two_rank_shards_loaded_from_index_file(tmp_path):
    from photo_search_engine_amd import faiss_format as F
    x = O.synth_rows(O.SEED_CORPUS, 0, 777, 20, True, "f32")
    p = str(tmp_path / "corpus.index")
    F.write_flat(p, x, 0)
    _run(tmp_path, N=777, d=20, nq=4, k=9, from_file=p)


@pytest.mark.parametrize("metric", ["ip", "l2"])
@pytest.mark.parametrize("world", [2, 3])
def test_two_phase_exchange_matches_single_index(tmp_path, metric, world):
    # phase A lists -> all-gather + merge -> floor -> phase B -> all-gather + merge: the global
    # exact answer, with each shard scoring only rows at least as good as the floor in phase B
    _run(tmp_path, N=1500, d=16, nq=6, k=40, metric=metric, world=world, two_phase=True)


def test_two_phase_empty_shard_and_k_beyond_rows(tmp_path):
    outs = _run(tmp_path, N=1, d=8, nq=2, k=4, two_phase=True)
    assert (outs[0]["I"][:, 1:] == -1).all()
