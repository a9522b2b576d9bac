"""The multi-rank search path on a real GPU: two ranks (gloo, both on cuda:0 -- the box has one
GPU; the driver's 8-GPU runs use nccl/RCCL with one GPU per rank) run the product's
ShardedFlatIndex with its default HIP local search and HIP device merge, and every rank's merged
answer must equal the oracle's exact answer over the whole corpus (ids and fp64 scores)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, d, dtype, nq, k, metric, outdir, screen="native", backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = rank if backend == "nccl" else 0  # nccl (RCCL over xGMI): one GPU per rank
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from photo_search_engine_amd.distributed import ShardedFlatIndex
        sh = ShardedFlatIndex(d, metric, dtype, device=dev)
        sh.add_synthetic(O.SEED_CORPUS, N, True)
        sh.index.set_screen(screen)
        q = torch.from_numpy(O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, dtype)).cuda()
        if rank != 0:
            q.zero_()  # rank 0's batch arrives by broadcast
        D, I, S = sh.search(q, k, src=0)
        D, I, S = sh.search(q, k, src=0)  # (a second call: the pending-search state is released)
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), D=D.cpu().numpy(), I=I.cpu().numpy(), S=S.cpu().numpy(),
                 row0=sh.row0, n=sh.n_local, two=sh.index.two_phase_ok(nq, k),
                 full_scan=sh.full_scan_count())
        sh.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("metric,dtype,nq,k,N", [("ip", "bf16", 40, 25, 20011), ("l2", "f32", 3, 10, 20011),
                                                 ("ip", "bf16", 12, 10, 15)])  # last: shards smaller than k
def test_two_ranks_one_gpu_match_oracle(tmp_path, metric, dtype, nq, k, N):
    d = 64
    mp.spawn(_worker, args=(2, _free_port(), N, d, dtype, nq, k, metric, str(tmp_path)), nprocs=2, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(2)]
    assert int(outs[0]["row0"]) == 0 and int(outs[1]["row0"]) == int(outs[0]["n"])
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, dtype)
    Se, Ie = O.knn_exact(x, q, k, metric)
    for o in outs:
        np.testing.assert_array_equal(o["I"], Ie)
        valid = Ie >= 0
        np.testing.assert_array_equal(o["S"][valid], Se[valid])
        np.testing.assert_array_equal(o["D"][valid], Se[valid].astype(np.float32))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one rank per GPU over RCCL); "
                    "the one-GPU box runs the same path over gloo above")
@pytest.mark.parametrize("screen,metric,dtype,nq,k,N", [("native", "ip", "bf16", 40, 25, 40011),
                                                        ("int8", "ip", "bf16", 64, 20, 40011),
                                                        ("native", "l2", "f32", 3, 10, 20011)])
def test_ranks_on_distinct_gpus_nccl_match_oracle(tmp_path, screen, metric, dtype, nq, k, N):
    # the driver's multi-GPU shape: one process per GPU, the exchanges over RCCL / xGMI
    world, d = min(torch.cuda.device_count(), 4), 256
    mp.spawn(_worker, args=(world, _free_port(), N, d, dtype, nq, k, metric, str(tmp_path), screen, "nccl"),
             nprocs=world, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert sum(int(o["n"]) for o in outs) == N
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, dtype)
    Se, Ie = O.knn_exact(x, q, k, metric)
    for o in outs:
        np.testing.assert_array_equal(o["I"], Ie)
        np.testing.assert_array_equal(o["S"], Se)
        assert int(o["full_scan"]) == 0


def test_four_ranks_one_gpu_match_oracle(tmp_path):
    # G = 4: the all-gather of packed (score, id) pairs and the 4-way device merge
    N, d, nq, k = 30001, 48, 20, 15
    mp.spawn(_worker, args=(4, _free_port(), N, d, "bf16", nq, k, "ip", str(tmp_path)), nprocs=4, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(4)]
    assert sum(int(o["n"]) for o in outs) == N
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    Se, Ie = O.knn_exact(x, q, k, "ip")
    for o in outs:
        np.testing.assert_array_equal(o["I"], Ie)
        np.testing.assert_array_equal(o["S"], Se)


@pytest.mark.parametrize("world,metric,dtype,nq,k,N,d", [
    (2, "ip", "bf16", 40, 25, 20011, 64),
    (2, "l2", "f16", 64, 10, 30000, 256),
    (4, "ip", "bf16", 256, 100, 4 * 256 * 4 * 256 + 333, 256),  # >= 4 tiles per CU per shard: seeded
    (4, "l2", "bf16", 100, 50, 4 * 256 * 4 * 256 + 333, 512),
    (3, "ip", "f16", 20, 30, 50, 64),                          # shards smaller than k
])
def test_two_phase_int8_ranks_one_gpu_match_oracle(tmp_path, world, metric, dtype, nq, k, N, d):
    # the int8 screen on bf16/f16 shards takes the two-phase search: phase-A lists exchanged and
    # merged into each query's floor, phase B per shard, then the final exchange -- the same exact
    # global answer as one index
    mp.spawn(_worker, args=(world, _free_port(), N, d, dtype, nq, k, metric, str(tmp_path), "int8"),
             nprocs=world, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert all(bool(o["two"]) for o in outs)
    assert sum(int(o["full_scan"]) for o in outs) == 0
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, dtype)
    Se, Ie = O.knn_exact(x, q, k, metric)
    for o in outs:
        np.testing.assert_array_equal(o["I"], Ie)
        valid = Ie >= 0
        np.testing.assert_array_equal(o["S"][valid], Se[valid])
        np.testing.assert_array_equal(o["D"][valid], Se[valid].astype(np.float32))


@pytest.mark.parametrize("metric", ["ip", "l2"])
def test_two_phase_single_index_with_external_floor(metric):
    # phase B with a floor taken from the WHOLE corpus's exact answer, on an index holding only a
    # slice of it: every row of the slice at least as good as the floor must come back exactly
    # (rows below it may be skipped); with its own phase-A lists as the floor it equals the
    # one-phase search
    from photo_search_engine_amd.index import FlatIndex
    N, d, nq, k = 300_000, 256, 64, 50
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, "bf16")
    q = O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")
    Sg, Ig = O.knn_exact(x, q, k, metric)
    lo, hi = 100_000, 250_000
    ix = FlatIndex(d, metric, "bf16")
    ix.add(x[lo:hi])
    ix.set_screen("int8")
    assert ix.two_phase_ok(nq, k) and not ix.two_phase_ok(8, k) and not ix.two_phase_ok(257, k)
    qd = torch.from_numpy(q).cuda()
    Sa = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    Ia = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    S = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    # (1) own floor
    p = ix.search_phase_a(qd.data_ptr(), nq, k, 1, Sa.data_ptr(), Ia.data_ptr(), lo)
    ix.search_phase_b(p, Sa.data_ptr(), D.data_ptr(), I.data_ptr(), S.data_ptr())
    Sl, Il = O.knn_exact(x[lo:hi], q, k, metric)
    np.testing.assert_array_equal(I.cpu().numpy(), Il + lo)
    np.testing.assert_array_equal(S.cpu().numpy(), Sl)
    # (2) the global floor: the slice's rows within the global top-k are all found, exactly
    floor = torch.from_numpy(Sg).cuda()
    p = ix.search_phase_a(qd.data_ptr(), nq, k, 4, Sa.data_ptr(), Ia.data_ptr(), lo)
    ix.search_phase_b(p, floor.data_ptr(), D.data_ptr(), I.data_ptr(), S.data_ptr())
    Ih, Sh = I.cpu().numpy(), S.cpu().numpy()
    for qi in range(nq):
        mine = [(s, i) for s, i in zip(Sg[qi], Ig[qi]) if lo <= i < hi]
        got = list(zip(Sh[qi][:len(mine)], Ih[qi][:len(mine)]))
        assert got == mine, qi
    assert ix.full_scan_count() == 0
    # (3) a pending search dropped without phase B releases the index (an add must not block)
    p = ix.search_phase_a(qd.data_ptr(), nq, k, 2, Sa.data_ptr(), Ia.data_ptr(), lo)
    ix.search_pending_free(p)
    ix.add(x[hi:hi + 10])
    ix.close()


def _nccl_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from photo_search_engine_amd.distributed import ShardedFlatIndex
        N, d, nq, k = 9000, 64, 24, 12
        sh = ShardedFlatIndex(d, "ip", "bf16", device=0)
        sh.add_synthetic(O.SEED_CORPUS, N, True)
        q = torch.from_numpy(O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "bf16")).cuda()
        D, I, S = sh.search(q, k, src=0)
        # the exchange step itself on RCCL: all_gather_into_tensor of the packed (score, id) pairs
        # and the device merge of the gathered lists (G = 1 here)
        SI = torch.stack([S.contiguous().view(torch.int64), I.contiguous()], dim=-1)
        g = sh._gather(SI)
        S2, I2, D2 = sh._merge(sh.metric, g[..., 0].contiguous().view(torch.float64), g[..., 1].contiguous(), k)
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, "nccl.npz"), D=D.cpu().numpy(), I=I.cpu().numpy(), S=S.cpu().numpy(),
                 D2=D2.cpu().numpy(), I2=I2.cpu().numpy(), S2=S2.cpu().numpy(), backend=dist.get_backend())
        sh.close()
    finally:
        dist.destroy_process_group()


def test_rccl_backend_one_rank_exchange_and_merge(tmp_path):
    # the nccl (= RCCL) branch of ShardedFlatIndex._gather, which the gloo tests above never take:
    # one rank (the box has one GPU; RCCL does not run two ranks on one device), all_gather_into_tensor
    # + the device merge, equal to the oracle
    mp.spawn(_nccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    o = np.load(tmp_path / "nccl.npz")
    assert str(o["backend"]) == "nccl"
    x = O.synth_rows(O.SEED_CORPUS, 0, 9000, 64, True, "bf16")
    q = O.synth_rows(O.SEED_QUERIES, 0, 24, 64, True, "bf16")
    Se, Ie = O.knn_exact(x, q, 12, "ip")
    for sfx in ("", "2"):
        np.testing.assert_array_equal(o["I" + sfx], Ie, err_msg="I" + sfx)
        np.testing.assert_array_equal(o["S" + sfx], Se, err_msg="S" + sfx)
        np.testing.assert_array_equal(o["D" + sfx], Se.astype(np.float32), err_msg="D" + sfx)


def _tie_worker(rank, world, port, N, d, dtype, copies, nq, k, metric, screen, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from photo_search_engine_amd.distributed import ShardedFlatIndex, shard_range
        x, q = _tie_corpus(N, d, dtype, copies, nq)
        sh = ShardedFlatIndex(d, metric, dtype, device=0)
        row0, n = shard_range(N, rank, world)
        sh.add_shard(x[row0:row0 + n], row0, N)
        sh.index.set_screen(screen)
        D, I, S = sh.search(torch.from_numpy(q).cuda(), k)
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), D=D.cpu().numpy(), I=I.cpu().numpy(), S=S.cpu().numpy(),
                 full_scan=sh.full_scan_count())
        sh.close()
    finally:
        dist.destroy_process_group()


def _tie_corpus(N, d, dtype, copies, nq):
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, True, dtype)
    v = x[N // 2 + 5].copy()
    pos = np.random.default_rng(5).choice(N, copies, replace=False)  # spread over every shard
    x[pos] = v
    q = np.concatenate([np.repeat(v[None], nq - 1, axis=0), O.synth_rows(O.SEED_QUERIES, 0, 1, d, True, dtype)])
    return x, q


@pytest.mark.parametrize("screen,metric,nq,copies", [("native", "ip", 3, 9000), ("native", "l2", 3, 20000),
                                                     ("int8", "ip", 12, 20000)])
def test_two_ranks_ties_split_across_shards(tmp_path, screen, metric, nq, copies):
    # thousands of identical rows spread over both shards (more per shard than any bounded screen
    # lists): each shard's device path ends in its exact full scan, the exchange merges exact shard
    # lists, and every rank returns faiss's answer -- the k lowest ids of the tie
    N, d, k, dtype = 2 * 24_000, 64, 10, "bf16"
    mp.spawn(_tie_worker, args=(2, _free_port(), N, d, dtype, copies, nq, k, metric, screen, str(tmp_path)),
             nprocs=2, join=True)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(2)]
    x, q = _tie_corpus(N, d, dtype, copies, nq)
    x = O.round_dtype(x, dtype)
    Se, Ie = O.knn_exact(x, O.round_dtype(q, dtype), k, metric)
    for o in outs:
        np.testing.assert_array_equal(o["I"], Ie)
        np.testing.assert_array_equal(o["S"], Se)
        np.testing.assert_array_equal(o["D"], Se.astype(np.float32))
    if copies // 2 > 8192:  # (beyond the adaptive refine's 8192 rows: only the full scan certifies)
        assert sum(int(o["full_scan"]) for o in outs) >= 1
