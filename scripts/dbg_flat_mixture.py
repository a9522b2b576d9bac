"""Diagnostic (GPU): flat search on Gaussian-mixture rows vs the CPU oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    import torch

    import bench
    from oracle import oracle as O
    from photo_search_engine_amd.index import FlatIndex, synthesize_device

    d, nlist, N, chunk, nq, k = 1536, 4096, int(sys.argv[1]), 1 << 20, 256, 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    c = torch.empty((nlist, d), dtype=torch.float32, device=dev)
    synthesize_device(0, bench.SEED_CENTROIDS, 0, nlist, d, c.data_ptr(), True, "bf16", stream)
    fx = FlatIndex(d, "ip", "bf16", device=0)
    for r0 in range(0, N, chunk):
        x = bench._mixture_rows(bench.SEED_CORPUS, r0, min(chunk, N - r0), d, c, 1.0, dev, stream)
        fx.add_device(x.data_ptr(), x.shape[0], stream)
        del x
    q = bench._mixture_rows(bench.SEED_QUERIES, 0, nq, d, c, 1.0, dev, stream).contiguous()
    Id = torch.empty((nq, k), dtype=torch.int64, device=dev)
    Sd = torch.empty((nq, k), dtype=torch.float64, device=dev)
    fx.search_device(q.data_ptr(), nq, k, None, Id.data_ptr(), Sd.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    Idh = Id.cpu().numpy()
    print("uncertified:", fx.uncertified_count(), flush=True)
    dup = [a for a in range(nq) if len(set(Idh[a].tolist())) < k]
    print("queries with duplicate ids:", len(dup))
    qh = q.cpu().numpy()
    _, Ih = fx.search(qh, k)
    print("host vs device ids equal:", np.mean(Ih == Idh), flush=True)
    xs = fx.reconstruct_n(0, N)
    sel = list(range(8))
    S, Ie = O.knn_exact(xs, qh[sel], k, "ip")
    print("device vs oracle ids equal (8 q):", np.mean(Idh[sel] == Ie))
    print("host   vs oracle ids equal (8 q):", np.mean(Ih[sel] == Ie))
    for a in sel[:2]:
        print(" q", a, "dev", Idh[a].tolist(), "\n   oracle", Ie[a].tolist())
        print("   dev S", np.round(Sd.cpu().numpy()[a], 6).tolist(), "\n   oracle S", np.round(S[a], 6).tolist())
        for i in Idh[a][:3]:
            print("   row", int(i), "fp64 score", float(xs[i].astype(np.float64) @ qh[a].astype(np.float64)))
    # small-scale isolation: the same rows in a fresh index through vs_add (host)
    if os.environ.get("DBG_HOST_ADD"):
        fy = FlatIndex(d, "ip", "bf16", device=0)
        fy.add(xs)
        _, Iy = fy.search(qh[sel], k)
        print("host-added index vs oracle:", np.mean(Iy == Ie))


if __name__ == "__main__":
    main()
