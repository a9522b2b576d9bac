"""Diagnostic (GPU): IVF and flat search on Gaussian-mixture data vs the CPU oracles."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import ivf_oracle as IO  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    import torch  # noqa: F401

    from photo_search_engine_amd.index import FlatIndex
    from photo_search_engine_amd.ivf import IVFFlatIndex

    d, N, nlist, nq, k, nprobe = int(sys.argv[1]), int(sys.argv[2]), 256, 64, 10, 8
    dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    rng = np.random.default_rng(1)
    c = rng.standard_normal((nlist, d)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    c = O.round_dtype(c, dtype)
    cid = rng.integers(0, nlist, N)
    x = c[cid] + rng.standard_normal((N, d)).astype(np.float32) / np.sqrt(d)
    x = (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)
    xs = O.round_dtype(x, dtype)
    qc = rng.integers(0, nlist, nq)
    q = c[qc] + rng.standard_normal((nq, d)).astype(np.float32) / np.sqrt(d)
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)

    # flat: exact oracle vs host search (retries) vs device search (no retries)
    S, Ie = O.knn_exact(xs, q, k, "ip")
    fx = FlatIndex(d, "ip", dtype)
    fx.add(x)
    assert np.array_equal(fx.reconstruct_n(0, N), xs)
    _, Ih = fx.search(q, k)
    qd = torch.from_numpy(q).cuda()
    Id = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    Sd = torch.empty((nq, k), dtype=torch.float64, device="cuda")
    fx.search_device(qd.data_ptr(), nq, k, None, Id.data_ptr(), Sd.data_ptr(), 0, None)
    torch.cuda.synchronize()
    print("flat host  ids exact:", np.mean(Ih == Ie))
    print("flat dev   ids exact:", np.mean(Id.cpu().numpy() == Ie), "uncertified:", fx.uncertified_count())

    ix = IVFFlatIndex(d, nlist, "ip", dtype, nprobe=nprobe)
    ix.set_centroids(c)
    cs = ix.centroids()
    ix.add(x)
    lists = IO.assign(xs, cs, "ip")
    print("assign ok:", np.array_equal(ix.assign(xs[:2000]), lists[:2000]),
          "sizes ok:", np.array_equal(ix.list_sizes(), np.bincount(lists, minlength=nlist)))
    D, I = ix.search(q, k, nprobe)
    Sx, Ix = IO.search(xs, np.arange(N), lists, cs, q, k, nprobe, "ip")
    print("ivf ids exact vs ivf oracle:", np.mean(I == Ix))
    bad = np.where((I != Ix).any(axis=1))[0]
    for a in bad[:3]:
        print(" q", a, "got", I[a].tolist(), "\n   want", Ix[a].tolist())
        print("   got S", D[a].tolist(), "\n   want S", Sx[a].astype(np.float32).tolist())
    print("ivf recall@10 vs flat exact:", np.mean([len(set(I[a]) & set(Ie[a])) / k for a in range(nq)]))


if __name__ == "__main__":
    main()
