"""Diagnostic (GPU): chunked device adds of generated rows, read back."""
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    import torch

    import bench
    from photo_search_engine_amd.index import FlatIndex, synthesize_device
    from photo_search_engine_amd.ivf import IVFFlatIndex

    d, nlist, N, chunk = 1536, 4096, 2_000_000, 1 << 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    c = torch.empty((nlist, d), dtype=torch.float32, device=dev)
    synthesize_device(0, bench.SEED_CENTROIDS, 0, nlist, d, c.data_ptr(), True, "bf16", stream)
    gen = {}
    fx = FlatIndex(d, "ip", "bf16", device=0)
    for r0 in range(0, N, chunk):
        x = bench._mixture_rows(bench.SEED_CORPUS, r0, min(chunk, N - r0), d, c, 1.0, dev, stream)
        gen[r0] = x[:4].cpu().numpy()
        fx.add_device(x.data_ptr(), x.shape[0], stream)
        print("chunk", r0, "ptr", hex(x.data_ptr()), "contig", x.is_contiguous(), flush=True)
        del x
    for r0 in gen:
        got = fx.reconstruct_n(r0, 4)
        print("flat rows", r0, "max |got - gen(bf16)|:", float(np.max(np.abs(got - gen[r0]))), flush=True)
    print("rows 0 vs 2^20 equal in flat:", np.array_equal(fx.reconstruct_n(0, 4), fx.reconstruct_n(chunk, 4)))
    print("gen rows 0 vs 2^20 equal:", np.array_equal(gen[0], gen[chunk]))


if __name__ == "__main__":
    main()
