import sys, numpy as np
sys.path.insert(0, '.')
from oracle import oracle as O, ivf_oracle as IO
from photo_search_engine_amd.index import FlatIndex
d = 48
x = O.synth_rows(O.SEED_CORPUS, 0, 90000, d, True, "bf16")
c = IO.sample_centroids(x, 8, 9)
for dt in ("bf16", "f32"):
    ix = FlatIndex(d, "ip", dt)
    ix.add(c)
    for nq in (9, 256, 300, 5000, 90000):
        D, I = ix.search(x[:nq], 1)
        bad = np.flatnonzero((I[:, 0] < 0) | (I[:, 0] >= 8))
        S, Ie = O.knn_exact(ix.reconstruct_n(0, 8), x[:nq], 1, "ip")
        print(dt, nq, "bad", bad.size, bad[:5], "mismatch", int((I != Ie).sum()), flush=True)
