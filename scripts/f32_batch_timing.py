"""fp32 rows: batch timing of the native (fp32 MFMA) and int8 screens at 1M x 1536 (profiles/r03_f32_mfma_timing.txt)."""
import time, torch, numpy as np
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O
from photo_search_engine_amd.index import FlatIndex
for N, d, nq in ((1_000_000, 1536, 256), (1_000_000, 1536, 64)):
    ix = FlatIndex(d, "ip", "f32"); ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    q = torch.from_numpy(O.synth_rows(O.SEED_QUERIES, 0, nq, d, True, "f32")).cuda()
    I = torch.empty((nq, 100), dtype=torch.int64, device="cuda")
    for mode in ("native", "int8"):
        ix.set_screen(mode)
        for _ in range(2): ix.search_device_exact(q.data_ptr(), nq, 100, None, I.data_ptr(), None, 0, 0)
        torch.cuda.synchronize(); ix.set_timing(True); t = time.perf_counter()
        for _ in range(5): ix.search_device_exact(q.data_ptr(), nq, 100, None, I.data_ptr(), None, 0, 0)
        torch.cuda.synchronize(); el = (time.perf_counter() - t) / 5; ix.set_timing(False)
        km, kind = ix.timing_fetch()
        print(f"N={N} d={d} nq={nq} f32 {mode}: {el*1e3:.2f} ms/batch, screen {kind} {np.mean(km):.2f} ms", flush=True)
    ix.close()
