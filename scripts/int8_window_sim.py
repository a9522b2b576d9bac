"""How many rows an int8-screen certificate must list on one tight cluster (the window analysis of
DESIGN.md §5 "Group residuals"): one cluster of 156,250 rows normalise(c + sigma g), d = 1536,
stored bf16; queries from the same cluster; k = 100.  Keys as the screen computes them (per-row
bf16 scale, int8 codes, beta = ||x - s c||; query codes t_q c_q): a row must be listed when its
key can reach the k-th best true score minus the query-side margin.  Variants: codes of x or of
x - mu (the group mean), and an exact (fp32-split) query (query error / 127).  numpy, CPU.
python scripts/int8_window_sim.py SIGMA"""
import numpy as np, sys
rng = np.random.default_rng(0)
d, n, sigma, k = 1536, 156250, float(sys.argv[1]) if len(sys.argv) > 1 else 0.3, 100
def unit(a): return a / np.linalg.norm(a, axis=-1, keepdims=True)
def bf16(a):
    u = a.astype(np.float32).view(np.uint32)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)
c = unit(rng.standard_normal(d)).astype(np.float32)
x = np.empty((n, d), np.float32)
for a in range(0, n, 20000):
    g = unit(rng.standard_normal((min(20000, n - a), d))).astype(np.float32)
    x[a:a+len(g)] = bf16(unit(c + sigma * g))
mu = bf16(x.mean(0))
qs = []
for j in range(8):
    q = unit(c + sigma * unit(rng.standard_normal(d))).astype(np.float32)
    qs.append(q)
def quant(v):
    s = bf16(np.abs(v).max(-1, keepdims=True) / 127.0)
    cc = np.clip(np.rint(v / s), -127, 127)
    e = v - s * cc
    return s, cc, np.linalg.norm(e, axis=-1)
for res in (False, True):
    r = x - mu if res else x
    s, cx, beta = quant(r)
    X = np.linalg.norm(s * cx, axis=1).max()
    out = []
    for q in qs:
        t = np.abs(q).max() / 127
        cq = np.clip(np.rint(q / t), -127, 127)
        eq = np.linalg.norm(q - t * cq)
        true = x.astype(np.float64) @ q
        sk = np.sort(true)[-k]
        key = (s[:, 0] * t) * (cx @ cq) + beta * np.linalg.norm(q) + (mu @ q if res else 0)
        for split in (False, True):
            qeps = X * (eq / 127 if split else eq)
            out.append((split, int((key >= sk - qeps).sum())))
    for split in (False, True):
        v = [o[1] for o in out if o[0] == split]
        print(f"sigma {sigma} residual={res} query_split={split}: rows to list per query (of {n}): median {int(np.median(v))} max {max(v)}  X={X:.3f} beta~{np.median(beta):.4f}")
