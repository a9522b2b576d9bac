"""Planning study for the certified int8 pre-screen: how many candidates per
query an int8 screen must pass to the exact refine at cfg3 (N=10M, d=1536, k=100).

Host-only numpy, synthetic cfg3 rows (oracle.synth_rows, bf16-rounded as stored) on a sample.
Per row x (bf16 values): scale_x = max|x| / 127, x8 = round(x / scale_x), e_x = x - scale_x x8.
Per query q (fp32): the same with scale_q, or a (hi, lo) pair of int8 vectors (two MFMAs per K-step,
16-bit effective precision).  Screen score s8 = scale_x scale_q <x8, q8> (exact int32 accumulate).
Per-row bound: |<x, q> - s8| <= eps_x = ||e_x|| ||q|| + ||scale_x x8|| ||e_q||.

A row can be dropped when s8 + eps_x < L, L = the k-th best (s8 - eps) over the candidates.  The
expected number of survivors at N rows follows from the sampled joint distribution of (s8, eps):
count(N) = N * P(s8 + eps >= L(N)), with L(N) found from the same sample by quantiles.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def quantise(v, axis=-1):
    scale = np.abs(v).max(axis=axis, keepdims=True) / 127.0
    v8 = np.rint(v / scale)
    return v8, scale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--dim", type=int, default=1536)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--target-rows", type=int, default=10_000_000)
    args = ap.parse_args()
    from oracle import oracle as O
    d = args.dim
    x = O.synth_rows(O.SEED_CORPUS, 0, args.rows, d, True, "bf16").astype(np.float64)
    q = O.synth_rows(O.SEED_QUERIES, 0, args.queries, d, True, "f32").astype(np.float64)
    x8, sx = quantise(x)
    xh = x8 * sx
    ex = np.linalg.norm(x - xh, axis=1)
    nxh = np.linalg.norm(xh, axis=1)
    s_true = x @ q.T
    frac = args.k / args.target_rows  # the k-th best at N rows sits at this upper quantile
    for mode in ("int8 query", "int8 (hi, lo) query"):
        q8, sq = quantise(q)
        qh = q8 * sq
        if mode.startswith("int8 (hi"):
            r = q - qh
            r8, sr = quantise(r)
            qh = qh + r8 * sr
        eq = np.linalg.norm(q - qh, axis=1)
        nq = np.linalg.norm(q, axis=1)
        s8 = xh @ qh.T
        eps = ex[:, None] * nq[None, :] + nxh[:, None] * eq[None, :]
        assert np.all(np.abs(s_true - s8) <= eps * (1 + 1e-9) + 1e-12), "bound violated"
        counts, errs = [], []
        for j in range(args.queries):
            lo = s8[:, j] - eps[:, j]
            hi = s8[:, j] + eps[:, j]
            L = np.quantile(lo, 1.0 - frac)           # k-th best lower bound at target N
            counts.append(np.mean(hi >= L) * args.target_rows)
            errs.append(np.median(np.abs(s_true[:, j] - s8[:, j])))
        print(f"{mode}: eps median {np.median(eps):.5f} max {eps.max():.5f}; |err| median {np.median(errs):.5f}; "
              f"expected survivors per query at N={args.target_rows:,}, k={args.k}: "
              f"median {np.median(counts):,.0f}, max {np.max(counts):,.0f}")


if __name__ == "__main__":
    main()
