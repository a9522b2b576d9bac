#!/usr/bin/env python3
"""bench.py -- the BASELINE.json metric on MI355X: exact flat-IP k-NN queries/sec (+ recall@10 vs
the faiss-semantics CPU restatement), N=10M d=1536 bf16, batch=256, top-100 (BASELINE cfg3).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg1|cfg2|cfg4|cfg5]

One process per GPU: under torchrun (WORLD_SIZE set, which must equal --gpus), or -- when
--gpus N > 1 is given without a launcher -- this process spawns N fresh child processes with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set and never touches a GPU itself.  The corpus is row-sharded: rank r holds rows
[r*N/G, (r+1)*N/G) generated in place in HBM (counter-hash generator, bit-identical to
oracle/vs_oracle.c); every rank holds the same synthetic query batch.  One step = the hot path on
one batch: per-shard exact search (pack -> MFMA screen with fused top-k -> merge -> exact
refine) and, for N > 1, an RCCL all-gather of the per-shard (fp64 score, id) lists + the on-device
merge (photo_search_engine_amd/distributed.py, the product's multi-GPU layer).  Prints ONE JSON line on rank 0 with `roofline` (dominant kernel, HIP events on its own
stream) and `cpu_baseline` (faiss fp32 restatement on this host, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

WORKLOADS = {
    # name: (N, d, dtype, nq, k, description); stored rows are `dtype`
    "cfg3": (10_000_000, 1536, "bf16", 256, 100, "N=10M d=1536 bf16, batch=256, top-100 (MFMA path)"),
    "cfg2": (1_000_000, 1536, "f32", 1, 10, "N=1M d=1536 fp32, batch=1, top-10 (GEMV path)"),
    "cfg4": (100_000_000, 768, "f16", 256, 10, "N=100M d=768 fp16, batch=256, top-10 (row-sharded)"),
}
# BASELINE cfg1: the reference's plumbing config, one query per VectorStore.search call
CFG1 = (10_000, 1536, "f32", 1, 10, "N=10k d=1536 fp32, one query per VectorStore.search call, top-10 (plumbing)")
IVF_WORKLOADS = {
    # name: (N, d, dtype, nq, k, nlist, nprobe, description)
    "cfg5": (50_000_000, 1536, "bf16", 256, 10, 4096, 32,
             "IVF-Flat nlist=4096 nprobe=32, N=50M d=1536 bf16, batch=256, top-10 (coarse probe + list scans)"),
}
SEED_CORPUS = 20260417
SEED_QUERIES = 20260418
SEED_CENTROIDS = 20260419
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_BF16_PEAK_TF = 2500.0
MFMA_I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: I8 16x16x64 runs at 2x the BF16 rate per clock
DEFAULT_SCREEN = {"cfg3": "int8", "cfg2": "int8", "cfg4": "int8"}  # (all flat workloads: inner product)
METRICS = {
    "cfg3": "kNN queries/sec + recall@10 vs FAISS, N=10M d=1536 batch=256",
    "cfg2": "kNN queries/sec vs FAISS, N=1M d=1536 fp32 batch=1 top-10",
    "cfg4": "kNN queries/sec vs FAISS, N=100M d=768 fp16 batch=256 top-10",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS) + sorted(IVF_WORKLOADS) + ["cfg1"])
    ap.add_argument("--rows", type=int, default=0, help="override corpus rows (testing)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="measure ONE rank of a G-shard step on this GPU: its N/G-row shard, the two-phase "
                         "search and both exchanges over a one-rank process group (not the BASELINE line)")
    ap.add_argument("--one-phase", action="store_true",
                    help="N > 1 / --shard-of: keep the one-phase local search (A/B of the two-phase step)")
    ap.add_argument("--metric", default="ip", choices=["ip", "l2"],
                    help="flat workloads: the index metric (BASELINE's configs are inner product; l2 = the "
                         "reference's metric='l2' stores, utils/vector_store.py:79-81)")
    ap.add_argument("--screen", default=None, choices=["native", "int8"],
                    help="flat workloads: the screen of the timed steps (default: int8); "
                         "with int8 the native screen is timed too and reported beside it")
    ap.add_argument("--cpu-sample-rows", type=int, default=0,
                    help="rows of the corpus the CPU baseline scans (default: the whole corpus if host memory allows)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (with --dist-backend gloo on a 1-GPU box)")
    ap.add_argument("--no-recall", action="store_true", help="cfg5: skip the exact ground truth (profiling runs)")
    ap.add_argument("--skew", type=float, default=0.0,
                    help="cfg5: Zipf exponent of the cluster sizes (0 = equal-sized clusters; 1.1 = a heavy head)")
    ap.add_argument("--ivf-qtile", default="split", choices=["plain", "split"],
                    help="cfg5: query tiles of the MFMA list scans' first pass (the other mode runs beside)")
    ap.add_argument("--ivf-scan", default="auto", choices=["auto", "gemv", "mfma"],
                    help="cfg5: list-scan kernels (auto: MFMA screen for lists probed by many queries; "
                         "with auto the GEMV-only scan is timed too and reported beside it)")
    ap.add_argument("--data", default="iso", choices=["iso", "mixture", "mixture-sorted"],
                    help="flat workloads: isotropic rows (default, the BASELINE data), or a Gaussian mixture "
                         "(64 clusters, sigma --sigma) in random / cluster-sorted insertion order; the "
                         "mixture runs report no CPU baseline (their rows are made on the GPU)")
    ap.add_argument("--sigma", type=float, default=1.0, help="--data mixture: cluster spread")
    ap.add_argument("--iso-data", action="store_true",
                    help="cfg5: isotropic rows (the flat bench's data) instead of the Gaussian mixture")
    ap.add_argument("--k1-schedule", type=int, default=None, choices=[0, 1],
                    help="the direct K1 screens' K-step schedule (include/vs.h vs_set_k1_schedule; default: the library's)")
    ap.add_argument("--traffic-file", default=None,
                    help="rocprofv3 PMC summary giving HBM bytes per launch (default profiles/traffic_<workload>.json)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return int(so.getsockname()[1])


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: run N fresh children of this script, one per GPU (rank r on
    cuda:r), with the torch.distributed environment set; rank 0 prints the JSON line.  The parent
    never initialises a GPU (no torch import) and never re-execs itself; if a rank fails, the
    others are stopped (they would wait in a collective) and the parent exits non-zero."""
    import subprocess
    env = dict(os.environ)
    env.update({"WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()),
                "LOCAL_WORLD_SIZE": str(n)})
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                _progress(f"rank {procs.index(p)} exited with {code}: stopping the other ranks")
                for o in live:
                    o.terminate()
    return rc


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE={env_world} from the launcher")
    if args.workload == "cfg1":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            sys.exit("cfg1 is a single-GPU workload")
        return run_cfg1(args)
    if args.workload in IVF_WORKLOADS:
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            sys.exit("cfg5 is a single-GPU workload")
        return run_ivf(args)
    import torch
    import torch.distributed as dist

    from photo_search_engine_amd.distributed import ShardedFlatIndex, shard_range
    from photo_search_engine_amd.index import set_k1_schedule, synthesize_device

    if args.k1_schedule is not None:
        set_k1_schedule(args.k1_schedule)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(local)
        if args.shard_of > 1:  # the one-rank group that carries the exchanges of --shard-of
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(args.dist_backend, rank=0, world_size=1)
    dev = torch.device("cuda", local)

    N, d, dtype, nq, k, desc = WORKLOADS[args.workload]
    if args.rows:
        N = args.rows
    G = world
    row0, n_local = shard_range(N, rank, G)
    if args.shard_of > 1:
        row0, n_local = shard_range(N, 0, args.shard_of)

    t_build = time.time()
    # the product's multi-GPU layer: one row shard per rank, all-gather + device merge (G > 1)
    sh = ShardedFlatIndex(d, args.metric, dtype, device=local)
    if args.shard_of > 1:
        sh.shards_hint = args.shard_of
    if args.data != "iso":
        # clustered rows: normalise(c[cid] + sigma g) over 64 unit centroids (the cfg5 data model,
        # `_mixture_rows`); sorted = inserted cluster by cluster (cid non-decreasing in row order)
        C = 64
        cen = torch.empty((C, d), dtype=torch.float32, device=dev)
        synthesize_device(local, SEED_CENTROIDS, 0, C, d, cen.data_ptr(), True, dtype, torch.cuda.current_stream(dev).cuda_stream)
        sh.row0, sh.n_total = row0, N
        chunk = 1 << 18
        for r in range(0, n_local, chunk):
            m = min(chunk, n_local - r)
            if args.data == "mixture":
                xr = _mixture_rows(SEED_CORPUS, row0 + r, m, d, cen, args.sigma, dev, torch.cuda.current_stream(dev).cuda_stream)
            else:
                xr = _mixture_rows_sorted(SEED_CORPUS, row0 + r, m, N, d, cen, args.sigma, dev,
                                          torch.cuda.current_stream(dev).cuda_stream)
            sh.index.add_device(xr.data_ptr(), m, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize()
            del xr
    elif args.shard_of > 1:
        sh.row0, sh.n_total = row0, N
        sh.index.add_synthetic(SEED_CORPUS, row0, n_local, True)
    else:
        sh.add_synthetic(SEED_CORPUS, N, True)
    ix = sh.index
    q = torch.empty((nq, d), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    synthesize_device(local, SEED_QUERIES, 0, nq, d, q.data_ptr(), True, dtype, stream.cuda_stream)
    if args.data != "iso":
        q.copy_(_mixture_rows(SEED_QUERIES, 0, nq, d, cen, args.sigma, dev, stream.cuda_stream))
    torch.cuda.synchronize()
    screen = args.screen or DEFAULT_SCREEN.get(args.workload, "native")
    if args.one_phase:
        sh._two_phase_ok = lambda *a_: False
    elif args.shard_of > 1 and screen == "int8":
        sh.floor_override = _shard_floor(args, N, d, dtype, nq, k, q, local, dev, torch)
    t_build = time.time() - t_build
    result = {}
    per_rank = {}
    host_ms = {}
    host_in_loop = {}

    def step():
        result["D"], result["I"], result["S"] = sh.search(q, k)

    def timed(scr):
        """warmup + exactly `steps` timed steps on screen `scr`: (elapsed s over ranks, kernel ms, kind, uncert)"""
        t_sw = time.time()
        ix.set_screen(scr)  # int8: builds the int8 copy of the shard's rows (untimed)
        t_sw = time.time() - t_sw
        u0 = ix.uncertified_count()
        for _ in range(args.warmup):
            step()
            # (one step at a time: the index's screen-health feedback -- a batch's certificate
            # failures read back behind it -- then reaches the next warmup step, as it does between
            # the synchronous calls of a server; the timed steps are enqueued back to back)
            torch.cuda.synchronize()
        ix.timing_fetch()  # drop warmup events
        sh.exchange_times_fetch()
        ix.set_timing(True)
        sh.exchange_timing = True
        if G > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t_in = 0.0  # host time inside the step calls (diagnostic: ~ elapsed means host-bound)
        for _ in range(args.steps):
            ts = time.perf_counter()
            step()
            t_in += time.perf_counter() - ts
        torch.cuda.synchronize()
        if G > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        ix.set_timing(False)
        sh.exchange_timing = False
        km, kd = ix.timing_fetch()
        xm = sh.exchange_times_fetch()
        # host time to enqueue one step with the device idle (untimed diagnostic: a step whose host
        # side exceeds its device time leaves the device waiting on the host)
        hs = []
        for _ in range(3):
            torch.cuda.synchronize()
            th = time.perf_counter()
            step()
            hs.append((time.perf_counter() - th) * 1e3)
        torch.cuda.synchronize()
        host_ms[scr] = float(np.median(hs))
        host_in_loop[scr] = t_in * 1e3 / max(args.steps, 1)
        per_rank[scr] = [float(np.mean(km)) if km else float("nan"), sum(xm) / args.steps, len(xm) / args.steps,
                         el * 1e3 / args.steps, float(n_local)]
        if G > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
            per_rank[scr] = _gather_rows(per_rank[scr], G, dev, args.dist_backend, torch, dist)
        else:
            per_rank[scr] = [per_rank[scr]]
        return el, km, kd, ix.uncertified_count() - u0, t_sw

    es = 2 if dtype in ("bf16", "f16") else 4
    alt = None
    if screen == "int8":  # the native (bf16 MFMA) screen of the same corpus, reported beside it
        el_n, km_n, kind_n, unc_n, _ = timed("native")
        res_native = {k_: v.clone() for k_, v in result.items()}
        kn = float(np.mean(km_n)) if km_n else float("nan")
        bytes_n = n_local * d * es + nq * d * es + nq * k * 12 + (n_local * 4 if args.metric == "l2" else 0)
        alt = {"screen": "native", "kernel": _kernel_name(kind_n, dtype, d), "value": round(nq * args.steps / el_n, 2),
               "ms_per_step": round(el_n * 1e3 / args.steps, 4), "kernel_ms": round(kn, 4),
               "hbm_frac": round(bytes_n / (kn * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
               "uncertified_first_pass": unc_n}
    elapsed, kms, kind, uncert, t_switch = timed(screen)
    full_scan = ix.full_scan_count()  # queries no bounded screen certified (answered by the full scan)
    if G > 1:
        t = torch.tensor([full_scan], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        full_scan = int(t.item())
    if alt is not None:  # both screens return the same exact answer
        if sh.floor_override is not None:
            # --shard-of: the two-phase rank returns its share of the GLOBAL top-k exactly (entries at
            # least as good as the G-shard floor), the native beside it its local top-k: compare those
            fl = sh.floor_override[:, k - 1:k]
            m1 = result["S"] >= fl if args.metric == "ip" else result["S"] <= fl
            m2 = res_native["S"] >= fl if args.metric == "ip" else res_native["S"] <= fl
            alt["identical_results"] = bool(torch.equal(m1, m2) and torch.equal(result["I"][m1], res_native["I"][m2])
                                            and torch.equal(result["S"][m1], res_native["S"][m2]))
            alt["compared"] = "entries at least as good as the G-shard floor"
        else:
            alt["identical_results"] = bool(torch.equal(result["I"], res_native["I"]) and
                                            torch.equal(result["S"], res_native["S"]))
        del res_native

    ms_per_step = elapsed * 1e3 / args.steps
    qps = nq * args.steps / elapsed
    kavg = float(np.mean(kms)) if kms else float("nan")
    if kind in ("mfma_i8", "gemv_i8"):
        # streamed per launch: the int8 codes + per-row (scale, error norm) + the queries (int8 for
        # the MFMA screen, fp32 for the GEMV) + the candidate lists
        alg_bytes = n_local * d + n_local * 4 + nq * d * (1 if kind == "mfma_i8" else 4) + nq * k * 12
        if args.metric == "l2":
            alg_bytes += n_local * 4  # the rows' ||x||^2
        peak_flops = MFMA_I8_PEAK_TOPS
    else:
        alg_bytes = n_local * d * es + nq * d * es + nq * k * 12 + (n_local * 4 if args.metric == "l2" else 0)
        peak_flops = MFMA_BF16_PEAK_TF
    alg_flops = 2.0 * n_local * d * nq
    achieved_gbs = alg_bytes / (kavg * 1e-3) / 1e9
    traffic = _traffic(args.traffic_file, args.workload, n_local, kind)

    out = None
    if rank == 0:
        out = {
            # a --rows run is a different configuration: its metric names the rows it ran on
            "metric": (METRICS[args.workload] if not args.rows else
                       METRICS[args.workload].split(",")[0] + f" (rows override: N={N}, not the BASELINE config)") +
                      ("" if args.metric == "ip" else " [L2 metric, not the BASELINE config]") +
                      (f" [one rank of a {args.shard_of}-shard step: {n_local} rows, both merges on the "
                       "rank's own lists (a one-rank group exchanges nothing: the G-rank run adds two RCCL "
                       "all-gathers), the G-shard floor precomputed; not the BASELINE line]"
                       if args.shard_of > 1 else ""),
            "value": round(qps, 2),
            "unit": "queries/s",
            "n_gpus": G,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "host_enqueue_ms": round(host_ms.get(screen, float("nan")), 4),
            "host_ms_in_loop": round(host_in_loop.get(screen, float("nan")), 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            # the stored rows' precision: every returned score is the canonical score of the stored
            # (dtype) row; the int8 screen only pre-selects rows for the exact refine
            "dtype": dtype,
            "screen": "int8" if kind in ("mfma_i8", "gemv_i8") else "native",
            "data": ("synthetic (counter-hash N(0,1) rows, L2-normalised, seeds 20260417/20260418)" if args.data == "iso"
                     else f"synthetic Gaussian mixture ({args.data}, 64 clusters, sigma {args.sigma}), L2-normalised"),
            "config": {"workload": args.workload, "desc": desc, "N": N, "d": d, "batch": nq, "k": k, "metric": args.metric,
                       "n_local": n_local, "stored_rows": dtype, "screen": screen,
                       "shard_of": args.shard_of or None,
                       "two_phase": bool(sh._two_phase_ok(sh.index, nq, k)) and (G > 1 or args.shard_of > 1),
                       "parallelism": f"row-shard x{G}" + (
                           (" + RCCL all-gather" if args.dist_backend == "nccl" else f" + {args.dist_backend} all-gather")
                           if G > 1 else "")},
            "roofline": {
                # the int8 main pass runs the direct form when d is a multiple of 256 (vs_kernels.hip)
                "kernel": _kernel_name(kind, dtype, d, n_local, args.metric,
                                       bool(ix.screen_state()["group_residuals"]) if kind == "mfma_i8" else False),
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms": round(kavg, 4),
                "alg_bytes_per_launch": alg_bytes,
                "mfma_tflops": round(alg_flops / (kavg * 1e-3) / 1e12, 1),
                "mfma_frac": round(alg_flops / (kavg * 1e-3) / 1e12 / peak_flops, 4),
                "mfma_peak_tflops": peak_flops,
                # the same box's zero / real operand pair of the main screen kernels (vs_screen_probe)
                "power_pair": _power_pair(ix, q, nq, kind, alg_bytes,
                                          n_local * d * es + nq * d * es + nq * k * 12 +
                                          (n_local * 4 if args.metric == "l2" else 0),
                                          torch.cuda.current_stream(dev).cuda_stream),
            },
            # first-pass certificate failures; every one was re-searched exactly (search_device_exact)
            "uncertified_first_pass": uncert,
            "full_scan": full_scan,
            # group residuals, margins and the screen-health state after the timed steps (vs_screen_state)
            "screen_state": ix.screen_state(),
            "build_s": round(t_build, 2),
        }
        if G > 1 or args.shard_of > 1:
            # per rank: its dominant kernel's mean ms (HIP events in the library), the all-gathers'
            # ms per step (HIP events around each collective on the calling stream) and its wall ms
            out["per_rank"] = [{"rank": r, "n_local": int(v[4]), "k1_ms": round(v[0], 4), "exchange_ms": round(v[1], 4),
                                "exchanges_per_step": round(v[2], 2), "wall_ms_per_step": round(v[3], 4)}
                               for r, v in enumerate(per_rank[screen])]
        if kind in ("mfma_i8", "gemv_i8"):
            out["int8_copy"] = {"hbm_bytes": ix.screen_copy_bytes(), "build_s": round(t_switch, 2),
                                "note": "int8 codes + bf16 (scale, error norm) per row on top of the stored rows "
                                        "(allocated capacity)"}
        if alt is not None:
            out["native_screen"] = alt
    if rank == 0 and G == 1 and not args.no_cpu_baseline and args.data == "iso" and args.metric == "ip" and not args.shard_of:
        out["cpu_baseline"], out["recall@10"], out["parity"] = cpu_baseline_and_recall(
            args, N, d, dtype, nq, k, local, torch, (result["D"].cpu().numpy(), result["I"].cpu().numpy()))
    if rank == 0:
        print(json.dumps(out), flush=True)
    sh.close()
    if G > 1 or args.shard_of > 1:
        dist.destroy_process_group()


def _power_pair(ix, q, nq: int, kind: str, alg_bytes: int, alg_bytes_native: int, stream: int) -> dict:
    """The box's own zero / real operand pair, measured in this process after the timed steps
    (include/vs.h ``vs_screen_probe``): one launch of each main screen kernel over the same rows with
    every threshold at +inf (the K loop + the epilogue's bound test, no survivors), once with the real
    query tile and once with the tile zeroed (one MFMA operand all zeros).  Same code, same bytes,
    same cycles per K-step: what differs is the clock the board holds under the MFMAs on real
    operands (DESIGN §6 "Power").  A reference beside ``frac``, not a bound: boards differ by up
    to ~12 % (MI355X_MICROARCH DVFS), and the product kernel also inserts survivors."""
    if kind != "mfma_i8":
        return {}
    out = {}
    for scr, ab in (("int8", alg_bytes), ("native", alg_bytes_native)):
        try:
            real = ix.screen_probe(q.data_ptr(), nq, scr, False, stream)
            zero = ix.screen_probe(q.data_ptr(), nq, scr, True, stream)
        except Exception as e:  # (the probe needs the direct screens: d a multiple of 256)
            out[scr] = {"skipped": str(e)[:120]}
            continue
        out[scr] = {"loop_ms": round(real, 4), "zero_query_ms": round(zero, 4),
                    "loop_frac": round(ab / (real * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "zero_query_frac": round(ab / (zero * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    out["note"] = ("five launches back to back per form, the fastest; thresholds at +inf (no survivors); "
                   "zero_query = the packed query tile zeroed; same process and box as the timed steps")
    return out


def _gather_rows(row, G, dev, backend, torch, dist):
    """Every rank's list of floats -> rank-ordered list of lists (one small all-gather)."""
    t = torch.tensor(row, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    out = [torch.empty_like(t) for _ in range(G)]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def _kernel_name(kind: str, dtype: str, d: int, n_local: int = 0, metric: str = "ip", residual: bool = False) -> str:
    """The screen kernel the library ran (vs_kernels.hip): the main passes take the direct forms
    when the K-steps per padded row are a multiple of 4 (int8: 64-element K-steps; bf16 / f16: 32);
    int8 codes taken against group means (``residual``) run the inner-product form that adds
    <mu_g, q> to every key."""
    dpad = max(-(-d // 64) * 64, 64)
    if kind == "full_scan":
        return "k_full_scan"
    if kind == "mfma_i8" and dpad % 256 == 0 and dpad >= 512:
        from photo_search_engine_amd.index import k1_schedule  # (inner product: the mid-step forms)
        ms = "_ms" if metric == "ip" and k1_schedule() == 1 else ""
        if residual and metric == "ip":
            return "k_screen_i8d_res" + ms
        return "k_screen_i8d" + ms
    if kind == "mfma" and dtype in ("bf16", "f16") and dpad % 128 == 0 and dpad >= 256:
        return "k_screen_d16"
    return f"k_screen_{kind}"


def _shard_floor(args, N, d, dtype, nq, k, q, local, dev, torch):
    """--shard-of G (untimed setup): phase A of the two-phase search on each of the G shards in turn
    (a temporary index per shard), merged on the device -- the floor all G ranks would share after
    the first exchange, which the measured rank then uses in place of its one-rank exchange's."""
    from photo_search_engine_amd.distributed import METRIC_CODES, _device_merge, shard_range
    from photo_search_engine_amd.index import FlatIndex
    G = args.shard_of
    Sg = torch.empty((G, nq, k), dtype=torch.float64, device=dev)
    Ig = torch.empty((G, nq, k), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for s_ in range(G):
        r0, n = shard_range(N, s_, G)
        t = FlatIndex(d, args.metric, dtype, device=local)
        t.add_synthetic(SEED_CORPUS, r0, n, True)
        t.set_screen("int8")
        pend = t.search_phase_a(q.data_ptr(), nq, k, G, Sg[s_].data_ptr(), Ig[s_].data_ptr(), r0, stream)
        t.search_pending_free(pend)
        torch.cuda.synchronize()
        t.close()
    return _device_merge(METRIC_CODES[args.metric], Sg, Ig, k)[0]


def _host_mem_bytes() -> int:
    try:
        return os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError):
        return 0


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_and_recall(args, N, d, dtype, nq, k, local, torch, gpu_full):
    """CPU baseline: the faiss IndexFlatIP fp32 restatement (oracle/vs_oracle.c, OpenMP) on this
    host's cores, over the whole corpus when it fits the host-memory budget (cfg3: ~7 s of 16-thread
    work, so no extrapolation), else a leading row sample scaled by N / rows; plus recall@10 and the
    exact-id match of the GPU path against it on the same rows (the GPU re-searches the sample when
    it is not the whole corpus).  Batches of >= 20 queries take faiss' BLAS path on all threads;
    single queries take faiss' sequential scan, which runs on ONE thread (faiss parallelises that path
    over queries only), so batch=1 workloads report the one-thread rate and, beside it, the rate of
    `threads` concurrent single-query calls.  Every line also carries one single query's latency."""
    from oracle import oracle as O
    from photo_search_engine_amd.index import FlatIndex

    ns = args.cpu_sample_rows or N
    # keep the fp32 copy well inside host memory: 40% of the machine, and never above 96 GiB (the
    # GPU box caps a command's host memory well below the machine's total)
    budget = min(0.4 * (_host_mem_bytes() or 1 << 40), 96 * (1 << 30))
    if ns * d * 4 > budget:
        ns = int(budget // (d * 4))
    ns = min(ns, N)
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores) or cores))
    t0 = time.perf_counter()
    x = O.synth_rows(SEED_CORPUS, 0, ns, d, True, dtype)  # the GPU's stored values, upcast to fp32
    t_gen = time.perf_counter() - t0
    q = O.synth_rows(SEED_QUERIES, 0, nq, d, True, dtype)
    O.knn_faiss_fp32(x[:1000], q[:1], 5, "ip", 1)  # warm
    scale = N / ns
    # one query through faiss' sequential scan (one thread), scaled to the whole corpus
    t0 = time.perf_counter()
    D1, I1 = O.knn_faiss_fp32(x, q[:1], k, "ip", 1)
    t1 = (time.perf_counter() - t0) * scale
    if nq == 1:
        qm = O.synth_rows(SEED_QUERIES, 0, threads, d, True, dtype)
        t0 = time.perf_counter()
        O.knn_faiss_fp32(x, qm, k, "ip", threads)  # `threads` single queries at once (< 20: sequential path)
        tm = (time.perf_counter() - t0) * scale
        Dc, Ic = D1, I1
        cpu_qps, used = 1.0 / t1, 1
        how = (f"faiss IndexFlatIP fp32 restatement (oracle/vs_oracle.c), single query: faiss' sequential scan on one "
               f"thread, {t1 * 1e3:.1f} ms per query; {threads} concurrent single-query scans on {threads} threads: "
               f"{threads / tm:.2f} queries/s")
    else:
        t0 = time.perf_counter()
        Dc, Ic = O.knn_faiss_fp32(x, q, k, "ip", threads)
        tc = (time.perf_counter() - t0) * scale
        cpu_qps, used = nq / tc, threads
        how = (f"faiss IndexFlatIP fp32 restatement (oracle/vs_oracle.c: blocked fp32 GEMM + per-thread heaps, "
               f"{threads} OpenMP threads) for the same {nq} queries (k={k}): {tc:.2f} s of search")
    del x
    if ns == N:
        Dg, Ig = gpu_full
    else:  # GPU on the same sample
        ix = FlatIndex(d, "ip", dtype, device=local)
        ix.add_synthetic(SEED_CORPUS, 0, ns, True)
        Dg, Ig = ix.search(q, k)
        ix.close()
    rec10 = O.recall_at(Ig, Ic, min(10, k))
    exact_match = float(np.mean(Ig == Ic))
    max_err = float(np.max(np.abs(Dg.astype(np.float64) - Dc)))
    scope = "the whole corpus" if ns == N else f"the first {ns} rows, timings scaled by N/{ns}"
    cpu = {"value": round(cpu_qps, 3), "unit": "queries/s", "cores": used, "kind": "port",
           "cpu_model": _cpu_model(), "host_threads": threads,
           "latency_nq1_ms": round(t1 * 1e3, 2),
           "sample": f"{how}; over {scope} ({ns} x {d}); +{t_gen:.1f} s to generate the rows, untimed"}
    parity = {"rows": ns, "exact_id_match_vs_faiss32": round(exact_match, 6),
              "max_abs_score_err_vs_faiss32": max_err}
    return cpu, round(rec10, 6), parity


def _traffic(path, workload: str, n_local: int, kind: str = "", skew: float = 0.0):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary of this
    configuration (profiles/traffic_<workload>_<kind>[_n<rows>].json, scripts/prof_summary.py)."""
    import glob
    paths = [path] if path else sorted(glob.glob(os.path.join(REPO, "profiles", f"traffic_{workload}_{kind}*.json")))
    for p in paths:
        try:
            with open(p) as f:
                tr = json.load(f)
        except (OSError, ValueError):
            continue
        if tr.get("workload") == workload and tr.get("n_local") == n_local and float(tr.get("skew", 0.0)) == skew:
            return tr.get("hbm_bytes_per_launch")
    return None


def _progress(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class _heartbeat:
    """Print a progress line every 30 s while a long native call runs (ctypes releases the GIL)."""

    def __init__(self, msg: str) -> None:
        import threading
        self.msg, self.stop = msg, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self) -> None:
        t0 = time.time()
        while not self.stop.wait(30.0):
            _progress(f"{self.msg} ... {time.time() - t0:.0f} s")

    def __enter__(self):
        _progress(self.msg)
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()
        _progress(f"{self.msg}: done")


def _mixture_rows_sorted(seed, r0, m, n_total, d, centroids, sigma, dev, stream):
    """As `_mixture_rows`, with row i in cluster floor(i * C / n_total): the corpus inserted cluster
    by cluster (the int8 screen's seed sample then sees whole clusters per workgroup)."""
    import torch

    from photo_search_engine_amd.index import synthesize_device
    g = torch.empty((m, d), dtype=torch.float32, device=dev)
    synthesize_device(dev.index, seed, r0, m, d, g.data_ptr(), True, "f32", stream)
    rows = torch.arange(r0, r0 + m, dtype=torch.int64, device=dev)
    cid = torch.clamp(rows * centroids.shape[0] // n_total, max=centroids.shape[0] - 1)
    x = centroids[cid] + sigma * g
    return x / torch.linalg.vector_norm(x, dim=1, keepdim=True)


def _mixture_rows(seed, r0, m, d, centroids, sigma, dev, stream, cdf=None):
    """Synthetic IVF corpus / query rows: a Gaussian mixture over the coarse centroids (the data
    model IVF exists for).  Row i = normalise(c[cid(i)] + sigma * g_i), g_i the unit counter-hash
    Gaussian row i of `seed` (bit-identical generator of oracle/vs_oracle.c).  cid(i) = h(i) mod
    nlist for equal-sized clusters (h a multiplicative hash), or, with `cdf` (the cumulative cluster
    weights), the inverse CDF of the hashed uniform h(i) / 2^31: Zipf-sized clusters.
    Deterministic: elementwise torch ops + the row norm on the same device."""
    import torch

    from photo_search_engine_amd.index import synthesize_device
    g = torch.empty((m, d), dtype=torch.float32, device=dev)
    synthesize_device(dev.index, seed, r0, m, d, g.data_ptr(), True, "f32", stream)
    rows = torch.arange(r0, r0 + m, dtype=torch.int64, device=dev)
    h = ((rows * 2654435761) >> 7)
    if cdf is None:
        cid = h % centroids.shape[0]
    else:
        u = ((h * 0x9E3779B1) & 0x7FFFFFFF).to(torch.float64) / 2147483648.0
        cid = torch.clamp(torch.searchsorted(cdf, u), max=centroids.shape[0] - 1)
    x = centroids[cid] + sigma * g
    return x / torch.linalg.vector_norm(x, dim=1, keepdim=True)


def run_cfg1(args):
    """BASELINE cfg1 end to end through the drop-in: ``VectorStore(dimension=1536)`` over 10k raw
    rows (bulk ``add``; the store normalises them as the reference does), one step = ONE
    ``store.search(query_list, 10)`` call -- host normalisation, the C-ABI call (H2D query, the
    exact full scan of the 61 MB corpus in one launch, D2H) and the result dicts -- over a cycle of
    256 distinct queries.
    value = calls per second; the dominant kernel's time comes from the library's HIP events.
    Beside it: the faiss IndexFlatIP sequential scan (nq < 20) restated on one host thread, the
    per-call latency faiss-cpu gives the reference at this config, and the ids of every timed call
    checked against the oracle."""
    import tempfile

    import torch

    from photo_search_engine_amd.vector_store import VectorStore
    N, d, dtype, nq, k, desc = CFG1
    if args.rows:
        N = args.rows
    torch.cuda.set_device(0)
    from photo_search_engine_amd.index import synthesize_device
    tmp = tempfile.mkdtemp(prefix="bench-cfg1-")
    t_build = time.time()

    def raw_rows(seed, n):  # raw (un-normalised) embeddings, generated on the device, to the host
        t = torch.empty((n, d), dtype=torch.float32, device="cuda")
        synthesize_device(0, seed, 0, n, d, t.data_ptr(), False, "f32", torch.cuda.current_stream().cuda_stream)
        return t.cpu().numpy()

    x = raw_rows(SEED_CORPUS, N)
    qs = raw_rows(SEED_QUERIES, 256)
    store = VectorStore(dimension=d, index_path=os.path.join(tmp, "photo_search.index"),
                        metadata_path=os.path.join(tmp, "metadata.json"))
    store.add(x, [{"photo_path": f"/photos/{i:05d}.jpg", "row": i} for i in range(N)])
    t_build = time.time() - t_build
    qlists = [qs[i].tolist() for i in range(qs.shape[0])]  # the embedding service hands over lists
    ix = store.index
    for i in range(args.warmup):
        store.search(qlists[i % 256], k)
    ix.timing_fetch()
    ix.set_timing(True)
    got = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        got.append(store.search(qlists[i % 256], k))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ix.set_timing(False)
    kms, kinds = ix.timing_fetch()
    kavg = float(np.mean(kms)) if kms else float("nan")
    alg_bytes = N * d * 4 + d * 4 + k * 12
    lat_ms = el * 1e3 / args.steps
    out = {"metric": "VectorStore.search calls/sec (N=10k d=1536 fp32, batch=1, top-10, end to end)" +
                     ("" if not args.rows else f" (rows override: N={N}, not the BASELINE config)"),
           "value": round(args.steps / el, 2), "unit": "queries/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(lat_ms, 4), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": dtype, "screen": "native",
           "data": "synthetic raw counter-hash N(0,1) embeddings (seeds 20260417/20260418), normalised by the store",
           "config": {"workload": "cfg1", "desc": desc, "N": N, "d": d, "batch": 1, "k": k, "metric": "cosine",
                      "api": "VectorStore.search (host lists in, result dicts out)", "parallelism": "1 GPU"},
           "roofline": {"kernel": _kernel_name(kinds if kinds != "none" else "gemv", dtype, d), "bound": "hbm",
                        "achieved": round(alg_bytes / (kavg * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg_bytes / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "kernel_ms": round(kavg, 4), "alg_bytes_per_launch": alg_bytes,
                        "note": "61 MB per call is a few microseconds of HBM: the call is launch/latency-bound"},
           "build_s": round(t_build, 2)}
    if not args.no_cpu_baseline:
        from oracle import oracle as O
        xn = np.stack([np.asarray(O.np_normalize_like_reference(r), dtype=np.float32) for r in x])
        qn = np.stack([np.asarray(O.np_normalize_like_reference(r), dtype=np.float32) for r in qs])
        reps = 200
        O.knn_faiss_fp32(xn, qn[:1], k, "ip", 1)  # warm
        t0 = time.perf_counter()
        for i in range(reps):
            O.knn_faiss_fp32(xn, qn[i % 256:i % 256 + 1], k, "ip", 1)
        t1 = (time.perf_counter() - t0) / reps
        S, I = O.knn_exact(xn, qn, k, "ip")
        ok = sum(int([r["metadata"]["row"] for r in res] == I[i % 256].tolist() and
                     [r["distance"] for r in res] == S[i % 256].astype(np.float32).tolist())
                 for i, res in enumerate(got))
        out["cpu_baseline"] = {"value": round(1.0 / t1, 2), "unit": "queries/s", "cores": 1, "kind": "port",
                               "cpu_model": _cpu_model(), "latency_nq1_ms": round(t1 * 1e3, 4),
                               "sample": f"faiss IndexFlatIP fp32 restatement (oracle/vs_oracle.c), sequential scan "
                                         f"(nq < 20) on one thread, {reps} single-query calls over the {N} normalised "
                                         f"rows; index search only (no wrapper overhead)"}
        out["parity"] = {"calls_checked": len(got), "calls_identical_to_oracle": ok}
    print(json.dumps(out), flush=True)
    ix.close()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


def run_ivf(args):
    """BASELINE cfg5: IVF-Flat (photo_search_engine_amd.ivf) on one GPU.  One step = one batch:
    exact coarse probe -> list scans (k_ivf_scan) -> exact refine.  Centroids are 4096 synthetic
    unit vectors (seed 20260419; training is not part of the metric); corpus and queries are a
    Gaussian mixture around them (sigma 1, `_mixture_rows`); `--iso-data` uses the isotropic flat-
    bench rows instead (no cluster structure: IVF recall is then ~0.03 at nprobe 32 by nature of
    the data, whatever the implementation).  recall@10 is measured against the exact flat top-10
    of the whole corpus (FlatIndex row shards, merged); `probed_recall@10` checks the IVF exactness
    contract at full size: every exact top-10 row whose list was probed must be returned."""
    import torch

    from photo_search_engine_amd.index import FlatIndex, synthesize_device
    from photo_search_engine_amd.ivf import IVFFlatIndex

    N, d, dtype, nq, k, nlist, nprobe, desc = IVF_WORKLOADS[args.workload]
    if args.rows:
        N = args.rows
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sigma = 1.0
    chunk = 1 << 20
    t_build = time.time()
    ix = IVFFlatIndex(d, nlist, "ip", dtype, device=0, nprobe=nprobe)
    c = torch.empty((nlist, d), dtype=torch.float32, device=dev)
    synthesize_device(0, SEED_CENTROIDS, 0, nlist, d, c.data_ptr(), True, dtype, stream)
    torch.cuda.synchronize()
    ix.set_centroids(c.cpu().numpy())

    cdf = None
    if args.skew > 0:  # Zipf(skew) cluster weights over a seeded permutation of the centroids
        rng = np.random.default_rng(SEED_CENTROIDS)
        w = 1.0 / np.arange(1, nlist + 1, dtype=np.float64) ** args.skew
        w = w[rng.permutation(nlist)]
        cdf = torch.from_numpy(np.cumsum(w) / w.sum()).to(dev)

    def corpus_chunk(r0, m):
        return _mixture_rows(SEED_CORPUS, r0, m, d, c, sigma, dev, stream, cdf)

    if args.iso_data:
        with _heartbeat(f"cfg5 build (isotropic rows): assigning and packing {N} rows"):
            ix.add_synthetic(SEED_CORPUS, 0, N, True)
        q = torch.empty((nq, d), dtype=torch.float32, device=dev)
        synthesize_device(0, SEED_QUERIES, 0, nq, d, q.data_ptr(), True, dtype, stream)
    else:
        ix.reserve(N)  # one page-pool allocation for the whole corpus
        with _heartbeat(f"cfg5 build (Gaussian mixture, sigma {sigma}): assigning and packing {N} rows"):
            for r0 in range(0, N, chunk):
                x = corpus_chunk(r0, min(chunk, N - r0))
                ix.add_device(x.data_ptr(), x.shape[0], stream)
                del x
        q = _mixture_rows(SEED_QUERIES, 0, nq, d, c, sigma, dev, stream, cdf).contiguous()
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    S = torch.empty((nq, k), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t_build = time.time() - t_build

    def step():
        ix.search_device(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), nprobe, stream)

    ix.set_scan(args.ivf_scan)
    ix.set_query_tiles(args.ivf_qtile)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ix.timing_fetch()
    ix.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ix.set_timing(False)
    kms, kbytes = ix.timing_fetch()
    kavg = float(np.mean(kms))
    alg_bytes = float(np.mean(kbytes))
    achieved = alg_bytes / (kavg * 1e-3) / 1e9
    sizes = ix.list_sizes()
    Ig = I.cpu().numpy()
    mfma_lists, uncert, mfma_bytes, gemv_bytes = ix.last_search_detail()
    gemv_beside = None
    if args.ivf_scan == "auto" and mfma_lists > 0:  # the GEMV-only scan on the same batch, beside
        Sg0 = S.cpu().numpy()
        ix.set_scan("gemv")
        step()
        torch.cuda.synchronize()
        ix.set_timing(True)
        t1 = time.perf_counter()
        for _ in range(max(2, args.steps // 2)):
            step()
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t1
        ix.set_timing(False)
        kms1, _ = ix.timing_fetch()
        gemv_beside = {"ms_per_step": round(el1 * 1e3 / max(2, args.steps // 2), 4),
                       "scan_ms": round(float(np.mean(kms1)), 4),
                       "identical_results": bool(np.array_equal(I.cpu().numpy(), Ig) and
                                                 np.array_equal(S.cpu().numpy(), Sg0))}
        ix.set_scan(args.ivf_scan)
    qtile_beside = None
    if mfma_lists > 0:  # the other query-tile mode of the MFMA list scans on the same batch, beside
        Sg0 = S.cpu().numpy()
        other = "split" if args.ivf_qtile == "plain" else "plain"
        ix.set_query_tiles(other)
        step()
        torch.cuda.synchronize()
        ix.set_timing(True)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t1
        ix.set_timing(False)
        kms1, _ = ix.timing_fetch()
        qtile_beside = {"qtile": other, "ms_per_step": round(el1 * 1e3 / args.steps, 4),
                        "scan_ms": round(float(np.mean(kms1)), 4),
                        "uncertified_first_pass": ix.last_search_detail()[1],
                        "identical_results": bool(np.array_equal(I.cpu().numpy(), Ig) and
                                                  np.array_equal(S.cpu().numpy(), Sg0))}
        ix.set_query_tiles(args.ivf_qtile)

    # probes (exact coarse top-nprobe) and per-batch scan volume, for the CPU baseline
    cf = FlatIndex(d, "ip", dtype, device=0)
    cf.add(ix.centroids())
    qh = q.cpu().numpy()
    _, P = cf.search(qh, nprobe)
    cf.close()
    pairs = float(sum(int(sizes[l]) for l in P.reshape(-1)))  # (row, query) dot products per batch

    # exact flat ground truth over the whole corpus, shard by shard (the IVF stays resident)
    shard = 6_250_000 if not args.no_recall else N + 1
    if args.no_recall:
        N_gt = 0
    else:
        N_gt = N
    parts_S, parts_I, lists_of = [], [], {}
    for r0 in range(0, N_gt, shard):
        n = min(shard, N - r0)
        fx = FlatIndex(d, "ip", dtype, device=0)
        if args.iso_data:
            fx.add_synthetic(SEED_CORPUS, r0, n, True)
        else:
            for s0 in range(r0, r0 + n, chunk):
                x = corpus_chunk(s0, min(chunk, r0 + n - s0))
                fx.add_device(x.data_ptr(), x.shape[0], stream)
                del x
        # host API: exact, with certificate failures re-searched (the device API only counts them)
        _, Ih = fx.search(qh, k)
        for i in np.unique(Ih):
            lists_of[int(i) + r0] = fx.reconstruct(int(i))
        Ih = Ih + r0
        parts_S.append(np.array([[float(lists_of[int(i)].astype(np.float64) @ qh[a].astype(np.float64)) for i in Ih[a]]
                                 for a in range(nq)]))
        parts_I.append(Ih)
        fx.close()
        _progress(f"cfg5 ground truth: rows {r0}..{r0 + n} searched")
    Sall = np.concatenate(parts_S, axis=1) if parts_S else np.zeros((nq, 0))
    Iall = np.concatenate(parts_I, axis=1) if parts_I else np.zeros((nq, 0), dtype=np.int64)
    Itrue = np.empty((nq, k), dtype=np.int64)
    for a in range(nq if parts_S else 0):
        order = np.lexsort((Iall[a], -Sall[a]))[:k]
        Itrue[a] = Iall[a, order]
    ids = sorted(lists_of)
    lst = dict(zip(ids, ix.assign(np.stack([lists_of[i] for i in ids])).tolist())) if ids else {}
    hit = sum(len(set(Ig[a, :10].tolist()) & set(Itrue[a, :10].tolist())) for a in range(nq if parts_S else 0))
    need = got = 0
    for a in range(nq if parts_S else 0):
        probed = set(P[a].tolist())
        res = set(Ig[a].tolist())
        for i in Itrue[a, :10].tolist():
            if lst[i] in probed:
                need += 1
                got += int(i in res)

    if os.environ.get("VS_IVF_DEBUG"):
        Sg = S.cpu().numpy()
        for a in [a for a in range(nq) if set(Ig[a, :10].tolist()) != set(Itrue[a, :10].tolist())][:3]:
            _progress(f"q{a} ivf  {Ig[a, :10].tolist()} {np.round(Sg[a, :10], 6).tolist()}")
            ts = [float(Sall[a][np.where(Iall[a] == i)[0][0]]) for i in Itrue[a, :10]]
            _progress(f"q{a} flat {Itrue[a, :10].tolist()} {np.round(ts, 6).tolist()}")
            _progress(f"q{a} lists of flat ids {[lst[i] for i in Itrue[a, :10].tolist()]} probed {sorted(P[a].tolist())}")
            for i in Itrue[a, :4].tolist():
                xi = lists_of[i]
                _progress(f"   id {i}: flat row == ivf row: {np.array_equal(xi, ix.reconstruct(i))}  "
                          f"flat-row score {float(xi.astype(np.float64) @ qh[a].astype(np.float64)):.9f}  "
                          f"gen row[:3] {corpus_chunk(i, 1).cpu().numpy()[0, :3].tolist()} flat row[:3] {xi[:3].tolist()}")
    data = ("synthetic isotropic (counter-hash N(0,1) rows, L2-normalised, seeds 20260417/20260418)" if args.iso_data
            else f"synthetic Gaussian mixture: normalise(centroid[cid(i)] + {sigma} * unit counter-hash Gaussian row i), "
                 + (f"Zipf({args.skew}) cluster sizes" if args.skew > 0 else f"cid = hash(i) % {nlist}")
                 + ", seeds 20260417 (rows) / 20260418 (queries) / 20260419 (centroids)")
    out = {
        "metric": f"kNN queries/sec + recall@10 vs exact flat, IVF-Flat nlist={nlist} nprobe={nprobe} N=50M d=1536 batch=256",
        "value": round(nq * args.steps / elapsed, 2),
        "unit": "queries/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": dtype,
        "data": data,
        "config": {"workload": args.workload, "desc": desc, "N": N, "d": d, "batch": nq, "k": k, "nlist": nlist,
                   "nprobe": nprobe, "list_rows_min_max": [int(sizes.min()), int(sizes.max())],
                   "list_rows_median": int(np.median(sizes)), "skew": args.skew,
                   "list_scan": args.ivf_scan, "mfma_query_tiles": args.ivf_qtile, "mfma_list_scans": mfma_lists,
                   "scan_bytes_read": {"mfma": mfma_bytes, "gemv": gemv_bytes},
                   "parallelism": "1 GPU"},
        "roofline": {
            "kernel": "k_ivf_scan",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": _traffic(None, "cfg5", N, "ivf_scan", args.skew),
            "kernel_ms": round(kavg, 4),
            "alg_bytes_per_launch": alg_bytes,
        },
        "uncertified_first_pass": uncert,
        "gemv_scan": gemv_beside,
        "mfma_query_tiles_beside": qtile_beside,
        "build_s": round(t_build, 2),
        "recall@10": round(hit / (nq * 10.0), 6) if parts_S else None,
        "probed_recall@10": round(got / max(need, 1), 6) if parts_S else None,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = ivf_cpu_baseline(d, dtype, qh, k, pairs, ix.centroids(), nprobe)
    print(json.dumps(out), flush=True)
    ix.close()


def ivf_cpu_baseline(d, dtype, qh, k, pairs, centroids, nprobe):
    """faiss IndexIVFFlat search restated on the host: the coarse probe (the faiss fp32 flat
    restatement over the centroids, BLAS path, all threads) timed in full, plus the list scans
    (oracle/vs_oracle.c fp32 sequential scan, one query per OpenMP thread as faiss parallelises IVF
    search over queries) timed on a contiguous row sample and scaled to the batch's (row, query)
    pair count."""
    from oracle import oracle as O
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores) or cores), 16)
    qa = np.ascontiguousarray(qh, dtype=np.float32)
    O.knn_faiss_fp32(centroids[:256], qa[:32], 4, "ip", threads)  # warm
    t0 = time.perf_counter()
    O.knn_faiss_fp32(np.ascontiguousarray(centroids), qa, nprobe, "ip", threads)
    t_probe = time.perf_counter() - t0
    R = 400_000
    x = O.synth_rows(SEED_CORPUS, 0, R, d, True, dtype)
    qs = np.ascontiguousarray(qh[:threads])
    O.knn_faiss_fp32(x[:1000], qs, 5, "ip", threads)  # warm
    t0 = time.perf_counter()
    O.knn_faiss_fp32(x, qs, k, "ip", threads)
    t = time.perf_counter() - t0
    rate = R * qs.shape[0] / t  # (row, query) pairs per second
    nq = qh.shape[0]
    t_scan = pairs / rate
    return {"value": round(nq / (t_probe + t_scan), 3), "unit": "queries/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"coarse probe (faiss flat fp32 restatement, {nq} queries x {centroids.shape[0]} centroids, top-"
                      f"{nprobe}) {t_probe * 1e3:.1f} ms, timed in full; list scans restated (oracle/vs_oracle.c fp32 "
                      f"sequential scan, {threads} queries on {threads} OpenMP threads) over {R} rows in {t:.2f} s = "
                      f"{rate / 1e6:.1f} M row-query pairs/s, scaled to this batch's {pairs / 1e6:.1f} M pairs "
                      f"({t_scan:.2f} s)"}


if __name__ == "__main__":
    main()
