"""Diagnostic (not product code): where k_refine_wide's time goes.  Builds a copy of the library
with wall-clock stamps (100 MHz) taken by each block's thread 0 at k_refine_wide's phase boundaries
(abtmp/stamps_src -> abtmp/libvs_stamps.so; --build, here), then (--run, on the GPU) searches an int8
index of `--rows` counter-hash rows (d=1536 bf16, 256 queries, k=100) and prints the median /
max per phase over the blocks of the timed launches.
python scripts/refine_stamps.py --build ; python scripts/refine_stamps.py --run [--rows 1250000]"""
import argparse
import glob
import json
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
SRC = os.path.join(ROOT, "photo_search_engine_amd", "csrc")
OUT = os.path.join(ROOT, "diag", "stamps_src")
LIB = os.path.join(ROOT, "diag", "libvs_stamps.so")
NS = 12
PHASES = ["start", "keys+q", "select A", "ids A", "score A", "sort A", "ids B", "score B", "merge B",
          "sort F", "cert+out"]


def build():
    shutil.rmtree(OUT, ignore_errors=True)
    shutil.copytree(SRC, OUT)
    p = os.path.join(OUT, "vs_kernels.hip")
    s = open(p).read()
    head = s.index("__global__ void __launch_bounds__(RF_THREADS) k_refine_wide(RefineArgs a, int KA) {")
    end = s.index("\n}\n", head)
    body = s[head:end]
    anchors = [
        ("    if (a.redo && (*a.gate == 0 || a.cert[q] != 0)) return;\n", 0, "after"),
        ("    const double worst = -INFINITY;\n", 1, "before_sync"),
        ("    if (inreg) {\n        nA = block_write_ids<RF_E>(keys, tA, ~0ull, ids, RFW_CAP, red);", 2, "before_sync"),
        ("    nA = min(nA, RFW_CAP);\n    __syncthreads();\n", 3, "after"),
        ("    rfw_score<DT, METRIC, QLDS>(a, ids, sc, 0, nA, qs, qv);\n    __syncthreads();\n", 4, "after"),
        ("    rfw_sort(sc, ids, nA2);  // phase A best first", 5, "after_line"),
        ("            a.pa_tA[q] = tA;\n        }\n", 11, "after_sync"),
        ("    const bool overflow = nA2 + nB > RFW_CAP;\n", 6, "before_sync"),
        ("    rfw_score<DT, METRIC, QLDS>(a, ids, sc, nA2, nA2 + nB, qs, qv);\n    __syncthreads();\n", 7, "after"),
        ("    const int nF = nA + nb_s;\n", 8, "before"),
        ("    if (nb_s > 0) rfw_sort(sc, ids, nF2);\n", 9, "after"),
    ]
    for a, i, how in anchors:
        assert body.count(a) == 1, a
        st = f"    if (threadIdx.x == 0) g_rfw_stamps[(size_t)blockIdx.x * {NS} + {i}] = wall_clock64();\n"
        if how == "after":
            body = body.replace(a, a + st)
        elif how == "after_line":
            k = body.index(a)
            e = body.index("\n", k) + 1
            body = body[:e] + st + body[e:]
        elif how == "after_sync":
            body = body.replace(a, a + "        __syncthreads();\n" + st.replace("    if", "        if"))
        elif how == "before_sync":
            body = body.replace(a, "    __syncthreads();\n" + st + a)
        else:
            body = body.replace(a, st + a)
    body = body + f"\n    __syncthreads();\n    if (threadIdx.x == 0) g_rfw_stamps[(size_t)blockIdx.x * {NS} + 10] = wall_clock64();\n"
    s = s[:head] + body + s[end:]
    decl = f"__device__ unsigned long long g_rfw_stamps[256 * {NS}];\n"
    s = s.replace("constexpr int RF_THREADS = 1024;", decl + "constexpr int RF_THREADS = 1024;", 1)
    s += f'''
extern "C" int vs_diag_rfw_stamps(unsigned long long* out) {{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_rfw_stamps), sizeof(unsigned long long) * 256 * {NS});
}}
'''
    open(p, "w").write(s)
    objs = []
    for f in sorted(glob.glob(os.path.join(OUT, "*.hip"))):
        o = f[:-4] + ".o"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                        "-Wno-unused-result", "-Wno-unused-value", "-Wno-inline-asm", "-c", f, "-o", o], check=True)
        objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs, check=True)
    shutil.rmtree(OUT, ignore_errors=True)  # (only the library travels to the GPU box)
    print("built", LIB)


def run_two_phase(rows, world):
    """phase A (stamps 0-5, 11) and phase B (stamps 0, 6-10) of the two-phase search, timed apart;
    the floor is the shard's own phase-A lists (a looser floor than G shards' merged lists)."""
    import ctypes
    import numpy as np
    sys.path.insert(0, ROOT)
    from photo_search_engine_amd import _lib
    L = _lib.load(LIB)
    from photo_search_engine_amd.index import FlatIndex
    import torch
    d, nq, k = 1536, 256, 100
    ix = FlatIndex(d, "ip", "bf16", device=0)
    ix.add_synthetic(20260417, 0, rows, True)
    ix.set_screen("int8")
    rng = np.random.default_rng(3)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    qd = torch.from_numpy(q).cuda()
    SIa = torch.empty((nq, k, 2), dtype=torch.int64, device="cuda")
    SIb = torch.empty((nq, k, 2), dtype=torch.int64, device="cuda")
    res = {}
    names_a = {1: "A keys+q", 2: "A select", 3: "A ids", 4: "A score", 5: "A sort", 11: "A write"}
    names_b = {6: "B resume+ids", 7: "B score", 8: "B merge", 9: "B sort F", 10: "B cert+out"}
    for rep in range(6):
        buf = (ctypes.c_ulonglong * (256 * NS))()
        pend = ix.search_phase_a(qd.data_ptr(), nq, k, world, SIa.data_ptr(), SIa.data_ptr() + 8, 0, 0, stride=2)
        torch.cuda.synchronize()
        L.vs_diag_rfw_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(256, NS).astype(np.int64).copy()
        floor = SIa[..., 0].contiguous().view(torch.float64)
        ix.search_phase_b(pend, floor.data_ptr(), None, SIb.data_ptr() + 8, SIb.data_ptr(), 0, stride=2)
        torch.cuda.synchronize()
        L.vs_diag_rfw_stamps(buf)
        b = np.frombuffer(buf, dtype=np.uint64).reshape(256, NS).astype(np.int64).copy()
        if rep < 2:
            continue
        prev = 0
        for i in (1, 2, 3, 4, 5, 11):
            res.setdefault(names_a[i], []).extend(((a[:, i] - a[:, prev]) / 100.0).tolist())
            prev = i
        res.setdefault("A block span", []).extend(((a[:, 11] - a[:, 0]) / 100.0).tolist())
        res.setdefault("A launch span", []).append(float((a[:, 11].max() - a[:, 0].min()) / 100.0))
        prev = 0
        for i in (6, 7, 8, 9, 10):
            res.setdefault(names_b[i], []).extend(((b[:, i] - b[:, prev]) / 100.0).tolist())
            prev = i
        res.setdefault("B block span", []).extend(((b[:, 10] - b[:, 0]) / 100.0).tolist())
        res.setdefault("B launch span", []).append(float((b[:, 10].max() - b[:, 0].min()) / 100.0))
    out = {kk: {"median_us": round(float(np.median(v)), 2), "max_us": round(float(np.max(v)), 2)} for kk, v in res.items()}
    print(json.dumps({"rows": rows, "world": world, "phases": out}, indent=1))


def run(rows):
    import ctypes
    import numpy as np
    sys.path.insert(0, ROOT)
    from photo_search_engine_amd import _lib
    L = _lib.load(LIB)
    from photo_search_engine_amd.index import FlatIndex
    import torch
    d, nq, k = 1536, 256, 100
    ix = FlatIndex(d, "ip", "bf16", device=0)
    ix.add_synthetic(20260417, 0, rows, True)
    ix.set_screen("int8")
    rng = np.random.default_rng(3)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    qd = torch.from_numpy(q).cuda()
    I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
    res = {}
    for rep in range(6):
        ix.search_device_exact(qd.data_ptr(), nq, k, None, I.data_ptr(), None, 0, 0)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (256 * NS))()
        L.vs_diag_rfw_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(256, NS).astype(np.int64)
        t0 = a[:, 0].min()
        rel = (a - t0) / 100.0  # us (100 MHz)
        if rep >= 2:
            for i in range(1, 11):
                dt = a[:, i] - a[:, i - 1]
                res.setdefault(PHASES[i], []).extend((dt / 100.0).tolist())
            res.setdefault("block span", []).extend(((a[:, 10] - a[:, 0]) / 100.0).tolist())
            res.setdefault("launch span (first start -> last end)", []).append(float(rel[:, 10].max()))
            res.setdefault("start skew (last block start)", []).append(float(rel[:, 0].max()))
    out = {kk: {"median_us": round(float(np.median(v)), 2), "max_us": round(float(np.max(v)), 2)} for kk, v in res.items()}
    print(json.dumps({"rows": rows, "phases": out}, indent=1))


ap = argparse.ArgumentParser()
ap.add_argument("--build", action="store_true")
ap.add_argument("--run", action="store_true")
ap.add_argument("--rows", type=int, default=1_250_000)
ap.add_argument("--two-phase", type=int, default=0, help="G > 1: time the two-phase search's phases A and B")
args = ap.parse_args()
if args.build:
    build()
if args.run:
    if args.two_phase > 1:
        run_two_phase(args.rows, args.two_phase)
    else:
        run(args.rows)
