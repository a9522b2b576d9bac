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
        ("    sort_valid_best_first<METRIC_IP>(sc, ids, nA, nA2);  // phase A best first", 5, "after_line"),
        ("            a.pa_tA[q] = tA;\n        }\n", 11, "after_sync"),
        ("    const bool overflow = nA2 + nB > RFW_CAP;\n", 6, "before_sync"),
        ("    rfw_score<DT, METRIC, QLDS>(a, ids, sc, nA2, nA2 + nB, qs, qv);\n    __syncthreads();\n", 7, "after"),
        ("    const int nF = nA + nb_s;\n", 8, "before"),
        ("    if (nb_s > 0) sort_valid_best_first<METRIC_IP>(sc, ids, nF, nF2);\n", 9, "after"),
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
    # refine() (k_refine): query 0's workgroups (split slices), stamps [slice][NS]
    head = s.index("__device__ __forceinline__ void refine(const RefineArgs& a, int KP2) {")
    end = s.index("\n}\n", head)
    body = s[head:end]
    ranchors = [
        ("    const float* qv = a.q + (int64_t)q * a.d;\n", 0, "after"),
        ("    __syncthreads();\n    // the Kp-th best listed key bounds", 1, "after_first_line"),
        ("    const int nv = nv_s;\n", 2, "before"),
        ("    if (split) {\n        // the last of the query's workgroups takes over", 3, "before_sync"),
        ("    const double worst = METRIC == METRIC_IP ? -INFINITY : INFINITY;\n", 4, "before_sync"),
        ("    sort_valid_best_first<METRIC>(sc, ids, nv, KP2);  // best first\n", 5, "after"),
    ]
    for a_, i, how in ranchors:
        assert body.count(a_) == 1, a_
        st = (f"    if (threadIdx.x == 0 && blockIdx.x == 0) g_rf_stamps[(size_t)blockIdx.y * {NS} + {i}] = "
              "wall_clock64();\n")
        if how == "after":
            body = body.replace(a_, a_ + st)
        elif how == "after_first_line":
            k = body.index(a_)
            e = body.index("\n", k) + 1
            body = body[:e] + st + body[e:]
        elif how == "before_sync":
            body = body.replace(a_, "    __syncthreads();\n" + st + a_)
        else:
            body = body.replace(a_, st + a_)
    body = body + (f"\n    __syncthreads();\n    if (threadIdx.x == 0 && blockIdx.x == 0) g_rf_stamps[(size_t)blockIdx.y * {NS} + 6] = "
                   "wall_clock64();\n"
                   f"    if (threadIdx.x == 0 && blockIdx.x == 0) g_rf_stamps[(size_t)blockIdx.y * {NS} + 11] = clock64();\n")
    body = body.replace("    const float* qv = a.q + (int64_t)q * a.d;\n",
                        "    const float* qv = a.q + (int64_t)q * a.d;\n"
                        f"    if (threadIdx.x == 0 && blockIdx.x == 0) g_rf_stamps[(size_t)blockIdx.y * {NS} + 10] = clock64();\n", 1)
    s = s[:head] + body + s[end:]
    decl = f"__device__ unsigned long long g_rfw_stamps[256 * {NS}];\n__device__ unsigned long long g_rf_stamps[64 * {NS}];\n"
    s = s.replace("constexpr int RF_THREADS = 1024;", decl + "constexpr int RF_THREADS = 1024;", 1)
    s += f'''
extern "C" int vs_diag_rfw_stamps(unsigned long long* out) {{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_rfw_stamps), sizeof(unsigned long long) * 256 * {NS});
}}
extern "C" int vs_diag_rf_stamps(unsigned long long* out, int clear) {{
    if (clear) {{
        static unsigned long long z[64 * {NS}];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(vs::g_rf_stamps), z, sizeof(z));
    }}
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_rf_stamps), sizeof(unsigned long long) * 64 * {NS});
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


def run_single(rows):
    """k_refine of one query (BASELINE cfg2: fp32 rows, int8 screen, k = 10): stamps of query 0's
    split workgroups (0 start, 1 selection, 2 counts, 3 scored, 4 hand-off, 5 sort, 6 end)."""
    import ctypes
    import numpy as np
    sys.path.insert(0, ROOT)
    from photo_search_engine_amd import _lib
    L = _lib.load(LIB)
    from photo_search_engine_amd.index import FlatIndex
    import torch
    d, k = 1536, 10
    ix = FlatIndex(d, "ip", "f32", device=0)
    ix.add_synthetic(20260417, 0, rows, True)
    ix.set_screen("int8")
    rng = np.random.default_rng(3)
    names = {1: "select", 2: "counts", 3: "score (slice)", 4: "hand-off", 5: "sort", 6: "cert+out"}
    res = {}
    for rep in range(12):
        q = rng.standard_normal((1, d)).astype(np.float32)
        q /= np.linalg.norm(q)
        qd = torch.from_numpy(q).cuda()
        I = torch.empty((1, k), dtype=torch.int64, device="cuda")
        L.vs_diag_rf_stamps(None, 1)
        ix.search_device_exact(qd.data_ptr(), 1, k, None, I.data_ptr(), None, 0, 0)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (64 * NS))()
        L.vs_diag_rf_stamps(buf, 0)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(64, NS).astype(np.int64)
        used = a[:, 0] > 0
        if rep < 2:
            continue
        a = a[used]
        t0 = a[:, 0].min()
        res.setdefault("slices", []).append(int(used.sum()))
        for i in (1, 2, 3):
            res.setdefault(names[i], []).extend(((a[:, i] - a[:, i - 1]) / 100.0).tolist())
        last = a[a[:, 6] > 0]
        if len(last):
            for i in (4, 5, 6):
                res.setdefault(names[i], []).append(float((last[0, i] - last[0, i - 1]) / 100.0))
            res.setdefault("launch span", []).append(float((last[0, 6] - t0) / 100.0))
            # shader clock of the last workgroup over its span (clock64 cycles / wall time)
            res.setdefault("sclk MHz", []).append(float((last[0, 11] - last[0, 10]) / ((last[0, 6] - last[0, 0]) / 100.0)))
    out = {kk: {"median_us": round(float(np.median(v)), 2), "max_us": round(float(np.max(v)), 2)} for kk, v in res.items()}
    print(json.dumps({"rows": rows, "refine": "k_refine, one query", "phases": out}, indent=1))


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
ap.add_argument("--single", action="store_true", help="k_refine of one query over fp32 rows (cfg2)")
ap.add_argument("--two-phase", type=int, default=0, help="G > 1: time the two-phase search's phases A and B")
args = ap.parse_args()
if args.build:
    build()
if args.run:
    if args.single:
        run_single(args.rows)
    elif args.two_phase > 1:
        run_two_phase(args.rows, args.two_phase)
    else:
        run(args.rows)
