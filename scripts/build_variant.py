"""Diagnostic (not product code): build a variant of libvs.so for an in-box A/B.  Copies csrc to
diag/var_src, applies exact text replacements from a JSON file [[file, old, new], ...] (each old must
occur exactly once), builds diag/<name>.so.  Run with VS_LIB_PATH=diag/<name>.so on the GPU box.
python scripts/build_variant.py patches.json name"""
import glob
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
SRC = os.path.join(ROOT, "photo_search_engine_amd", "csrc")
OUT = os.path.join(ROOT, "diag", "var_src")


def main(patch_file, name):
    shutil.rmtree(OUT, ignore_errors=True)
    shutil.copytree(SRC, OUT)
    for f, old, new in json.load(open(patch_file)):
        p = os.path.join(OUT, f)
        s = open(p).read()
        assert s.count(old) == 1, (f, old[:80], s.count(old))
        open(p, "w").write(s.replace(old, new))
    objs, procs = [], []
    for f in sorted(glob.glob(os.path.join(OUT, "*.hip"))):  # (compiled concurrently)
        o = f[:-4] + ".o"
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                                       "-Wno-unused-result", "-Wno-unused-value", "-Wno-inline-asm", "-c", f, "-o", o],
                                      stderr=subprocess.DEVNULL))
        objs.append(o)
    assert all(p.wait() == 0 for p in procs), "variant build failed"
    lib = os.path.join(ROOT, "diag", name + ".so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    shutil.rmtree(OUT, ignore_errors=True)
    print("built", lib)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
