"""ISA check of the direct int8 screen (k_screen_i8d): build-time evidence that the inline-asm
corpus loads are only ever read by the MFMAs, i.e. that hipcc inserted no copy, spill or other
read of a fragment register that could run before the kernel's own s_waitcnt.

    python scripts/check_i8d_isa.py [vs_kernels.s]   (default: compiles vs_kernels.hip to asm)

Both instantiations are checked (inner product and L2), and the bf16 / f16 direct form
k_screen_d16 the same way.

Checks, for the kernel's code: no scratch (spill) traffic; every register written by a corpus load
(`global_load_dwordx4 ... nt`) is read only by v_mfma instructions; one s_barrier per K-step body.
Exit status 0 = pass.
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "photo_search_engine_amd", "csrc", "vs_kernels.hip")


def regs(spec: str):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", spec)
    return {int(m.group(1))} if m else set()


def operands(line: str):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    return parts[0], [o.strip() for o in parts[1].split(",")]


def main() -> int:
    if len(sys.argv) > 1:
        asm = open(sys.argv[1]).read()
    else:
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "k.s")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                            "-S", "-Wno-inline-asm", "-o", out, SRC], check=True)
            asm = open(out).read()
    rc = 0
    for metric, sym in (("ip", "_ZN2vs12k_screen_i8dILi0EEEvNS_10ScreenArgsEPKhi:"),
                        ("l2", "_ZN2vs12k_screen_i8dILi1EEEvNS_10ScreenArgsEPKhi:")):
        rc |= check(asm, metric, sym)
    # the mid-step-barrier form (SCHED 1, the default int8 main pass): its corpus loads and query
    # DMAs sit inside the K-step asm blocks, and the next step's first query fragments are read at
    # the end of a block (in flight across the loop code between blocks)
    # (inner product only: the L2 form keeps the head-barrier schedule)
    rc |= check(asm, "ip", "_ZN2vs15k_screen_i8d_msILi0EEEvNS_10ScreenArgsEPKhi:", name="k_screen_i8d_ms",
                frag_reads=True)
    # ... and over group-residual codes (4 VGPRs spilled outside the K-step blocks: the epilogue's
    # reloads, once per tile; the fragment checks still hold)
    rc |= check(asm, "ip", "_ZN2vs19k_screen_i8d_res_msENS_10ScreenArgsEPKhi:", name="k_screen_i8d_res_ms",
                frag_reads=True, allow_spill=True)
    # the main pass over group-residual codes (inner product; + <mu_g, q> per key)
    rc |= check(asm, "ip", "_ZN2vs16k_screen_i8d_resENS_10ScreenArgsEPKhi:", name="k_screen_i8d_res")
    # the bf16 / f16 direct form (k_screen_d16): its corpus loads are global_load_dwordx4 with and
    # without the nt hint (the first half of each 128 B line keeps the default policy)
    for dt, dcode in (("bf16", 1), ("f16", 2)):
        for metric, mcode in (("ip", 0), ("l2", 1)):
            rc |= check(asm, f"{dt}/{metric}", f"_ZN2vs12k_screen_d16ILi{dcode}ELi{mcode}EEEvNS_10ScreenArgsEPKhi:",
                        name="k_screen_d16", any_policy=True)
            # the IVF list scan form (page table; wide and narrow query tiles in one kernel)
            rc |= check(asm, f"{dt}/{metric}", f"_ZN2vs19k_screen_d16_mappedILi{dcode}ELi{mcode}EEEvNS_10ScreenArgsEPKhi:",
                        name="k_screen_d16_mapped", any_policy=True)

    return rc


def check(asm: str, metric: str, sym: str, name: str = "k_screen_i8d", any_policy: bool = False,
          frag_reads: bool = False, allow_spill: bool = False) -> int:
    start = asm.index(sym)
    end = asm.index(".Lfunc_end", start)
    raw = asm[start:end].split("\n")
    code, in_asm, inasm = [], [], False  # in_asm: the instruction comes from an inline-asm block
    for i, l in enumerate(raw):
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True
        elif t.startswith(";;#ASMEND"):
            inasm = False
        if t and not t.startswith((";", ".")):
            code.append(f"{l}  ;#L{i}")
            in_asm.append(inasm)
    bad = []
    if any("scratch_" in l for l in code):
        if not allow_spill:
            bad.append("scratch (spill) instructions present")
        elif any("scratch_" in l for l, a in zip(code, in_asm) if a):
            bad.append("scratch instructions inside an asm block")
    # Forward scan from every corpus load (in layout order, the load's fall-through path) to the
    # first MFMA that reads its registers or the first redefinition of them: no other instruction
    # may READ them in between (a copy or spill there would read the register before the kernel's
    # s_waitcnt lets the load land).  The compiler never writes a register it believes live, so
    # writes need no check.
    def split(l):
        op, ops = operands(l)
        if not ops:
            return op, set(), set()
        if op.startswith(("global_load_lds", "s_")) or op.startswith(("global_store", "ds_write")):
            return op, set(), set().union(*[regs(o) for o in ops])
        return op, regs(ops[0]), set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
    parsed = [split(l) for l in code]
    loaded = set()
    # (corpus loads come after the first barrier; a mapped scan's descriptor load before it is an
    # ordinary compiler-waited load)
    first_bar = next((i for i, l in enumerate(code) if l.strip().startswith("s_barrier")), 0)
    for i, l in enumerate(code):
        op, dst, _ = parsed[i]
        if i < first_bar:
            continue
        ins = l.split(";")[0].rstrip()
        # (the corpus loads are the inline-asm ones: 64-bit VGPR address, "off"; the compiler's own
        # loads of descriptors use the SGPR-base form and are waited for by the compiler)
        if not (op == "global_load_dwordx4" and ", off" in ins and (any_policy or ins.endswith("nt"))):
            continue
        loaded |= dst
        for j in range(i + 1, len(code)):
            op2, dst2, src2 = parsed[j]
            if op2.startswith("v_mfma") and src2 & dst:
                break
            if src2 & dst:
                bad.append(f"corpus fragment {sorted(dst)[0]}.. read before its MFMA by: {code[j].strip()}")
                break
            if dst2 & dst:
                break
    if frag_reads:
        # every query-fragment read (ds_read_b128) is consumed by an MFMA before any other
        # instruction reads its registers without an lgkmcnt(0) wait in between (a copy of a
        # prefetched fragment would read the register before the read lands)
        for i, l in enumerate(code):
            op, dst, _ = parsed[i]
            if op != "ds_read_b128" or i < first_bar or not in_asm[i]:
                continue  # (the compiler's own LDS reads are waited for by the compiler)
            for j in range(i + 1, len(code)):
                op2, dst2, src2 = parsed[j]
                if "lgkmcnt(0)" in code[j]:
                    break
                if op2.startswith("v_mfma") and src2 & dst:
                    break
                if src2 & dst:
                    bad.append(f"query fragment {sorted(dst)[0]}.. read before its wait by: {code[j].strip()}")
                    break
                if dst2 & dst:
                    break
    nmfma = sum(1 for l in code if l.strip().startswith("v_mfma"))
    nbar = sum(1 for l in code if l.strip().startswith("s_barrier"))
    print(f"{name}<{metric}>: {len(code)} instructions, {nmfma} MFMA, {nbar} s_barrier, "
          f"{len(loaded)} corpus-fragment VGPRs")
    for b in bad[:20]:
        print("FAIL:", b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
