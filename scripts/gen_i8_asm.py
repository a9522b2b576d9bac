"""Generate photo_search_engine_amd/csrc/vs_i8_asm.h: the K-step bodies of the direct screens.

One K-step of k_screen_i8d for one wave: 16 query fragments (16 queries x 64 B
each, one ds_read_b128 per lane) read from the LDS ring slot RA = 4 reads ahead of their MFMAs,
and 32 v_mfma_i32_16x16x64_i8 (2 corpus fragments x 16 query fragments) into 128 accumulator
VGPRs.  Written as ONE inline-asm block so the reads stay ahead of the MFMAs (hipcc schedules
the same source with one read in flight and an LDS wait per MFMA pair) and the compiler never
touches the corpus fragments between their load and their use.

  I8D_STEP()   accumulate: c += a * b
  I8D_STEP0()  first K-step of a tile: c = a * b (src2 = 0, no zeroing of the accumulators)
  BFD_STEP / BFD_STEP0, HFD_STEP / HFD_STEP0: the same for the bf16 / f16 direct screen
  (v_mfma_f32_16x16x32_bf16 / _f16: 32 elements per K-step, fp32 accumulators in the same VGPRs)
  *_N4: 4 query column groups instead of 16 (narrow query tiles: 8 MFMAs per K-step)

  I8D_LDSONLY: the 16 query-fragment reads and their waits alone (no MFMA; the K-loop probe)

Mid-step-barrier schedule (SCHED 1 of screen_direct): one asm block per K-step that also holds the
step's barrier and the issue of the K-step 3 ahead, so no wave leaves the matrix pipe idle around a
barrier:
  MS_<I8|BF|HF>_<F|N><O|P><P|N>: [4 own fragment reads (O) | the 4 prefetched by the previous step
  (P)] MFMA pairs 0-7 (reads 4 ahead) -> s_waitcnt vmcnt(6) + s_barrier (the next step's query
  slot has landed in every wave; every wave is done with the slot the issue below refills) -> MFMA
  pairs 8-15, the 2 query LDS-DMAs and 2 corpus loads of the K-step 3 ahead between them -> [the
  next step's first 4 fragment reads from its slot (P) | none (N)].  F = first K-step of a tile
  (src2 = 0).

Usage: python scripts/gen_i8_asm.py > photo_search_engine_amd/csrc/vs_i8_asm.h
"""
RA = 4  # query-fragment reads in flight


def body(first: bool, last: bool, op: str = "v_mfma_i32_16x16x64_i8", ng: int = 16) -> str:
    lines = []
    for n in range(RA):
        lines.append(f"ds_read_b128 %[b{n % RA}], %[addr] offset:{n * 1024}")
    for n in range(ng):
        issued = min(ng, n + RA)
        lines.append(f"s_waitcnt lgkmcnt({issued - (n + 1)})")
        for m in range(2):
            src2 = "0" if first else f"%[c{m}_{n}]"
            lines.append(f"{op} %[c{m}_{n}], %[a{m}], %[b{n % RA}], {src2}")
        if n + RA < ng:
            lines.append(f"ds_read_b128 %[b{n % RA}], %[addr] offset:{(n + RA) * 1024}")
    if last:
        lines += ["s_nop 7", "s_nop 7", "s_nop 7"]
    return "\\n\\t".join(lines)


def lds_only() -> str:
    lines = []
    for n in range(RA):
        lines.append(f"ds_read_b128 %[b{n % RA}], %[addr] offset:{n * 1024}")
    for n in range(16):
        issued = min(16, n + RA)
        lines.append(f"s_waitcnt lgkmcnt({issued - (n + 1)})")
        if n + RA < 16:
            lines.append(f"ds_read_b128 %[b{n % RA}], %[addr] offset:{(n + RA) * 1024}")
    outs = ", ".join(f'[b{i}] "=&v"(bt[{i}])' for i in range(RA))
    body_ = "\\n\\t".join(lines)
    return f'#define I8D_LDSONLY() asm volatile("{body_}" : {outs} : [addr] "v"(slot_lds) : "memory")'


def ms_step(op: str, first: bool, own: bool, pre: bool, nt: bool) -> str:
    """One K-step of the mid-step-barrier schedule (module docstring)."""
    ld = "global_load_dwordx4 %[an{}], %[cs], off" + (" offset:{}" ) + (" nt" if nt else "")
    vmem = [["s_mov_b32 m0, %[ql0]", "s_nop 0", "global_load_lds_dwordx4 %[qs0], off"],
            ["s_mov_b32 m0, %[ql1]", "s_nop 0", "global_load_lds_dwordx4 %[qs1], off"],
            [ld.format(0, 0).replace(" offset:0", "")],
            [ld.format(1, "%[a2off]").replace("%[a2off]", "{A2}")]]
    lines = []
    if own:
        for n in range(RA):
            lines.append(f"ds_read_b128 %[b{n}], %[addr] offset:{n * 1024}")
    for n in range(16):
        if n == 8:
            lines += ["s_waitcnt vmcnt(6)", "s_barrier"]
        # fragment reads in flight before pair n: min(16, n + RA) issued (+ the prefetch lines come last)
        issued = min(16, n + RA)
        lines.append(f"s_waitcnt lgkmcnt({issued - (n + 1)})")
        for m in range(2):
            src2 = "0" if first else f"%[c{m}_{n}]"
            lines.append(f"{op} %[c{m}_{n}], %[a{m}], %[b{n % RA}], {src2}")
        if n + RA < 16:
            lines.append(f"ds_read_b128 %[b{n % RA}], %[addr] offset:{(n + RA) * 1024}")
        if 8 <= n < 12:
            lines += vmem[n - 8]
    if pre:
        for n in range(RA):
            lines.append(f"ds_read_b128 %[b{n}], %[naddr] offset:{n * 1024}")
    return "\\n\\t".join(lines)


def ms_macro(name: str, op: str, first: bool, own: bool, pre: bool, nt: bool, a2: int) -> str:
    outs = ", ".join([f'[c{m}_{n}] "+v"(acc[{m}][{n}])' for m in range(2) for n in range(16)] +
                     [f'[b{i}] "+v"(bt[{i}])' for i in range(RA)] + ['[an0] "+v"(AN0_)', '[an1] "+v"(AN1_)'])
    ins = ('[a0] "v"(A0_), [a1] "v"(A1_), [addr] "v"(slot_lds), [naddr] "v"(next_lds), [qs0] "v"(QS0_), '
           '[qs1] "v"(QS1_), [ql0] "s"(QL0_), [ql1] "s"(QL1_), [cs] "v"(CS_)')
    body_ = ms_step(op, first, own, pre, nt).replace("{A2}", str(a2))
    return (f'#define {name}(A0_, A1_, AN0_, AN1_, QS0_, QS1_, QL0_, QL1_, CS_) asm volatile("{body_}" : {outs} : '
            f'{ins} : "memory", "m0")')


def macro(name: str, first: bool, last: bool, op: str = "v_mfma_i32_16x16x64_i8", ng: int = 16) -> str:
    # "+v" in every variant (I8D_STEP0 ignores the old values): identical operand constraints let
    # the register allocator keep the accumulators in place across the runtime choice of variant
    acc_c = "+v"
    outs = ", ".join([f'[c{m}_{n}] "{acc_c}"(acc[{m}][{n}])' for m in range(2) for n in range(ng)] +
                     [f'[b{i}] "=&v"(bt[{i}])' for i in range(RA)])
    ins = '[a0] "v"(A0_), [a1] "v"(A1_), [addr] "v"(slot_lds)'
    return f'#define {name}(A0_, A1_) asm volatile("{body(first, last, op, ng)}" : {outs} : {ins} : "memory")'


if __name__ == "__main__":
    print("// vs_i8_asm.h -- GENERATED by scripts/gen_i8_asm.py; do not edit.")
    print("// K-step bodies of the direct screens k_screen_i8d / k_screen_d16 (vs_kernels.hip): operands in scope at")
    print("// the expansion site: intx4 acc[2][16], intx4 bt[4], uint32_t slot_lds; the arguments are the")
    print("// wave's two corpus fragments (intx4) of the K-step.")
    print("#pragma once")
    print(macro("I8D_STEP", False, False))
    print(macro("I8D_STEP0", True, False))
    print(macro("BFD_STEP", False, False, "v_mfma_f32_16x16x32_bf16"))
    print(macro("BFD_STEP0", True, False, "v_mfma_f32_16x16x32_bf16"))
    print(macro("HFD_STEP", False, False, "v_mfma_f32_16x16x32_f16"))
    print(macro("HFD_STEP0", True, False, "v_mfma_f32_16x16x32_f16"))
    # narrow query tiles (the IVF list scans of lists probed by <= 32 queries): 4 column groups
    print(macro("BFD_STEP_N4", False, False, "v_mfma_f32_16x16x32_bf16", 4))
    print(macro("BFD_STEP0_N4", True, False, "v_mfma_f32_16x16x32_bf16", 4))
    print(macro("HFD_STEP_N4", False, False, "v_mfma_f32_16x16x32_f16", 4))
    print(macro("HFD_STEP0_N4", True, False, "v_mfma_f32_16x16x32_f16", 4))
    print(lds_only())
    # mid-step-barrier K-steps of the int8 screen (corpus loads nt, fragments 1 KiB apart)
    for first, own, pre in ((True, True, False), (False, True, True), (False, False, True), (False, False, False)):
        nm = f"MS_I8_{'F' if first else 'N'}{'O' if own else 'P'}{'P' if pre else 'N'}"
        print(ms_macro(nm, "v_mfma_i32_16x16x64_i8", first, own, pre, True, 1024))
