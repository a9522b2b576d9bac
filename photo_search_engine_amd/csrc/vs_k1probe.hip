// vs_k1probe.hip -- diagnostic forms of the direct K1 screens (DESIGN §5 "Where K1 int8's time
// goes"), not on any search path: the int8 direct screen's loop taken apart (the loads and barriers
// alone, + the query-fragment reads, + the MFMAs, the whole loop), and the whole loop under the
// schedules compared in-process (SCHED 0 / the mid-step barrier, static priority for waves 4-7), each
// with s_memtime / s_memrealtime stamps per workgroup around the loop, so a launch's time splits
// into cycles and clock.  Entry: vs_k1_probe (vs_api.hip, include/vs.h).
#include "vs_screen.h"

namespace vs {

template <int DT, int PROBE, int SCHED, bool PRIO>
__global__ void __launch_bounds__(512, 2) k_k1_probe(ScreenArgs a, const uint8_t* __restrict__ qt, int nqb) {
    screen_direct<DT, METRIC_IP, false, 16, false, PROBE, SCHED, PRIO>(a, qt, nqb);
}

template <int DT, int PROBE, int SCHED, bool PRIO>
static hipError_t launch_one(const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    const void* fn = (const void*)k_k1_probe<DT, PROBE, SCHED, PRIO>;
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, I8D_LDS);
    (void)hipGetLastError();
    hipLaunchKernelGGL((k_k1_probe<DT, PROBE, SCHED, PRIO>), dim3(a.G), dim3(MF_THREADS), I8D_LDS, st, a, qt, nqb);
    return hipGetLastError();
}

hipError_t launch_k1_probe(int variant, int dt, const ScreenArgs& a, const uint8_t* qt, int nqb, hipStream_t st) {
    if (!a.stamps || a.metric != METRIC_IP || a.seed_acc || a.gate || a.gT || a.tile_map) return hipErrorInvalidValue;
    if (dt == DT_I8) {
        if (!i8_direct_ok(a.dpad) || !a.rsb || !a.qfac) return hipErrorInvalidValue;
        switch (variant) {
            case VS_K1P_LOADS: return launch_one<DT_I8, PR_LOADS, 0, false>(a, qt, nqb, st);
            case VS_K1P_LDS: return launch_one<DT_I8, PR_LDS, 0, false>(a, qt, nqb, st);
            case VS_K1P_MFMA: return launch_one<DT_I8, PR_MFMA, 0, false>(a, qt, nqb, st);
            case VS_K1P_FULL: return launch_one<DT_I8, PR_FULL, 0, false>(a, qt, nqb, st);
            case VS_K1P_FULL_MS: return launch_one<DT_I8, PR_FULL, 1, false>(a, qt, nqb, st);
            case VS_K1P_FULL_PRIO: return launch_one<DT_I8, PR_FULL, 0, true>(a, qt, nqb, st);
            case VS_K1P_FULL_MS_PRIO: return launch_one<DT_I8, PR_FULL, 1, true>(a, qt, nqb, st);
            default: return hipErrorInvalidValue;
        }
    }
    if (dt == DT_BF16) {
        if (!d16_direct_ok(a.dpad)) return hipErrorInvalidValue;
        switch (variant) {
            case VS_K1P_LOADS: return launch_one<DT_BF16, PR_LOADS, 0, false>(a, qt, nqb, st);
            case VS_K1P_MFMA: return launch_one<DT_BF16, PR_MFMA, 0, false>(a, qt, nqb, st);
            case VS_K1P_FULL: return launch_one<DT_BF16, PR_FULL, 0, false>(a, qt, nqb, st);
            default: return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
}

}  // namespace vs
