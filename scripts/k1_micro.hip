// k1_micro.hip -- diagnostic microbenchmark of the int8 screen's inner loop (not product code).
//
// Question it answers: can the int8 K1 screen (cfg3: 10M rows x 1536 int8, 256 queries) overlap
// its MFMAs with the corpus stream if the corpus fragments go HBM -> VGPRs directly (each wave
// owns 32 rows of the 256-row tile and prefetches P K-steps ahead in rotating register sets), and
// only the query stream (L2-resident, shared by all waves) goes through an LDS ring?
//
// Variants (template MODE): 0 = loads only (A loads + query DMA, no reads, no MFMA),
// 1 = + B fragment reads, 2 = + MFMAs (full loop, column-max epilogue), 3/4 = dump accumulators
// (correctness check on a small corpus against a host int32 GEMM), 5 = no barrier, 6 = loads issued
// after the MFMAs, 8 = per-value float epilogue, 9 = bound epilogue (the product's), P = lead;
// 10 / 11 = compiler-scheduled v_mfma_i32_32x32x32_i8 / 16x16x64_i8 over the same bytes (run ids
// 20 / 21: does the 32x32 shape's half operand traffic per MAC lower the power-limited time?).
// Results (MI355X, 10M x 1536, int8 codes of Gaussian rows): DESIGN.md §5.
// Run: ./abtmp/k1_micro [N] [d] [iters] [data: 0 random, 1 zero, 2 Gaussian codes] [mode]
//
// build: hipcc --offload-arch=gfx950 -O3 -o abtmp/k1_micro scripts/k1_micro.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../photo_search_engine_amd/csrc/vs_i8_asm.h"

typedef int intx4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef int intx16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int THREADS = 512;
constexpr int TR = 256;
constexpr int QB = 256;
constexpr int KB = 16384;  // one K-step block: 256 rows x 64 B

typedef __attribute__((address_space(3))) uint8_t* lds_u8_t;
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) { return (uint32_t)(uintptr_t)(lds_u8_t)(p); }
__device__ __forceinline__ int swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
__device__ __forceinline__ void gld16(intx4& v, const void* p) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm(intx4& a, intx4& b) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
__device__ __forceinline__ void barrier_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int QOPS = 2;    // query DMAs per wave per K-step (16 KiB / 8 waves)
constexpr int OPS = QOPS + 2;

template <int MODE, int P = 5>
__global__ void __launch_bounds__(THREADS, 2)
    k_micro(const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ qt, int tiles, int nks,
            int* __restrict__ hits, int* __restrict__ dump) {
    constexpr int U = P + 1;  // register sets / LDS slots
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    asm volatile("; lds ring escapes: %0" ::"v"(smem) : "memory");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int blk = blockIdx.x, G = gridDim.x;
    const int t0 = (int)((int64_t)tiles * blk / G), t1 = (int)((int64_t)tiles * (blk + 1) / G);
    const int S = (t1 - t0) * nks;
    const uint32_t ring = lds_addr(smem);
    const int r16 = lane & 15;
    const int lane_off = r16 * 64 + (((lane >> 4) ^ swz(r16)) << 4);
    // A: this wave's 32 rows of a K-step block, lane's 16 B of each 16-row fragment
    const int a_off = w * 2048 + r16 * 64 + (lane >> 4) * 16;
    const int64_t tbytes = (int64_t)TR * nks * 64;

    intx4 A[U][2];
    intx4 acc[2][16];
    intx16 acc32[8];  // MODE 10: 8 blocks of 32 rows x 32 queries (v_mfma_i32_32x32x32_i8)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc32[n] = intx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 16; ++n) acc[m][n] = intx4{0, 0, 0, 0};

    // issue step j (query DMA into slot j % U, A loads into set jset)
    int iti = t0, iks = 0;
#define ISSUE_STEP(J, SET)                                                                            \
    do {                                                                                              \
        const uint32_t sbase = __builtin_amdgcn_readfirstlane(ring + (uint32_t)(((J) % U) * KB) + w * 1024); \
        _Pragma("unroll") for (int it = 0; it < QOPS; ++it) {                                         \
            const int g = it * 512 + w * 64 + lane;                                                   \
            const int row = g >> 2, pos = g & 3;                                                      \
            glds16(qt + (int64_t)iks * KB + (row << 6) + ((pos ^ swz(row)) << 4), sbase + it * 8192); \
        }                                                                                             \
        const uint8_t* ab = corpus + (int64_t)min(iti, t1 - 1) * tbytes + (int64_t)iks * KB + a_off;  \
        gld16(A[SET][0], ab);                                                                         \
        gld16(A[SET][1], ab + 1024);                                                                  \
        if (++iks == nks) { iks = 0; ++iti; }                                                         \
    } while (0)

    // prologue: steps 0 .. P-1 into sets 0 .. P-1
#pragma unroll
    for (int j = 0; j < P; ++j) ISSUE_STEP(j, j);

    int ti = t0, ks = 0;
    int nhit = 0;
    for (int s0 = 0; s0 < S; s0 += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int s = s0 + u;
            if (s < S) {
                // uniform count: past the end the issue below loads clamped dummy steps
                if constexpr (P == 3) wait_vm<2 * OPS>(A[u][0], A[u][1]);
                else if constexpr (P == 5) wait_vm<4 * OPS>(A[u][0], A[u][1]);
                else wait_vm<6 * OPS>(A[u][0], A[u][1]);
                if constexpr (MODE != 5) barrier_lgkm();
                if constexpr (MODE != 6) ISSUE_STEP(s + P, (u + P) % U);
                const uint8_t* slot = smem + (s % U) * KB + lane_off;
                if constexpr (MODE == 10 || MODE == 11 || MODE == 12) {
                    // compiler-scheduled MFMAs over the same bytes: 10 = 32x32x32 (16 per K-step, half
                    // the operand reads per MAC), 11 = 16x16x64 (32 per K-step); the operand mapping
                    // is not the product's (timing only)
                    intx4 b[16];
#pragma unroll
                    for (int n = 0; n < 16; ++n) b[n] = *(const intx4*)(slot + n * 1024);
                    if constexpr (MODE == 10) {
#pragma unroll
                        for (int h = 0; h < 2; ++h)
#pragma unroll
                            for (int n = 0; n < 8; ++n)
                                acc32[n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[u][h], b[8 * h + n], acc32[n], 0, 0, 0);
                    } else if constexpr (MODE == 11) {  // corpus fragment held for 16 MFMAs in a row
#pragma unroll
                        for (int m = 0; m < 2; ++m)
#pragma unroll
                            for (int n = 0; n < 16; ++n)
                                acc[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[u][m], b[n], acc[m][n], 0, 0, 0);
                    } else {  // 12: MFMA pairs per query fragment (the product's order)
#pragma unroll
                        for (int n = 0; n < 16; ++n)
#pragma unroll
                            for (int m = 0; m < 2; ++m)
                                acc[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[u][m], b[n], acc[m][n], 0, 0, 0);
                    }
                } else if constexpr (MODE == 2 || MODE >= 5 || MODE == 3 || MODE == 4) {
                    // one asm block per K-step: 16 B-fragment reads RA = 4 ahead of their MFMA pairs
                    intx4 bt[4];
                    const uint32_t slot_lds = lds_addr(slot);
                    I8D_STEP(A[u][0], A[u][1]);  // the product's K-step body (vs_i8_asm.h)
                    if constexpr (MODE == 6) ISSUE_STEP(s + P, (u + P) % U);
                } else if constexpr (MODE == 1) {
                    intx4 b[16];
#pragma unroll
                    for (int n = 0; n < 16; ++n) b[n] = *(const intx4*)(slot + n * 1024);
                    int x = 0;
#pragma unroll
                    for (int n = 0; n < 16; ++n) x ^= b[n].x ^ b[n].y ^ b[n].z ^ b[n].w;
                    nhit += x == 0x12345678;
                } else {
                    nhit += (A[u][0].x ^ A[u][1].y) == 0x12345678;
                }
                if (MODE == 1) nhit += (A[u][0].x ^ A[u][1].y) == 0x12345678;
                if (ks == nks - 1) {
                    if constexpr (MODE == 3 || MODE == 4) {
                        if constexpr (MODE == 4) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
                        // acc[m][n][r]: row 32 w + 16 m + 4 (lane >> 4) + r, query 16 n + (lane & 15)
#pragma unroll
                        for (int m = 0; m < 2; ++m)
#pragma unroll
                            for (int n = 0; n < 16; ++n)
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const int row = 32 * w + 16 * m + 4 * (lane >> 4) + r;
                                    const int q = 16 * n + (lane & 15);
                                    dump[((int64_t)ti * TR + row) * QB + q] = acc[m][n][r];
                                }
                    } else if constexpr (MODE == 8 || MODE == 9) {
                        // realistic epilogues: keys s_x acc t_q + beta_x ||q|| against per-query thresholds
                        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // MFMA (asm) -> VALU read
                        const uint32_t* side = (const uint32_t*)(smem + U * KB);
                        const float2* qf = (const float2*)(smem + U * KB + 1024);
                        const float* thr = (const float*)(smem + U * KB + 3072);
                        float sq[2][4], rb[2][4];
#pragma unroll
                        for (int m = 0; m < 2; ++m) {
                            const uint4 wv = *(const uint4*)(side + w * 32 + m * 16 + (lane >> 4) * 4);
                            const uint32_t w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                sq[m][r] = __uint_as_float(w4[r] << 16);
                                rb[m][r] = __uint_as_float(w4[r] & 0xFFFF0000u);
                            }
                        }
                        if constexpr (MODE == 8) {
#pragma unroll
                            for (int n = 0; n < 16; ++n) {
                                const int q = 16 * n + (lane & 15);
                                const float2 f = qf[q];
                                float mx = -INFINITY;
#pragma unroll
                                for (int m = 0; m < 2; ++m)
#pragma unroll
                                    for (int r = 0; r < 4; ++r)
                                        mx = fmaxf(mx, __builtin_fmaf(rb[m][r], f.y, (float)acc[m][n][r] * sq[m][r]));
                                nhit += mx * f.x >= thr[q];
                            }
                        } else {
                            float smax = sq[0][0], smin = sq[0][0], bmax = rb[0][0];
#pragma unroll
                            for (int m = 0; m < 2; ++m)
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    smax = fmaxf(smax, sq[m][r]);
                                    smin = fminf(smin, sq[m][r]);
                                    bmax = fmaxf(bmax, rb[m][r]);
                                }
#pragma unroll
                            for (int n = 0; n < 16; ++n) {
                                const int q = 16 * n + (lane & 15);
                                const float2 f = qf[q];
                                int mi = acc[0][n][0];
#pragma unroll
                                for (int m = 0; m < 2; ++m)
#pragma unroll
                                    for (int r = 0; r < 4; ++r) mi = max(mi, acc[m][n][r]);
                                const float fm = (float)mi;
                                const float bound = fmaxf(smax * fm, smin * fm);
                                nhit += __builtin_fmaf(bmax, f.y, bound) * f.x >= thr[q];
                            }
                        }
                    } else if constexpr (MODE == 10) {
#pragma unroll
                        for (int n = 0; n < 8; ++n) {
                            int mx = INT32_MIN;
#pragma unroll
                            for (int r = 0; r < 16; ++r) mx = max(mx, acc32[n][r]);
                            nhit += mx > 2000000;
                            acc32[n] = intx16{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
                        }
                    } else if constexpr (MODE == 2 || MODE >= 5) {
#pragma unroll
                        for (int n = 0; n < 16; ++n) {
                            int mx = INT32_MIN;
#pragma unroll
                            for (int m = 0; m < 2; ++m)
#pragma unroll
                                for (int r = 0; r < 4; ++r) mx = max(mx, acc[m][n][r]);
                            nhit += mx > 2000000;
                        }
                    }
#pragma unroll
                    for (int m = 0; m < 2; ++m)
#pragma unroll
                        for (int n = 0; n < 16; ++n) acc[m][n] = intx4{0, 0, 0, 0};
                }
                if (++ks == nks) { ks = 0; ++ti; }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (nhit) atomicAdd(hits, nhit);
}

int main(int argc, char** argv) {
    const int64_t N = argc > 1 ? atoll(argv[1]) : 10000000;
    const int d = argc > 2 ? atoi(argv[2]) : 1536;
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const int data = argc > 4 ? atoi(argv[4]) : 0;  // 0 random bytes, 1 all zero (clock test), 2 int8 codes
                                                    // of Gaussian rows (sigma ~ 127 / 3.9, as the screen copy)
    const bool zero = data == 1;
    const int only = argc > 5 ? atoi(argv[5]) : -1;     // run only this mode (profiling)
    const int nks = d / 64;
    const int tiles = (int)((N + TR - 1) / TR);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int G = prop.multiProcessorCount;
    const size_t cbytes = (size_t)tiles * TR * d;
    uint8_t *corpus, *qt;
    int *hits, *dump;
    CK(hipMalloc(&corpus, cbytes));
    CK(hipMalloc(&qt, (size_t)QB * d));
    CK(hipMalloc(&hits, 4));
    // random bytes
    {
        std::vector<uint8_t> h(64 << 20);
        uint64_t x = 88172645463325252ull;
        for (auto& b : h) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            if (data == 2) {  // sum of 4 uniforms ~ Gaussian, scaled so |c| <= 127 at ~3.9 sigma
                const int u = (int)((x >> 8) & 255) + (int)((x >> 16) & 255) + (int)((x >> 24) & 255) +
                              (int)((x >> 32) & 255) - 510;  // sigma ~ 147.8
                int c = (int)lrint(u * (32.5 / 147.8));
                b = (uint8_t)(int8_t)(c > 127 ? 127 : c < -127 ? -127 : c);
            } else {
                b = (uint8_t)(x >> 24);
            }
        }
        for (size_t off = 0; off < cbytes; off += h.size())
            CK(hipMemcpy(corpus + off, h.data(), std::min(h.size(), cbytes - off), hipMemcpyHostToDevice));
        CK(hipMemcpy(qt, h.data() + 12345, (size_t)QB * d, hipMemcpyHostToDevice));
    }
    if (zero) {
        CK(hipMemset(corpus, 0, cbytes));
        CK(hipMemset(qt, 0, (size_t)QB * d));
    }
    const size_t lds = (size_t)8 * KB + 4096;
    auto run = [&](auto kern, const char* name, int mode) {
        if (only >= 0 && mode != only) return;
        CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(THREADS), lds, 0, corpus, qt, tiles, nks, hits, nullptr);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(THREADS), lds, 0, corpus, qt, tiles, nks, hits, nullptr);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        const double bytes = (double)N * d + (double)QB * d;
        printf("%-28s N=%lld d=%d: %.4f ms  %.3f TB/s (corpus bytes)  %.2f POPS\n", name, (long long)N, d, ms,
               bytes / ms / 1e9, 2.0 * N * QB * d / ms / 1e9 / 1e3);
        fflush(stdout);
    };
    // correctness: small corpus, dump accumulators, compare with the host
    for (int dm = 3; dm <= 4 && only < 0 && !zero; ++dm) {
        auto dk = dm == 3 ? k_micro<3, 5> : k_micro<4, 5>;
        printf("dump mode %d\n", dm);
        const int tiles_s = 8;
        CK(hipMalloc(&dump, (size_t)tiles_s * TR * QB * 4));
        CK(hipFuncSetAttribute((const void*)dk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(dk, dim3(2), dim3(THREADS), lds, 0, corpus, qt, tiles_s, nks, hits, dump);
        CK(hipDeviceSynchronize());
        std::vector<int> got((size_t)tiles_s * TR * QB);
        CK(hipMemcpy(got.data(), dump, got.size() * 4, hipMemcpyDeviceToHost));
        std::vector<int8_t> hc((size_t)tiles_s * TR * d), hq((size_t)QB * d);
        CK(hipMemcpy(hc.data(), corpus, hc.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(hq.data(), qt, hq.size(), hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int t = 0; t < tiles_s; ++t)
            for (int r = 0; r < TR; ++r)
                for (int q = 0; q < QB; ++q) {
                    int s = 0;
                    for (int ks = 0; ks < nks; ++ks)
                        for (int e = 0; e < 64; ++e)
                            s += (int)hc[(size_t)t * TR * d + (size_t)ks * KB + r * 64 + e] *
                                 (int)hq[(size_t)ks * KB + q * 64 + e];
                    if (s != got[((size_t)t * TR + r) * QB + q]) {
                        ++bad;
                        if (bad <= 12) printf("  t %d row %d q %d: want %d got %d\n", t, r, q, s, got[((size_t)t * TR + r) * QB + q]);
                    }
                }
        {   // where do the values of tile 0 come from?  (row', q') with want == got
            std::vector<int> want((size_t)TR * QB);
            for (int r = 0; r < TR; ++r)
                for (int q = 0; q < QB; ++q) {
                    int s = 0;
                    for (int ks = 0; ks < nks; ++ks)
                        for (int e = 0; e < 64; ++e)
                            s += (int)hc[(size_t)ks * KB + r * 64 + e] * (int)hq[(size_t)ks * KB + q * 64 + e];
                    want[(size_t)r * QB + q] = s;
                }
            int hist[16] = {0};
            for (int r = 0; r < TR; ++r)
                for (int q = 0; q < QB; ++q)
                    if (want[(size_t)r * QB + q] != got[(size_t)r * QB + q]) hist[r & 15]++;
            for (int i = 0; i < 16; ++i) printf("row%%16=%d bad %d\n", i, hist[i]);
            for (int r = 1; r < 4; ++r)
                for (int q = 0; q < 2; ++q) {
                    const int g = got[(size_t)r * QB + q];
                    for (int r2 = 0; r2 < TR; ++r2)
                        for (int q2 = 0; q2 < QB; ++q2)
                            if (want[(size_t)r2 * QB + q2] == g) printf("got(%d,%d) = want(%d,%d)\n", r, q, r2, q2);
                }
        }
        printf("dump check: %lld mismatches of %lld\n", (long long)bad, (long long)tiles_s * TR * QB);
        fflush(stdout);
    }
    run(k_micro<0>, "loads only", 0);
    run(k_micro<1>, "loads + B reads", 1);
    run(k_micro<2>, "full (MFMA)", 2);
    run(k_micro<5>, "full, no barrier", 5);
    run(k_micro<6>, "full, issue after MFMAs", 6);

    run(k_micro<8>, "full, per-value float epi", 8);
    run(k_micro<9>, "full, bound epilogue", 9);

    run(k_micro<0, 3>, "loads only P=3", 11);
    run(k_micro<2, 3>, "full P=3", 12);
    run(k_micro<0, 7>, "loads only P=7", 13);
    run(k_micro<2, 7>, "full P=7", 14);
    run(k_micro<2>, "full (MFMA)", 2);
    run(k_micro<10>, "MFMA 32x32x32 (builtins)", 20);
    run(k_micro<11>, "MFMA 16x16x64 (builtins)", 21);
    run(k_micro<12>, "MFMA 16x16x64 pairs (builtins)", 22);
    return 0;
}
