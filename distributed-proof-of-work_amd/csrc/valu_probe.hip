// valu_probe.hip -- diagnostic: sustained VALU issue rate of the instructions the
// MD5 search is made of (v_add_u32, v_add3_u32, v_alignbit_b32, v_bitop3_b32),
// plus v_fma_f32 for reference, and the shader clock under that load.  It pins
// the roofline "peak" that bench.py divides by: 8 independent dependency chains
// per lane, 8 waves per SIMD, every CU busy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../include/dpow_diag.h"

namespace {

constexpr int kChains = 8;
constexpr int kUnroll = 16;
constexpr int kThreads = 256;

template <int KIND>
__device__ __forceinline__ void op(uint32_t &a, uint32_t b, uint32_t c) {
    if constexpr (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (KIND == 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
    if constexpr (KIND == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 6) asm volatile("v_lshl_add_u32 %0, %0, 7, %1" : "+v"(a) : "v"(b));
    if constexpr (KIND == 7) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a) : "v"(b));
    if constexpr (KIND == 8) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 9) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 10) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a));
    if constexpr (KIND == 11) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 12) asm volatile("v_add_u32 %0, 0x5a827999, %0" : "+v"(a));
    if constexpr (KIND == 13) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(a));
    if constexpr (KIND == 14) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 15) asm volatile("v_add_lshl_u32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
    if constexpr (KIND == 16) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (KIND == 17) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "s"(b), "v"(c));
    if constexpr (KIND == 18) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    if constexpr (KIND == 28) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 29) asm volatile("v_dot2_u32_u16 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    if constexpr (KIND == 30) asm volatile("v_bitop3_b16 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
    // SDWA halves of b + rot16(t): b + t.hi (32-bit add, src1 = WORD_1), then the
    // top half += t.lo (16-bit add into WORD_1, low half preserved)
    if constexpr (KIND == 34)
        asm volatile("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                     : "+v"(a) : "v"(b));
    if constexpr (KIND == 35)
        asm volatile("v_add_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0"
                     : "+v"(a) : "v"(b));
}

template <int KIND>
__global__ void __launch_bounds__(kThreads) valu_probe_kernel(uint32_t *out, uint32_t iters, uint64_t *clk) {
    uint32_t x[kChains];
    const uint32_t b = KIND == 17 ? __builtin_amdgcn_readfirstlane(blockIdx.x * 0x9E3779B9u)
                                  : threadIdx.x * 0x9E3779B9u;
    const uint32_t c = blockIdx.x + 0x7F4A7C15u + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kChains; ++j) x[j] = threadIdx.x + 17u * j;
    const uint32_t ks = __builtin_amdgcn_readfirstlane(c);
    uint32_t tqv = x[5] ^ ks;  // kind 25: q's pending half step
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
            for (int j = 0; j < kChains; ++j) {
                if constexpr (KIND == 19 || KIND == 20) {
                    // MD5-step mix interleaved at instruction granularity across chains:
                    // 19: all 8 chains per instruction; 20: pairs of chains (the NC = 2 shape)
                    constexpr int G = KIND == 19 ? kChains : 2;
                    if (j % G == 0) {
                        uint32_t f[G];
#pragma unroll
                        for (int q = 0; q < G; ++q)
                            asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(f[q]) : "v"(x[j + q]), "v"(b), "v"(c));
#pragma unroll
                        for (int q = 0; q < G; ++q)
                            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[j + q]) : "v"(f[q]), "v"(c));
#pragma unroll
                        for (int q = 0; q < G; ++q) asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[j + q]));
#pragma unroll
                        for (int q = 0; q < G; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j + q]) : "v"(b));
                    }
                } else if constexpr (KIND == 21) {
                    // two adds instead of add3, pairs of chains interleaved
                    if (j % 2 == 0) {
                        uint32_t f[2];
#pragma unroll
                        for (int q = 0; q < 2; ++q)
                            asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(f[q]) : "v"(x[j + q]), "v"(b), "v"(c));
#pragma unroll
                        for (int q = 0; q < 2; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j + q]) : "v"(c));
#pragma unroll
                        for (int q = 0; q < 2; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j + q]) : "v"(f[q]));
#pragma unroll
                        for (int q = 0; q < 2; ++q) asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[j + q]));
#pragma unroll
                        for (int q = 0; q < 2; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j + q]) : "v"(b));
                    }
                } else if constexpr (KIND == 22) {
                    // two chains software-pipelined so full- and half-rate instructions
                    // alternate: F(p) H(q) F(q) H(p) F(q) H(p) F(p) H(q)
                    if (j % 2 == 0) {
                        uint32_t &p = x[j], &q = x[j + 1];
                        uint32_t fp, fq;
                        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(fp) : "v"(p), "v"(b), "v"(c));
                        asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(q));
                        asm volatile("v_add_u32 %0, %0, %1" : "+v"(q) : "v"(b));
                        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(p) : "v"(fp), "v"(c));
                        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(fq) : "v"(q), "v"(b), "v"(c));
                        asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(p));
                        asm volatile("v_add_u32 %0, %0, %1" : "+v"(p) : "v"(b));
                        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(q) : "v"(fq), "v"(c));
                    }
                } else if constexpr (KIND == 24) {
                    // real MD5 dependency structure: 2 candidates x 4 state words
                    // (x[0..3], x[4..7]), step I = 4 u + j / 2, compiler-ordered
                    if (j % 2 == 0) {
                        const int I = 4 * u + j / 2;
                        const int a = (64 - I) % 4, bb = (a + 1) % 4, cc = (a + 2) % 4, d = (a + 3) % 4;
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            uint32_t *y = x + 4 * q;
                            const uint32_t f = __builtin_amdgcn_bitop3_b32(y[bb], y[cc], y[d], 0xCA);
                            y[a] = y[bb] + __builtin_rotateleft32(y[a] + f + ks, 7 + (I % 4) * 5);
                        }
                    }
                } else if constexpr (KIND == 25) {
                    // the same in the search kernel's hand-ordered alternating groups
                    if (j % 2 == 0) {
                        const int I = 4 * u + j / 2;
                        const int a = (64 - I) % 4, bb = (a + 1) % 4, cc = (a + 2) % 4, d = (a + 3) % 4;
                        uint32_t fp, fq, rq, tp;
                        asm volatile(
                            "v_bitop3_b32 %[fp], %[pb], %[pc], %[pd] bitop3:0xca\n\t"
                            "v_alignbit_b32 %[rq], %[tq], %[tq], 25\n\t"
                            "v_add_u32_e32 %[qb], %[qc], %[rq]\n\t"
                            "v_add3_u32 %[tp], %[pa], %[fp], %[kp]\n\t"
                            "v_bitop3_b32 %[fq], %[qb], %[qc], %[qd] bitop3:0xca\n\t"
                            "v_alignbit_b32 %[tp], %[tp], %[tp], 25\n\t"
                            "v_add_u32_e32 %[pa], %[pb], %[tp]\n\t"
                            "v_add3_u32 %[tq], %[qa], %[fq], %[kq]"
                            : [pa] "+v"(x[a]), [qb] "=&v"(x[4 + bb]), [tq] "+v"(tqv), [fp] "=&v"(fp), [fq] "=&v"(fq),
                              [rq] "=&v"(rq), [tp] "=&v"(tp)
                            : [pb] "v"(x[bb]), [pc] "v"(x[cc]), [pd] "v"(x[d]), [qc] "v"(x[4 + cc]), [qd] "v"(x[4 + d]),
                              [qa] "v"(x[4 + a]), [kp] "s"(ks), [kq] "s"(ks));
                    }
                } else if constexpr (KIND == 36 || KIND == 37) {
                    // the search kernel's order-2 step pair with its padding; 37 replaces
                    // each rotate + add by the two SDWA adds of b + rot16(t)
                    if (j % 2 == 0) {
                        const int I = 4 * u + j / 2;
                        const int a = (64 - I) % 4, bb = (a + 1) % 4, cc = (a + 2) % 4, d = (a + 3) % 4;
                        uint32_t fp, fq, rq, tp;
                        if constexpr (KIND == 36)
                            asm volatile(
                                "v_bitop3_b32 %[fp], %[pb], %[pc], %[pd] bitop3:0x96\n\t"
                                "v_alignbit_b32 %[rq], %[tq], %[tq], 16\n\ts_nop 0\n\t"
                                "v_add3_u32 %[tp], %[pa], %[fp], %[kp]\n\ts_nop 2\n\t"
                                "v_add_u32_e32 %[qb], %[qc], %[rq]\n\t"
                                "v_alignbit_b32 %[tp], %[tp], %[tp], 16\n\ts_nop 0\n\t"
                                "v_bitop3_b32 %[fq], %[qb], %[qc], %[qd] bitop3:0x96\n\t"
                                "v_add_u32_e32 %[pa], %[pb], %[tp]\n\t"
                                "v_add3_u32 %[tq], %[qa], %[fq], %[kq]\n\ts_nop 2"
                                : [pa] "+v"(x[a]), [qb] "=&v"(x[4 + bb]), [tq] "+v"(tqv), [fp] "=&v"(fp), [fq] "=&v"(fq),
                                  [rq] "=&v"(rq), [tp] "=&v"(tp)
                                : [pb] "v"(x[bb]), [pc] "v"(x[cc]), [pd] "v"(x[d]), [qc] "v"(x[4 + cc]),
                                  [qd] "v"(x[4 + d]), [qa] "v"(x[4 + a]), [kp] "s"(ks), [kq] "s"(ks));
                        else
                            asm volatile(
                                "v_bitop3_b32 %[fp], %[pb], %[pc], %[pd] bitop3:0x96\n\t"
                                "v_add_u32_sdwa %[qb], %[qc], %[tq] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
                                "v_add3_u32 %[tp], %[pa], %[fp], %[kp]\n\ts_nop 2\n\t"
                                "v_add_u16_sdwa %[qb], %[qb], %[tq] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t"
                                "v_add_u32_sdwa %[pa], %[pb], %[tp] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
                                "v_bitop3_b32 %[fq], %[qb], %[qc], %[qd] bitop3:0x96\n\t"
                                "v_add_u16_sdwa %[pa], %[pa], %[tp] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t"
                                "v_add3_u32 %[tq], %[qa], %[fq], %[kq]\n\ts_nop 2"
                                : [pa] "+v"(x[a]), [qb] "=&v"(x[4 + bb]), [tq] "+v"(tqv), [fp] "=&v"(fp), [fq] "=&v"(fq),
                                  [rq] "=&v"(rq), [tp] "=&v"(tp)
                                : [pb] "v"(x[bb]), [pc] "v"(x[cc]), [pd] "v"(x[d]), [qc] "v"(x[4 + cc]),
                                  [qd] "v"(x[4 + d]), [qa] "v"(x[4 + a]), [kp] "s"(ks), [kq] "s"(ks));
                        (void)rq;
                    }
                } else if constexpr (KIND == 26 || KIND == 27) {
                    // kind 22's alternating pairs on fixed registers (4 pairs p/q = v24+4k / v25+4k):
                    // 26 reads operands from distinct VGPR banks (index mod 4), 27 from one bank
                    if (j % 2 == 0) {
#define DPOW_PAIR(P, Q, B, C, FP, FQ)                                                          \
    "v_bitop3_b32 " FP ", " P ", " B ", " C " bitop3:0xca\n\t"                                 \
    "v_alignbit_b32 " Q ", " Q ", " Q ", 25\n\t"                                               \
    "v_add_u32_e32 " Q ", " Q ", " B "\n\t"                                                    \
    "v_add3_u32 " P ", " P ", " FP ", " C "\n\t"                                              \
    "v_bitop3_b32 " FQ ", " Q ", " B ", " C " bitop3:0xca\n\t"                                 \
    "v_alignbit_b32 " P ", " P ", " P ", 25\n\t"                                               \
    "v_add_u32_e32 " P ", " P ", " B "\n\t"                                                    \
    "v_add3_u32 " Q ", " Q ", " FQ ", " C "\n\t"
                        if constexpr (KIND == 26) {
                            if (j == 0) asm volatile(DPOW_PAIR("v24", "v25", "v14", "v19", "v41", "v40") ::: "v24", "v25", "v40", "v41");
                            if (j == 2) asm volatile(DPOW_PAIR("v28", "v29", "v14", "v19", "v41", "v40") ::: "v28", "v29", "v40", "v41");
                            if (j == 4) asm volatile(DPOW_PAIR("v32", "v33", "v14", "v19", "v41", "v40") ::: "v32", "v33", "v40", "v41");
                            if (j == 6) asm volatile(DPOW_PAIR("v36", "v37", "v14", "v19", "v41", "v40") ::: "v36", "v37", "v40", "v41");
                        } else {
                            if (j == 0) asm volatile(DPOW_PAIR("v24", "v25", "v12", "v16", "v40", "v41") ::: "v24", "v25", "v40", "v41");
                            if (j == 2) asm volatile(DPOW_PAIR("v28", "v29", "v12", "v16", "v40", "v41") ::: "v28", "v29", "v40", "v41");
                            if (j == 4) asm volatile(DPOW_PAIR("v32", "v33", "v12", "v16", "v40", "v41") ::: "v32", "v33", "v40", "v41");
                            if (j == 6) asm volatile(DPOW_PAIR("v36", "v37", "v12", "v16", "v40", "v41") ::: "v36", "v37", "v40", "v41");
                        }
#undef DPOW_PAIR
                    }
                } else if constexpr (KIND == 23) {
                    // MD5 step mix with the K operand from an SGPR (as in the kernel)
                    uint32_t f;
                    const uint32_t k = __builtin_amdgcn_readfirstlane(c);
                    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(f) : "v"(x[j]), "v"(b), "v"(c));
                    asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(f), "s"(k));
                    asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[j]));
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(b));
                } else if constexpr (KIND == 31 || KIND == 32 || KIND == 33) {
                    // 64-bit shifts / shift-add and the packed 64-bit move, on register pairs
                    if (j % 2 == 0) {
                        uint64_t v64 = ((uint64_t)x[j + 1] << 32) | x[j];
                        const uint64_t w64 = ((uint64_t)b << 32) | c;
                        if constexpr (KIND == 31) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(v64));
                        if constexpr (KIND == 32) asm volatile("v_lshl_add_u64 %0, %0, 7, %1" : "+v"(v64) : "v"(w64));
                        if constexpr (KIND == 33) asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(v64) : "v"(w64));
                        x[j] = (uint32_t)v64;
                        x[j + 1] = (uint32_t)(v64 >> 32);
                    }
                } else if constexpr (KIND == 5) {
                    uint32_t f = x[j];
                    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(f) : "v"(x[j]), "v"(b), "v"(c));
                    asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(f), "v"(c));
                    asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[j]));
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(b));
                } else {
                    op<KIND>(x[j], b, c);
                }
            }
        }
    }
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
    uint32_t acc = tqv;
#pragma unroll
    for (int j = 0; j < kChains; ++j) acc ^= x[j];
    out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

template <int KIND>
hipError_t run(uint32_t blocks, uint32_t iters, uint32_t *out, uint64_t *clk, hipStream_t s) {
    hipLaunchKernelGGL(valu_probe_kernel<KIND>, dim3(blocks), dim3(kThreads), 0, s, out, iters, clk);
    return hipGetLastError();
}

}  // namespace

extern "C" int dpow_diag_valu_rate(int device, int kind, double *lane_ops_per_s, double *clock_ghz) {
    if (kind < 0 || kind > 37 || !lane_ops_per_s || !clock_ghz) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return -2;
    const uint32_t blocks = (uint32_t)prop.multiProcessorCount * 8;  // 32 waves per CU = 8 per SIMD
    const uint32_t iters = 4096;
    uint32_t *out = nullptr;
    uint64_t *clk = nullptr;
    if (hipMalloc(&out, (size_t)blocks * kThreads * 4) != hipSuccess) return -2;
    if (hipMalloc(&clk, (size_t)blocks * 16) != hipSuccess) return -2;
    hipStream_t s;
    hipEvent_t e0, e1;
    (void)hipStreamCreate(&s);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto launch = [&]() -> hipError_t {
        switch (kind) {
            case 0: return run<0>(blocks, iters, out, clk, s);
            case 1: return run<1>(blocks, iters, out, clk, s);
            case 2: return run<2>(blocks, iters, out, clk, s);
            case 3: return run<3>(blocks, iters, out, clk, s);
            case 4: return run<4>(blocks, iters, out, clk, s);
            case 5: return run<5>(blocks, iters, out, clk, s);
            case 6: return run<6>(blocks, iters, out, clk, s);
            case 7: return run<7>(blocks, iters, out, clk, s);
            case 8: return run<8>(blocks, iters, out, clk, s);
            case 9: return run<9>(blocks, iters, out, clk, s);
            case 10: return run<10>(blocks, iters, out, clk, s);
            case 11: return run<11>(blocks, iters, out, clk, s);
            case 12: return run<12>(blocks, iters, out, clk, s);
            case 13: return run<13>(blocks, iters, out, clk, s);
            case 14: return run<14>(blocks, iters, out, clk, s);
            case 15: return run<15>(blocks, iters, out, clk, s);
            case 16: return run<16>(blocks, iters, out, clk, s);
            case 17: return run<17>(blocks, iters, out, clk, s);
            case 18: return run<18>(blocks, iters, out, clk, s);
            case 19: return run<19>(blocks, iters, out, clk, s);
            case 20: return run<20>(blocks, iters, out, clk, s);
            case 21: return run<21>(blocks, iters, out, clk, s);
            case 22: return run<22>(blocks, iters, out, clk, s);
            case 23: return run<23>(blocks, iters, out, clk, s);
            case 24: return run<24>(blocks, iters, out, clk, s);
            case 25: return run<25>(blocks, iters, out, clk, s);
            case 26: return run<26>(blocks, iters, out, clk, s);
            case 27: return run<27>(blocks, iters, out, clk, s);
            case 28: return run<28>(blocks, iters, out, clk, s);
            case 29: return run<29>(blocks, iters, out, clk, s);
            case 30: return run<30>(blocks, iters, out, clk, s);
            case 31: return run<31>(blocks, iters, out, clk, s);
            case 32: return run<32>(blocks, iters, out, clk, s);
            case 34: return run<34>(blocks, iters, out, clk, s);
            case 35: return run<35>(blocks, iters, out, clk, s);
            case 36: return run<36>(blocks, iters, out, clk, s);
            case 37: return run<37>(blocks, iters, out, clk, s);
            default: return run<33>(blocks, iters, out, clk, s);
        }
    };
    hipError_t err = hipSuccess;
    for (int w = 0; w < 3 && err == hipSuccess; ++w) err = launch();  // warm the clock
    (void)hipEventRecord(e0, s);
    const int reps = 5;
    for (int r = 0; r < reps && err == hipSuccess; ++r) err = launch();
    (void)hipEventRecord(e1, s);
    (void)hipStreamSynchronize(s);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(2 * blocks);
    (void)hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    double ratio = 0;
    uint32_t n = 0;
    for (uint32_t bI = 0; bI < blocks; ++bI)
        if (h[2 * bI + 1]) {
            ratio += (double)h[2 * bI] / (double)h[2 * bI + 1];
            ++n;
        }
    const double instr_per_lane =
        (double)iters * kUnroll * kChains * (kind == 5 || kind == 19 || kind == 20 || (kind >= 22 && kind <= 27) || kind == 36 || kind == 37 ? 4
         : kind == 21 ? 5 : (kind >= 31 && kind <= 33) ? 0.5 : 1);
    *lane_ops_per_s = instr_per_lane * (double)blocks * kThreads * reps / (ms * 1e-3);
    *clock_ghz = n ? ratio / n * 0.1 : 0.0;  // s_memrealtime ticks at 100 MHz
    (void)hipFree(out);
    (void)hipFree(clk);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return err == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------
// Launch round-trip floor of the platform (what bounds time-to-secret at small N).
namespace {
__global__ void ping_kernel(uint32_t *host_flag, uint32_t v) {
    if (threadIdx.x == 0 && host_flag) __hip_atomic_store(host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

extern "C" int dpow_diag_launch_latency(int device, int mode, int reps, double *median_us) {
    if (mode < 0 || mode > 2 || reps < 1 || !median_us) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -2;
    uint32_t *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0) != hipSuccess)
        return -2;
    *h = 0;
    std::vector<double> us;
    int rc = 0;
    for (int r = 0; r < reps + 5 && rc == 0; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        if (mode == 0) {  // launch + hipStreamSynchronize
            hipLaunchKernelGGL(ping_kernel, dim3(1), dim3(64), 0, s, (uint32_t *)nullptr, 0u);
            if (hipStreamSynchronize(s) != hipSuccess) rc = -2;
        } else if (mode == 1) {  // launch + spin on a pinned word the kernel writes
            const uint32_t v = (uint32_t)r + 1u;
            hipLaunchKernelGGL(ping_kernel, dim3(1), dim3(64), 0, s, d, v);
            while (__atomic_load_n(h, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
        } else {  // 16-byte device->host copy + hipStreamSynchronize
            if (hipMemcpyAsync(h + 4, d, 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                rc = -2;
        }
        const double dt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (r >= 5) us.push_back(dt);
    }
    (void)hipStreamSynchronize(s);
    std::sort(us.begin(), us.end());
    *median_us = us.empty() ? 0.0 : us[us.size() / 2];
    (void)hipHostFree(h);
    (void)hipStreamDestroy(s);
    return rc;
}
