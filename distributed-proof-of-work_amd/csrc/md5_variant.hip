// md5_variant.hip -- instantiates md5_search_kernel for one (NBLK, SH) pair and
// every word position W0 of that pair.  Compiled once per pair by the Makefile
// (-DDPOW_VNBLK=<1|2> -DDPOW_VSH=<0..3>) so the 72 layouts (154 kernels with the one-block
// D-equality ones and SH = 3's narrow ones) build in parallel.
#include "md5_search_kernel.h"
#include "md5_variants.h"

#include <hip/hip_ext.h>

#ifndef DPOW_VNBLK
#error "DPOW_VNBLK must be defined"
#endif
#ifndef DPOW_VSH
#error "DPOW_VSH must be defined"
#endif

namespace dpow {

namespace {
using namespace DPOW_KNS;
using KernelFn = void (*)(Launch);
// EQ kernels (the D-equality test, use_d_equality) exist for one final block only.
// The kernel of a layout: the long-SGPR-budget template for long nonces and two
// final blocks (md5_search_kernel.h kLongSgpr), a slightly larger budget for the two-block
// W0 = 15 layouts and a few more (kW15Sgpr); only the chosen one is instantiated.
template <int NBLK, int W0, int SH, bool EQ, bool KSPAN>
constexpr KernelFn kernel_of() {
    if constexpr (kSgprOf<NBLK, W0, SH, KSPAN> == 2) return md5_search_kernel_w15sgpr<NBLK, W0, SH, EQ, KSPAN>;
    else if constexpr (kSgprOf<NBLK, W0, SH, KSPAN> == 1) return md5_search_kernel_lsgpr<NBLK, W0, SH, EQ, KSPAN>;
    else return md5_search_kernel<NBLK, W0, SH, EQ, KSPAN>;
}
// [EQ][narrow][w0 - kW0Lo]: narrow = the SH = 3 kernel without the lanes' k offset
// (md5_search_kernel.h hash_wave_block KSPAN), for launches with R >= 64, where narrow_knobs
// has one; other layouts have one kernel for both.
#define DPOW_K(w, e, nar) \
    kernel_of<DPOW_VNBLK, w, DPOW_VSH, e, !(DPOW_VSH == 3 && nar && narrow_knobs(DPOW_VNBLK, w).on)>()
#if DPOW_VNBLK == 1
constexpr int kW0Lo = 0;
#define DPOW_ROW(e, n)                                                                                              \
    {DPOW_K(0, e, n), DPOW_K(1, e, n), DPOW_K(2, e, n),  DPOW_K(3, e, n),  DPOW_K(4, e, n),  DPOW_K(5, e, n),        \
     DPOW_K(6, e, n), DPOW_K(7, e, n), DPOW_K(8, e, n),  DPOW_K(9, e, n),  DPOW_K(10, e, n), DPOW_K(11, e, n),       \
     DPOW_K(12, e, n), DPOW_K(13, e, n)}
const KernelFn kTable[2][2][14] = {{DPOW_ROW(false, false), DPOW_ROW(false, true)},
                                   {DPOW_ROW(true, false), DPOW_ROW(true, true)}};
#else
constexpr int kW0Lo = 12;
#define DPOW_ROW(e, n) {DPOW_K(12, e, n), DPOW_K(13, e, n), DPOW_K(14, e, n), DPOW_K(15, e, n)}
const KernelFn kTable[2][2][4] = {{DPOW_ROW(false, false), DPOW_ROW(false, true)},
                                  {DPOW_ROW(false, false), DPOW_ROW(false, true)}};
#endif
#undef DPOW_ROW
#undef DPOW_K
constexpr int kW0N = sizeof(kTable[0][0]) / sizeof(kTable[0][0][0]);

// narrow: the launch's R >= 64 (rbits >= 6), so no wave-block's lanes span two k
KernelFn pick(int w0, bool eq, bool narrow) {
    return (w0 >= kW0Lo && w0 < kW0Lo + kW0N) ? kTable[eq ? 1 : 0][narrow ? 1 : 0][w0 - kW0Lo] : nullptr;
}
}  // namespace

#if DPOW_VLS  // the chunk-length-spanning SH = 0 kernels: variant_launch_<n>_0_ls
#define DPOW_SFX _ls
#else
#define DPOW_SFX
#endif
#define DPOW_CAT4(a, b, c, d) a##b##_##c##d
#define DPOW_NAME2(a, b, c, d) DPOW_CAT4(a, b, c, d)
#define DPOW_NAME(a, b, c) DPOW_NAME2(a, b, c, DPOW_SFX)

hipError_t DPOW_NAME(variant_launch_, DPOW_VNBLK, DPOW_VSH)(int w0, const Launch &L, uint32_t grid,
                                                           hipStream_t stream) {
    KernelFn fn = pick(w0, use_d_equality(DPOW_VNBLK, L.ntz), L.rbits >= 6u);
    if (!fn) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlockThreads), 0, stream, L);
    return hipGetLastError();
}

// Resolve every kernel of this translation unit on the current device (dpow_open, once per
// device and process).  HIP loads a translation unit's code object on the first use of any
// of its kernels: round 3's first search after dpow_open waited 972.8 us between its k = 0
// kernel and its first md5 launch, the "_ls" unit's load (profiles/r03_final_tts_timeline.json).
hipError_t DPOW_NAME(variant_prepare_, DPOW_VNBLK, DPOW_VSH)() {
    for (const auto &eq : kTable)
        for (const auto &row : eq)
            for (KernelFn fn : row) {
                hipFuncAttributes a;
                const hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(fn));
                if (e != hipSuccess) return e;
            }
    return hipSuccess;
}

hipError_t DPOW_NAME(variant_occupancy_, DPOW_VNBLK, DPOW_VSH)(int w0, int *blocks_per_cu) {
    KernelFn fn = pick(w0, false, true);  // the sweep's (workerBits 0) kernel
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void *>(fn),
                                                        kBlockThreads, 0);
}

}  // namespace dpow

#if DPOW_WAVE_TRACE && DPOW_VNBLK == 1 && DPOW_VSH == 0
// Diagnostic builds only: the per-wave trace of the last one-block, SH = 0 launch
// (dpow_diag_wave_trace_ls: of the last chunk-length-spanning one, below k = 2^24).
#if DPOW_VLS
extern "C" int dpow_diag_wave_trace_ls(unsigned long long *out, size_t n) {
#else
extern "C" int dpow_diag_wave_trace(unsigned long long *out, size_t n) {
#endif
    if (n > dpow::DPOW_KNS::kTraceWaves * dpow::DPOW_KNS::kTraceFields)
        n = dpow::DPOW_KNS::kTraceWaves * dpow::DPOW_KNS::kTraceFields;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(dpow::DPOW_KNS::g_wave_trace), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -2;
}
#endif
