// md5_variant.hip -- instantiates md5_search_kernel for one (NBLK, SH) pair and
// every word position W0 of that pair.  Compiled once per pair by the Makefile
// (-DDPOW_VNBLK=<1|2> -DDPOW_VSH=<0..3>) so the 72 variants build in parallel.
#include "md5_search_kernel.h"
#include "md5_variants.h"

#ifndef DPOW_VNBLK
#error "DPOW_VNBLK must be defined"
#endif
#ifndef DPOW_VSH
#error "DPOW_VSH must be defined"
#endif

namespace dpow {

namespace {
using KernelFn = void (*)(Launch);
#define DPOW_K(w) md5_search_kernel<DPOW_VNBLK, w, DPOW_VSH>
#if DPOW_VNBLK == 1
constexpr int kW0Lo = 0;
const KernelFn kTable[] = {DPOW_K(0), DPOW_K(1), DPOW_K(2),  DPOW_K(3),  DPOW_K(4),  DPOW_K(5),  DPOW_K(6),
                           DPOW_K(7), DPOW_K(8), DPOW_K(9), DPOW_K(10), DPOW_K(11), DPOW_K(12), DPOW_K(13)};
#else
constexpr int kW0Lo = 12;
const KernelFn kTable[] = {DPOW_K(12), DPOW_K(13), DPOW_K(14), DPOW_K(15)};
#endif
#undef DPOW_K
constexpr int kW0N = sizeof(kTable) / sizeof(kTable[0]);

KernelFn pick(int w0) { return (w0 >= kW0Lo && w0 < kW0Lo + kW0N) ? kTable[w0 - kW0Lo] : nullptr; }
}  // namespace

#define DPOW_CAT3(a, b, c) a##b##_##c
#define DPOW_NAME(a, b, c) DPOW_CAT3(a, b, c)

hipError_t DPOW_NAME(variant_launch_, DPOW_VNBLK, DPOW_VSH)(int w0, const Launch &L, uint32_t grid,
                                                           hipStream_t stream) {
    KernelFn fn = pick(w0);
    if (!fn) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlockThreads), 0, stream, L);
    return hipGetLastError();
}

hipError_t DPOW_NAME(variant_occupancy_, DPOW_VNBLK, DPOW_VSH)(int w0, int *blocks_per_cu) {
    KernelFn fn = pick(w0);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void *>(fn),
                                                        kBlockThreads, 0);
}

}  // namespace dpow
