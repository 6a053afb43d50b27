// md5_variants.h -- per-(NBLK, SH) launch entry points (defined in md5_variant.hip)
// and the dispatcher over them (md5_dispatch.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "dpow_common.h"

namespace dpow {

#define DPOW_DECL_VARIANT(n, s)                                                                  \
    hipError_t variant_launch_##n##_##s(int w0, const Launch &L, uint32_t grid, hipStream_t st); \
    hipError_t variant_occupancy_##n##_##s(int w0, int *blocks_per_cu);                        \
    hipError_t variant_prepare_##n##_##s();
DPOW_DECL_VARIANT(1, 0)
DPOW_DECL_VARIANT(1, 1)
DPOW_DECL_VARIANT(1, 2)
DPOW_DECL_VARIANT(1, 3)
DPOW_DECL_VARIANT(2, 0)
DPOW_DECL_VARIANT(2, 1)
DPOW_DECL_VARIANT(2, 2)
DPOW_DECL_VARIANT(2, 3)
DPOW_DECL_VARIANT(1, 0_ls)  // chunk-length-spanning SH = 0 kernels (launches below k = 2^24)
DPOW_DECL_VARIANT(2, 0_ls)
#undef DPOW_DECL_VARIANT

// True when a kernel variant exists for (nblk, w0, sh).
inline bool variant_exists(int nblk, int w0, int sh) {
    if (sh < 0 || sh > 3) return false;
    if (nblk == 1) return w0 >= 0 && w0 <= 13;
    if (nblk == 2) return w0 >= 12 && w0 <= 15;
    return false;
}

// Launches whose template is chunk length 0's (L.seg0 == kLsegBase: SH = 0 below k = 2^24)
// run the "_ls" kernels.  (No timing events: the kernel stamps its start and end into its
// completion record.)
hipError_t search_launch(int nblk, int w0, int sh, const Launch &L, uint32_t grid, hipStream_t stream);
hipError_t search_occupancy(int nblk, int w0, int sh, int *blocks_per_cu);
// Load and resolve every search kernel (all layouts, the "_ls" ones, the k = 0 and init
// kernels) on the current device, so no search pays a code object's first-use load.
hipError_t search_prepare();

// The k = 0 kernel (search_ctrl.hip): hashes the k = 0 candidates (msg = nonce ||
// threadByte, R of them) and writes k0.snap's record with their first hit.
struct StartK0 {
    uint32_t r;        // threadBytes of the partition (R)
    uint32_t base_tb;  // uint8(worker_byte << R_bits)
    uint32_t nblk;     // final blocks of the k = 0 message
    uint32_t p;        // byte offset of the threadByte in them
    uint32_t ntz;
    uint32_t seq;      // record value (launch sequence + 1)
    Snap *snap;        // completion record (device alias of the pinned slot)
    uint32_t iv[4];    // chaining value entering the final blocks
    uint32_t T[32];    // their words, threadByte zeroed (plan.cpp build_template)
};
hipError_t search_k0(const StartK0 &k0, hipStream_t stream);
hipError_t search_k0_prepare();
// A context's initial control state (search_ctrl.hip): n_ctrl clean control blocks, n_claims
// zero claim counters.
hipError_t context_init(Ctrl *ctrl, uint32_t n_ctrl, unsigned long long *claims, uint32_t n_claims,
                        hipStream_t stream);
// One thread stamps s_memrealtime into *out (system scope): the host/device clock pairing of
// dpow_diag_clock_sync.
hipError_t clock_probe(unsigned long long *out, hipStream_t stream);

}  // namespace dpow
