// md5_dispatch.cpp -- routes a launch to the kernel variant of its message layout.
#include "md5_variants.h"

namespace dpow {

hipError_t search_launch(int nblk, int w0, int sh, const Launch &L, uint32_t grid, hipStream_t stream) {
    if (!variant_exists(nblk, w0, sh)) return hipErrorInvalidValue;
    if (L.seg0 == kLsegBase) {
        if (sh != 0) return hipErrorInvalidValue;
        return nblk == 1 ? variant_launch_1_0_ls(w0, L, grid, stream)
                         : variant_launch_2_0_ls(w0, L, grid, stream);
    }
#define DPOW_CASE(n, s) \
    if (nblk == n && sh == s) return variant_launch_##n##_##s(w0, L, grid, stream);
    DPOW_CASE(1, 0) DPOW_CASE(1, 1) DPOW_CASE(1, 2) DPOW_CASE(1, 3)
    DPOW_CASE(2, 0) DPOW_CASE(2, 1) DPOW_CASE(2, 2) DPOW_CASE(2, 3)
#undef DPOW_CASE
    return hipErrorInvalidValue;
}

hipError_t search_occupancy(int nblk, int w0, int sh, int *blocks_per_cu) {
    if (!variant_exists(nblk, w0, sh)) return hipErrorInvalidValue;
#define DPOW_CASE(n, s) \
    if (nblk == n && sh == s) return variant_occupancy_##n##_##s(w0, blocks_per_cu);
    DPOW_CASE(1, 0) DPOW_CASE(1, 1) DPOW_CASE(1, 2) DPOW_CASE(1, 3)
    DPOW_CASE(2, 0) DPOW_CASE(2, 1) DPOW_CASE(2, 2) DPOW_CASE(2, 3)
#undef DPOW_CASE
    return hipErrorInvalidValue;
}

hipError_t search_prepare() {
    hipError_t e = search_k0_prepare();
#define DPOW_PREP(n, s) \
    if (e == hipSuccess) e = variant_prepare_##n##_##s();
    DPOW_PREP(1, 0) DPOW_PREP(1, 1) DPOW_PREP(1, 2) DPOW_PREP(1, 3)
    DPOW_PREP(2, 0) DPOW_PREP(2, 1) DPOW_PREP(2, 2) DPOW_PREP(2, 3)
    DPOW_PREP(1, 0_ls) DPOW_PREP(2, 0_ls)
#undef DPOW_PREP
    return e;
}

}  // namespace dpow
