// search_ctrl.hip -- per-search reset of a context's device control state.
//
// One small kernel on the context stream replaces a host->device copy of the
// control block and a memset of the claim counters (each an SDMA round trip of
// tens of microseconds on the time-to-secret path).
#include <hip/hip_runtime.h>

#include "dpow_common.h"
#include "md5_variants.h"

namespace dpow {

namespace {
// Control block (when ctrl != nullptr) and claim counters [0, n_claims).
__global__ void __launch_bounds__(kBlockThreads) search_reset_kernel(Ctrl *ctrl, unsigned long long *claims,
                                                                     uint32_t n_claims, unsigned long long bound) {
    if (ctrl && threadIdx.x == 0) {
        ctrl->best = bound;
        ctrl->stop = 0u;
        ctrl->done = 0u;
    }
    for (uint32_t i = threadIdx.x; i < n_claims; i += kBlockThreads) claims[i] = 0ull;
}
}  // namespace

hipError_t search_reset(Ctrl *ctrl, unsigned long long *claims, uint32_t n_claims, unsigned long long bound,
                        hipStream_t stream) {
    hipLaunchKernelGGL(search_reset_kernel, dim3(1), dim3(kBlockThreads), 0, stream, ctrl, claims, n_claims, bound);
    return hipGetLastError();
}

}  // namespace dpow
