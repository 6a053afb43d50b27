// search_ctrl.hip -- per-search reset of a context's device control state.
//
// One small kernel on the context stream replaces a host->device copy of the
// control block and a memset of the claim counters (each an SDMA round trip of
// tens of microseconds on the time-to-secret path).
#include <hip/hip_runtime.h>

#include "dpow_common.h"
#include "md5_variants.h"

#include <hip/hip_ext.h>

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
// Lower Ctrl::best to an external bound (dpow_search_bound) while a search runs:
// its waves stop claiming work at or above it at their next group.
__global__ void search_bound_kernel(Ctrl *ctrl, unsigned long long g) {
    if (threadIdx.x == 0) __hip_atomic_fetch_min(&ctrl->best, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

hipError_t search_bound(Ctrl *ctrl, unsigned long long g, hipStream_t stream) {
    hipLaunchKernelGGL(search_bound_kernel, dim3(1), dim3(64), 0, stream, ctrl, g);
    return hipGetLastError();
}

hipError_t search_reset(Ctrl *ctrl, unsigned long long *claims, uint32_t n_claims, unsigned long long bound,
                        hipStream_t stream, hipEvent_t done_ev) {
    hipExtLaunchKernelGGL(search_reset_kernel, dim3(1), dim3(kBlockThreads), 0, stream, nullptr, done_ev, 0, ctrl,
                          claims, n_claims, bound);
    return hipGetLastError();
}

}  // namespace dpow
