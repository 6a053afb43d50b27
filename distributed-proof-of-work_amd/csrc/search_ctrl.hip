// search_ctrl.hip -- the start kernel of a search: resets a context's device control
// state and hashes the chunk of zero bytes (k = 0).
//
// One small kernel on the context stream replaces a host->device copy of the
// control block and a memset of the claim counters (each an SDMA round trip of
// tens of microseconds on the time-to-secret path).  k = 0 is the one chunk whose
// message layout (msg = nonce || threadByte, the 0x80 pad right behind it) differs
// from every other chunk's within a wave: a wave of an md5 launch holds 64 / R
// consecutive k, so for R <= 64 it would mix k = 0 and k = 1.  Its R <= 256 candidates
// are hashed here instead, one per thread, before the search's first md5 launch
// (which then starts at k = 1 and may span chunk lengths 1..3: plan.cpp).
#include <hip/hip_runtime.h>

#include "dpow_common.h"
#include "md5_variants.h"

#include <hip/hip_ext.h>

namespace dpow {

namespace {
// One MD5 compression (RFC 1321 3.4), compiler-scheduled: the start kernel hashes at
// most 256 candidates, once per search.
__device__ void md5_block(uint32_t st[4], const uint32_t M[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        if (i < 16) f = (b & c) | (~b & d);
        else if (i < 32) f = (d & b) | (~d & c);
        else if (i < 48) f = b ^ c ^ d;
        else f = c ^ (b | ~d);
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + __builtin_rotateleft32(a + f + kMd5K[i] + M[md5_word(i)], md5_shift(i));
        a = t;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

// Control block and claim counters [0, n_claims); then the k = 0 candidates, one per
// thread (worker.go:318-356 for chunk_0 = []: msg = nonce || threadByte).
__global__ void __launch_bounds__(kBlockThreads) search_start_kernel(Ctrl *ctrl, unsigned long long *claims,
                                                                     uint32_t n_claims, unsigned long long bound,
                                                                     const StartK0 k0) {
    if (threadIdx.x == 0) {
        ctrl->best = bound;
        ctrl->stop = 0u;
        ctrl->done = 0u;
    }
    for (uint32_t i = threadIdx.x; i < n_claims; i += kBlockThreads) claims[i] = 0ull;
    if (k0.r == 0u) return;
    __threadfence();
    __syncthreads();  // Ctrl::best holds the bound before any hit is min'ed into it
    if (threadIdx.x < k0.r) {
        const uint32_t tb = k0.base_tb | threadIdx.x;
        uint32_t st[4] = {k0.iv[0], k0.iv[1], k0.iv[2], k0.iv[3]};
        for (uint32_t b = 0; b < k0.nblk; ++b) {
            uint32_t M[16];
#pragma unroll
            for (int w = 0; w < 16; ++w) M[w] = k0.T[16 * b + w];
            const uint32_t q = k0.p - 64 * b;  // the threadByte's byte in this block (if any)
            if (k0.p / 64 == b) {
#pragma unroll
                for (int w = 0; w < 16; ++w)
                    if ((uint32_t)w == q / 4) M[w] += tb << (8 * (q % 4));
            }
            md5_block(st, M);
        }
        if (trailing_zero_nibbles(st[0], st[1], st[2], st[3]) >= k0.ntz) {
            // g = 0 * 256 + threadByte; a returning atomic, consumed: performed before the barrier
            const unsigned long long prev =
                __hip_atomic_fetch_min(&ctrl->best, (unsigned long long)tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("; dpow: k0 atomicMin performed (%0)" ::"v"(prev));
        }
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long best = __hip_atomic_load(&ctrl->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&k0.snap->best, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->stop, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->seq, k0.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
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

hipError_t search_start(Ctrl *ctrl, unsigned long long *claims, uint32_t n_claims, unsigned long long bound,
                        const StartK0 &k0, hipStream_t stream, hipEvent_t start, hipEvent_t stop) {
    hipExtLaunchKernelGGL(search_start_kernel, dim3(1), dim3(kBlockThreads), 0, stream, start, stop, 0, ctrl, claims,
                          n_claims, bound, k0);
    return hipGetLastError();
}

}  // namespace dpow
