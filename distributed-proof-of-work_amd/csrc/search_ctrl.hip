// search_ctrl.hip -- the k = 0 kernel of a search window that starts at k = 0.
//
// k = 0 is the one chunk whose message layout (msg = nonce || threadByte, the 0x80 pad
// right behind it) differs from every other chunk's within a wave: a wave of an md5
// launch holds 64 / R consecutive k, so for R <= 64 it would mix k = 0 and k = 1.  Its
// R <= 256 candidates are hashed here instead, one per thread, on the search stream ahead
// of the search's first md5 launch (which starts at k = 1 and may span chunk lengths 1..3:
// plan.cpp).  (Round 3 start: this kernel also reset the control block and
// claim counters, in front of the first md5 launch on the same stream -- 15 us on every
// search's time-to-secret path; the launches now reset the next search's control block
// themselves, md5_search_kernel.h publish().)
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

// The k = 0 candidates, one per thread (worker.go:318-356 for chunk_0 = []: msg = nonce ||
// threadByte), and the kernel's own completion record: {its first hit, or kNoHit}.  It
// touches no control block; the host consumes its record first (the lowest indices of the
// window), so a hit here ends the search and the md5 launches queued behind it are
// stopped as stale.
__global__ void __launch_bounds__(kBlockThreads) search_k0_kernel(const StartK0 k0) {
    __shared__ unsigned long long hit;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) hit = kNoHit;
    __syncthreads();
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
        // g = 0 * 256 + threadByte
        if (trailing_zero_nibbles(st[0], st[1], st[2], st[3]) >= k0.ntz) atomicMin(&hit, (unsigned long long)tb);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&k0.snap->best, hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->stop, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->t_start, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->t_end, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&k0.snap->seq, k0.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__global__ void context_init_kernel(Ctrl *ctrl, uint32_t n_ctrl, unsigned long long *claims, uint32_t n_claims) {
    for (uint32_t i = threadIdx.x; i < n_ctrl; i += blockDim.x) {
        ctrl[i].best = kNoHit;
        ctrl[i].stop = 0u;
        ctrl[i].done = 0u;
    }
    for (uint32_t i = threadIdx.x; i < n_claims; i += blockDim.x) claims[i] = 0ull;
}
__global__ void clock_probe_kernel(unsigned long long *out) {
    if (threadIdx.x == 0)
        __hip_atomic_store(out, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

hipError_t clock_probe(unsigned long long *out, hipStream_t stream) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, stream, out);
    return hipGetLastError();
}

hipError_t context_init(Ctrl *ctrl, uint32_t n_ctrl, unsigned long long *claims, uint32_t n_claims,
                        hipStream_t stream) {
    hipLaunchKernelGGL(context_init_kernel, dim3(1), dim3(kBlockThreads), 0, stream, ctrl, n_ctrl, claims, n_claims);
    return hipGetLastError();
}

hipError_t search_k0_prepare() {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(search_k0_kernel));
    if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(context_init_kernel));
    return e;
}

hipError_t search_k0(const StartK0 &k0, hipStream_t stream) {
    hipLaunchKernelGGL(search_k0_kernel, dim3(1), dim3(kBlockThreads), 0, stream, k0);
    return hipGetLastError();
}

}  // namespace dpow
