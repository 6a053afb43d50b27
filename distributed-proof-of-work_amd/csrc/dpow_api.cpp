// dpow_api.cpp -- the C ABI (include/dpow.h) over the gfx950 search kernels.
//
// dpow_search replaces the reference miner's enumeration loop
// (worker.go:301-400): plan the window into launches (plan.cpp), queue them on
// the context's stream behind one control-block reset with at most kDepth in
// flight (a pinned snapshot of the control block follows each launch), and
// re-verify a hit with the host MD5 before returning it.  Launches queued after
// a hit (or a cancel) retire at once: every worker wave compares its first
// index against Ctrl::best / Ctrl::stop before hashing.
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/dpow.h"
#include "dpow_common.h"
#include "md5_host.h"
#include "md5_variants.h"
#include "plan.h"

using namespace dpow;

namespace {

thread_local std::string g_last_error;

int set_error(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return set_error(DPOW_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define DPOW_HIP(call)                                    \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

// Persistent grid: one round of resident workgroups (8 four-wave workgroups per
// CU at <= 80 SGPRs), work handed out by in-order chunk claims.  A chunk is
// sized for >= 16 claims per wave (small tail) and at most 32 wave-blocks
// (one claim counter serves < 88 claims/us, MI355X_MICROARCH.md "dequeue").
constexpr uint64_t kBlocksPerCu = 8;
constexpr uint64_t kClaimsPerWave = 16;
constexpr uint64_t kMaxChunk = 32;
constexpr size_t kClaimRing = 1024;  // per-launch claim counters, zeroed per search
// Launches kept in flight: launch j is queued only after the control block
// snapshot behind launch j - kDepth shows no hit and no cancel, so a hit or a
// cancel leaves at most kDepth launches to retire (each exits at its first check).
constexpr size_t kDepth = 3;
constexpr size_t kRing = 8;  // pinned control-block snapshots and event slots (>= kDepth + 1)

}  // namespace

struct dpow_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Ctrl *d_ctrl = nullptr;
    unsigned long long *d_claims = nullptr;  // kClaimRing claim counters
    Ctrl *h_ctrl = nullptr;        // pinned staging: [0] reset image, [1 + j % kRing] snapshots
    uint32_t *h_cancel = nullptr;  // pinned, host-coherent, mapped
    uint32_t *d_cancel = nullptr;  // device alias
    uint32_t cus = 0;
    std::vector<hipEvent_t> events;  // 3 per ring slot: start, kernel end, snapshot landed
    dpow_stats stats{};
};

extern "C" {

const char *dpow_last_error(void) { return g_last_error.c_str(); }
int dpow_abi_version(void) { return DPOW_ABI_VERSION; }

int dpow_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int dpow_open(int device, dpow_ctx **out) {
    if (!out) return set_error(DPOW_EINVAL, "dpow_open: out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return set_error(DPOW_EHIP, "dpow_open: no HIP device visible");
    if (device < 0 || device >= n) return set_error(DPOW_EINVAL, "dpow_open: bad device ordinal");
    DPOW_HIP(hipSetDevice(device));
    dpow_ctx *c = new (std::nothrow) dpow_ctx();
    if (!c) return set_error(DPOW_ENOMEM, "dpow_open: out of memory");
    c->device = device;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) {
        delete c;
        return hip_fail(e, "hipGetDeviceProperties");
    }
    c->cus = (uint32_t)prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&c->d_ctrl, sizeof(Ctrl))) != hipSuccess ||
        (e = hipMalloc(&c->d_claims, kClaimRing * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipHostMalloc(&c->h_ctrl, (1 + kRing) * sizeof(Ctrl), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_cancel, 64, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_cancel), c->h_cancel, 0)) != hipSuccess) {
        dpow_close(c);
        return hip_fail(e, "dpow_open: allocation");
    }
    memset(c->h_cancel, 0, 64);
    *out = c;
    return 0;
}

void dpow_close(dpow_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t ev : c->events) (void)hipEventDestroy(ev);
    if (c->d_ctrl) (void)hipFree(c->d_ctrl);
    if (c->d_claims) (void)hipFree(c->d_claims);
    if (c->h_ctrl) (void)hipHostFree(c->h_ctrl);
    if (c->h_cancel) (void)hipHostFree(c->h_cancel);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

volatile uint32_t *dpow_cancel_flag(dpow_ctx *c) { return c ? c->h_cancel : nullptr; }
void *dpow_stream(dpow_ctx *c) { return c ? (void *)c->stream : nullptr; }
int dpow_device(dpow_ctx *c) { return c ? c->device : -1; }

int dpow_geometry(dpow_ctx *c, uint32_t *cus, uint32_t *blocks_per_cu, uint32_t *threads_per_block) {
    if (!c) return set_error(DPOW_EINVAL, "dpow_geometry: ctx is NULL");
    if (cus) *cus = c->cus;
    if (blocks_per_cu) *blocks_per_cu = (uint32_t)kBlocksPerCu;
    if (threads_per_block) *threads_per_block = kBlockThreads;
    return 0;
}

int dpow_get_stats(dpow_ctx *c, dpow_stats *out) {
    if (!c || !out) return set_error(DPOW_EINVAL, "dpow_get_stats: NULL argument");
    *out = c->stats;
    return 0;
}

void dpow_reset_stats(dpow_ctx *c) {
    if (c) c->stats = dpow_stats{};
}

int dpow_secret_from_index(uint64_t g, uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len) {
    if (!secret_out || !secret_len) return set_error(DPOW_EINVAL, "dpow_secret_from_index: NULL argument");
    if (g == DPOW_NO_HIT) return set_error(DPOW_EINVAL, "dpow_secret_from_index: no hit");
    size_t n = 0;
    secret_out[n++] = (uint8_t)(g & 0xFF);
    for (uint64_t k = g >> 8; k; k >>= 8) secret_out[n++] = (uint8_t)(k & 0xFF);
    *secret_len = n;
    return 0;
}

void dpow_md5(const uint8_t *msg, size_t len, uint8_t digest_out[16]) { md5_digest(msg, len, digest_out); }

uint32_t dpow_trailing_zero_nibbles(const uint8_t digest[16]) { return digest_trailing_zero_nibbles(digest); }

int dpow_verify(const uint8_t *nonce, size_t nonce_len, const uint8_t *secret, size_t secret_len, uint32_t ntz) {
    std::vector<uint8_t> msg(nonce_len + secret_len);
    if (nonce_len) memcpy(msg.data(), nonce, nonce_len);
    if (secret_len) memcpy(msg.data() + nonce_len, secret, secret_len);
    uint8_t d[16];
    md5_digest(msg.data(), msg.size(), d);
    return digest_trailing_zero_nibbles(d) >= ntz ? 1 : 0;
}

int dpow_plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t worker_byte, uint32_t worker_bits,
                     uint64_t k_begin, uint64_t k_end, dpow_plan_launch *out, size_t max_launches) {
    std::vector<PlannedLaunch> plan;
    int n = plan_window(nonce, nonce_len, 0, worker_byte, worker_bits, k_begin, k_end, plan);
    if (n < 0) return set_error(n, "dpow_plan_window: bad arguments");
    for (size_t i = 0; i < plan.size() && i < max_launches && out; ++i) out[i] = plan[i].info;
    return n;
}

int dpow_plan_candidate(const uint8_t *nonce, size_t nonce_len, uint32_t worker_byte, uint32_t worker_bits,
                        uint64_t local_idx, uint32_t iv_out[4], uint32_t words_out[32], uint32_t *nblk_out) {
    if (!iv_out || !words_out || !nblk_out) return set_error(DPOW_EINVAL, "dpow_plan_candidate: NULL argument");
    const uint64_t k = local_idx >> remainder_bits(worker_bits);
    std::vector<PlannedLaunch> plan;
    int n = plan_window(nonce, nonce_len, 0, worker_byte, worker_bits, k, k + 1, plan);
    if (n != 1) return set_error(n < 0 ? n : DPOW_EINVAL, "dpow_plan_candidate: bad arguments");
    for (int w = 0; w < 4; ++w) iv_out[w] = plan[0].L.iv[w];
    memset(words_out, 0, 32 * sizeof(uint32_t));
    candidate_words(plan[0], local_idx, words_out);
    *nblk_out = plan[0].info.nblk;
    return 0;
}

int dpow_search(dpow_ctx *c, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, uint64_t *best_global_idx,
                uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len) {
    if (!c || !best_global_idx || !secret_out || !secret_len)
        return set_error(DPOW_EINVAL, "dpow_search: NULL argument");
    if (nonce_len && !nonce) return set_error(DPOW_EINVAL, "dpow_search: nonce is NULL");
    if (worker_byte > 255u) return set_error(DPOW_EINVAL, "dpow_search: worker_byte > 255");
    if (k_end > DPOW_K_LIMIT) return set_error(DPOW_ERANGE, "dpow_search: k_end beyond DPOW_K_LIMIT");
    *secret_len = 0;
    c->stats.searches++;
    if (k_begin >= k_end) return DPOW_EXHAUSTED;
    if (__atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) return DPOW_CANCELLED;

    WindowPlanner planner;
    int rc = planner.init(nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end);
    if (rc < 0) return set_error(rc, "dpow_search: planning failed");
    DPOW_HIP(hipSetDevice(c->device));
    while (c->events.size() < 3 * kRing) {  // {start, kernel end, snapshot landed} per ring slot
        hipEvent_t ev;
        DPOW_HIP(hipEventCreate(&ev));
        c->events.push_back(ev);
    }
    auto ev = [&](size_t li, int which) { return c->events[3 * (li % kRing) + which]; };

    const uint64_t bound = *best_global_idx;
    c->h_ctrl->best = bound;
    c->h_ctrl->stop = 0;
    c->h_ctrl->done = 0;
    DPOW_HIP(hipMemcpyAsync(c->d_ctrl, c->h_ctrl, sizeof(Ctrl), hipMemcpyHostToDevice, c->stream));
    DPOW_HIP(hipMemsetAsync(c->d_claims, 0, kClaimRing * sizeof(unsigned long long), c->stream));

    constexpr uint32_t wpb = kBlockThreads / 64;
    uint32_t done_target = 0;
    uint64_t candidates = 0;
    double ms_total = 0.0;
    size_t launched = 0, retired = 0;
    // Kernel time of a launch whose snapshot has landed (its events are complete).
    auto retire = [&](size_t li) -> int {
        float ms = 0.f;
        DPOW_HIP(hipEventElapsedTime(&ms, ev(li, 0), ev(li, 1)));
        ms_total += ms;
        return 0;
    };
    PlannedLaunch pl;
    while (planner.next(pl)) {
        const size_t li = launched;
        if (li >= kDepth) {  // the snapshot behind launch li - kDepth decides whether to go on
            const size_t lj = li - kDepth;
            DPOW_HIP(hipEventSynchronize(ev(lj, 2)));
            if (retire(lj) < 0) return DPOW_EHIP;
            retired = lj + 1;
            const Ctrl &snap = c->h_ctrl[1 + lj % kRing];
            if (snap.best < bound || snap.stop != 0u || __atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) break;
        }
        Launch &L = pl.L;
        unsigned long long *claim = c->d_claims + li % kClaimRing;
        if (li >= kClaimRing) DPOW_HIP(hipMemsetAsync(claim, 0, sizeof(unsigned long long), c->stream));
        uint64_t worker_blocks = (L.n_wblocks + wpb - 1) / wpb;
        if (worker_blocks > (uint64_t)c->cus * kBlocksPerCu) worker_blocks = (uint64_t)c->cus * kBlocksPerCu;
        uint64_t chunk = L.n_wblocks / (worker_blocks * wpb * kClaimsPerWave);
        if (chunk < 1) chunk = 1;
        if (chunk > kMaxChunk) chunk = kMaxChunk;
        done_target += (uint32_t)(worker_blocks * wpb);
        L.chunk = (uint32_t)chunk;
        L.n_chunks = (L.n_wblocks + chunk - 1) / chunk;
        L.claim = claim;
        L.done_target = done_target;
        L.ctrl = c->d_ctrl;
        L.cancel = c->d_cancel;
        DPOW_HIP(hipEventRecord(ev(li, 0), c->stream));
        hipError_t e = search_launch((int)pl.info.nblk, (int)pl.info.w0, (int)pl.info.sh, L,
                                     (uint32_t)(worker_blocks + 1), c->stream);
        if (e != hipSuccess) return hip_fail(e, "search_launch");
        DPOW_HIP(hipEventRecord(ev(li, 1), c->stream));
        DPOW_HIP(hipMemcpyAsync(&c->h_ctrl[1 + li % kRing], c->d_ctrl, sizeof(Ctrl), hipMemcpyDeviceToHost,
                                c->stream));
        DPOW_HIP(hipEventRecord(ev(li, 2), c->stream));
        candidates += L.i_end - L.i_begin;
        ++launched;
    }
    DPOW_HIP(hipStreamSynchronize(c->stream));
    for (size_t lj = retired; lj < launched; ++lj)
        if (retire(lj) < 0) return DPOW_EHIP;
    const Ctrl fin = c->h_ctrl[1 + (launched - 1) % kRing];
    c->stats.launches += launched;
    c->stats.candidates += candidates;
    c->stats.kernel_ms += ms_total;

    const uint64_t best = fin.best;
    if (best < bound) {
        dpow_secret_from_index(best, secret_out, secret_len);
        if (!dpow_verify(nonce, nonce_len, secret_out, *secret_len, ntz)) {
            *secret_len = 0;
            return set_error(DPOW_EVERIFY, "dpow_search: kernel hit failed host MD5 verification");
        }
        *best_global_idx = best;
        return DPOW_FOUND;
    }
    if (fin.stop != 0u || __atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) return DPOW_CANCELLED;
    return DPOW_EXHAUSTED;
}

}  // extern "C"
