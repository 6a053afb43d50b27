// dpow_api.cpp -- the C ABI (include/dpow.h) over the gfx950 search kernels.
//
// dpow_search replaces the reference miner's enumeration loop
// (worker.go:301-400): plan the window into launches (plan.cpp), queue them on
// the context's stream (behind the k = 0 kernel when the window holds k = 0) with at most kDepth in flight,
// and re-verify a hit with the host MD5 before returning it.  Each launch's
// last retiring workgroup writes a completion record (the control block as of
// the end of the launch) to pinned host memory; the host polls that record rather
// than synchronising on events, so a hit is seen one PCIe write after the
// kernel publishes it.  Launches queued behind a hit (or a cancel) are not
// waited for: they retire at once (every worker wave compares its first index
// against Ctrl::best / Ctrl::stop before hashing), in stream order ahead of
// the next search on the context.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dpow.h"
#include "../../include/dpow_worker.h"
#include "dpow_common.h"
#include "md5_host.h"
#include "md5_variants.h"
#include "node.h"
#include "plan.h"
#include "../../include/dpow_diag.h"


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

// The calling thread's current device (HIP per-thread state) for the duration of an
// entry point, restored on return: a host thread that drives several GPUs -- one rank's
// coordinator mirror with a worker per GPU, torch's current device -- keeps its own.
struct DeviceScope {
    int prev = -1;
    hipError_t e = hipSuccess;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) e = hipSetDevice(dev);
        if (prev == dev) prev = -1;  // nothing to restore
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

// Internal status of consume(): the window holds nothing below a bound injected
// by dpow_search_bound (reported as DPOW_EXHAUSTED).
constexpr int DPOW_BOUNDED = 3;

#define DPOW_HIP(call)                                    \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

// Persistent grid: one round of resident workgroups (6 four-wave workgroups per
// CU; the kernel's <= 80 SGPRs would admit 8), work handed out by in-order
// chunk claims from 8 per-XCD counters.  A chunk is sized for >= 16 claims per
// wave (small tail) and within [kMinChunk, kMaxChunk] wave-blocks: a contended
// counter serves < 90 claims/us (MI355X_MICROARCH.md "dequeue") and a wave
// hashes one wave-block in ~6 us, so 8k waves at chunk c ask ~1300/c claims/us
// of the 8 counters.  Small launches get fewer workgroups instead of smaller
// chunks.  Why 6, not 8: the SIMD issues oldest-first, and the five oldest
// waves of a SIMD already take ~all its VALU cycles (tools/wave_trace.py); the
// youngest ones hash ~1/60 of the mean and sit on the early chunks they
// claimed, which a first hit has to wait for.  6 vs 8 (profiles/r01_ab_tail_prio.log):
// throughput equal in every layout, time-to-secret N = 7 1.49 -> 1.37 ms.
// (The grid of a short launch is smaller: plan.h launch_blocks_per_cu.)
constexpr uint64_t kBlocksPerCu = kMaxBlocksPerCu;
// Claim-counter slots (kClaimSlot counters each) used round-robin by the launches
// of a search: zeroed at search start, re-zeroed by each launch's last workgroup.
constexpr size_t kClaimRing = 64;
// Launches kept in flight: launch j is queued only after the completion record
// of launch j - kDepth shows no hit and no cancel, so a hit or a cancel leaves
// at most kDepth launches to retire (each exits at its first check).
constexpr size_t kDepth = 3;
static_assert(kDepth < kClaimRing, "a claim slot is reused only after its launch completed");
constexpr size_t kRing = 8;  // completion records and event pairs, indexed by launch seq (>= kDepth + 1)
// Words of the pinned cancel page: the stale launch sequence (Launch::stale) and the
// 64-bit bound injected by dpow_search_bound (Launch::ext_bound, relayed by the watcher).
constexpr size_t kStaleWord = 8;
constexpr size_t kBoundWord = 16;  // uint32 index of an 8-byte-aligned 64-bit word
constexpr size_t kEarlyWord = 20;  // uint32 index of kCtrlRing 64-bit early-hit words (Launch::early)
constexpr size_t kCancelPage = 128;
static_assert(kEarlyWord * 4 + kCtrlRing * 8 <= kCancelPage, "the early-hit words fit the pinned page");
// Completion-record wait: spin for the first kSpinNs of a search (time-to-secret) -- or
// longer, up to kSpinMaxNs, for twice the time its first hit is expected in (round 3 spun for
// 200 us only, so an 8-GPU rank's N = 7 search, whose hit comes ~200 us in, saw its records
// and posted its hit one 5-7 us sleep late) -- then poll at kPollNs (20 us in round 2: a
// record waited up to that long to be seen once a search ran past the spin; the thread
// sleeps between polls either way).
constexpr int64_t kSpinNs = 200000;
constexpr int64_t kSpinMaxNs = 4000000;
constexpr long kPollNs = 5000;
constexpr int64_t kNoDeadline = INT64_MAX;
// Deferred queueing.  A launch is queued only once the launches ahead of it are
// expected to finish within kQueueLeadNs, so a hit leaves (almost) nothing queued
// behind it: every queued launch of a persistent grid costs 10-20 us of dispatch
// and retirement even when it claims nothing (profiles/r02_tts_timeline.json),
// which the next search on the stream, and a device synchronize, wait out.  The
// estimate is early on purpose (kEstRate is above every layout's measured rate,
// the fixed cost below the measured one), so a window without a hit runs its
// launches back to back.
constexpr int64_t kQueueLeadNs = 60000;
// (kEstRate: plan.h)
constexpr int64_t kEstFixedNs = 8000;

// Searches in flight per device in this process.  Several logical workers may
// share one GPU (the coordinator mirror places W workers round-robin on the
// node's devices; BASELINE config 4 runs 8 on one in the 1-GPU bench): each
// search then sizes its persistent grids to its share of the device and keeps its
// launches short (plan.h grid_share, cap_shared_launch), so the device stays full and
// every search's grid follows the others that start or end beside it.
constexpr int kMaxDevices = 64;
std::atomic<int> g_active[kMaxDevices];
// Contexts open per device in this process, each with the time it was last used (opened, or a
// search started): several used recently means other searches may start beside this one at any
// moment (the coordinator mirror's logical workers); contexts idle in a pool do not count.
std::mutex g_ctx_mu;
std::vector<dpow_ctx *> g_ctxs;

struct ActiveSearch {
    int dev;
    explicit ActiveSearch(int d) : dev(d) { g_active[dev].fetch_add(1, std::memory_order_relaxed); }
    ~ActiveSearch() { g_active[dev].fetch_sub(1, std::memory_order_relaxed); }
};

// One queued launch: its completion record slot (seq % kRing) and what its record adds
// to dpow_stats once consumed (launches, candidates, and the kernel time the launch
// stamps into the record itself).
struct LaunchSlot {
    uint64_t seq = 0;       // launch sequence number of the slot's last user
    bool in_flight = false; // its record was not consumed: it may still be running
    uint64_t candidates = 0;
    uint64_t g_end = 0;    // global indices of this launch are below g_end = k_end * 256
    hipStream_t stream = nullptr;  // the stream it was queued on (the k = 0 kernel: the second one)
};

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Per-search wait state: the search's start (the spin window), the caller thread's
// timer slack (lowered for the sleeping polls, restored when the search returns --
// the thread is the caller's own, e.g. a cgo goroutine's), and the node slot
// (dpow_node_attach) as last seen.
struct SearchWait {
    int64_t t0 = now_ns();
    int64_t spin_ns = kSpinNs;  // spin_for(): this search's spin window
    long old_slack = -1;
    uint64_t node_seen = DPOW_NO_HIT;  // lowest node best injected into this search
    bool node_stop = false;            // the node slot's stop was seen
    // Early Found fan-out (attached node): the pinned word the running launch's watcher relays
    // Ctrl::best to, the lowest value seen there, and what a hit is verified against.
    const uint64_t *early = nullptr;
    uint64_t early_seen = DPOW_NO_HIT;
    uint64_t own_posted = DPOW_NO_HIT;  // the lowest hit of ours posted early: the slot's best, not a bound
    // Every candidate of this window below `covered` has been searched without a hit: the
    // g_end of the last consumed launch (round 5).  Once an injected bound (another rank's
    // hit, dpow_search_bound) is at or below it, the search is over -- the launches still in
    // flight hold nothing below the bound -- and it returns without waiting for their drain.
    uint64_t covered = 0;
    const uint8_t *nonce = nullptr;
    size_t nonce_len = 0;
    uint32_t ntz = 0;
    uint32_t rbits = 8, base_tb = 0;    // the partition: g is ours iff (g & 255) >> rbits == base_tb >> rbits
    void lower_slack() {
        if (old_slack >= 0) return;
        // Linux pads a normal thread's nanosleep by its 50 us default timer slack,
        // which a hit's record would wait out; 1 us keeps the poll at ~kPollNs.
        const int r = prctl(PR_GET_TIMERSLACK, 0UL, 0UL, 0UL, 0UL);
        if (r <= 0) return;
        old_slack = r;
        (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
    }
    ~SearchWait() {
        if (old_slack >= 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)old_slack, 0UL, 0UL, 0UL);
    }
};

}  // namespace

struct dpow_ctx {
    int device = 0;
    bool counted = false;  // in g_ctxs
    hipStream_t stream = nullptr;
    Ctrl *d_ctrl = nullptr;  // kCtrlRing control blocks (kCtrlStride apart, aligned to the ring's size);
                             //  ctrl_idx's is clean
    Ctrl *d_ctrl_alloc = nullptr;
    uint32_t ctrl_idx = 0;
    unsigned long long *d_claims = nullptr;  // kClaimRing slots of kClaimSlot claim counters
    Snap *h_snap = nullptr;        // kRing completion records: pinned, host-coherent, mapped
    Snap *d_snap = nullptr;        // device alias
    uint32_t *h_cancel = nullptr;  // pinned, host-coherent, mapped: [0] the cancel flag, [kStaleWord] stale seq,
                                   //  [kBoundWord] the injected bound (64-bit)
    uint32_t *d_cancel = nullptr;  // device alias
    uint32_t cus = 0;
    uint64_t seq = 0;  // launches ever queued on this context (record/slot index = seq % kRing)
    LaunchSlot slots[kRing];
    dpow_stats stats{};
    // External bound (dpow_search_bound): lowered from another thread while a
    // search runs, written to the pinned bound word, which the running launch's
    // watcher relays to Ctrl::best (as it relays the node slot's best).
    std::mutex bound_mu;
    bool searching = false;                      // under bound_mu
    std::atomic<uint64_t> ext_bound{DPOW_NO_HIT};  // the lowest bound injected into the running search
    // Node slot (dpow_node_attach): shared by the ranks of one node, polled while a
    // search waits for its records.
    dpow_node_slot *node = nullptr;
    dpow_node_slot *d_node = nullptr;  // its device alias (the watcher polls it)
    // A/B overrides of the launch policy (dpow_diag.h): DPOW_DIAG_POLL_WB (wave-blocks per poll
    // group), DPOW_DIAG_BPC (worker workgroups per CU), DPOW_DIAG_MIN_CHUNK (minimum wave-blocks
    // per claim, a power of two), DPOW_DIAG_CPW (big claims per wave), DPOW_DIAG_SHARE_LAUNCH_US
    // (launch length on a shared device), DPOW_DIAG_SHARE_MAX (grid share cap); 0 = the policy.
    LaunchKnobs knobs;
    int64_t diag_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // the last search's host timeline (dpow_diag_search_times)
    // The last search's launches, in launch order (dpow_diag_search_launches): host times of
    // each queueing and record consumption (absolute now_ns), the search's start.
    struct DiagLaunch {
        uint64_t seq = 0, candidates = 0, g_end = 0;
        int32_t kind = 0;  // 0: the k = 0 kernel, 1: an md5 launch
        int64_t queued = -1, seen = -1;
    };
    static constexpr size_t kDiagLaunches = 32;
    DiagLaunch diag_l[kDiagLaunches];
    size_t diag_nl = 0;
    int64_t diag_t0 = 0;
    uint64_t dev_key = 0;  // the GPU's identity across processes: a hash of its PCI bus id (dpow::device_key)
    std::atomic<int64_t> last_use{0};  // now_ns() of dpow_open / the last search start (recent_contexts)
    bool solo = false;  // dpow_board_search's node-wide role: no young-search sharing (plan.h kYoungNs)
};

namespace {

// Before a record slot is reused: a launch whose record was never consumed (queued behind
// a hit, a cancel or an error, possibly on the other stream) may still be running; wait
// for its record, so it cannot land on the slot's next user.
int retire_slot(dpow_ctx *c, LaunchSlot &s);

uint64_t *bound_word(dpow_ctx *c) { return reinterpret_cast<uint64_t *>(c->h_cancel + kBoundWord); }

// Lower Ctrl::best of the running search to g (dpow_search_bound): the pinned bound
// word, which the running launch's watcher relays to Ctrl::best within its poll (about
// 1 us).  Round 2 launched a one-thread atomicMin kernel on a second stream instead,
// which took 50-160 us to start beside the running grid.  The caller holds bound_mu.
int inject_bound_locked(dpow_ctx *c, uint64_t g) {
    if (g >= c->ext_bound.load(std::memory_order_relaxed)) return 0;
    c->ext_bound.store(g, std::memory_order_release);
    __atomic_store_n(bound_word(c), g, __ATOMIC_RELEASE);
    return 0;
}

// The node slot, polled between record polls: a lower best of another rank is
// injected as a bound; a stop marks every launch queued so far stale, so their
// watchers stop them (the search then returns DPOW_CANCELLED).
int poll_node(dpow_ctx *c, SearchWait &sw) {
    dpow_node_slot *n = c->node;
    if (!n) return 0;
    const uint64_t nb = __atomic_load_n(&n->best, __ATOMIC_ACQUIRE);
    if (nb < sw.node_seen) {
        // The running launch's watcher lowers Ctrl::best to it on the device; the host
        // keeps the injected bound (ext_bound) that tells another rank's index from ours.
        // Our own hit, posted early (poll_early), is not a bound.
        sw.node_seen = nb;
        if (nb != sw.own_posted) {
            std::lock_guard<std::mutex> g(c->bound_mu);
            uint64_t cur = c->ext_bound.load(std::memory_order_relaxed);
            if (nb < cur) c->ext_bound.store(nb, std::memory_order_release);
        }
    }
    if (!sw.node_stop && __atomic_load_n(&n->stop, __ATOMIC_ACQUIRE) != 0u) {
        sw.node_stop = true;
        __atomic_store_n(&c->h_cancel[kStaleWord], (uint32_t)c->seq, __ATOMIC_RELEASE);
    }
    return 0;
}

// The early-hit word (attached node): a value below what was seen there is this launch's
// Ctrl::best -- a hit of ours, or a bound that is itself a hit of another rank.  It is
// verified with the host MD5 and posted to the node slot at once, so the other ranks stop at
// it while this launch drains; the search's final answer is still taken from the records.
void poll_early(dpow_ctx *c, SearchWait &sw) {
    const uint64_t g = __atomic_load_n(sw.early, __ATOMIC_ACQUIRE);
    if (g >= sw.early_seen) return;
    sw.early_seen = g;
    // only a hit of this search's partition (Ctrl::best also holds the bounds the watcher relays)
    if ((((uint32_t)g & 0xFFu) >> sw.rbits) != (sw.base_tb >> sw.rbits)) return;
    uint8_t sec[DPOW_MAX_SECRET];
    size_t len = 0;
    if (dpow_secret_from_index(g, sec, &len) != 0) return;
    if (!dpow_verify(sw.nonce, sw.nonce_len, sec, len, sw.ntz)) return;  // not a hit (a bound): left to the record
    if (g < sw.own_posted) sw.own_posted = g;  // before the post: poll_node must not take it for a bound
    dpow_node_post(c->node, g);
    if (c->diag_t[7] < 0) c->diag_t[7] = now_ns() - sw.t0;
}

// Wait for the completion record of launch `seq`, until `deadline` (now_ns()
// clock; kNoDeadline: none).  Returns 1 when the record is there, 0 at the
// deadline, 2 when an injected bound reached what the consumed launches cover
// (SearchWait::covered: nothing of ours is left below it), < 0 on error.  Spins in the first kSpinNs of the search (the record
// of a launch holding a hit is the time-to-secret path), then sleeps between
// polls; the stream is queried now and then so a failed launch, or a stream
// that went idle without writing the record, ends the wait with an error.
int wait_record(dpow_ctx *c, uint64_t seq, int64_t deadline, SearchWait &sw) {
    const uint32_t *p = &c->h_snap[seq % kRing].seq;
    const uint32_t want = (uint32_t)(seq + 1);
    for (uint64_t it = 1;; ++it) {
        if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == want) return 1;
        const int64_t t = now_ns();
        if (t >= deadline) return 0;
        const bool spinning = t - sw.t0 < sw.spin_ns;
        if (spinning ? (it % 4096 == 0) : (it % 16 == 0)) {
            const hipError_t q = hipStreamQuery(c->slots[seq % kRing].stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == want) return 1;
                return set_error(DPOW_EHIP, "dpow_search: stream idle without the launch's completion record");
            }
            if (q != hipErrorNotReady) return hip_fail(q, "hipStreamQuery");
        }
        if (sw.early && (!spinning || it % 8 == 0)) poll_early(c, sw);
        if (!spinning || it % 64 == 0) {
            if (c->node) {
                const int rc = poll_node(c, sw);
                if (rc < 0) return rc;
            }
            if (c->ext_bound.load(std::memory_order_acquire) <= sw.covered) return 2;
        }
        if (spinning) {
            __builtin_ia32_pause();
        } else {
            sw.lower_slack();
            int64_t ns = kPollNs;
            if (deadline != kNoDeadline && deadline - t < ns) ns = deadline - t;
            const struct timespec ts = {0, (long)ns};
            nanosleep(&ts, nullptr);
        }
    }
}

int retire_slot(dpow_ctx *c, LaunchSlot &s) {
    if (!s.in_flight) return 0;
    const uint32_t *p = &c->h_snap[s.seq % kRing].seq;
    const uint32_t want = (uint32_t)(s.seq + 1);
    for (uint64_t it = 1; __atomic_load_n(p, __ATOMIC_ACQUIRE) != want; ++it) {
        if (it % 1024 == 0) {
            const hipError_t q = hipStreamQuery(s.stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == want) break;
                return set_error(DPOW_EHIP, "dpow_search: stream idle without a queued launch's completion record");
            }
            if (q != hipErrorNotReady) return hip_fail(q, "hipStreamQuery");
        }
        __builtin_ia32_pause();
    }
    s.in_flight = false;
    return 0;
}

// Contexts of `device` used within kRecentNs (the young-search rule above).
int recent_contexts(int device) {
    const int64_t t = now_ns();
    int n = 0;
    std::lock_guard<std::mutex> g(g_ctx_mu);
    for (dpow_ctx *x : g_ctxs)
        if (x->device == device && t - x->last_use.load(std::memory_order_relaxed) < kRecentNs) ++n;
    return n;
}

// The body of dpow_search (arguments checked).
int search_window(dpow_ctx *c, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                  uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, uint64_t *best_global_idx,
                  uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len) {
    WindowPlanner planner;
    int rc = planner.init(nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end);
    if (rc < 0) return set_error(rc, "dpow_search: planning failed");
    const DeviceScope on_device(c->device);
    if (on_device.e != hipSuccess) return hip_fail(on_device.e, "hipSetDevice");
    if (c->device >= kMaxDevices) return set_error(DPOW_EINVAL, "dpow_search: device ordinal too large");
    const ActiveSearch active(c->device);
    SearchWait sw;
    {   // Spin while the first hit is expected (memoryless: from any start), 2x, within [kSpinNs,
        // kSpinMaxNs].  The expected time is at this search's share of the device (the searches
        // in flight on it).  A search whose hit is not expected within a few spin windows (the
        // sweep, N >= 9, N = 8 on one GPU) spins kSpinNs only: busy-spinning a host core for
        // 4 ms of a long search buys nothing.
        const double searches = (double)std::max(1, g_active[c->device].load(std::memory_order_relaxed));
        const double expect_ns =
            (double)expected_first_hit(ntz, remainder_bits(worker_bits)) / kEstRate * 1e9 * searches;
        sw.spin_ns = expect_ns > 2.0 * (double)kSpinMaxNs
                         ? kSpinNs
                         : (int64_t)std::min<double>(std::max<double>(2.0 * expect_ns, (double)kSpinNs),
                                                     (double)kSpinMaxNs);
    }

    {   // keep the stale mark within 2^30 launches of the present (int32 distance in the watcher)
        uint32_t *st = &c->h_cancel[kStaleWord];
        const uint32_t next = (uint32_t)(c->seq + 1);
        if ((int32_t)(next - __atomic_load_n(st, __ATOMIC_RELAXED)) > (1 << 30))
            __atomic_store_n(st, next - (1u << 30), __ATOMIC_RELAXED);
    }
    const uint64_t bound = *best_global_idx;
    // Another rank's hit already on the node slot bounds this search from the start
    // (as an injected bound: a record at or above it is not a hit of ours).
    const uint64_t node_best = c->node ? __atomic_load_n(&c->node->best, __ATOMIC_ACQUIRE) : DPOW_NO_HIT;
    sw.node_seen = node_best;
    const uint64_t seq0 = c->seq;
    sw.covered = k_begin << 8;  // nothing of this window is searched yet
    for (int64_t &t : c->diag_t) t = -1;
    c->diag_nl = 0;
    c->diag_t0 = sw.t0;
    auto diag_queued = [c](size_t li, uint64_t seq, int32_t kind, uint64_t cands, uint64_t g_end) {
        if (li >= dpow_ctx::kDiagLaunches) return;
        c->diag_l[li] = {seq, cands, g_end, kind, now_ns(), -1};
        c->diag_nl = li + 1;
    };
    if (c->node) {  // the early Found fan-out: this search's control block's early-hit word
        uint64_t *ew = reinterpret_cast<uint64_t *>(c->h_cancel + kEarlyWord) + c->ctrl_idx;
        __atomic_store_n(ew, (uint64_t)DPOW_NO_HIT, __ATOMIC_RELEASE);
        sw.early = ew;
        sw.nonce = nonce;
        sw.nonce_len = nonce_len;
        sw.ntz = ntz;
        sw.rbits = remainder_bits(worker_bits);
        sw.base_tb = base_thread_byte(worker_byte, worker_bits);
    }
    size_t launched = 0, consumed = 0;
    int64_t busy_until = 0;  // expected end of the launches queued so far (now_ns clock)
    PlannedLaunch pl;
    bool have = planner.next(pl);
    c->diag_t[4] = now_ns() - sw.t0;
    // A window holding k = 0 starts with the k = 0 kernel (search_ctrl.hip), ahead of the
    // first md5 launch on the search stream: launch 0 of the search, with a completion record
    // of its own that holds its own first hit only.  (On a second stream beside the first md5
    // launch it started 2-4 us sooner, but one more busy device queue per process pushed 8
    // processes sharing a GPU into queue oversubscription: profiles/r03_rehearsal_queues.json.)
    hipError_t e = hipSuccess;
    if (have && pl.k0) {
        LaunchSlot &k0slot = c->slots[seq0 % kRing];
        if ((rc = retire_slot(c, k0slot)) < 0) return rc;
        c->diag_t[5] = now_ns() - sw.t0;
        StartK0 k0{};
        k0.r = (uint32_t)(pl.L.i_end - pl.L.i_begin);
        k0.base_tb = pl.L.base_tb;
        k0.nblk = pl.info.nblk;
        k0.p = 4 * pl.info.w0 + pl.info.sh;
        k0.ntz = ntz;
        k0.seq = (uint32_t)(seq0 + 1);
        k0.snap = c->d_snap + seq0 % kRing;
        memcpy(k0.iv, pl.L.iv, sizeof k0.iv);
        memcpy(k0.T, pl.L.T, sizeof k0.T);
        e = search_k0(k0, c->stream);
        if (e != hipSuccess) return hip_fail(e, "search_k0");
        c->diag_t[0] = now_ns() - sw.t0;
        diag_queued(0, seq0, 0, k0.r, 1ull << 8);
        k0slot.in_flight = true;
        k0slot.seq = seq0;
        k0slot.candidates = k0.r;
        k0slot.g_end = 1ull << 8;
        k0slot.stream = c->stream;
        c->seq = seq0 + 1;
        launched = 1;
        have = planner.next(pl);
    }
    // This search's control block (clean: reset by the previous search's launches, or at
    // dpow_open); its md5 launches reset the next one.
    Ctrl *const ctrl = c->d_ctrl + (size_t)c->ctrl_idx * kCtrlStride;
    Ctrl *const ctrl_next = c->d_ctrl + (size_t)((c->ctrl_idx + 1) % kCtrlRing) * kCtrlStride;
    bool md5_queued = false;
    struct CtrlAdvance {  // once an md5 launch is queued, the next search uses the next block
        dpow_ctx *c;
        const bool &queued;
        ~CtrlAdvance() {
            if (queued) c->ctrl_idx = (c->ctrl_idx + 1) % kCtrlRing;
        }
    } ctrl_advance{c, md5_queued};
    const uint64_t bound0 = node_best < bound ? node_best : bound;
    // Open the window for dpow_search_bound (the bound word starts at "none" for this
    // search; stale launches of the previous one may still read it, harmlessly).
    struct BoundWindow {
        dpow_ctx *c;
        BoundWindow(dpow_ctx *cc, uint64_t start) : c(cc) {
            std::lock_guard<std::mutex> g(c->bound_mu);
            c->ext_bound.store(start, std::memory_order_relaxed);
            __atomic_store_n(bound_word(c), (uint64_t)DPOW_NO_HIT, __ATOMIC_RELEASE);
            c->searching = true;
        }
        ~BoundWindow() {
            std::lock_guard<std::mutex> g(c->bound_mu);
            c->searching = false;
        }
    } bound_window(c, node_best);

    uint32_t done_target = 0;
    // Launches still queued when the search returns -- behind a hit, a bound, a
    // cancel or an error -- are marked stale, so their watchers stop them at once
    // even if the caller clears the cancel flag for its next task before they
    // start.
    struct StaleOnReturn {
        dpow_ctx *c;
        const size_t &launched, &consumed;
        ~StaleOnReturn() {
            if (consumed < launched) __atomic_store_n(&c->h_cancel[kStaleWord], (uint32_t)c->seq, __ATOMIC_RELEASE);
        }
    } stale_on_return{c, launched, consumed};
    uint64_t best = bound;
    int status = DPOW_EXHAUSTED;
    // Consume the completion record of launch lj (in launch order): FOUND or
    // CANCELLED ends the search, EXHAUSTED goes on, < 0 is an error.  Ctrl::best
    // persists across the launches of a search and later launches hold higher
    // indices, so the first record below the bound carries the answer.
    auto consume = [&](size_t lj) -> int {
        const uint64_t seq = seq0 + lj;
        const int rc = wait_record(c, seq, kNoDeadline, sw);
        if (rc < 0) return rc;
        if (rc == 2) return DPOW_BOUNDED;  // the launch stays in flight; marked stale on return
        LaunchSlot &slot = c->slots[seq % kRing];
        const Snap &sn = c->h_snap[seq % kRing];
        slot.in_flight = false;
        c->stats.launches++;
        c->stats.candidates += slot.candidates;
        if (sn.t_start != 0ull && sn.t_end >= sn.t_start)
            c->stats.kernel_ms += (double)(sn.t_end - sn.t_start) * kRealtimeNs * 1e-6;
        if (consumed == 0) c->diag_t[2] = now_ns() - sw.t0;
        if (lj < dpow_ctx::kDiagLaunches) c->diag_l[lj].seen = now_ns();
        consumed = lj + 1;
        // The watcher may have put the node slot's best into Ctrl::best before this thread
        // saw it: read the slot now (its best only decreases) so ext_bound covers it.
        if (c->node) {
            const int prc = poll_node(c, sw);
            if (prc < 0) return prc;
        }
        if (sn.best < bound) {
            // Ctrl::best = min(this search's hits, bounds injected by dpow_search_bound
            // or from the node slot).  At or above the lowest injected bound it is not a
            // hit of ours.  The search is over only when that bound lies within the
            // launches consumed so far (every candidate below it has been searched);
            // otherwise the later launches still hold candidates below it: go on
            // (they skip chunks at or above Ctrl::best, and a hit of ours there shows
            // in their records as a value below the bound).
            const uint64_t eb = c->ext_bound.load(std::memory_order_acquire);
            if (sn.best >= eb) return eb <= slot.g_end ? DPOW_BOUNDED : DPOW_EXHAUSTED;
            best = sn.best;
            return DPOW_FOUND;
        }
        if (sn.stop != 0u || sw.node_stop || __atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u)
            return DPOW_CANCELLED;
        sw.covered = slot.g_end;
        if (c->ext_bound.load(std::memory_order_acquire) <= sw.covered) return DPOW_BOUNDED;
        return DPOW_EXHAUSTED;
    };
    while (status == DPOW_EXHAUSTED && have) {
        if (sw.node_stop) {
            status = DPOW_CANCELLED;
            break;
        }
        const size_t li = launched;
        if (li - consumed >= kDepth) {  // the record of the oldest launch decides whether to go on
            const int r = consume(consumed);
            if (r < 0) return r;
            if (r != DPOW_EXHAUSTED) status = r;
            continue;
        }
        if (li > consumed && busy_until - now_ns() > kQueueLeadNs) {
            // Deferred queueing: wait for the oldest record until the launches ahead
            // are expected to be within kQueueLeadNs of their end.
            const size_t lj = consumed;
            const int w = wait_record(c, seq0 + lj, busy_until - kQueueLeadNs, sw);
            if (w < 0) return w;
            if (w == 2) {
                status = DPOW_BOUNDED;
                continue;
            }
            if (w == 1) {
                const int r = consume(lj);
                if (r < 0) return r;
                if (r != DPOW_EXHAUSTED) status = r;
                continue;
            }
        }
        {   // a launch wholly at or above the bound (the caller's, an injected one) holds nothing
            const uint64_t eb = c->ext_bound.load(std::memory_order_acquire);
            if ((pl.info.k_begin << 8) >= (eb < bound ? eb : bound)) break;
        }
        const uint64_t seq = seq0 + li;
        LaunchSlot &slot = c->slots[seq % kRing];
        if ((rc = retire_slot(c, slot)) < 0) return rc;  // the slot's previous user
        if (!md5_queued) c->diag_t[6] = now_ns() - sw.t0;
        Launch &L = pl.L;
        // This search's share of the device's resident workgroups (searches sharing the device:
        // plan.h grid_share, cap_shared_launch).
        uint64_t active = (uint64_t)std::max(1, g_active[c->device].load(std::memory_order_relaxed));
        if (active == 1 && !c->solo && now_ns() - sw.t0 < kYoungNs) {
            // A young search that looks alone while other contexts of this process were used on
            // the device recently plans as if they all searched: its first long launch no longer
            // takes the whole device for its full length just because it registered first
            // (round 4: one 16-28 ms full-device launch, config 4's one nonce 8.5-23 ms over runs).
            const int recent = recent_contexts(c->device);
            if (recent > 1) active = (uint64_t)recent;
        }
        const uint64_t share = grid_share(active, c->knobs);
        cap_shared_launch(planner, pl, active, c->knobs);
        uint64_t worker_blocks = 0;
        rc = size_search_launch(pl, ntz, c->cus, share, c->knobs, &worker_blocks, active);
        if (rc < 0) return set_error(rc, "dpow_search: launch grid leaves a claim counter without waves");
        done_target += (uint32_t)worker_blocks;  // retirement is counted per workgroup
        L.claim = c->d_claims + (li % kClaimRing) * kClaimSlot;
        L.done_target = done_target;
        L.ctrl = ctrl;
        L.ctrl_next = ctrl_next;
        L.bound0 = bound0;
        L.cancel = c->d_cancel;
        L.stale = c->d_cancel + kStaleWord;
        L.ext_bound = reinterpret_cast<const unsigned long long *>(c->d_cancel + kBoundWord);
        L.snap = c->d_snap + seq % kRing;
        L.seq = (uint32_t)(seq + 1);
        L.node_best = c->d_node ? reinterpret_cast<const unsigned long long *>(&c->d_node->best) : nullptr;
        L.node_stop = c->d_node ? &c->d_node->stop : nullptr;
        L.early = c->d_node ? reinterpret_cast<unsigned long long *>(c->d_cancel + kEarlyWord) + c->ctrl_idx : nullptr;
        e = search_launch((int)pl.info.nblk, (int)pl.info.w0, (int)pl.info.sh, L, (uint32_t)(worker_blocks + 1),
                          c->stream);
        if (e != hipSuccess) return hip_fail(e, "search_launch");
        if (!md5_queued) c->diag_t[1] = now_ns() - sw.t0;
        diag_queued(li, seq, 1, L.i_end - L.i_begin, pl.info.k_end << 8);
        md5_queued = true;
        slot.seq = seq;
        slot.in_flight = true;
        slot.candidates = L.i_end - L.i_begin;
        slot.g_end = pl.info.k_end << 8;
        slot.stream = c->stream;
        c->seq = seq + 1;
        ++launched;
        const int64_t t = now_ns();
        busy_until = std::max(busy_until, t) + kEstFixedNs +
                     (int64_t)((double)slot.candidates * (double)active / kEstRate * 1e9);
        have = planner.next(pl);
    }
    while (status == DPOW_EXHAUSTED && consumed < launched) {  // the window is queued: drain in order
        const int r = consume(consumed);
        if (r < 0) return r;
        status = r;
    }
    if (status == DPOW_BOUNDED) status = DPOW_EXHAUSTED;  // no hit below the (injected) bound
    c->diag_t[3] = now_ns() - sw.t0;

    if (status == DPOW_FOUND) {
        dpow_secret_from_index(best, secret_out, secret_len);
        if (!dpow_verify(nonce, nonce_len, secret_out, *secret_len, ntz)) {
            *secret_len = 0;
            return set_error(DPOW_EVERIFY, "dpow_search: kernel hit failed host MD5 verification");
        }
        *best_global_idx = best;
    }
    return status;
}

// Host pages registered for node slots (hipHostRegister: process-wide, not per context).  A
// context that attaches a slot holds its pages until dpow_close (detaching keeps them, so
// node_mine's attach / detach per node search costs no registration); a page is registered by
// its first holder and unregistered when its last holder closes, so two contexts of one
// process attached to one slot (one per GPU, or the 2-rank rehearsal) never see the page
// unregistered under a running watcher.  Memory about to be unmapped is released explicitly
// (dpow_node_release: NodeBoard.close), so a new mapping at the same address is registered
// afresh instead of reusing the old registration's device alias.
// The registration is portable (every device of the process may map the page) and the device
// alias is looked up per device, under that device, the first time a context of that device
// holds the page: a process whose contexts on several GPUs share one slot (a node scheduler with
// a context per GPU, the board's workers) never hands one GPU's alias to another's watcher
// (VERDICT r05 item 2(i)).
struct PageEntry {
    void *page;
    bool foreign;                    // registered outside this library: never unregistered here
    std::vector<dpow_ctx *> holders;
    char *dev[kMaxDevices] = {};     // the page's alias on each device (hipHostGetDevicePointer, once per device)
};
std::mutex g_page_mu;
std::vector<PageEntry> g_pages;

// Drop entry i (every holder's streams drained by the caller).  g_page_mu held.
void page_drop_locked(size_t i) {
    if (!g_pages[i].foreign) (void)hipHostUnregister(g_pages[i].page);
    g_pages.erase(g_pages.begin() + (long)i);
}

// A reference of ctx on `page` (registering it if no context holds it).  g_page_mu held, the
// calling thread on ctx's device.  *dev: the page's alias on ctx's device.
hipError_t page_hold_locked(dpow_ctx *c, void *page, char **dev) {
    PageEntry *pe = nullptr;
    for (PageEntry &x : g_pages)
        if (x.page == page) {
            pe = &x;
            break;
        }
    if (!pe) {
        hipError_t e = hipHostRegister(page, 4096, hipHostRegisterMapped | hipHostRegisterPortable);
        bool foreign = false;
        if (e == hipErrorHostMemoryAlreadyRegistered) {
            (void)hipGetLastError();
            e = hipSuccess;
            foreign = true;
        }
        if (e != hipSuccess) return e;
        g_pages.push_back(PageEntry{page, foreign, {}, {}});
        pe = &g_pages.back();
    }
    if (!pe->dev[c->device]) {
        void *d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, page, 0);
        if (e != hipSuccess) {
            if (pe->holders.empty()) page_drop_locked((size_t)(pe - g_pages.data()));
            return e;
        }
        pe->dev[c->device] = static_cast<char *>(d);
    }
    if (std::find(pe->holders.begin(), pe->holders.end(), c) == pe->holders.end()) pe->holders.push_back(c);
    *dev = pe->dev[c->device];
    return hipSuccess;
}

// dpow_close: ctx's references go (its stream has drained); pages without holders are unregistered.
void pages_release_ctx(dpow_ctx *c) {
    std::lock_guard<std::mutex> g(g_page_mu);
    for (size_t i = g_pages.size(); i-- > 0;) {
        auto &h = g_pages[i].holders;
        h.erase(std::remove(h.begin(), h.end(), c), h.end());
        if (h.empty()) page_drop_locked(i);
    }
}

// Kernels loaded per device in this process (search_prepare): once, under a lock.
hipError_t prepare_device(int device) {
    static std::mutex mu;
    static bool prepared[kMaxDevices] = {};
    std::lock_guard<std::mutex> g(mu);
    if (device < kMaxDevices && prepared[device]) return hipSuccess;
    const hipError_t e = search_prepare();
    if (e == hipSuccess && device < kMaxDevices) prepared[device] = true;
    return e;
}

}  // namespace

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
    const DeviceScope on_device(device);
    if (on_device.e != hipSuccess) return hip_fail(on_device.e, "hipSetDevice");
    dpow_ctx *c = new (std::nothrow) dpow_ctx();
    if (!c) return set_error(DPOW_ENOMEM, "dpow_open: out of memory");
    c->device = device;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) {
        delete c;
        return hip_fail(e, "hipGetDeviceProperties");
    }
    c->cus = (uint32_t)prop.multiProcessorCount;
    {   // FNV-1a of the PCI bus id: the same GPU gives the same key in every process of the host
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, device) != hipSuccess) {
            (void)hipGetLastError();
            snprintf(bus, sizeof bus, "ordinal-%d-pid-%d", device, (int)getpid());  // never matches another process
        }
        uint64_t h = 1469598103934665603ull;
        for (const char *q = bus; *q; ++q) h = (h ^ (uint8_t)*q) * 1099511628211ull;
        c->dev_key = h | 1ull;
    }
    if (const char *pw = getenv("DPOW_DIAG_POLL_WB")) c->knobs.poll_wb = (uint32_t)std::max(0, atoi(pw));
    if (const char *pw = getenv("DPOW_DIAG_BPC")) c->knobs.bpc = (uint32_t)std::max(0, atoi(pw));
    if (const char *pw = getenv("DPOW_DIAG_CPW")) c->knobs.cpw = (uint32_t)std::max(0, atoi(pw));
    if (const char *pw = getenv("DPOW_DIAG_SHARE_LAUNCH_US")) c->knobs.share_launch_us = (uint32_t)std::max(0, atoi(pw));
    if (const char *pw = getenv("DPOW_DIAG_SHARE_MAX")) c->knobs.share_max = (uint32_t)std::max(0, atoi(pw));
    if (const char *pw = getenv("DPOW_DIAG_MIN_CHUNK")) {
        const uint32_t v = (uint32_t)std::max(0, atoi(pw));
        if (v && !(v & (v - 1))) c->knobs.min_chunk = v;
    }
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&c->d_ctrl_alloc, 2 * kCtrlRing * kCtrlStride * sizeof(Ctrl))) != hipSuccess ||
        (e = hipMalloc(&c->d_claims, kClaimRing * kClaimSlot * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipHostMalloc(&c->h_snap, kRing * sizeof(Snap), hipHostMallocCoherent | hipHostMallocMapped)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_snap), c->h_snap, 0)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_cancel, kCancelPage, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_cancel), c->h_cancel, 0)) != hipSuccess) {
        dpow_close(c);
        return hip_fail(e, "dpow_open: allocation");
    }
    {   // the control-block ring, aligned to its size (publish() derives the next block's address)
        const uintptr_t rb = kCtrlRing * kCtrlStride * sizeof(Ctrl);
        c->d_ctrl = reinterpret_cast<Ctrl *>((reinterpret_cast<uintptr_t>(c->d_ctrl_alloc) + rb - 1) & ~(rb - 1));
    }
    memset(c->h_snap, 0, kRing * sizeof(Snap));
    memset(c->h_cancel, 0, kCancelPage);
    *bound_word(c) = DPOW_NO_HIT;
    // Clean control blocks and zero claim counters (the launches keep them so): a kernel on
    // the context's own stream, which stays the only device queue a context uses (no null-
    // stream copy: with 8 processes sharing one GPU, every extra queue a process keeps busy
    // pushed the device into queue oversubscription, whose time slices held each search
    // ~10 ms, profiles/r03_rehearsal_queues.json).
    if ((e = context_init(c->d_ctrl, kCtrlRing * kCtrlStride, c->d_claims, (uint32_t)(kClaimRing * kClaimSlot),
                          c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess) {
        dpow_close(c);
        return hip_fail(e, "dpow_open: control state");
    }
    // Every search kernel resolved on this device before the first search (once per device and
    // process): a translation unit's code object loads on its first use, which cost round 3's
    // first search ~1 ms (the k = 0 kernel, then a 972.8 us gap before the "_ls" md5 launch).
    if ((e = prepare_device(device)) != hipSuccess) {
        dpow_close(c);
        return hip_fail(e, "dpow_open: loading the search kernels");
    }
    c->last_use.store(now_ns(), std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(g_ctx_mu);
        g_ctxs.push_back(c);
        c->counted = true;
    }
    *out = c;
    return 0;
}

void dpow_close(dpow_ctx *c) {
    if (!c) return;
    if (c->counted) {
        std::lock_guard<std::mutex> g(g_ctx_mu);
        g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), c), g_ctxs.end());
    }
    const DeviceScope on_device(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    // Drained: no watcher of ours reads the node pages any more.  Leave the page registry
    // before the stream is destroyed (dpow_node_release synchronizes every holder's stream).
    c->node = c->d_node = nullptr;
    pages_release_ctx(c);
    if (c->d_ctrl_alloc) (void)hipFree(c->d_ctrl_alloc);
    if (c->d_claims) (void)hipFree(c->d_claims);
    if (c->h_snap) (void)hipHostFree(c->h_snap);
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
    if (!c) return;
    c->stats = dpow_stats{};
}

int dpow_search_bound(dpow_ctx *c, uint64_t global_idx) {
    if (!c) return set_error(DPOW_EINVAL, "dpow_search_bound: ctx is NULL");
    std::lock_guard<std::mutex> g(c->bound_mu);
    if (!c->searching) return 0;  // no search in flight: the caller passes its bound to the next one
    return inject_bound_locked(c, global_idx);
}

int dpow_node_attach(dpow_ctx *c, dpow_node_slot *slot) {
    if (!c) return set_error(DPOW_EINVAL, "dpow_node_attach: ctx is NULL");
    if (!slot) {  // detach: the pages stay held (registered) until dpow_close or dpow_node_release
        c->node = c->d_node = nullptr;
        return 0;
    }
    if (((uintptr_t)slot & 7u) != 0u) return set_error(DPOW_EINVAL, "dpow_node_attach: slot not 8-byte aligned");
    if (c->device >= kMaxDevices) return set_error(DPOW_EINVAL, "dpow_node_attach: device ordinal too large");
    // Map the slot's host page(s) for the watcher (fine-grained: hipHostRegister's default).
    const DeviceScope on_device(c->device);
    if (on_device.e != hipSuccess) return hip_fail(on_device.e, "hipSetDevice");
    // The device alias of a slot within one page comes from its page's, looked up once when the
    // page is registered: a node search attaches once per call, and hipHostGetDevicePointer per
    // attach cost every node search its call (a board's slots are 64-byte aligned; a slot
    // across two pages still asks the runtime).
    const uintptr_t pg = 4096;
    const bool one_page = (((uintptr_t)slot & (pg - 1)) + sizeof(dpow_node_slot)) <= pg;
    char *dev = nullptr;
    {
        std::lock_guard<std::mutex> g(g_page_mu);
        for (uintptr_t a = (uintptr_t)slot & ~(pg - 1); a < (uintptr_t)slot + sizeof(dpow_node_slot); a += pg) {
            char *d = nullptr;
            const hipError_t e = page_hold_locked(c, (void *)a, &d);
            if (e != hipSuccess) return hip_fail(e, "dpow_node_attach: hipHostRegister");
            if (!dev) dev = d;
        }
    }
    void *d = dev + ((uintptr_t)slot & (pg - 1));
    if (!one_page) DPOW_HIP(hipHostGetDevicePointer(&d, slot, 0));
    c->node = slot;
    c->d_node = (dpow_node_slot *)d;
    return 0;
}

int dpow_node_release(void *mem, size_t len) {
    if (!mem || !len) return 0;
    const uintptr_t pg = 4096;
    const uintptr_t lo = (uintptr_t)mem & ~(pg - 1), hi = (uintptr_t)mem + len;
    std::lock_guard<std::mutex> g(g_page_mu);
    for (const PageEntry &pe : g_pages) {
        const uintptr_t p = (uintptr_t)pe.page;
        if (p < lo || p >= hi) continue;
        for (dpow_ctx *h : pe.holders)
            if (h->node && (uintptr_t)h->node < p + pg && (uintptr_t)h->node + sizeof(dpow_node_slot) > p)
                return set_error(DPOW_EINVAL, "dpow_node_release: a context is still attached to a slot in the range");
    }
    for (size_t i = g_pages.size(); i-- > 0;) {
        const uintptr_t p = (uintptr_t)g_pages[i].page;
        if (p < lo || p >= hi) continue;
        // launches a holder left queued behind its last search may still read the page
        for (dpow_ctx *h : g_pages[i].holders) {
            const DeviceScope on_device(h->device);
            const hipError_t e = hipStreamSynchronize(h->stream);
            if (e != hipSuccess) return hip_fail(e, "dpow_node_release: hipStreamSynchronize");
        }
        page_drop_locked(i);
    }
    return 0;
}

void dpow_node_slot_reset(dpow_node_slot *slot) {
    if (!slot) return;
    __atomic_store_n(&slot->stop, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&slot->best, DPOW_NO_HIT, __ATOMIC_RELEASE);
}

void dpow_node_post(dpow_node_slot *slot, uint64_t global_idx) {
    if (!slot) return;
    uint64_t cur = __atomic_load_n(&slot->best, __ATOMIC_RELAXED);
    while (global_idx < cur &&
           !__atomic_compare_exchange_n(&slot->best, &cur, global_idx, true, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
    }
}

int dpow_node_vote(dpow_node_vote_entry *votes, uint32_t rank, uint32_t world, uint64_t epoch, const int64_t in[3],
                   int64_t out[3], int64_t timeout_ns) {
    return dpow::node_vote(votes, rank, world, epoch, in, out, timeout_ns, nullptr);
}

}  // extern "C"

// dpow_node_vote, and the wait of a board search (dpow_board_search): `abort_flag` non-NULL and
// raised (the rank's cancel flag: its task was killed) ends the wait with DPOW_CANCELLED, the
// vote left behind -- every rank of a board task is killed by the same Found / Cancel fan-out
// (coordinator.go:210-230), so none is left waiting for it.
int dpow::node_vote(dpow_node_vote_entry *votes, uint32_t rank, uint32_t world, uint64_t epoch, const int64_t in[3],
                    int64_t out[3], int64_t timeout_ns, const uint32_t *abort_flag) {
    if (!votes || !in || !out || world == 0 || rank >= world || epoch == 0)
        return set_error(DPOW_EINVAL, "dpow_node_vote: bad argument");
    dpow_node_vote_entry &mine = votes[2 * rank + (epoch & 1)];
    for (int i = 0; i < 3; ++i) __atomic_store_n(&mine.v[i], in[i], __ATOMIC_RELAXED);
    __atomic_store_n(&mine.epoch, epoch, __ATOMIC_RELEASE);
    int64_t acc[3] = {in[0], in[1], in[2]};
    const int64_t t0 = now_ns();
    // Spin while the other ranks are expected soon (a node's ranks end a search within tens of
    // microseconds of each other), then poll every 2 us with the thread's timer slack lowered
    // (a 2 us nanosleep under Linux's default 50 us slack wakes ~50 us late).
    constexpr int64_t kVoteSpinNs = 500000;
    long old_slack = -1;
    struct SlackRestore {
        long &old;
        ~SlackRestore() {
            if (old >= 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)old, 0UL, 0UL, 0UL);
        }
    } slack_restore{old_slack};
    for (uint32_t r = 0; r < world; ++r) {
        if (r == rank) continue;
        const dpow_node_vote_entry &e = votes[2 * r + (epoch & 1)];
        for (uint64_t it = 0; __atomic_load_n(&e.epoch, __ATOMIC_ACQUIRE) != epoch; ++it) {
            if (abort_flag && it % 64 == 0 && __atomic_load_n(abort_flag, __ATOMIC_ACQUIRE) != 0u) return DPOW_CANCELLED;
            if (it % 64 != 0 || now_ns() - t0 < std::min(kVoteSpinNs, timeout_ns)) {
                __builtin_ia32_pause();
                continue;
            }
            if (now_ns() - t0 > timeout_ns)
                return set_error(DPOW_EPROTO, "dpow_node_vote: rank " + std::to_string(r) + " did not vote at epoch " +
                                                  std::to_string(epoch));
            if (old_slack < 0) {
                const int sl = prctl(PR_GET_TIMERSLACK, 0UL, 0UL, 0UL, 0UL);
                if (sl > 0) {
                    old_slack = sl;
                    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
                }
            }
            const struct timespec d = {0, 2000};
            nanosleep(&d, nullptr);
        }
        for (int i = 0; i < 3; ++i) {
            const int64_t v = __atomic_load_n(&e.v[i], __ATOMIC_RELAXED);
            if (v < acc[i]) acc[i] = v;
        }
    }
    for (int i = 0; i < 3; ++i) out[i] = acc[i];
    return 0;
}

extern "C" int dpow_node_mine(dpow_ctx *c, dpow_node_slot *slot, dpow_node_vote_entry *votes, uint32_t rank,
                              uint32_t world, uint64_t *epoch, int64_t vote_timeout_ns, const uint8_t *nonce,
                              size_t nonce_len, uint32_t ntz, uint64_t k_begin, uint64_t k_limit, uint64_t first_k,
                              uint64_t batch_k, uint64_t *best_global_idx, uint8_t secret_out[DPOW_MAX_SECRET],
                              size_t *secret_len, uint32_t *batches) {
    return dpow::node_mine(c, slot, votes, rank, world, epoch, vote_timeout_ns, nonce, nonce_len, ntz, k_begin, k_limit,
                           first_k, batch_k, best_global_idx, secret_out, secret_len, batches, false, 0);
}

// dpow_node_mine; `abandon_on_cancel` (a board search, dpow_board_search): a rank whose cancel flag
// is raised -- its task was killed by Found or Cancel -- stops the slot and returns DPOW_CANCELLED
// at once instead of voting running = 0 and waiting for the other ranks' votes.  The fan-out kills
// every rank of the task, so each leaves on its own kill, also when some rank never joined (a
// worker that answered from its cache, worker.go:261-299).
int dpow::node_mine(dpow_ctx *c, dpow_node_slot *slot, dpow_node_vote_entry *votes, uint32_t rank, uint32_t world,
                    uint64_t *epoch, int64_t vote_timeout_ns, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                    uint64_t k_begin, uint64_t k_limit, uint64_t first_k, uint64_t batch_k, uint64_t *best_global_idx,
                    uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len, uint32_t *batches, bool abandon_on_cancel,
                    int role) {
    if (!c || !slot || !epoch || !best_global_idx || !secret_out || !secret_len || !batches)
        return set_error(DPOW_EINVAL, "dpow_node_mine: NULL argument");
    if (world == 0 || (world & (world - 1)) != 0 || world > 256 || rank >= world)
        return set_error(DPOW_EINVAL, "dpow_node_mine: world must be a power of two <= 256, rank < world");
    if (batch_k == 0 || k_limit > DPOW_K_LIMIT) return set_error(DPOW_EINVAL, "dpow_node_mine: bad window");
    // The partition of rank r of world 2^b: worker_byte = r, worker_bits = b (coordinator.go:127,326).
    const uint32_t wbits = (uint32_t)__builtin_ctz(world);
    *batches = 0;
    *secret_len = 0;
    // A rank that cannot attach the slot fails its first batch: it stops the slot (the other
    // ranks' searches end at once) and votes healthy = 0 at the first boundary.
    int err = dpow_node_attach(c, slot);
    if (err < 0) dpow_node_stop(slot);
    uint64_t k = k_begin, window = first_k ? first_k : batch_k;
    uint8_t sec[DPOW_MAX_SECRET];
    size_t slen = 0;
    uint64_t own = DPOW_NO_HIT;  // this rank's verified hit (the secret bytes are ours)
    int status = DPOW_EXHAUSTED;
    while (k < k_limit) {
        const uint64_t ke = k_limit - k > window ? k + window : k_limit;
        window = batch_k;
        int rc = DPOW_EXHAUSTED;
        if (err == 0) {
            uint64_t best = DPOW_NO_HIT;
            // role 0: this rank's partition; 1: every partition of the node (the ranks share this
            // GPU, dpow_board_search); 2: none (the role-1 rank covers this one's window)
            if (role == 2) rc = DPOW_EXHAUSTED;
            else rc = dpow_search(c, nonce, nonce_len, ntz, role == 1 ? 0 : rank, role == 1 ? 0 : wbits, k, ke, &best,
                                  sec, &slen);
            if (rc < 0) {
                err = rc;
                dpow_node_stop(slot);
            } else if (rc == DPOW_FOUND && best < own) {
                own = best;
                memcpy(secret_out, sec, slen);
                *secret_len = slen;
            }
        }
        const int64_t running =
            (err != 0 || rc == DPOW_CANCELLED || __atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) ? 0 : 1;
        const uint64_t posted = __atomic_load_n(&slot->best, __ATOMIC_ACQUIRE);
        const int64_t in[3] = {(int64_t)(own < posted ? own : posted), running, err != 0 ? 0 : 1};
        int64_t out[3] = {in[0], in[1], in[2]};
        if (abandon_on_cancel && err == 0 && __atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) {
            // this rank was killed: leave without the vote
            dpow_node_stop(slot);
            status = DPOW_CANCELLED;
            break;
        }
        if (votes) {
            const int vr = node_vote(votes, rank, world, ++*epoch, in, out, vote_timeout_ns,
                                     abandon_on_cancel ? c->h_cancel : nullptr);
            if (vr == DPOW_CANCELLED) {
                dpow_node_stop(slot);
                status = DPOW_CANCELLED;
                break;
            }
            if (vr < 0) {
                err = err ? err : vr;
                out[2] = 0;
            }
        }
        ++*batches;
        if (out[2] == 0) {  // a rank failed: the node's search is lost (coordinator.go:202-206)
            status = err ? err : set_error(DPOW_EPROTO, "dpow_node_mine: another rank's search failed");
            break;
        }
        if ((uint64_t)out[0] != DPOW_NO_HIT) {
            *best_global_idx = (uint64_t)out[0];
            if ((uint64_t)out[0] != own) dpow_secret_from_index((uint64_t)out[0], secret_out, secret_len);
            status = DPOW_FOUND;
            break;
        }
        if (out[1] == 0) {
            status = DPOW_CANCELLED;
            break;
        }
        k = ke;
    }
    if (c->node == slot) c->node = c->d_node = nullptr;  // detach (the pages stay held: dpow_node_attach)
    if (status != DPOW_FOUND) *secret_len = 0;
    return status;
}

int dpow::fail(int code, const char *msg) { return set_error(code, msg); }

uint64_t dpow::device_key(const dpow_ctx *c) { return c ? c->dev_key : 0; }

void dpow::set_solo(dpow_ctx *c, bool solo) {
    if (c) c->solo = solo;
}

extern "C" {

int dpow_diag_node_post_at(dpow_node_slot *slot, uint64_t global_idx, int64_t t_ns) {
    if (!slot) return set_error(DPOW_EINVAL, "dpow_diag_node_post_at: slot is NULL");
    // One poster thread per process, spinning while requests may come (it exits after 2 s
    // without one): queueing a request costs the caller a lock, not a thread creation --
    // round 3 started a thread per post, on the emulated rank's clock.  The state is never
    // destroyed (the detached thread may still run while the process exits).
    struct Poster {
        std::mutex mu;
        std::vector<std::pair<int64_t, std::pair<dpow_node_slot *, uint64_t>>> q;
        std::atomic<int> pending{0};
        bool alive = false;
    };
    static Poster *const P = new Poster;
    std::lock_guard<std::mutex> g(P->mu);
    P->q.push_back({t_ns, {slot, global_idx}});
    P->pending.fetch_add(1, std::memory_order_release);
    if (!P->alive) {
        P->alive = true;
        std::thread([]() {
            auto mono = []() {
                struct timespec ts;
                clock_gettime(CLOCK_MONOTONIC, &ts);
                return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
            };
            int64_t idle_since = mono();
            for (;;) {
                if (P->pending.load(std::memory_order_acquire) == 0) {
                    if (mono() - idle_since > 2000000000) {
                        std::lock_guard<std::mutex> g2(P->mu);
                        if (P->pending.load(std::memory_order_acquire) == 0) {
                            P->alive = false;
                            return;
                        }
                    }
                    __builtin_ia32_pause();
                    continue;
                }
                // The earliest request first (a request queued mid-batch with an
                // earlier time waited for the whole batch before): take it, and while waiting
                // for its time go back to the queue whenever another request arrives.
                std::pair<int64_t, std::pair<dpow_node_slot *, uint64_t>> w;
                int rest = 0;  // requests left in the queue when w was taken
                {
                    std::lock_guard<std::mutex> g2(P->mu);
                    auto it = std::min_element(P->q.begin(), P->q.end(),
                                               [](const auto &x, const auto &y) { return x.first < y.first; });
                    w = *it;
                    P->q.erase(it);
                    rest = P->pending.fetch_sub(1, std::memory_order_acq_rel) - 1;
                }
                bool requeued = false;
                for (;;) {
                    const int64_t left = w.first - mono();
                    if (left <= 0) break;
                    if (P->pending.load(std::memory_order_acquire) > rest) {  // a new one: maybe earlier
                        std::lock_guard<std::mutex> g2(P->mu);
                        P->q.push_back(w);
                        P->pending.fetch_add(1, std::memory_order_release);
                        requeued = true;
                        break;
                    }
                    if (left > 100000) {
                        const struct timespec d = {0, (long)std::min<int64_t>(left - 50000, 50000)};
                        nanosleep(&d, nullptr);
                    } else {
                        __builtin_ia32_pause();
                    }
                }
                if (requeued) continue;
                dpow_node_post(w.second.first, w.second.second);
                idle_since = mono();
            }
        }).detach();
    }
    return 0;
}

int dpow_diag_vote_latency(uint32_t world, int reps, double *last_us, double *all_us) {
    if (world < 2 || world > 256 || reps < 1 || !last_us || !all_us)
        return set_error(DPOW_EINVAL, "dpow_diag_vote_latency: world in [2, 256], reps >= 1, outputs non-NULL");
    void *mem = aligned_alloc(64, (size_t)2 * world * sizeof(dpow_node_vote_entry));
    if (!mem) return set_error(DPOW_EINVAL, "dpow_diag_vote_latency: out of memory");
    memset(mem, 0, (size_t)2 * world * sizeof(dpow_node_vote_entry));
    auto *votes = static_cast<dpow_node_vote_entry *>(mem);
    // The ranks on CPUs spread over this thread's affinity set, as a node's processes would be.
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    std::vector<int> cpus;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int i = 0; i < CPU_SETSIZE; ++i) {
            if (!CPU_ISSET(i, &allowed)) continue;
            // one hardware thread per core (the first of its siblings): two ranks on SMT
            // siblings would share a core's caches, which a node's processes do not
            char path[96];
            snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", i);
            if (FILE *f = fopen(path, "r")) {
                int first = -1;
                const int n = fscanf(f, "%d", &first);
                fclose(f);
                if (n == 1 && first != i) continue;
            }
            cpus.push_back(i);
        }
    auto pin = [&](uint32_t r) {
        if (cpus.empty()) return;
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpus[(size_t)r * cpus.size() / world], &one);
        (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
    };
    std::atomic<int> go{0};
    std::vector<std::atomic<int64_t>> done_at(world);
    for (auto &d : done_at) d.store(0);
    std::atomic<int> failed{0};
    std::vector<std::thread> others;
    for (uint32_t r = 1; r < world; ++r)
        others.emplace_back([&, r]() {
            pin(r);
            for (int rep = 1; rep <= reps; ++rep) {
                while (go.load(std::memory_order_acquire) < rep) __builtin_ia32_pause();
                if (failed.load()) break;  // rank 0 stopped: no rank waits for a vote that will not come
                const int64_t in[3] = {(int64_t)(1000 + r), 1, 1};
                int64_t out[3];
                if (dpow_node_vote(votes, r, world, (uint64_t)rep, in, out, 1000000000) != 0) failed.store(1);
                done_at[r].store(now_ns(), std::memory_order_release);
                while (go.load(std::memory_order_acquire) == rep) __builtin_ia32_pause();  // rank 0 collects
            }
        });
    // Rank 0 (this thread) arrives last: it waits until every other rank has voted and sits in
    // the vote's spin, then votes; last_us is its own vote, all_us the time until every rank
    // holds the result -- the node vote's share of a node's time-to-secret.
    cpu_set_t caller;
    const bool have_caller = pthread_getaffinity_np(pthread_self(), sizeof caller, &caller) == 0;
    pin(0);
    std::vector<double> last, all;
    int64_t t_prev_done = 0;
    for (int rep = 1; rep <= reps && !failed.load(); ++rep) {
        go.store(rep, std::memory_order_release);
        for (uint32_t r = 1; r < world; ++r)
            while (__atomic_load_n(&votes[2 * r + (rep & 1)].epoch, __ATOMIC_ACQUIRE) != (uint64_t)rep &&
                   !failed.load())
                __builtin_ia32_pause();
        for (const int64_t t_wait = now_ns(); now_ns() - t_wait < 2000;) __builtin_ia32_pause();
        const int64_t t0 = now_ns();
        const int64_t in[3] = {1000, 1, 1};
        int64_t out[3];
        if (dpow_node_vote(votes, 0, world, (uint64_t)rep, in, out, 1000000000) != 0 || out[0] != 1000) failed.store(1);
        const int64_t t1 = now_ns();
        int64_t t_all = t1;
        for (uint32_t r = 1; r < world && !failed.load(); ++r) {
            int64_t t;
            while ((t = done_at[r].load(std::memory_order_acquire)) <= t_prev_done && !failed.load())
                __builtin_ia32_pause();
            t_all = std::max(t_all, t);
        }
        t_prev_done = t_all;
        last.push_back((t1 - t0) / 1e3);
        all.push_back((t_all - t0) / 1e3);
    }
    go.store(reps + 1, std::memory_order_release);
    for (auto &t : others) t.join();
    if (have_caller) (void)pthread_setaffinity_np(pthread_self(), sizeof caller, &caller);
    free(mem);
    if (failed.load() || last.empty()) return set_error(DPOW_EPROTO, "dpow_diag_vote_latency: a vote failed");
    std::sort(last.begin(), last.end());
    std::sort(all.begin(), all.end());
    *last_us = last[last.size() / 2];
    *all_us = all[all.size() / 2];
    return 0;
}

void dpow_node_stop(dpow_node_slot *slot) {
    if (slot) __atomic_store_n(&slot->stop, 1u, __ATOMIC_RELEASE);
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

int dpow_plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                     uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, dpow_plan_launch *out,
                     size_t max_launches) {
    std::vector<PlannedLaunch> plan;
    int n = plan_window(nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end, plan);
    if (n < 0) return set_error(n, "dpow_plan_window: bad arguments");
    for (size_t i = 0; i < plan.size() && i < max_launches && out; ++i) out[i] = plan[i].info;
    return n;
}

int dpow_plan_candidate(const uint8_t *nonce, size_t nonce_len, uint32_t worker_byte, uint32_t worker_bits,
                        uint64_t local_idx, uint32_t iv_out[4], uint32_t words_out[32], uint32_t *nblk_out) {
    if (!iv_out || !words_out || !nblk_out) return set_error(DPOW_EINVAL, "dpow_plan_candidate: NULL argument");
    const uint64_t k = local_idx >> remainder_bits(worker_bits);
    // The launch a search from the start of k's chunk-length segment would use
    // (it spans the 2^24-k segments up to k: the segment-word path of the kernel).
    const uint32_t clen = chunk_len_of(k);
    uint64_t k_first = clen == 0 ? k : 1ull << (8 * (clen - 1));
    if (const uint64_t w2 = word2_period((uint32_t)(nonce_len % 64) % 4))  // the planner's W0 + 2 split
        if (k_first < k / w2 * w2) k_first = k / w2 * w2;
    std::vector<PlannedLaunch> plan;
    int n = plan_window(nonce, nonce_len, 0, worker_byte, worker_bits, k_first, k + 1, plan);
    if (n != 1) return set_error(n < 0 ? n : DPOW_EINVAL, "dpow_plan_candidate: bad arguments");
    for (int w = 0; w < 4; ++w) iv_out[w] = plan[0].L.iv[w];
    memset(words_out, 0, 32 * sizeof(uint32_t));
    candidate_words(plan[0], local_idx, words_out);
    *nblk_out = plan[0].info.nblk;
    return 0;
}

int dpow_diag_launch_geometry(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                              uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, uint32_t cus, uint32_t share,
                              dpow_diag_launch *out, size_t max_launches) {
    if (cus == 0 || share == 0) return set_error(DPOW_EINVAL, "dpow_diag_launch_geometry: cus and share must be > 0");
    WindowPlanner planner;
    const int rc = planner.init(nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end);
    if (rc < 0) return set_error(rc, "dpow_diag_launch_geometry: bad arguments");
    PlannedLaunch pl;
    size_t n = 0;
    const LaunchKnobs policy{};
    while (planner.next(pl)) {
        if (pl.k0) continue;  // k = 0: the search's k = 0 kernel, not an md5 launch
        // share = searches in flight on the device, as dpow_search sees them (g_active)
        cap_shared_launch(planner, pl, share, policy);
        uint64_t wblocks = 0;
        const int r = size_search_launch(pl, ntz, cus, grid_share(share, policy), policy, &wblocks, share);
        if (r < 0) return set_error(r, "dpow_diag_launch_geometry: launch grid leaves a claim counter without waves");
        if (out && n < max_launches) {
            dpow_diag_launch &d = out[n];
            d.k_begin = pl.info.k_begin;
            d.k_end = pl.info.k_end;
            d.i_begin = pl.L.i_begin;
            d.i_end = pl.L.i_end;
            d.wb_begin = pl.L.wb_begin;
            d.n_wblocks = pl.L.n_wblocks;
            d.n_big = pl.L.n_big;
            d.n_chunks = pl.L.n_chunks;
            d.worker_blocks = wblocks;
            d.chunk = pl.L.chunk;
            d.chunk_tail = pl.L.chunk_tail;
            d.rbits = pl.L.rbits;
            d.wave_block = kWaveBlock;
            d.n_static = pl.L.n_static;
            d.poll_wb = pl.L.poll_wb;
        }
        ++n;
    }
    return (int)n;
}

int dpow_diag_node_alias(dpow_ctx *c, void **cached, void **lookup) {
    if (!c || !cached || !lookup) return set_error(DPOW_EINVAL, "dpow_diag_node_alias: NULL argument");
    if (!c->node) return set_error(DPOW_EINVAL, "dpow_diag_node_alias: no slot attached");
    const DeviceScope on_device(c->device);
    if (on_device.e != hipSuccess) return hip_fail(on_device.e, "hipSetDevice");
    *cached = c->d_node;
    DPOW_HIP(hipHostGetDevicePointer(lookup, c->node, 0));
    return 0;
}

int dpow_diag_search_times(dpow_ctx *c, int64_t out[8]) {
    if (!c || !out) return set_error(DPOW_EINVAL, "dpow_diag_search_times: NULL argument");
    for (int i = 0; i < 8; ++i) out[i] = c->diag_t[i];
    return 0;
}

int dpow_diag_search_launches(dpow_ctx *c, int64_t *t0_ns, dpow_diag_launch_time *out, size_t max_launches) {
    if (!c || !t0_ns) return set_error(DPOW_EINVAL, "dpow_diag_search_launches: NULL argument");
    *t0_ns = c->diag_t0;
    const size_t n = c->diag_nl;
    for (size_t i = 0; out && i < n && i < max_launches; ++i) {
        const dpow_ctx::DiagLaunch &d = c->diag_l[i];
        dpow_diag_launch_time &o = out[i];
        o.seq = d.seq;
        o.kind = d.kind;
        o.queued_ns = d.queued;
        o.seen_ns = d.seen;
        o.candidates = d.candidates;
        o.g_end = d.g_end;
        const Snap &sn = c->h_snap[d.seq % kRing];
        const bool rec = __atomic_load_n(&sn.seq, __ATOMIC_ACQUIRE) == (uint32_t)(d.seq + 1);
        o.recorded = rec ? 1 : 0;
        o.t_start_tick = rec ? sn.t_start : 0;
        o.t_end_tick = rec ? sn.t_end : 0;
        o.best = rec ? sn.best : DPOW_NO_HIT;
    }
    return (int)n;
}

int dpow_diag_clock_sync(dpow_ctx *c, int reps, int64_t *offset_ns) {
    if (!c || !offset_ns || reps < 1) return set_error(DPOW_EINVAL, "dpow_diag_clock_sync: bad argument");
    const DeviceScope on_device(c->device);
    if (on_device.e != hipSuccess) return hip_fail(on_device.e, "hipSetDevice");
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(e, "dpow_diag_clock_sync: hipStreamSynchronize");
    unsigned long long *h = nullptr, *d = nullptr;
    if ((e = hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
        return hip_fail(e, "dpow_diag_clock_sync: hipHostMalloc");
    if ((e = hipHostGetDevicePointer(reinterpret_cast<void **>(&d), h, 0)) != hipSuccess) {
        (void)hipHostFree(h);
        return hip_fail(e, "dpow_diag_clock_sync: hipHostGetDevicePointer");
    }
    int64_t best = INT64_MAX;
    int rc = 0;
    for (int r = 0; r < reps && rc == 0; ++r) {
        __atomic_store_n(h, 0ull, __ATOMIC_RELEASE);
        if ((e = clock_probe(d, c->stream)) != hipSuccess) {
            rc = hip_fail(e, "dpow_diag_clock_sync: clock_probe");
            break;
        }
        const int64_t t_launch = now_ns();
        unsigned long long tick = 0;
        int64_t t = 0;
        while ((tick = __atomic_load_n(h, __ATOMIC_ACQUIRE)) == 0ull) {
            t = now_ns();
            if (t - t_launch > 1000000000) {
                rc = set_error(DPOW_EHIP, "dpow_diag_clock_sync: the probe's stamp never arrived");
                break;
            }
            __builtin_ia32_pause();
        }
        if (rc) break;
        t = now_ns();
        // The stamp reached host memory at or before t: the least delayed pairing bounds the offset.
        const int64_t off = t - (int64_t)((double)tick * kRealtimeNs);
        if (off < best) best = off;
    }
    e = hipStreamSynchronize(c->stream);
    if (rc == 0 && e != hipSuccess) rc = hip_fail(e, "dpow_diag_clock_sync: hipStreamSynchronize");
    (void)hipHostFree(h);
    if (rc == 0) *offset_ns = best;
    return rc;
}

uint64_t dpow_diag_blocks_per_cu(uint64_t candidates, uint32_t ntz, uint32_t worker_bits) {
    return launch_blocks_per_cu(candidates, ntz, remainder_bits(worker_bits));
}

int dpow_diag_dword_test(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint64_t k, uint32_t iv_d,
                         uint32_t state_d) {
    std::vector<PlannedLaunch> plan;
    const int n = plan_window(nonce, nonce_len, ntz, 0, 0, k, k + 1, plan);
    if (n != 1) return set_error(n < 0 ? n : DPOW_EINVAL, "dpow_diag_dword_test: bad arguments");
    const Launch &L = plan[0].L;
    const uint32_t nblk = plan[0].info.nblk;
    // one final block: the chaining value is the planner's (midstate or RFC IV)
    if (nblk == 1 && iv_d != L.iv[3]) return set_error(DPOW_EINVAL, "dpow_diag_dword_test: iv_d != iv[3]");
    const uint32_t D = iv_d + state_d;
    const bool pre = use_d_equality(nblk, ntz) ? state_d == L.deq : D <= L.dle;
    return pre && (D & L.dmask) == 0u ? 1 : 0;
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
    c->last_use.store(now_ns(), std::memory_order_relaxed);
    if (k_begin >= k_end) return DPOW_EXHAUSTED;
    // A node slot whose stop is raised (another rank was cancelled or failed), or a
    // raised cancel flag: nothing to do.  A node slot's stop is raised by every
    // attached rank that returns DPOW_CANCELLED or an error, so the other ranks end
    // their searches too (node_stop below).
    dpow_node_slot *const node = c->node;
    if (node && __atomic_load_n(&node->stop, __ATOMIC_ACQUIRE) != 0u) return DPOW_CANCELLED;
    if (__atomic_load_n(c->h_cancel, __ATOMIC_ACQUIRE) != 0u) {
        dpow_node_stop(node);
        return DPOW_CANCELLED;
    }
    const int status = search_window(c, nonce, nonce_len, ntz, worker_byte, worker_bits, k_begin, k_end,
                                     best_global_idx, secret_out, secret_len);
    if (node) {
        if (status == DPOW_FOUND) dpow_node_post(node, *best_global_idx);
        else if (status != DPOW_EXHAUSTED) dpow_node_stop(node);
    }
    return status;
}

}  // extern "C"
