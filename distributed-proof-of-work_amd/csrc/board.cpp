// board.cpp -- the node board (include/dpow.h, ABI 5): the node scheduler under the reference
// coordinator's unchanged protocol.
//
// The coordinator fans one task out to W workers, worker i searching prefix partition i
// (coordinator.go:122-129,179-199,326; worker.go:302-316), and returns whichever result comes
// first (coordinator.go:202).  When the W workers of a task share one host, their miners meet on
// the board: one entry per task, keyed by (nonce, numTrailingZeros, W), holding the task's node
// slot (the Found fan-out between the GPUs, dpow_node_attach) and its vote entries
// (dpow_node_vote).  Each worker runs the node search for its partition there (rank = workerByte,
// world = W), and every rank gets the node's first hit: the minimum global index over the
// partitions, i.e. the workerBits = 0 enumeration's first hit.  Only the owner of that index --
// the worker whose partition holds it -- reports it (WorkerResult); the others wait for their
// kill, as the reference workers still searching would (worker.go:320-342).  So the first result
// the coordinator receives is the deterministic answer, over the reference's message protocol.
//
// Layout (all-zero is a valid empty board, so a freshly created shared-memory object needs no
// initialiser and openers cannot race one): a 64-byte header (magic, lock) and kEntries task
// entries.  Join and leave take the header's spin lock (a few hundred nanoseconds, once per
// task and rank; a lock held for 10 s -- a process that died inside -- is an error, not a
// hang); the search itself never does.
#include <errno.h>
#include <stdlib.h>
#include <fcntl.h>
#include <sched.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <time.h>

#include <chrono>
#include <new>
#include <string>

#include "../../include/dpow.h"
#include "../../include/dpow_worker.h"
#include "node.h"

namespace {

constexpr uint64_t kMagic = 0x64706f77626f6105ull;  // "dpowboa" + layout 5
constexpr uint32_t kEntries = DPOW_BOARD_TASKS;
constexpr uint32_t kMaxWorld = DPOW_BOARD_MAX_WORLD;
// A rank that never votes (a dead worker process, or W workers that do not all share this
// host's board): the others fail the task after this long (their error reaches the coordinator).
constexpr int64_t kVoteTimeoutNs = 120ll * 1000000000ll;
// Each rank's node-search windows: 2^33 candidates (the node slot ends every rank's window at the
// first posted hit, so a window costs its vote only when it holds no hit; distpow/node.py
// BOARD_BATCH_CANDIDATES).
constexpr uint64_t kBatchCandidates = 1ull << 33;

struct alignas(64) Header {
    uint64_t magic;
    uint32_t lock;
    uint32_t pad0;
    uint64_t tasks;   // task entries created over the board's life (diagnostics)
    uint64_t shared;  // of which every rank ran on one GPU (one search for the node: dpow_board_search)
    uint64_t pad[4];
};

struct alignas(64) Entry {
    uint32_t state;      // 0 free, 1 active
    uint32_t refs;       // ranks inside (joined, not yet left)
    uint32_t ntz, world;
    uint64_t joined;     // bit r: rank r has joined this task
    uint64_t nonce_len;
    uint64_t pad[4];
    uint64_t dev_key[kMaxWorld];  // rank r's GPU (dpow::device_key; 0: unknown), written before its joined bit
    uint8_t nonce[DPOW_MAX_NONCE];
    dpow_node_slot slot;
    dpow_node_vote_entry votes[2 * kMaxWorld];
};
static_assert(sizeof(Header) == 64, "one line");
static_assert(sizeof(dpow_node_slot) == 64 && sizeof(dpow_node_vote_entry) == 64, "dpow.h layouts");
static_assert(offsetof(Entry, slot) % 64 == 0, "slot on its own line");

struct Layout {
    Header h;
    Entry e[kEntries];
};

// The board's spin lock (join, leave, counters: a few hundred ns each).  A holder never blocks
// inside it, so a wait of kLockTimeoutNs means a process died holding it: the caller then gets
// DPOW_EPROTO instead of spinning forever.
constexpr int64_t kLockTimeoutNs = 10ll * 1000000000ll;

int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

class Lock {
   public:
    explicit Lock(uint32_t *w) : w_(w) {
        int64_t t0 = 0;
        for (uint32_t it = 0;; ++it) {
            uint32_t z = 0;
            if (__atomic_compare_exchange_n(w_, &z, 1u, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) {
                held_ = true;
                return;
            }
            if (it % 64 != 63) {
                __builtin_ia32_pause();
                continue;
            }
            sched_yield();
            const int64_t t = mono_ns();
            if (!t0) t0 = t;
            else if (t - t0 > kLockTimeoutNs) return;
        }
    }
    ~Lock() {
        if (held_) __atomic_store_n(w_, 0u, __ATOMIC_RELEASE);
    }
    bool held() const { return held_; }
    Lock(const Lock &) = delete;
    Lock &operator=(const Lock &) = delete;

   private:
    uint32_t *w_;
    bool held_ = false;
};

int lock_lost(const char *who) {
    return dpow::fail(DPOW_EPROTO, (std::string(who) + ": the board's lock was held for 10 s (a worker process "
                                                       "died inside a join or leave?)").c_str());
}

bool key_matches(const Entry &e, const uint8_t *nonce, size_t len, uint32_t ntz, uint32_t world) {
    return e.state == 1 && e.ntz == ntz && e.world == world && e.nonce_len == len &&
           (len == 0 || memcmp(e.nonce, nonce, len) == 0);
}

}  // namespace

struct dpow_board {
    Layout *mem = nullptr;
    int fd = -1;
    bool shared = false;
};

namespace {

int board_join(dpow_board *b, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t world, uint32_t rank,
               uint64_t dev_key, Entry **out);
int same_gpu(const Entry &e, uint32_t world, uint64_t mine, const volatile uint32_t *cancel);

}  // namespace

extern "C" {

int dpow_board_open(const char *name, dpow_board **out) {
    if (!out) return dpow::fail(DPOW_EINVAL, "dpow_board_open: out is NULL");
    *out = nullptr;
    const size_t len = sizeof(Layout);
    dpow_board *b = new (std::nothrow) dpow_board();
    if (!b) return dpow::fail(DPOW_ENOMEM, "dpow_board_open: out of memory");
    void *m = MAP_FAILED;
    if (!name) {  // the workers of this process only
        m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    } else {      // every worker process of this host that opens the same name
        if (name[0] != '/' || strchr(name + 1, '/')) {
            delete b;
            return dpow::fail(DPOW_EINVAL, "dpow_board_open: name must be \"/name\" (one POSIX shm object)");
        }
        b->fd = shm_open(name, O_RDWR | O_CREAT, 0600);
        struct stat st;
        if (b->fd < 0 || fstat(b->fd, &st) != 0 ||
            ((size_t)st.st_size < len && ftruncate(b->fd, (off_t)len) != 0)) {
            const std::string err = std::string("dpow_board_open: ") + name + ": " + strerror(errno);
            if (b->fd >= 0) close(b->fd);
            delete b;
            return dpow::fail(DPOW_EINVAL, err.c_str());
        }
        m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, b->fd, 0);
        b->shared = true;
    }
    if (m == MAP_FAILED) {
        if (b->fd >= 0) close(b->fd);
        delete b;
        return dpow::fail(DPOW_ENOMEM, "dpow_board_open: mmap failed");
    }
    b->mem = static_cast<Layout *>(m);
    uint64_t z = 0;
    if (!__atomic_compare_exchange_n(&b->mem->h.magic, &z, kMagic, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE) &&
        z != kMagic) {
        munmap(m, len);
        if (b->fd >= 0) close(b->fd);
        delete b;
        return dpow::fail(DPOW_EPROTO, "dpow_board_open: the shared object holds another board layout");
    }
    *out = b;
    return 0;
}

void dpow_board_close(dpow_board *b) {
    if (!b) return;
    if (b->mem) {
        // The library's HIP registrations of the entries' slot pages go first (every search on
        // the board has detached: dpow_board_search detaches before it returns).
        (void)dpow_node_release(b->mem, sizeof(Layout));
        munmap(b->mem, sizeof(Layout));
    }
    if (b->fd >= 0) close(b->fd);
    delete b;
}

int dpow_board_unlink(const char *name) {
    if (!name) return dpow::fail(DPOW_EINVAL, "dpow_board_unlink: name is NULL");
    if (shm_unlink(name) != 0 && errno != ENOENT)
        return dpow::fail(DPOW_EINVAL, (std::string("dpow_board_unlink: ") + strerror(errno)).c_str());
    return 0;
}

int dpow_board_join(dpow_board *b, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t world,
                    uint32_t rank, dpow_node_slot **slot, dpow_node_vote_entry **votes) {
    if (!slot || !votes) return dpow::fail(DPOW_EINVAL, "dpow_board_join: NULL argument");
    Entry *e = nullptr;
    const int rc = board_join(b, nonce, nonce_len, ntz, world, rank, 0, &e);
    if (rc < 0) return rc;
    *slot = &e->slot;
    *votes = e->votes;
    return 0;
}

int dpow_board_leave(dpow_board *b, dpow_node_slot *slot) {
    if (!b || !b->mem || !slot) return dpow::fail(DPOW_EINVAL, "dpow_board_leave: NULL argument");
    Layout &L = *b->mem;
    const uintptr_t off = (uintptr_t)slot - (uintptr_t)&L.e[0].slot;
    if ((uintptr_t)slot < (uintptr_t)&L.e[0].slot || off % sizeof(Entry) != 0 || off / sizeof(Entry) >= kEntries)
        return dpow::fail(DPOW_EINVAL, "dpow_board_leave: not a slot of this board");
    Entry &e = L.e[off / sizeof(Entry)];
    Lock lk(&L.h.lock);
    if (!lk.held()) return lock_lost("dpow_board_leave");
    if (e.state != 1 || e.refs == 0) return dpow::fail(DPOW_EPROTO, "dpow_board_leave: the entry is not joined");
    // The last rank out frees the entry, whether or not every rank joined (a worker that
    // answered from its cache never does; the others left on their kill).
    if (--e.refs == 0) __atomic_store_n(&e.state, 0u, __ATOMIC_RELEASE);
    return 0;
}

int dpow_board_counters(dpow_board *b, uint64_t *tasks, uint64_t *shared_gpu) {
    if (!b || !b->mem || !tasks || !shared_gpu) return dpow::fail(DPOW_EINVAL, "dpow_board_counters: NULL argument");
    Lock lk(&b->mem->h.lock);
    if (!lk.held()) return lock_lost("dpow_board_counters");
    *tasks = b->mem->h.tasks;
    *shared_gpu = __atomic_load_n(&b->mem->h.shared, __ATOMIC_RELAXED);
    return 0;
}

int dpow_board_tasks(dpow_board *b) {
    if (!b || !b->mem) return dpow::fail(DPOW_EINVAL, "dpow_board_tasks: board is NULL");
    Lock lk(&b->mem->h.lock);
    if (!lk.held()) return lock_lost("dpow_board_tasks");
    int n = 0;
    for (uint32_t i = 0; i < kEntries; ++i) n += b->mem->e[i].state == 1 ? 1 : 0;
    return n;
}

int dpow_board_search(dpow_board *b, dpow_ctx *ctx, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                      uint32_t worker_byte, uint32_t worker_bits, uint64_t *best_global_idx,
                      uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len, uint32_t *owner) {
    if (!b || !ctx || !best_global_idx || !secret_out || !secret_len || !owner)
        return dpow::fail(DPOW_EINVAL, "dpow_board_search: NULL argument");
    *owner = 0;
    *secret_len = 0;
    if (worker_bits < 1 || (1u << worker_bits) > kMaxWorld || worker_byte >= (1u << worker_bits))
        return dpow::fail(DPOW_EINVAL, "dpow_board_search: needs 1 <= worker_bits <= 6 and worker_byte < 2^worker_bits");
    const uint32_t world = 1u << worker_bits;
    const uint64_t key = dpow::device_key(ctx);
    Entry *e = nullptr;
    int rc = board_join(b, nonce, nonce_len, ntz, world, worker_byte, key, &e);
    if (rc < 0) return rc;
    dpow_node_slot *const slot = &e->slot;
    // Ranks that share one GPU (more workers than GPUs: the coordinator mirror's W logical workers
    // on one device) would split the device W ways and progress in the runtime's time slices, so
    // the node's answer waited for the slowest one's slice (tools/coord_fresh.py: 1.4-1.9x the
    // first-arrived race).  Then rank 0 searches every partition of each window (worker_bits 0:
    // the node's first hit directly) and the others only vote; on distinct GPUs each rank searches
    // its own partition.
    const int same = same_gpu(*e, world, key, dpow_cancel_flag(ctx));
    if (same < 0) {
        if (same == DPOW_CANCELLED) dpow_node_stop(slot);
        const std::string err = same == DPOW_CANCELLED ? "" : dpow_last_error();
        (void)dpow_board_leave(b, slot);
        return same == DPOW_CANCELLED ? DPOW_CANCELLED : dpow::fail(same, err.c_str());
    }
    // DPOW_DIAG_BOARD_SPLIT=1: every rank searches its own partition even on a shared GPU (tests
    // cover the multi-GPU role on one GPU with it; dpow_diag.h)
    const char *split = getenv("DPOW_DIAG_BOARD_SPLIT");
    const int role = same && !(split && split[0] == '1') ? (worker_byte == 0 ? 1 : 2) : 0;
    if (role == 1) __atomic_fetch_add(&b->mem->h.shared, 1ull, __ATOMIC_RELAXED);
    uint64_t epoch = 0;  // the entry's votes start at zero (board_join)
    uint32_t batches = 0;
    const uint64_t batch_k = kBatchCandidates >> (8 - worker_bits);
    dpow::set_solo(ctx, role == 1);
    rc = dpow::node_mine(ctx, slot, e->votes, worker_byte, world, &epoch, kVoteTimeoutNs, nonce, nonce_len, ntz, 0,
                         DPOW_K_LIMIT, 0, batch_k, best_global_idx, secret_out, secret_len, &batches, true, role);
    dpow::set_solo(ctx, false);
    const std::string err = rc < 0 ? dpow_last_error() : "";
    (void)dpow_board_leave(b, slot);
    if (rc < 0) return dpow::fail(rc, err.c_str());
    if (rc == DPOW_FOUND) *owner = (((uint32_t)*best_global_idx & 0xFFu) >> (8 - worker_bits)) == worker_byte ? 1u : 0u;
    return rc;
}

}  // extern "C"

namespace {

int board_join(dpow_board *b, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t world, uint32_t rank,
               uint64_t dev_key, Entry **out) {
    if (!b || !b->mem || (nonce_len && !nonce)) return dpow::fail(DPOW_EINVAL, "dpow_board_join: NULL argument");
    if (nonce_len > DPOW_MAX_NONCE) return dpow::fail(DPOW_EINVAL, "dpow_board_join: nonce too long");
    if (world < 2 || world > kMaxWorld || (world & (world - 1)) != 0 || rank >= world)
        return dpow::fail(DPOW_EINVAL, "dpow_board_join: world must be a power of two in [2, 64], rank < world");
    Layout &L = *b->mem;
    const uint64_t bit = 1ull << rank;
    Lock lk(&L.h.lock);
    if (!lk.held()) return lock_lost("dpow_board_join");
    // The task's entry: the active one with this key that rank has not joined yet (an entry the
    // rank already joined belongs to an earlier task with the same key whose other ranks are
    // still leaving it).
    Entry *free_e = nullptr;
    for (uint32_t i = 0; i < kEntries; ++i) {
        Entry &e = L.e[i];
        if (key_matches(e, nonce, nonce_len, ntz, world) && !(e.joined & bit)) {
            e.dev_key[rank] = dev_key;
            __atomic_store_n(&e.joined, e.joined | bit, __ATOMIC_RELEASE);
            e.refs++;
            *out = &e;
            return 0;
        }
        if (e.state == 0 && !free_e) free_e = &e;
    }
    if (!free_e) return dpow::fail(DPOW_ENOMEM, "dpow_board_join: every task entry of the board is in use");
    Entry &e = *free_e;
    e.ntz = ntz;
    e.world = world;
    e.nonce_len = nonce_len;
    if (nonce_len) memcpy(e.nonce, nonce, nonce_len);
    dpow_node_slot_reset(&e.slot);
    memset(e.votes, 0, sizeof e.votes);
    memset(e.dev_key, 0, sizeof e.dev_key);
    e.dev_key[rank] = dev_key;
    e.refs = 1;
    L.h.tasks++;
    __atomic_store_n(&e.joined, bit, __ATOMIC_RELEASE);
    __atomic_store_n(&e.state, 1u, __ATOMIC_RELEASE);
    *out = &e;
    return 0;
}

// Whether every rank of the task searches on this rank's GPU: 1 yes (all W joined, one device
// key), 0 no (some rank's GPU differs, or is unknown), DPOW_CANCELLED when the rank's cancel flag
// rises first (its task was killed; a rank that answers from its cache never joins), DPOW_EPROTO
// after kVoteTimeoutNs.  Every rank reaches the same verdict: "no" is final as soon as one other
// GPU is seen, "yes" needs the full set of W keys, which all ranks then read alike.
int same_gpu(const Entry &e, uint32_t world, uint64_t mine, const volatile uint32_t *cancel) {
    const uint64_t full = world == 64 ? ~0ull : (1ull << world) - 1;
    const int64_t t0 = mono_ns();
    for (uint64_t it = 0;; ++it) {
        const uint64_t m = __atomic_load_n(&e.joined, __ATOMIC_ACQUIRE);
        for (uint32_t r = 0; r < world; ++r)
            if ((m >> r & 1) && (e.dev_key[r] == 0 || e.dev_key[r] != mine)) return 0;
        if (m == full) return 1;
        if (__atomic_load_n(cancel, __ATOMIC_ACQUIRE) != 0u) return DPOW_CANCELLED;
        if (it < 4096) {
            __builtin_ia32_pause();
            continue;
        }
        const int64_t t = mono_ns();
        if (t - t0 > kVoteTimeoutNs)
            return dpow::fail(DPOW_EPROTO, "dpow_board_search: the task's other ranks never joined the board");
        const struct timespec d = {0, 2000};
        nanosleep(&d, nullptr);
    }
}

}  // namespace
