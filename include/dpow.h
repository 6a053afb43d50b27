/*
 * dpow.h -- C ABI of the MI355X proof-of-work search (libdpow.so).
 *
 * The drop-in boundary for philipjesic/Distributed-Proof-Of-Work's hot path:
 * the worker's brute-force search, `miner` (worker.go:258-401), whose search
 * loop (worker.go:301-400) is replaced by GPU dispatch.  The reference has no
 * FFI of its own; these entry points are what its Go worker would bind through
 * cgo (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Plain C types only (pointers + sizes); no HIP / torch types cross the ABI.
 * Ownership: the caller owns every host buffer passed in or out; the library
 * owns all device memory and the pinned cancel flag of a context.
 * Threading: one search in flight per context (the caller serialises); the
 * cancel flag may be written from any thread while a search runs.  An entry point
 * that works on a context's GPU makes it the calling thread's current HIP device
 * for the call and restores the caller's device on return.
 * Errors are returned as negative codes; nothing longjmps, throws or aborts.
 */
#ifndef DPOW_H
#define DPOW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: dpow_worker_result gained `error` (dpow_worker.h), DPOW_K_LIMIT = 2^55 - 1 and
 * 7-byte chunks (round 2); dpow_node_* (round 3).
 * 3 (round 4): dpow_diag_launch_geometry takes ntz (dpow_diag.h); dpow_node_release.
 * 4 (round 5): dpow_node_mine.
 * 5 (round 6): the node board, dpow_board_* (the node scheduler under the coordinator protocol).
 * A consumer built against another version must refuse the library before any
 * other call (distpow/_lib.py check_abi, tests/c/abi_harness.c). */
#define DPOW_ABI_VERSION 5

/* "no hit" sentinel for global indices: INT64_MAX, so that signed (RCCL/gloo
 * int64 MIN) and unsigned (device atomicMin u64) reductions agree. */
#define DPOW_NO_HIT 0x7FFFFFFFFFFFFFFFull

/* Longest secret the search can return: 1 thread byte + 7 chunk bytes
 * (k < DPOW_K_LIMIT).  Buffers are sized 16 for headroom. */
#define DPOW_MAX_SECRET 16

/* k (the number of nextChunk applications, worker.go:234-244/399) is limited to
 * k < DPOW_K_LIMIT = 2^55 - 1: chunks of at most 7 bytes, and every global index
 * k * 256 + threadByte stays below DPOW_NO_HIT (about 2^63 candidates: decades of
 * a GPU node, so the reference's unbounded loop is never cut short in practice). */
#define DPOW_K_LIMIT ((1ull << 55) - 1)

/* dpow_search return codes */
#define DPOW_EXHAUSTED 0   /* window searched, no hit (the reference keeps looping) */
#define DPOW_FOUND 1       /* hit; *best_global_idx / secret filled, MD5 re-verified on host */
#define DPOW_CANCELLED 2   /* the cancel flag was raised (Found/Cancel RPC, worker.go:194,209) */
#define DPOW_EINVAL (-1)   /* bad argument */
#define DPOW_EHIP (-2)     /* HIP runtime error (see dpow_last_error) */
#define DPOW_EVERIFY (-3)  /* kernel hit failed host MD5 re-verification (never expected) */
#define DPOW_ERANGE (-4)   /* k window beyond DPOW_K_LIMIT */
#define DPOW_ENOMEM (-5)

typedef struct dpow_ctx dpow_ctx;

/* ---------------------------------------------------------------------------
 * Context: one per GPU.  Owns persistent device buffers (control block), the
 * HIP stream the kernels run on, and a pinned host-coherent cancel flag.
 * Replaces the per-task setup of worker.go:301-316 (buffers + threadBytes).
 * ------------------------------------------------------------------------- */
int dpow_open(int device, dpow_ctx **out);
void dpow_close(dpow_ctx *ctx);

/* Pinned, host-coherent cancel flag polled by the running kernel.  Writing a
 * non-zero value stops the search mid-launch (dpow_search returns
 * DPOW_CANCELLED).  Replaces the per-candidate `select` on killChan
 * (worker.go:320-345) and the writes at worker.go:194 (Cancel) / 209 (Found).
 * The caller clears it (writes 0) before the next task. */
volatile uint32_t *dpow_cancel_flag(dpow_ctx *ctx);

/* ---------------------------------------------------------------------------
 * The hot path.  Replaces worker.go:301-400 (the miner's enumeration loop).
 *
 * Searches the worker partition (worker_byte, worker_bits) -- threadBytes
 * uint8((worker_byte << R_bits) | t), R_bits = 8 - worker_bits % 9
 * (worker.go:302-316) -- over chunks k in [k_begin, k_end) (chunk_k = the
 * minimal little-endian bytes of k, i.e. nextChunk applied k times), in the
 * reference's order (k outer, t inner), for the first candidate whose
 * hex(MD5(nonce || threadByte || chunk_k)) ends in `ntz` '0' characters
 * (worker.go:353-356, hasNumZeroesSuffix worker.go:246-256).
 *
 * best_global_idx (in/out): on input an upper bound (DPOW_NO_HIT = none); only
 * hits with global index below it are reported.  Global index
 * g = k * 256 + threadByte; it is monotone in the worker's local order, so the
 * minimum over partitions equals the worker_bits = 0 answer.
 * On DPOW_FOUND, secret_out[0..*secret_len) = threadByte || chunk_k (the
 * `Secret` of WorkerResult, worker.go:357-362), recomputed and verified with
 * a host MD5 before returning.
 * ------------------------------------------------------------------------- */
int dpow_search(dpow_ctx *ctx, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                uint32_t worker_byte, uint32_t worker_bits, uint64_t k_begin, uint64_t k_end,
                uint64_t *best_global_idx, uint8_t secret_out[DPOW_MAX_SECRET],
                size_t *secret_len);

/* Lower the bound of the search running on ctx, from any thread: candidates at
 * or above global_idx are no longer wanted (another partition -- another GPU of
 * the node -- has a hit there).  The running kernel stops claiming work at or
 * above it within one group of wave-blocks, and dpow_search returns
 * DPOW_EXHAUSTED unless it finds a hit below the bound (then DPOW_FOUND with
 * that hit).  Used by the multi-GPU node (distpow.node.node_mine_async) to stop
 * every rank at the node's best hit without waiting for batch boundaries; the
 * reference has no counterpart (its coordinator's Found fan-out,
 * coordinator.go:210-230, cancels instead).  No effect when no search runs.
 * Returns 0 or a negative error code. */
int dpow_search_bound(dpow_ctx *ctx, uint64_t global_idx);

/* ---------------------------------------------------------------------------
 * Node slot (round 3): the Found fan-out of one node's ranks, in shared memory.
 *
 * The reference coordinator fans Found out to every worker once the first
 * result arrives (coordinator.go:210-230).  Here the G GPUs of one node search
 * the prefix partitions of the same k-window, one process each, and share a
 * dpow_node_slot (e.g. a POSIX shared-memory page mapped by every rank).  A
 * search on a context attached to a slot
 *   - takes the slot's best as a bound from its start and whenever it drops
 *     while the search waits for its launches (as dpow_search_bound), so every
 *     rank stops at the node's lowest hit without waiting for a batch boundary;
 *   - posts its own verified hit to the slot (atomic min) before it returns
 *     DPOW_FOUND;
 *   - returns DPOW_CANCELLED when the slot's stop is raised, and raises it when
 *     it returns DPOW_CANCELLED or an error itself, so a cancelled or failed rank
 *     ends the node's search on every GPU at once.
 * The node's answer is still the minimum over the ranks' results, taken once per
 * batch (distpow.node.node_mine): through dpow_node_vote below when every rank
 * shares the host, else one RCCL MIN all-reduce.  It equals the workerBits = 0
 * first hit.
 * ------------------------------------------------------------------------- */
typedef struct dpow_node_slot {
    uint64_t best;     /* lowest verified hit of any rank; DPOW_NO_HIT = none */
    uint32_t stop;     /* non-zero: every attached search ends (DPOW_CANCELLED) */
    uint32_t pad[13];  /* one 64-byte line per slot */
} dpow_node_slot;
/* Attach a slot to ctx for its next searches (NULL detaches).  Not thread-safe
 * against a running search on ctx.  The slot's host page is registered with HIP once
 * per process and stays registered while any context that attached it is open, so
 * detaching and re-attaching costs nothing and several contexts may share a slot. */
int dpow_node_attach(dpow_ctx *ctx, dpow_node_slot *slot);
/* Memory holding slots is about to be unmapped or freed: waits for the launches of every
 * context that attached a slot in [mem, mem + len), then drops the library's HIP
 * registration of those pages (so a later mapping at the same address is registered
 * afresh).  DPOW_EINVAL if a context is still attached to a slot there (ABI 3).
 * Mandatory before any memory that held an attached slot is unmapped or freed, whoever
 * owns it (a shared mapping, a heap buffer, a Go or Python array): the library keys its
 * registrations on the page address, so a later slot at the same address would otherwise
 * be matched to the old registration and its stale device alias. */
int dpow_node_release(void *mem, size_t len);
/* best = DPOW_NO_HIT, stop = 0 (before the node's search that uses the slot). */
void dpow_node_slot_reset(dpow_node_slot *slot);
/* Atomic min of a verified hit into the slot. */
void dpow_node_post(dpow_node_slot *slot, uint64_t global_idx);
/* Raise the slot's stop. */
void dpow_node_stop(dpow_node_slot *slot);

/* Node vote (round 3): node_mine's batch boundary among the G ranks of one host, through
 * the same shared memory instead of a collective -- MIN over the ranks of three int64
 * values ([best index, running, healthy]); every rank gets the same result.  `votes` is
 * an array of world * 2 dpow_node_vote_entry (zeroed before the first vote), shared by the
 * ranks; each rank votes once per boundary with the same increasing epoch (1, 2, ...),
 * into entry [rank][epoch % 2] (a rank is at most one boundary ahead of the slowest),
 * then waits for every rank's entry of that epoch.  An RCCL all-reduce of the same 24
 * bytes costs 33 us at world 1 on an MI355X (tests/test_gpu_rccl.py); this costs the
 * slowest rank's arrival plus a cache-line transfer.  Returns 0, or DPOW_EPROTO (dpow_worker.h) when some
 * rank's vote has not arrived within timeout_ns (a dead rank; the node's search is lost). */
typedef struct dpow_node_vote_entry {
    uint64_t epoch;
    int64_t v[3];
    uint64_t pad[4];   /* one 64-byte line per entry */
} dpow_node_vote_entry;
int dpow_node_vote(dpow_node_vote_entry *votes, uint32_t rank, uint32_t world, uint64_t epoch,
                   const int64_t in[3], int64_t out[3], int64_t timeout_ns);

/* One node search of this rank, natively (ABI 4): distpow.node.node_mine's batch loop over a
 * shared board, without a Python round per batch -- what a Go node scheduler would call.
 * Rank `rank` of `world` (a power of two <= 256) searches its partition (worker_byte = rank,
 * worker_bits = log2 world; coordinator.go:127,326) window by window from k_begin: the first
 * window first_k chunks (0: batch_k), every later one batch_k, up to k_limit.  The context is
 * attached to `slot` for the call (the Found fan-out, dpow_node_attach) and detached after it.
 * Each window ends in the node vote through `votes` (dpow_node_vote, epoch advanced from
 * *epoch, which the caller keeps across calls), a MIN of [the lower of its own hit and the
 * slot's posted best, running, healthy]; votes = NULL takes this rank's values alone (one rank,
 * or the one-GPU emulation of tools/node_probe.py).  Returns DPOW_FOUND with *best_global_idx =
 * the node's first hit (the workerBits = 0 answer) and its secret (this rank's verified bytes,
 * or dpow_secret_from_index of another rank's hit), DPOW_CANCELLED when some rank was
 * cancelled (the context's cancel flag, the slot's stop), DPOW_EXHAUSTED at k_limit; this
 * rank's error code when its own search failed (it stopped the slot and voted healthy = 0),
 * DPOW_EPROTO when another rank's did or a vote timed out.  *batches = windows voted. */
int dpow_node_mine(dpow_ctx *ctx, dpow_node_slot *slot, dpow_node_vote_entry *votes, uint32_t rank,
                   uint32_t world, uint64_t *epoch, int64_t vote_timeout_ns, const uint8_t *nonce,
                   size_t nonce_len, uint32_t ntz, uint64_t k_begin, uint64_t k_limit, uint64_t first_k,
                   uint64_t batch_k, uint64_t *best_global_idx, uint8_t secret_out[DPOW_MAX_SECRET],
                   size_t *secret_len, uint32_t *batches);

/* ---------------------------------------------------------------------------
 * Node board (ABI 5): the node scheduler under the reference coordinator's unchanged protocol.
 *
 * The coordinator fans a task out to W workers, worker i searching prefix partition i
 * (coordinator.go:122-129,179-199,326), and answers with the first result to arrive
 * (coordinator.go:202).  When the W workers of a coordinator share one host (one worker per GPU
 * of the node), they open one board, and each miner runs its partition's node search there
 * (dpow_board_search): the task's entry -- keyed by (nonce, ntz, W), created by the first rank
 * to arrive -- carries its node slot and votes, and every rank gets the node's first hit, the
 * minimum global index over the partitions (the workerBits = 0 answer).  Only its owner reports
 * it; the other workers wait for their kill (worker.go:320-342).  So the coordinator's first
 * result is the deterministic answer, with the reference's messages unchanged: 2 per worker.
 *
 * Requirements: W a power of two in [2, DPOW_BOARD_MAX_WORLD]; all W workers of the
 * coordinator on this host, sharing one board; one live task per (nonce, ntz) at a time (the
 * reference's task maps, worker.go:173 and coordinator.go:175, key on the same).  A worker with
 * W = 1 or a non-power-of-two W (coordinator.go:326 floor(log2 W) leaves partitions that
 * overlap) searches alone with dpow_search, and the first result wins as in the reference.
 * ------------------------------------------------------------------------- */
#define DPOW_BOARD_MAX_WORLD 64
#define DPOW_BOARD_TASKS 64      /* tasks in flight on one board at once */
typedef struct dpow_board dpow_board;
/* name NULL: a board private to this process (workers of one process, the coordinator mirror);
 * else a POSIX shared-memory object "/name", created by the first worker process that opens it
 * (zero-filled: an empty board) and mapped by every other. */
int dpow_board_open(const char *name, dpow_board **out);
/* Unmaps the board (no search may run on it); the shared object stays (dpow_board_unlink). */
void dpow_board_close(dpow_board *b);
int dpow_board_unlink(const char *name);
/* Rank `rank` of `world` joins the task (nonce, ntz, world): its entry's slot and 2 * world vote
 * entries (zeroed by the rank that created the entry).  dpow_board_leave: the last rank out
 * frees the entry.  dpow_board_search does both; they are exposed for node schedulers that call
 * dpow_node_mine themselves, and for tests. */
int dpow_board_join(dpow_board *b, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t world,
                    uint32_t rank, dpow_node_slot **slot, dpow_node_vote_entry **votes);
int dpow_board_leave(dpow_board *b, dpow_node_slot *slot);
/* Task entries in use (0 once every joined rank has left). */
int dpow_board_tasks(dpow_board *b);
/* Task entries created over the board's life, and of those the tasks whose W ranks all ran on one
 * GPU (dpow_board_search then searched the node's windows once, on rank 0, instead of W ways). */
int dpow_board_counters(dpow_board *b, uint64_t *tasks, uint64_t *shared_gpu);
/* One worker's search of a task on the board: replaces the miner's loop (worker.go:301-400) when
 * the node's W = 2^worker_bits workers share the board.  Joins the task's entry, runs
 * dpow_node_mine for partition worker_byte (rank = worker_byte, world = 2^worker_bits) from k = 0,
 * and leaves.  Returns DPOW_FOUND with *best_global_idx = the node's first hit and its secret;
 * *owner = 1 when the hit lies in this worker's partition (this worker sends WorkerResult),
 * 0 when another worker owns it (this worker waits for its kill, then sends the two nil
 * messages of the cancel path).  DPOW_CANCELLED when the context's cancel flag is raised (the
 * task's kill: Found or Cancel; the rank leaves at once, without waiting for the others' votes),
 * or another rank's cancel stopped the task; a negative code when a search failed or another
 * rank's did, or a vote timed out (120 s: a rank that never joined).  DPOW_EINVAL unless
 * 1 <= worker_bits <= 6 and worker_byte < 2^worker_bits.
 * A rank first waits until the task's other ranks have joined or one of them is seen on another
 * GPU (microseconds: the Mine fan-out's skew).  When all W ranks share one GPU (more workers than
 * GPUs), rank 0 searches every partition of each window (worker_bits 0) and the others only
 * vote: the same answer, without splitting one device W ways. */
int dpow_board_search(dpow_board *b, dpow_ctx *ctx, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                      uint32_t worker_byte, uint32_t worker_bits, uint64_t *best_global_idx,
                      uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len, uint32_t *owner);

/* ---------------------------------------------------------------------------
 * Host helpers (no GPU needed).
 * ------------------------------------------------------------------------- */
/* Secret bytes of a global index: threadByte = g & 255, chunk = minimal LE bytes of g >> 8. */
int dpow_secret_from_index(uint64_t global_idx, uint8_t secret_out[DPOW_MAX_SECRET],
                           size_t *secret_len);
/* Host MD5 (RFC 1321) of msg -> 16-byte digest. */
void dpow_md5(const uint8_t *msg, size_t len, uint8_t digest_out[16]);
/* Number of trailing '0' characters of the 32-char hex form of a digest. */
uint32_t dpow_trailing_zero_nibbles(const uint8_t digest[16]);
/* 1 if hex(MD5(nonce || secret)) ends in >= ntz '0' characters, else 0. */
int dpow_verify(const uint8_t *nonce, size_t nonce_len, const uint8_t *secret,
                size_t secret_len, uint32_t ntz);

/* Launch plan of a window (host logic of dpow_search, exposed for testing):
 * one entry per kernel launch, as dpow_search with these arguments would queue them
 * (ntz matters: chunk lengths 1..3 share a launch only when a hit is expected early).  Returns the number of launches (may exceed
 * max_launches, in which case only the first max_launches are written), or a
 * negative error code. */
typedef struct dpow_plan_launch {
    uint64_t k_begin, k_end;   /* chunk range of this launch */
    uint64_t i_begin, i_end;   /* local index range (k * R + t) */
    uint32_t nblk;             /* final MD5 blocks computed per candidate (1 or 2) */
    uint32_t w0, sh;           /* variable bytes start at word w0, byte shift sh */
    uint32_t chunk_len;        /* L: chunk bytes of k_begin ... */
    uint32_t chunk_len_last;   /* ... and of k_end - 1 (one launch may span chunk lengths 1..3) */
    uint32_t start_kernel;     /* 1: k = 0, hashed by the search's k = 0 kernel, not an md5 launch */
} dpow_plan_launch;
int dpow_plan_window(const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                     uint32_t worker_bits, uint64_t k_begin, uint64_t k_end,
                     dpow_plan_launch *out, size_t max_launches);

/* Final-block message words and chaining value the kernel hashes for local
 * index `local_idx` of a partition, assembled with the same template + lane
 * arithmetic the kernel uses.  words_out: 16 * (*nblk_out) words. */
int dpow_plan_candidate(const uint8_t *nonce, size_t nonce_len, uint32_t worker_byte,
                        uint32_t worker_bits, uint64_t local_idx, uint32_t iv_out[4],
                        uint32_t words_out[32], uint32_t *nblk_out);

/* ---------------------------------------------------------------------------
 * Introspection / measurement.
 * ------------------------------------------------------------------------- */
typedef struct dpow_stats {
    uint64_t searches;     /* dpow_search calls */
    uint64_t launches;     /* kernel launches whose completion record a search consumed */
    uint64_t candidates;   /* candidates covered by those launches' windows */
    double kernel_ms;      /* sum of their durations, as each launch stamps them into its
                              completion record (s_memrealtime at its start and at the record) */
} dpow_stats;
int dpow_get_stats(dpow_ctx *ctx, dpow_stats *out);
void dpow_reset_stats(dpow_ctx *ctx);
/* The hipStream_t the context's kernels run on (as void*, for event timing). */
void *dpow_stream(dpow_ctx *ctx);
/* Device ordinal of the context. */
int dpow_device(dpow_ctx *ctx);
/* Worker waves per launch and CUs used (for reporting). */
int dpow_geometry(dpow_ctx *ctx, uint32_t *cus, uint32_t *blocks_per_cu, uint32_t *threads_per_block);
/* Thread-local description of the last error. */
const char *dpow_last_error(void);
int dpow_abi_version(void);
/* Source hash the library was built from: 16 hex digits of sha256 over the
 * kernel/host sources, the Makefile, these headers and the build flags.  The
 * Python host (distpow/_lib.py) refuses a library whose id does not match the
 * tree it runs in, so a stale build is never tested or benched. */
const char *dpow_build_id(void);
/* Number of visible HIP devices (0 when none; never an error). */
int dpow_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* DPOW_H */
