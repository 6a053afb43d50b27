/*
 * dpow_worker.h -- C ABI of the GPU worker (libdpow.so): the reference
 * worker's RPC handler (worker.go:108-232), miner (worker.go:258-401) and
 * result cache (worker.go:424-506), with the search loop on the GPU.
 *
 * A Go maintainer keeps worker.go's net/rpc shell and forwards its three RPCs
 * here: WorkerRPCHandler.Mine -> dpow_worker_mine,
 * .Found -> dpow_worker_found, .Cancel -> dpow_worker_cancel, and drains
 * dpow_worker_next_result into CoordRPCHandler.Result (cmd/worker/main.go:27-36).
 *
 * Protocol kept from the reference: every Mine task produces exactly two
 * messages -- (result, nil ACK) when the miner found a secret or hit its cache
 * (worker.go:279/291, 373/389), or (nil, nil) when the kill arrives while it
 * searches (worker.go:327-341) -- and a Found for a task that is no longer
 * running produces one nil ACK (worker.go:212-229).  Trace actions carry the
 * reference's type names (WorkerMine, WorkerResult, WorkerCancel, CacheHit,
 * CacheMiss, CacheAdd, CacheRemove).
 */
#ifndef DPOW_WORKER_H
#define DPOW_WORKER_H

#include <stddef.h>
#include <stdint.h>

#include "dpow.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DPOW_MAX_NONCE 1024
#define DPOW_EPROTO (-6)    /* protocol violation the reference log.Fatal's on (worker.go:192) */
#define DPOW_ETIMEOUT (-7)  /* dpow_worker_next_result timed out */

typedef struct dpow_worker dpow_worker;

/* One message of the worker's ResultChannel (WorkerResultWithToken, worker.go:38-44).
 * has_secret == 0 is the nil-secret cancellation ACK.  error != 0 (a negative
 * DPOW_E* code) reports a search that failed on the GPU side -- a case the Go
 * reference cannot have: the task is over, no further message follows for it,
 * and the coordinator fails the request at once instead of waiting for ACKs. */
typedef struct dpow_worker_result {
    uint32_t num_trailing_zeros;
    uint32_t worker_byte;
    uint32_t has_secret;
    uint32_t secret_len;
    int32_t error;
    uint8_t secret[DPOW_MAX_SECRET];
    uint64_t token;      /* the task's trace token (opaque, passed through) */
    uint64_t nonce_len;
    uint8_t nonce[DPOW_MAX_NONCE];
} dpow_worker_result;

/* NewWorker + InitializeWorkerRPCs (worker.go:116-165), network excluded:
 * a worker whose miners search on GPU `device`. */
int dpow_worker_new(int device, dpow_worker **out);
/* Cancels running miners, joins their threads, frees all resources. */
void dpow_worker_free(dpow_worker *w);

/* Node mode (ABI 5): the miners of this worker search on the node board `b` (dpow.h
 * dpow_board_search) whenever the task's worker_bits is in [1, 6] and worker_byte <
 * 2^worker_bits, so the node's W workers return the deterministic first hit through the
 * unchanged protocol: the owner of the node's minimum index sends (result, nil ACK), every other
 * worker (nil, nil) on its kill.  b = NULL turns node mode off.  Every worker of the coordinator
 * must share the board (one process: one board; worker processes: dpow_board_open of one name);
 * the board must outlive the worker's tasks.  Set it before the first Mine. */
int dpow_worker_set_board(dpow_worker *w, dpow_board *b);

/* WorkerRPCHandler.Mine (worker.go:169-185): register the task (key
 * hex(nonce)|ntz|workerByte), record WorkerMine, start the miner thread. */
int dpow_worker_mine(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                     uint32_t worker_byte, uint32_t worker_bits, uint64_t token);

/* WorkerRPCHandler.Found (worker.go:202-232): cache the secret; kill the
 * running task, or -- when it is no longer running -- record WorkerCancel and
 * send one nil ACK. */
int dpow_worker_found(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                      uint32_t worker_byte, const uint8_t *secret, size_t secret_len, uint64_t token);

/* WorkerRPCHandler.Cancel (worker.go:189-198): kill the running task;
 * DPOW_EPROTO when there is none (the reference log.Fatal's). */
int dpow_worker_cancel(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                       uint32_t worker_byte);

/* Receive from the ResultChannel (worker.go:112,133).  timeout_ms < 0 blocks.
 * Returns 0, or DPOW_ETIMEOUT. */
int dpow_worker_next_result(dpow_worker *w, dpow_worker_result *out, int timeout_ms);

/* Trace actions recorded so far, one JSON object per line, e.g.
 * {"trace":7,"action":"WorkerMine","Nonce":[1,2,3,4],"NumTrailingZeros":5,"WorkerByte":0}.
 * Copies at most cap bytes (NUL-terminated when cap > 0); returns the full length. */
size_t dpow_worker_trace(dpow_worker *w, char *buf, size_t cap);

/* Tasks currently registered (mineTasks size). */
int dpow_worker_active_tasks(dpow_worker *w);

#ifdef __cplusplus
}
#endif
#endif /* DPOW_WORKER_H */
