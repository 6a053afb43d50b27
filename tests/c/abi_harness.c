/* abi_harness.c -- the C ABI consumed from plain C11, as cgo consumes it.
 *
 * cgo compiles a Go file's preamble as C and links the shared library; this
 * harness does the same with gcc: it includes include/dpow.h and
 * include/dpow_worker.h, links libdpow.so and calls the host-side entry points
 * (no GPU needed).  tests/test_abi.py builds and runs it.  On a host with a GPU
 * it also runs one search (argument "gpu").
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include "dpow.h"
#include "dpow_worker.h"

static int fail(const char *what) {
    fprintf(stderr, "abi_harness: %s (%s)\n", what, dpow_last_error());
    return 1;
}

static void sleep_ms(long ms) {
    struct timespec ts = {ms / 1000, (ms % 1000) * 1000000L};
    nanosleep(&ts, NULL);
}

/* The Found/Cancel handler's side (worker.go:194,209): another thread raises the
 * pinned flag while dpow_search runs. */
static void *raise_cancel(void *ctx) {
    sleep_ms(100);
    *dpow_cancel_flag((dpow_ctx *)ctx) = 1u;
    return NULL;
}

/* the worker's trace holds an action line naming `action` */
static int traced(dpow_worker *w, const char *action) {
    static char buf[1 << 16];
    dpow_worker_trace(w, buf, sizeof buf);
    return strstr(buf, action) != NULL;
}

int main(int argc, char **argv) {
    /* A consumer built against another ABI version refuses the library (dpow.h) before it
     * calls anything else: struct layouts and signatures may differ. */
    if (dpow_abi_version() != DPOW_ABI_VERSION) {
        fprintf(stderr, "abi_harness: libdpow.so implements ABI %d, this program was built for %d: refused\n",
                dpow_abi_version(), DPOW_ABI_VERSION);
        return 3;
    }
    const uint8_t nonce[4] = {1, 2, 3, 4};
    uint8_t secret[DPOW_MAX_SECRET];
    size_t len = 0;
    /* worker.go:357-362: the Secret of global index 2532284 (config 2's answer) */
    if (dpow_secret_from_index(2532284u, secret, &len) != 0 || len != 3 || secret[0] != 188 || secret[1] != 163 ||
        secret[2] != 38)
        return fail("dpow_secret_from_index");
    if (dpow_verify(nonce, sizeof nonce, secret, len, 6) != 1 || dpow_verify(nonce, sizeof nonce, secret, len, 7) != 0)
        return fail("dpow_verify");
    uint8_t d[16];
    dpow_md5((const uint8_t *)"abc", 3, d);
    if (d[0] != 0x90 || d[15] != 0x72) return fail("dpow_md5 (RFC 1321 'abc')");
    if (dpow_trailing_zero_nibbles(d) != 0) return fail("dpow_trailing_zero_nibbles");
    dpow_plan_launch plan[8];
    const int n = dpow_plan_window(nonce, sizeof nonce, 0, 0, 0, 0, (1u << 24) + 5, plan, 8);
    /* k = 0 (start kernel), k in [1, 2^24) (chunk lengths 1..3 in one launch), then L = 4 */
    if (n != 3 || !plan[0].start_kernel || plan[1].chunk_len != 1 || plan[1].chunk_len_last != 3 ||
        plan[2].chunk_len != 4)
        return fail("dpow_plan_window");
    /* the node slot (host memory shared by a node's ranks): reset, post = atomic min, stop */
    dpow_node_slot slot;
    dpow_node_slot_reset(&slot);
    dpow_node_post(&slot, 1000);
    dpow_node_post(&slot, 2000);
    if (slot.best != 1000 || slot.stop != 0 || sizeof slot != 64) return fail("dpow_node_post");
    dpow_node_stop(&slot);
    if (slot.stop == 0 || dpow_node_attach(NULL, &slot) != DPOW_EINVAL) return fail("dpow_node_stop");
    if (dpow_search(NULL, nonce, 4, 6, 0, 0, 0, 1, NULL, secret, &len) != DPOW_EINVAL) return fail("NULL ctx");
    /* the node board (ABI 5): two ranks of one task share an entry; the last one out frees it */
    {
        dpow_board *b = NULL;
        dpow_node_slot *s0 = NULL, *s1 = NULL;
        dpow_node_vote_entry *v0 = NULL, *v1 = NULL;
        uint32_t owner = 9;
        if (dpow_board_open(NULL, &b) != 0) return fail("dpow_board_open");
        if (dpow_board_join(b, nonce, 4, 7, 4, 0, &s0, &v0) != 0 || dpow_board_join(b, nonce, 4, 7, 4, 3, &s1, &v1) != 0 ||
            s0 != s1 || v0 != v1 || s0->best != DPOW_NO_HIT || dpow_board_tasks(b) != 1)
            return fail("dpow_board_join");
        if (dpow_board_leave(b, s0) != 0 || dpow_board_tasks(b) != 1 || dpow_board_leave(b, s1) != 0 ||
            dpow_board_tasks(b) != 0 || dpow_board_leave(b, s1) != DPOW_EPROTO)
            return fail("dpow_board_leave");
        if (dpow_board_search(b, NULL, nonce, 4, 7, 0, 2, &slot.best, secret, &len, &owner) != DPOW_EINVAL ||
            owner != 9)
            return fail("dpow_board_search: NULL ctx");
        dpow_board_close(b);
    }
    if (sizeof(dpow_worker_result) != 56 + DPOW_MAX_NONCE) return fail("dpow_worker_result layout");
    const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    /* The worker mirror as worker.go's RPC shell would drive it (include/dpow_worker.h). */
    dpow_worker *w = NULL;
    dpow_worker_result res;
    if (dpow_worker_new(0, &w) != 0) return fail("dpow_worker_new");
    if (dpow_worker_mine(w, nonce, 4, 6, 0, 0, 11u) != 0) return fail("dpow_worker_mine");
    if (dpow_worker_next_result(w, &res, 30000) != 0 || res.token != 11u) return fail("dpow_worker_next_result");
    if (!gpu) {
        /* no GPU: the failed search is reported at once, one message, the task is over */
        if (res.error != DPOW_EHIP || res.has_secret || dpow_worker_active_tasks(w) != 0)
            return fail("worker: failed search not reported");
        if (!traced(w, "\"MinerError\"")) return fail("worker trace: MinerError");
    } else {
        /* config 2's answer, then the coordinator's Found kills the task: one nil ACK */
        if (res.error != 0 || !res.has_secret || res.secret_len != 3 || res.secret[0] != 188 ||
            res.secret[1] != 163 || res.secret[2] != 38)
            return fail("worker: config 2 secret");
        if (dpow_worker_found(w, nonce, 4, 6, 0, res.secret, res.secret_len, 11u) != 0)
            return fail("dpow_worker_found");
        if (dpow_worker_next_result(w, &res, 5000) != 0 || res.has_secret) return fail("worker: nil ACK");
        if (dpow_worker_next_result(w, &res, 100) != DPOW_ETIMEOUT) return fail("worker: exactly two messages");
        if (!traced(w, "\"WorkerResult\"") || !traced(w, "\"WorkerCancel\"")) return fail("worker trace");
    }
    dpow_worker_free(w);
    printf("{\"build_id\": \"%s\", \"abi\": %d, \"devices\": %d", dpow_build_id(), dpow_abi_version(),
           dpow_device_count());
    if (gpu) {
        dpow_ctx *ctx = NULL;
        if (dpow_open(0, &ctx) != 0) return fail("dpow_open");
        uint64_t best = DPOW_NO_HIT;
        int rc = dpow_search(ctx, nonce, 4, 6, 0, 0, 0, 1u << 20, &best, secret, &len);
        if (rc != DPOW_FOUND || best != 2532284u) return fail("dpow_search");
        printf(", \"search\": %llu", (unsigned long long)best);
        /* an unreachable search (N = 32 over 2^40 k) stopped by the flag from another thread */
        pthread_t th;
        if (pthread_create(&th, NULL, raise_cancel, ctx) != 0) return fail("pthread_create");
        best = DPOW_NO_HIT;
        rc = dpow_search(ctx, nonce, 4, 32, 0, 0, 1u << 24, 1ull << 40, &best, secret, &len);
        pthread_join(th, NULL);
        *dpow_cancel_flag(ctx) = 0u;
        if (rc != DPOW_CANCELLED) return fail("dpow_search: cancel flag from another thread");
        rc = dpow_search(ctx, nonce, 4, 3, 0, 0, 0, 1u << 10, &best, secret, &len);  /* the ctx is reusable */
        dpow_close(ctx);
        if (rc != DPOW_FOUND || best != 97u) return fail("dpow_search after cancel");
        printf(", \"cancelled\": true");
    }
    printf("}\n");
    return 0;
}
