/* fake_search.c -- a CPU stand-in of the five entry points INTEGRATION.md's Option A calls
 * on the GPU (dpow_open, dpow_close, dpow_cancel_flag, dpow_search, dpow_board_search), linked in front of
 * libdpow.so so that tests/c/option_a.c's state machine runs without a GPU (test
 * infrastructure only; the product never links it).
 *
 * dpow_search keeps dpow.h's contract: the partition's threadBytes
 * uint8((worker_byte << R_bits) | t), R_bits = 8 - worker_bits % 9 (worker.go:302-316),
 * k outer / t inner over [k_begin, k_end) (worker.go:318-319, 399), the suffix test on the
 * host MD5 (libdpow's dpow_md5, worker.go:353-356), the in/out bound, and -- what Option A's
 * control flow depends on -- the pinned cancel flag polled during the search (every 64
 * candidates, as the kernel's waves poll it), DPOW_CANCELLED when it is raised.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dpow.h"
#include "dpow_worker.h" /* DPOW_EPROTO */

struct dpow_ctx {
    volatile uint32_t flag;
};

int dpow_open(int device, dpow_ctx **out) {
    (void)device;
    if (!out) return DPOW_EINVAL;
    *out = calloc(1, sizeof **out);
    return *out ? 0 : DPOW_ENOMEM;
}

void dpow_close(dpow_ctx *ctx) { free(ctx); }

volatile uint32_t *dpow_cancel_flag(dpow_ctx *ctx) { return ctx ? &ctx->flag : NULL; }

int dpow_search(dpow_ctx *ctx, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                uint32_t worker_bits, uint64_t k_begin, uint64_t k_end, uint64_t *best_global_idx,
                uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len) {
    if (!ctx || !best_global_idx || !secret_out || !secret_len || nonce_len > 64) return DPOW_EINVAL;
    if (k_end > DPOW_K_LIMIT) return DPOW_ERANGE;
    const uint32_t rbits = 8 - worker_bits % 9;
    uint8_t msg[64 + DPOW_MAX_SECRET];
    memcpy(msg, nonce, nonce_len);
    uint64_t polled = 0;
    for (uint64_t k = k_begin; k < k_end; k++) {
        size_t clen = 0;
        for (uint64_t x = k; x; x >>= 8) msg[nonce_len + 1 + clen++] = (uint8_t)x;
        for (uint32_t t = 0; t < (1u << rbits); t++) {
            if ((polled++ & 63) == 0 && __atomic_load_n(&ctx->flag, __ATOMIC_SEQ_CST)) return DPOW_CANCELLED;
            const uint8_t tb = (uint8_t)((worker_byte << rbits) | t);
            const uint64_t g = k * 256 + tb;
            if (g >= *best_global_idx) return DPOW_EXHAUSTED; /* the bound: nothing wanted beyond */
            msg[nonce_len] = tb;
            uint8_t d[16];
            dpow_md5(msg, nonce_len + 1 + clen, d);
            if (dpow_trailing_zero_nibbles(d) >= ntz) {
                *best_global_idx = g;
                memcpy(secret_out, msg + nonce_len, 1 + clen);
                *secret_len = 1 + clen;
                return DPOW_FOUND;
            }
        }
    }
    return DPOW_EXHAUSTED;
}

/* dpow_board_search over the stand-in search, for option_a.c's fanout_node scenario on the CPU:
 * the library's board entry (dpow_board_join / dpow_board_leave, host code) and node vote
 * (dpow_node_vote), around the same windowed node search dpow_node_mine runs on the GPU -- each
 * window of this partition bounded by the slot's best (another rank's hit), its hit posted to the
 * slot, the window's end voted [min(own, posted), running, healthy] over the ranks; a rank whose
 * cancel flag is raised stops the slot and leaves without its vote (dpow.h dpow_board_search). */
int dpow_board_search(dpow_board *b, dpow_ctx *ctx, const uint8_t *nonce, size_t nonce_len, uint32_t ntz,
                      uint32_t worker_byte, uint32_t worker_bits, uint64_t *best_global_idx,
                      uint8_t secret_out[DPOW_MAX_SECRET], size_t *secret_len, uint32_t *owner) {
    if (!b || !ctx || !best_global_idx || !secret_out || !secret_len || !owner) return DPOW_EINVAL;
    *owner = 0;
    *secret_len = 0;
    if (worker_bits < 1 || worker_bits > 6 || worker_byte >= (1u << worker_bits)) return DPOW_EINVAL;
    const uint32_t world = 1u << worker_bits;
    dpow_node_slot *slot = NULL;
    dpow_node_vote_entry *votes = NULL;
    int rc = dpow_board_join(b, nonce, nonce_len, ntz, world, worker_byte, &slot, &votes);
    if (rc < 0) return rc;
    uint64_t own = DPOW_NO_HIT, epoch = 0;
    uint8_t sec[DPOW_MAX_SECRET];
    size_t slen = 0;
    int status = DPOW_EXHAUSTED;
    for (uint64_t k = 0; status == DPOW_EXHAUSTED; k += 16) {
        uint64_t bound = __atomic_load_n(&slot->best, __ATOMIC_ACQUIRE);
        rc = dpow_search(ctx, nonce, nonce_len, ntz, worker_byte, worker_bits, k, k + 16, &bound, sec, &slen);
        if (rc == DPOW_FOUND && bound < own) {
            own = bound;
            memcpy(secret_out, sec, slen);
            *secret_len = slen;
            dpow_node_post(slot, own);
        }
        if (__atomic_load_n(dpow_cancel_flag(ctx), __ATOMIC_SEQ_CST) != 0u) {  /* killed */
            dpow_node_stop(slot);
            status = DPOW_CANCELLED;
            break;
        }
        const uint64_t posted = __atomic_load_n(&slot->best, __ATOMIC_ACQUIRE);
        const int64_t in[3] = {(int64_t)(own < posted ? own : posted), slot->stop ? 0 : 1, 1};
        int64_t out[3];
        ++epoch;
        /* the vote, abandoned on this rank's kill: re-casting the same epoch is idempotent */
        while ((rc = dpow_node_vote(votes, worker_byte, world, epoch, in, out, 1000000)) == DPOW_EPROTO &&
               __atomic_load_n(dpow_cancel_flag(ctx), __ATOMIC_SEQ_CST) == 0u) {
        }
        if (rc != 0) {
            dpow_node_stop(slot);
            status = DPOW_CANCELLED;
            break;
        }
        if ((uint64_t)out[0] != DPOW_NO_HIT) {
            *best_global_idx = (uint64_t)out[0];
            if ((uint64_t)out[0] != own) dpow_secret_from_index((uint64_t)out[0], secret_out, secret_len);
            status = DPOW_FOUND;
        } else if (out[1] == 0) {
            status = DPOW_CANCELLED;
        }
    }
    dpow_board_leave(b, slot);
    if (status == DPOW_FOUND) *owner = ((*best_global_idx & 255u) >> (8 - worker_bits)) == worker_byte;
    else *secret_len = 0;
    return status;
}
