/* fake_search.c -- a CPU stand-in of the four entry points INTEGRATION.md's Option A calls
 * on the GPU (dpow_open, dpow_close, dpow_cancel_flag, dpow_search), linked in front of
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
