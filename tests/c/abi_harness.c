/* abi_harness.c -- the C ABI consumed from plain C11, as cgo consumes it.
 *
 * cgo compiles a Go file's preamble as C and links the shared library; this
 * harness does the same with gcc: it includes include/dpow.h and
 * include/dpow_worker.h, links libdpow.so and calls the host-side entry points
 * (no GPU needed).  tests/test_abi.py builds and runs it.  On a host with a GPU
 * it also runs one search (argument "gpu").
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "dpow.h"
#include "dpow_worker.h"

static int fail(const char *what) {
    fprintf(stderr, "abi_harness: %s (%s)\n", what, dpow_last_error());
    return 1;
}

int main(int argc, char **argv) {
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
    const int n = dpow_plan_window(nonce, sizeof nonce, 0, 0, 0, (1u << 24) + 5, plan, 8);
    if (n != 5 || plan[4].chunk_len != 4) return fail("dpow_plan_window");
    if (dpow_abi_version() != DPOW_ABI_VERSION) return fail("dpow_abi_version");
    if (dpow_search(NULL, nonce, 4, 6, 0, 0, 0, 1, NULL, secret, &len) != DPOW_EINVAL) return fail("NULL ctx");
    if (sizeof(dpow_worker_result) != 56 + DPOW_MAX_NONCE) return fail("dpow_worker_result layout");
    printf("{\"build_id\": \"%s\", \"abi\": %d, \"devices\": %d", dpow_build_id(), dpow_abi_version(),
           dpow_device_count());
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) {
        dpow_ctx *ctx = NULL;
        if (dpow_open(0, &ctx) != 0) return fail("dpow_open");
        uint64_t best = DPOW_NO_HIT;
        const int rc = dpow_search(ctx, nonce, 4, 6, 0, 0, 0, 1u << 20, &best, secret, &len);
        dpow_close(ctx);
        if (rc != DPOW_FOUND || best != 2532284u) return fail("dpow_search");
        printf(", \"search\": %llu", (unsigned long long)best);
    }
    printf("}\n");
    return 0;
}
