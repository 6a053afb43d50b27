// dpow_cli.cpp -- native command-line harness over the C ABI (no Python).
//
//   dpow_cli mine  <nonce-hex> <ntz> [worker_byte worker_bits [device]]
//       the reference miner's answer for one partition (worker.go:301-400), verified on the host
//   dpow_cli sweep <log2-candidates> [device]
//       hash 2^n candidates of nonce 01020304 at N=32 (unreachable) from k = 2^24, report GH/s
//   dpow_cli latency [reps [device]]
//       time-to-secret floor: platform launch round trips (dpow_diag.h) and median dpow_search
//       latency for hits at N = 0 / 3 / 5 (in-process, warm context)
//   dpow_cli worker <nonce-hex> <ntz> [device]
//       one Mine -> result -> Found -> ACK round trip through the native worker (worker.go:169-232)
// Each command prints one JSON line.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include <algorithm>

#include "../../include/dpow.h"
#include "../../include/dpow_diag.h"
#include "../../include/dpow_worker.h"

static std::vector<uint8_t> from_hex(const char *s) {
    std::vector<uint8_t> out;
    const size_t n = strlen(s);
    for (size_t i = 0; i + 1 < n; i += 2) {
        unsigned v = 0;
        sscanf(s + i, "%2x", &v);
        out.push_back((uint8_t)v);
    }
    return out;
}

static std::string bytes_json(const uint8_t *b, size_t n) {
    std::string s = "[";
    for (size_t i = 0; i < n; ++i) s += (i ? "," : "") + std::to_string(b[i]);
    return s + "]";
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, dpow_last_error());
    return 1;
}

static int cmd_mine(int argc, char **argv) {
    if (argc < 4) return 2;
    std::vector<uint8_t> nonce = from_hex(argv[2]);
    const uint32_t ntz = (uint32_t)atoi(argv[3]);
    const uint32_t wb = argc > 5 ? (uint32_t)atoi(argv[4]) : 0, wbits = argc > 5 ? (uint32_t)atoi(argv[5]) : 0;
    const int dev = argc > 6 ? atoi(argv[6]) : 0;
    dpow_ctx *ctx = nullptr;
    int rc = dpow_open(dev, &ctx);
    if (rc) return fail("dpow_open", rc);
    uint8_t secret[DPOW_MAX_SECRET];
    size_t slen = 0;
    uint64_t best = DPOW_NO_HIT;
    const double t0 = now_s();
    uint64_t k = 0, window = 1ull << 16;
    rc = DPOW_EXHAUSTED;
    while (rc == DPOW_EXHAUSTED && k < DPOW_K_LIMIT) {
        const uint64_t ke = k + window < DPOW_K_LIMIT ? k + window : DPOW_K_LIMIT;
        rc = dpow_search(ctx, nonce.data(), nonce.size(), ntz, wb, wbits, k, ke, &best, secret, &slen);
        k = ke;
        if (window < (1ull << 26)) window <<= 2;
    }
    const double dt = now_s() - t0;
    if (rc < 0) return fail("dpow_search", rc);
    printf("{\"status\":%d,\"global_idx\":%llu,\"secret\":%s,\"verified\":%d,\"ms\":%.3f}\n", rc,
           (unsigned long long)best, bytes_json(secret, slen).c_str(),
           rc == DPOW_FOUND ? dpow_verify(nonce.data(), nonce.size(), secret, slen, ntz) : 0, dt * 1e3);
    dpow_close(ctx);
    return 0;
}

static int cmd_sweep(int argc, char **argv) {
    const int lg = argc > 2 ? atoi(argv[2]) : 36;
    const int dev = argc > 3 ? atoi(argv[3]) : 0;
    if (lg < 8 || lg > 44) return 2;
    const uint8_t nonce[4] = {1, 2, 3, 4};
    dpow_ctx *ctx = nullptr;
    int rc = dpow_open(dev, &ctx);
    if (rc) return fail("dpow_open", rc);
    uint8_t secret[DPOW_MAX_SECRET];
    size_t slen;
    uint64_t best = DPOW_NO_HIT;
    const uint64_t k0 = 1ull << 24, nk = 1ull << (lg - 8);
    rc = dpow_search(ctx, nonce, 4, 32, 0, 0, k0 - (1ull << 20), k0, &best, secret, &slen);  // warm-up
    if (rc < 0) return fail("dpow_search", rc);
    dpow_reset_stats(ctx);
    const double t0 = now_s();
    rc = dpow_search(ctx, nonce, 4, 32, 0, 0, k0, k0 + nk, &best, secret, &slen);
    const double dt = now_s() - t0;
    if (rc < 0) return fail("dpow_search", rc);
    dpow_stats st;
    dpow_get_stats(ctx, &st);
    printf("{\"candidates\":%llu,\"status\":%d,\"wall_ghs\":%.3f,\"kernel_ghs\":%.3f,\"launches\":%llu}\n",
           (unsigned long long)st.candidates, rc, (double)st.candidates / dt / 1e9,
           (double)st.candidates / (st.kernel_ms * 1e-3) / 1e9, (unsigned long long)st.launches);
    dpow_close(ctx);
    return 0;
}

static int cmd_latency(int argc, char **argv) {
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    const int dev = argc > 3 ? atoi(argv[3]) : 0;
    double floor_us[3] = {0, 0, 0};
    for (int m = 0; m < 3; ++m)
        if (dpow_diag_launch_latency(dev, m, reps, &floor_us[m]) != 0) return fail("dpow_diag_launch_latency", -2);
    dpow_ctx *ctx = nullptr;
    int rc = dpow_open(dev, &ctx);
    if (rc) return fail("dpow_open", rc);
    const uint8_t nonce[4] = {1, 2, 3, 4};
    const uint8_t nonce5[4] = {2, 2, 2, 2};
    struct Case { const uint8_t *n; uint32_t ntz; uint64_t k_end; const char *name; int idle_us; } cases[] = {
        {nonce, 0, 1, "n0_k1", 0},           {nonce, 3, 1, "n3_k1", 0},
        {nonce, 3, 256, "n3_k256", 0},       {nonce, 3, 65536, "n3_k64k", 0},
        {nonce, 3, 1ull << 24, "n3_k16M", 0}, {nonce, 3, 1ull << 26, "n3", 0},
        {nonce, 3, 1ull << 26, "n3_idle", 3000}, {nonce5, 5, 1ull << 26, "n5_02020202", 0},
        {nonce5, 5, 1ull << 26, "n5_02020202_idle", 3000}};
    std::string out = "{\"launch_sync_us\":" + std::to_string(floor_us[0]) +
                      ",\"launch_pinned_poll_us\":" + std::to_string(floor_us[1]) +
                      ",\"memcpy16_d2h_sync_us\":" + std::to_string(floor_us[2]);
    for (const Case &c : cases) {
        std::vector<double> us;
        for (int r = 0; r < reps + 5; ++r) {
            uint64_t best = DPOW_NO_HIT;
            uint8_t secret[DPOW_MAX_SECRET];
            size_t slen = 0;
            if (c.idle_us) {  // let the previous search's queued launches drain first
                const double tw = now_s();
                while ((now_s() - tw) * 1e6 < c.idle_us) {
                }
            }
            const double t0 = now_s();
            rc = dpow_search(ctx, c.n, 4, c.ntz, 0, 0, 0, c.k_end, &best, secret, &slen);
            const double dt = (now_s() - t0) * 1e6;
            if (rc != DPOW_FOUND) return fail("dpow_search", rc);
            if (r >= 5) us.push_back(dt);
        }
        std::sort(us.begin(), us.end());
        out += std::string(",\"search_") + c.name + "_us\":" + std::to_string(us[us.size() / 2]);
    }
    dpow_close(ctx);
    printf("%s}\n", out.c_str());
    return 0;
}

static int cmd_worker(int argc, char **argv) {
    if (argc < 4) return 2;
    std::vector<uint8_t> nonce = from_hex(argv[2]);
    const uint32_t ntz = (uint32_t)atoi(argv[3]);
    const int dev = argc > 4 ? atoi(argv[4]) : 0;
    dpow_worker *w = nullptr;
    int rc = dpow_worker_new(dev, &w);
    if (rc) return fail("dpow_worker_new", rc);
    const double t0 = now_s();
    rc = dpow_worker_mine(w, nonce.data(), nonce.size(), ntz, 0, 0, 1);
    if (rc) return fail("dpow_worker_mine", rc);
    dpow_worker_result r;
    rc = dpow_worker_next_result(w, &r, 600000);
    if (rc) return fail("dpow_worker_next_result", rc);
    const double dt = now_s() - t0;
    rc = dpow_worker_found(w, nonce.data(), nonce.size(), ntz, 0, r.secret, r.secret_len, 1);
    if (rc) return fail("dpow_worker_found", rc);
    dpow_worker_result ack;
    rc = dpow_worker_next_result(w, &ack, 10000);
    if (rc) return fail("dpow_worker_next_result", rc);
    printf("{\"secret\":%s,\"ack_is_nil\":%d,\"ms_to_result\":%.3f}\n", bytes_json(r.secret, r.secret_len).c_str(),
           ack.has_secret == 0, dt * 1e3);
    dpow_worker_free(w);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "mine")) return cmd_mine(argc, argv);
    if (argc >= 2 && !strcmp(argv[1], "sweep")) return cmd_sweep(argc, argv);
    if (argc >= 2 && !strcmp(argv[1], "worker")) return cmd_worker(argc, argv);
    if (argc >= 2 && !strcmp(argv[1], "latency")) return cmd_latency(argc, argv);
    fprintf(stderr,
            "usage: dpow_cli mine <nonce-hex> <ntz> [worker_byte worker_bits [device]]\n"
            "       dpow_cli sweep <log2-candidates> [device]\n"
            "       dpow_cli worker <nonce-hex> <ntz> [device]\n"
            "       dpow_cli latency [reps [device]]\n");
    return 2;
}
