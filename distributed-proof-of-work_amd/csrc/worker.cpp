// worker.cpp -- native mirror of the reference worker (worker.go) over the GPU search.
//
//   WorkerRPCHandler.Mine   worker.go:169-185  -> dpow_worker_mine
//   WorkerRPCHandler.Cancel worker.go:189-198  -> dpow_worker_cancel
//   WorkerRPCHandler.Found  worker.go:202-232  -> dpow_worker_found
//   miner                   worker.go:258-401  -> Worker::miner (search loop = dpow_search windows, or
//                                                 the node board's search, dpow_board_search)
//   WorkerResultCache       worker.go:424-506  -> Worker::cache_get / cache_add
//
// A task's cancel channel (cap 1, worker.go:172) becomes a kill counter plus
// the pinned cancel flag of the dpow_ctx its miner searches with, so a
// Found/Cancel stops the kernel mid-launch instead of at the next candidate.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dpow.h"
#include "../../include/dpow_worker.h"

namespace {

std::string hex(const std::vector<uint8_t> &b) {
    static const char d[] = "0123456789abcdef";
    std::string s;
    for (uint8_t x : b) {
        s += d[x >> 4];
        s += d[x & 15];
    }
    return s;
}

std::string json_bytes(const std::vector<uint8_t> &b) {
    std::string s = "[";
    for (size_t i = 0; i < b.size(); ++i) {
        if (i) s += ",";
        s += std::to_string(b[i]);
    }
    return s + "]";
}

std::string json_escape(const std::string &in) {
    std::string s;
    for (char ch : in) {
        if (ch == '"' || ch == '\\') s += '\\';
        if ((unsigned char)ch < 0x20) continue;
        s += ch;
    }
    return s;
}

// worker.go:508-510 generateWorkerTaskKey
std::string task_key(const std::vector<uint8_t> &nonce, uint32_t ntz, uint32_t wb) {
    return hex(nonce) + "|" + std::to_string(ntz) + "|" + std::to_string(wb);
}

// bytes.Compare(a, b) > 0 (worker.go:487)
bool bytes_greater(const std::vector<uint8_t> &a, const std::vector<uint8_t> &b) {
    const size_t n = a.size() < b.size() ? a.size() : b.size();
    int c = n ? memcmp(a.data(), b.data(), n) : 0;
    if (c != 0) return c > 0;
    return a.size() > b.size();
}

struct Task {
    std::vector<uint8_t> nonce;
    uint32_t ntz = 0, wb = 0, wbits = 0;
    uint64_t token = 0;
    std::mutex m;
    std::condition_variable cv;
    int kills = 0;              // messages sent on the cap-1 cancel channel
    dpow_ctx *ctx = nullptr;    // set while the miner searches
};

struct CacheEntry {
    uint32_t ntz;
    std::vector<uint8_t> secret;
};

}  // namespace

struct dpow_worker {
    int device = 0;
    std::atomic<dpow_board *> board{nullptr};                // node mode (dpow_worker_set_board)
    std::mutex tasks_mu;                                    // WorkerMineTasks.mu
    std::map<std::string, std::shared_ptr<Task>> tasks;     // WorkerMineTasks.tasks
    std::mutex cache_mu;                                    // WorkerResultCache.mu
    std::map<std::string, CacheEntry> cache;                // keyed by string(nonce)
    std::mutex res_mu;                                      // ResultChannel
    std::condition_variable res_cv;
    std::deque<dpow_worker_result> results;
    std::mutex trace_mu;
    std::vector<std::string> trace;
    std::mutex pool_mu;                                     // one dpow_ctx per concurrent search
    std::vector<dpow_ctx *> pool;
    // The miner goroutines (worker.go:182): a pool of threads, each running one task's miner at
    // a time.  A Mine hands its task to an idle pool thread (a condition-variable wake) or starts
    // a new one: creating a thread per Mine cost ~20 us of the Mine call, which a node's ranks
    // wait out before their search starts (dpow_board_search waits for all W ranks to join).
    std::mutex thr_mu;
    std::condition_variable thr_cv;
    std::deque<std::shared_ptr<Task>> pending;      // handed over, not yet picked up
    std::vector<std::shared_ptr<Task>> running;     // picked up by a pool thread, miner not returned
    std::vector<std::thread> threads;
    size_t idle = 0;
    bool closing = false;

    void pool_thread() {
        std::unique_lock<std::mutex> g(thr_mu);
        for (;;) {
            ++idle;
            thr_cv.wait(g, [&] { return closing || !pending.empty(); });
            --idle;
            if (pending.empty()) return;  // closing, nothing left
            std::shared_ptr<Task> t = pending.front();
            pending.pop_front();
            running.push_back(t);  // with the pop, under one lock: a closing worker kills it
            g.unlock();
            miner(t);
            g.lock();
            running.erase(std::find(running.begin(), running.end(), t));
        }
    }

    // -- tracing.Trace.RecordAction ------------------------------------------
    void record(uint64_t token, const std::string &action, const std::string &fields) {
        std::lock_guard<std::mutex> g(trace_mu);
        trace.push_back("{\"trace\":" + std::to_string(token) + ",\"action\":\"" + action + "\"" +
                        (fields.empty() ? "" : "," + fields) + "}");
    }
    static std::string fields(const std::vector<uint8_t> &nonce, uint32_t ntz, const std::vector<uint8_t> *secret,
                              const uint32_t *wb) {
        std::string s = "\"Nonce\":" + json_bytes(nonce) + ",\"NumTrailingZeros\":" + std::to_string(ntz);
        if (wb) s += ",\"WorkerByte\":" + std::to_string(*wb);
        if (secret) s += ",\"Secret\":" + json_bytes(*secret);
        return s;
    }

    // -- resultChan <- ----------------------------------------------------------
    void send(const std::vector<uint8_t> &nonce, uint32_t ntz, uint32_t wb, const std::vector<uint8_t> *secret,
              uint64_t token, int32_t error = 0) {
        dpow_worker_result r;
        memset(&r, 0, sizeof r);
        r.error = error;
        r.num_trailing_zeros = ntz;
        r.worker_byte = wb;
        r.token = token;
        r.nonce_len = nonce.size();
        memcpy(r.nonce, nonce.data(), nonce.size());
        if (secret) {
            r.has_secret = 1;
            r.secret_len = (uint32_t)secret->size();
            memcpy(r.secret, secret->data(), secret->size());
        }
        {
            std::lock_guard<std::mutex> g(res_mu);
            results.push_back(r);
        }
        res_cv.notify_all();
    }

    // -- worker.go:424-452 cacheGet ---------------------------------------------
    bool cache_get(const std::vector<uint8_t> &nonce, uint32_t ntz, uint64_t token, std::vector<uint8_t> &out) {
        std::lock_guard<std::mutex> g(cache_mu);
        auto it = cache.find(std::string(nonce.begin(), nonce.end()));
        if (it != cache.end() && it->second.ntz >= ntz) {
            record(token, "CacheHit", fields(nonce, ntz, &it->second.secret, nullptr));
            out = it->second.secret;
            return true;
        }
        record(token, "CacheMiss", fields(nonce, ntz, nullptr, nullptr));
        return false;
    }

    // -- worker.go:454-506 cacheAdd ---------------------------------------------
    void cache_add(const std::vector<uint8_t> &nonce, uint32_t ntz, const std::vector<uint8_t> &secret,
                   uint64_t token) {
        std::lock_guard<std::mutex> g(cache_mu);
        const std::string key(nonce.begin(), nonce.end());
        auto it = cache.find(key);
        if (it == cache.end()) {
            cache[key] = CacheEntry{ntz, secret};
            record(token, "CacheAdd", fields(nonce, ntz, &secret, nullptr));
        } else if (ntz > it->second.ntz ||
                   (ntz == it->second.ntz && bytes_greater(secret, it->second.secret))) {
            record(token, "CacheRemove", fields(nonce, it->second.ntz, &it->second.secret, nullptr));
            cache.erase(it);
            record(token, "CacheAdd", fields(nonce, ntz, &secret, nullptr));
            cache[key] = CacheEntry{ntz, secret};
        }
    }

    // -- cancelChan <- struct{}{} (worker.go:194, 209) ------------------------
    static void kill(Task &t) {
        std::lock_guard<std::mutex> g(t.m);
        t.kills++;
        if (t.ctx) *dpow_cancel_flag(t.ctx) = 1u;
        t.cv.notify_all();
    }
    static void wait_kill(Task &t) {  // <-killChan
        std::unique_lock<std::mutex> g(t.m);
        t.cv.wait(g, [&] { return t.kills > 0; });
        t.kills--;
    }

    dpow_ctx *acquire_ctx() {
        {
            std::lock_guard<std::mutex> g(pool_mu);
            if (!pool.empty()) {
                dpow_ctx *c = pool.back();
                pool.pop_back();
                return c;
            }
        }
        dpow_ctx *c = nullptr;
        const int rc = dpow_open(device, &c);
        return rc == 0 ? c : nullptr;
    }
    void release_ctx(dpow_ctx *c) {
        *dpow_cancel_flag(c) = 0u;
        std::lock_guard<std::mutex> g(pool_mu);
        pool.push_back(c);
    }

    // -- worker.go:258-401 miner --------------------------------------------------
    void miner(std::shared_ptr<Task> tp) {
        Task &t = *tp;
        const uint32_t wb = t.wb;
        std::vector<uint8_t> secret;
        if (cache_get(t.nonce, t.ntz, t.token, secret)) {  // worker.go:261-299
            record(t.token, "WorkerResult", fields(t.nonce, t.ntz, &secret, &wb));
            send(t.nonce, t.ntz, wb, &secret, t.token);
            wait_kill(t);
            record(t.token, "WorkerCancel", fields(t.nonce, t.ntz, nullptr, &wb));
            send(t.nonce, t.ntz, wb, nullptr, t.token);
            return;
        }
        dpow_ctx *ctx = acquire_ctx();
        if (ctx) {
            std::lock_guard<std::mutex> g(t.m);
            t.ctx = ctx;
            if (t.kills > 0) *dpow_cancel_flag(ctx) = 1u;
        }
        int status = DPOW_EXHAUSTED;
        bool own_hit = true;
        dpow_board *const nb = board.load();
        const bool node = nb && t.wbits >= 1 && t.wbits <= 6 && t.wb < (1u << t.wbits);
        if (ctx && node) {
            // The node's search of this task (dpow.h dpow_board_search): the deterministic first
            // hit of all W partitions; reported by its owner only.
            uint64_t best = DPOW_NO_HIT;
            uint8_t sec[DPOW_MAX_SECRET];
            size_t slen = 0;
            uint32_t owner = 0;
            status = dpow_board_search(nb, ctx, t.nonce.data(), t.nonce.size(), t.ntz, t.wb, t.wbits, &best, sec,
                                       &slen, &owner);
            if (status == DPOW_FOUND) {
                secret.assign(sec, sec + slen);
                own_hit = owner != 0;
            }
        }
        uint64_t k = 0, window = 1ull << 16;
        while (ctx && !node && status == DPOW_EXHAUSTED && k < DPOW_K_LIMIT) {  // worker.go:318-400
            const uint64_t ke = k + window < DPOW_K_LIMIT ? k + window : DPOW_K_LIMIT;
            uint64_t best = DPOW_NO_HIT;
            uint8_t sec[DPOW_MAX_SECRET];
            size_t slen = 0;
            status = dpow_search(ctx, t.nonce.data(), t.nonce.size(), t.ntz, t.wb, t.wbits, k, ke, &best, sec,
                                 &slen);
            if (status == DPOW_FOUND) secret.assign(sec, sec + slen);
            k = ke;
            if (window < (1ull << 24)) window <<= 4;
        }
        if (ctx) {
            std::lock_guard<std::mutex> g(t.m);
            t.ctx = nullptr;
        }
        if (ctx) release_ctx(ctx);
        if (status < 0 || !ctx) {
            // The GPU search failed (no device, a HIP error, a hit that failed host
            // verification).  The Go miner cannot fail here; waiting for a kill
            // would hang the coordinator until its timeout.  Report the error on
            // the result channel and end the task.
            const int32_t code = ctx ? status : DPOW_EHIP;
            const std::string err = dpow_last_error();
            record(t.token, "MinerError", fields(t.nonce, t.ntz, nullptr, &wb) + ",\"Code\":" +
                                              std::to_string(code) + ",\"Error\":\"" + json_escape(err) + "\"");
            fprintf(stderr, "dpow worker: search failed (%d): %s\n", code, err.c_str());
            {
                std::lock_guard<std::mutex> g(tasks_mu);
                auto it = tasks.find(task_key(t.nonce, t.ntz, t.wb));
                if (it != tasks.end() && it->second == tp) tasks.erase(it);
            }
            send(t.nonce, t.ntz, wb, nullptr, t.token, code);
            return;
        }
        if (status == DPOW_FOUND && own_hit) {  // worker.go:356-396
            record(t.token, "WorkerResult", fields(t.nonce, t.ntz, &secret, &wb));
            send(t.nonce, t.ntz, wb, &secret, t.token);
            wait_kill(t);
            record(t.token, "WorkerCancel", fields(t.nonce, t.ntz, nullptr, &wb));
            send(t.nonce, t.ntz, wb, nullptr, t.token);
            return;
        }
        // Killed while searching (worker.go:320-342).  A window exhausted up to
        // DPOW_K_LIMIT waits for the kill like the reference's never-ending
        // loop would, and so does a node rank whose partition does not hold the node's
        // first hit: the reference worker of that partition would still be searching.
        wait_kill(t);
        record(t.token, "WorkerCancel", fields(t.nonce, t.ntz, nullptr, &wb));
        send(t.nonce, t.ntz, wb, nullptr, t.token);
        send(t.nonce, t.ntz, wb, nullptr, t.token);  // the extra ACK for the first cancellation round
    }
};

extern "C" {

int dpow_worker_new(int device, dpow_worker **out) {
    if (!out) return DPOW_EINVAL;
    *out = new (std::nothrow) dpow_worker();
    if (!*out) return DPOW_ENOMEM;
    (*out)->device = device;
    // Open one search context up front (stream, control block, pinned flag) so
    // the first Mine does not pay for it.  Without a visible GPU this is skipped;
    // a miner then fails its search loudly when it needs one.
    if (dpow_device_count() > device) {
        dpow_ctx *c = nullptr;
        if (dpow_open(device, &c) == 0) (*out)->pool.push_back(c);
    }
    return 0;
}

void dpow_worker_free(dpow_worker *w) {
    if (!w) return;
    {
        // every miner, running or still pending, ends at its next kill wait (a pending one at once)
        std::lock_guard<std::mutex> g(w->thr_mu);
        w->closing = true;
        for (auto &t : w->running) dpow_worker::kill(*t);
        for (auto &t : w->pending) dpow_worker::kill(*t);
        w->thr_cv.notify_all();
    }
    for (auto &th : w->threads) th.join();
    for (dpow_ctx *c : w->pool) dpow_close(c);
    delete w;
}

int dpow_worker_set_board(dpow_worker *w, dpow_board *b) {
    if (!w) return DPOW_EINVAL;
    w->board.store(b);
    return 0;
}

int dpow_worker_mine(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                     uint32_t worker_bits, uint64_t token) {
    if (!w || (nonce_len && !nonce) || nonce_len > DPOW_MAX_NONCE || worker_byte > 255) return DPOW_EINVAL;
    auto t = std::make_shared<Task>();
    t->nonce.assign(nonce, nonce + nonce_len);
    t->ntz = ntz;
    t->wb = worker_byte;
    t->wbits = worker_bits;
    t->token = token;
    {
        std::lock_guard<std::mutex> g(w->tasks_mu);
        w->tasks[task_key(t->nonce, ntz, worker_byte)] = t;  // mineTasks.set
    }
    const uint32_t wb = worker_byte;
    w->record(token, "WorkerMine", dpow_worker::fields(t->nonce, ntz, nullptr, &wb));
    std::lock_guard<std::mutex> g(w->thr_mu);
    w->pending.push_back(t);  // go miner(...)
    if (w->idle >= w->pending.size()) w->thr_cv.notify_one();
    else w->threads.emplace_back([w] { w->pool_thread(); });
    return 0;
}

int dpow_worker_found(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte,
                      const uint8_t *secret, size_t secret_len, uint64_t token) {
    if (!w || (nonce_len && !nonce) || nonce_len > DPOW_MAX_NONCE || secret_len > DPOW_MAX_SECRET ||
        (secret_len && !secret))
        return DPOW_EINVAL;
    std::vector<uint8_t> n(nonce, nonce + nonce_len), s(secret, secret + secret_len);
    std::shared_ptr<Task> t;
    {
        std::lock_guard<std::mutex> g(w->tasks_mu);
        auto it = w->tasks.find(task_key(n, ntz, worker_byte));
        if (it != w->tasks.end()) {
            t = it->second;
            w->tasks.erase(it);  // mineTasks.delete
        }
    }
    if (t) {
        w->cache_add(n, ntz, s, token);
        dpow_worker::kill(*t);
    } else {
        const uint32_t wb = worker_byte;
        w->record(token, "WorkerCancel", dpow_worker::fields(n, ntz, nullptr, &wb));
        w->cache_add(n, ntz, s, token);
        w->send(n, ntz, worker_byte, nullptr, token);
    }
    return 0;
}

int dpow_worker_cancel(dpow_worker *w, const uint8_t *nonce, size_t nonce_len, uint32_t ntz, uint32_t worker_byte) {
    if (!w || (nonce_len && !nonce) || nonce_len > DPOW_MAX_NONCE) return DPOW_EINVAL;
    std::vector<uint8_t> n(nonce, nonce + nonce_len);
    std::shared_ptr<Task> t;
    {
        std::lock_guard<std::mutex> g(w->tasks_mu);
        auto it = w->tasks.find(task_key(n, ntz, worker_byte));
        if (it == w->tasks.end()) return DPOW_EPROTO;  // "Received more than once cancellation"
        t = it->second;
        w->tasks.erase(it);
    }
    dpow_worker::kill(*t);
    return 0;
}

int dpow_worker_next_result(dpow_worker *w, dpow_worker_result *out, int timeout_ms) {
    if (!w || !out) return DPOW_EINVAL;
    std::unique_lock<std::mutex> g(w->res_mu);
    auto ready = [&] { return !w->results.empty(); };
    if (timeout_ms < 0) {
        w->res_cv.wait(g, ready);
    } else if (!w->res_cv.wait_for(g, std::chrono::milliseconds(timeout_ms), ready)) {
        return DPOW_ETIMEOUT;
    }
    *out = w->results.front();
    w->results.pop_front();
    return 0;
}

size_t dpow_worker_trace(dpow_worker *w, char *buf, size_t cap) {
    if (!w) return 0;
    std::string s;
    {
        std::lock_guard<std::mutex> g(w->trace_mu);
        for (auto &l : w->trace) s += l + "\n";
    }
    if (buf && cap) {
        const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size();
}

int dpow_worker_active_tasks(dpow_worker *w) {
    if (!w) return DPOW_EINVAL;
    std::lock_guard<std::mutex> g(w->tasks_mu);
    return (int)w->tasks.size();
}

}  // extern "C"
