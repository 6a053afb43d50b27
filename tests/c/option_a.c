/* option_a.c -- INTEGRATION.md Option A (gpu_miner.go and the miner's tail), restated in
 * C11 + pthreads over the real C ABI, statement for statement, so that its control flow
 * runs and is checked here, where no Go toolchain exists.
 *
 * Go construct            -> here
 *   chan struct{} (cap c) -> chan_t (count + closed flag under one global lock/condvar)
 *   go func() {...}()     -> a thread per goroutine (joined at the end: none may leak)
 *   sync.Mutex            -> pthread_mutex_t
 *   atomic.StoreUint32    -> __atomic_store_n(..., __ATOMIC_SEQ_CST)
 *   w.resultChan          -> results_send / results_recv (the coordinator's side)
 *   trace.RecordAction    -> record(t, ACT_*)
 * Each function names the INTEGRATION.md Go function it mirrors; the comments on the right
 * quote the Go statement.  The reference flow it slots into: worker.go:167-232 (the RPC
 * handlers), 258-401 (miner; Option A replaces 301-400), coordinator.go:237-248 (the
 * coordinator waits for exactly 2 messages per worker task).
 *
 * Built two ways (tests/test_option_a.py):
 *   - over the real libdpow.so (argument "gpu"): the searches run on the GPU (-m gpu);
 *   - with tests/c/fake_search.c linked in front of libdpow.so (argument "fake"): the same
 *     state machine over a CPU stand-in of dpow_open / dpow_search / dpow_cancel_flag that
 *     polls the flag as the kernel does (no GPU needed; the host MD5 is libdpow's).
 * -DOPTION_A_R04 compiles round 4's gpuSearch instead (the kill goroutine also returned
 * when the search did, so the kill was never re-delivered): its "late_found" scenario must
 * report the deadlock the judge found (exit 4), which shows the scenarios can see it.
 * -DOPTION_A_NAIVE keeps the goroutine waiting but lets it raise the flag after the search
 * returned: its "reuse" scenario must report the late kill cancelling the pooled context's
 * next search (exit 5).
 *
 * Scenarios (argv[2..], default all): late_found, early_found, race, cancel, reuse, fanout, fanout_node.
 * Exit 0 and one JSON line on success; 4 on a missing message (deadlock), 5 on a protocol
 * violation (a third message, a wrong order, a wrong secret, a leaked goroutine or context).
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "dpow.h"

/* ------------------------------------------------------------------ Go runtime stand-ins */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;

typedef struct chan_t {
    int cap, n, closed;
} chan_t;

static void chan_send(chan_t *c) { /* c <- struct{}{} */
    pthread_mutex_lock(&g_mu);
    while (c->n >= c->cap) pthread_cond_wait(&g_cv, &g_mu);
    c->n++;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
}

static void chan_recv(chan_t *c) { /* <-c (a value, or the channel closed) */
    pthread_mutex_lock(&g_mu);
    while (c->n == 0 && !c->closed) pthread_cond_wait(&g_cv, &g_mu);
    if (c->n > 0) c->n--;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
}

static void chan_close(chan_t *c) { /* close(c) */
    pthread_mutex_lock(&g_mu);
    c->closed = 1;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
}

#ifdef OPTION_A_R04
/* select { case <-a: return 0; case <-b: return 1 } */
static int chan_select2(chan_t *a, chan_t *b) {
    pthread_mutex_lock(&g_mu);
    for (;;) {
        if (a->n > 0 || a->closed) {
            if (a->n > 0) a->n--;
            pthread_cond_broadcast(&g_cv);
            pthread_mutex_unlock(&g_mu);
            return 0;
        }
        if (b->n > 0 || b->closed) {
            if (b->n > 0) b->n--;
            pthread_cond_broadcast(&g_cv);
            pthread_mutex_unlock(&g_mu);
            return 1;
        }
        pthread_cond_wait(&g_cv, &g_mu);
    }
}
#endif

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void sleep_ms(long ms) {
    struct timespec ts = {ms / 1000, (ms % 1000) * 1000000L};
    nanosleep(&ts, NULL);
}

/* Every goroutine the binding starts is a thread counted here: at the end none may still be
 * running (a goroutine left waiting on a channel is a leak in Go). */
#define MAX_THREADS 1024
static pthread_t g_threads[MAX_THREADS];
static int g_nthreads, g_live;

typedef struct go_call {
    void *(*fn)(void *);
    void *arg;
} go_call;

static void *go_trampoline(void *p) {
    go_call c = *(go_call *)p;
    free(p);
    c.fn(c.arg);
    pthread_mutex_lock(&g_mu);
    g_live--;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
    return NULL;
}

static void go(void *(*fn)(void *), void *arg) { /* go fn(arg) */
    go_call *c = malloc(sizeof *c);
    c->fn = fn;
    c->arg = arg;
    pthread_mutex_lock(&g_mu);
    if (g_nthreads == MAX_THREADS) {
        fprintf(stderr, "option_a: too many goroutines\n");
        exit(1);
    }
    g_live++;
    pthread_t *th = &g_threads[g_nthreads++];
    pthread_mutex_unlock(&g_mu);
    if (pthread_create(th, NULL, go_trampoline, c) != 0) {
        fprintf(stderr, "option_a: pthread_create failed\n");
        exit(1);
    }
}

/* ------------------------------------------------ the worker's state (worker.go:86-114) */
enum { ACT_MINE = 1, ACT_RESULT = 2, ACT_CANCEL = 3 };

typedef struct task {
    int id;
    uint8_t nonce[8];
    size_t nonce_len;
    uint32_t ntz, worker_byte, worker_bits;
    chan_t kill;      /* cancelCh := make(chan struct{}, 1)        worker.go:172 */
    int registered;   /* w.mineTasks.set / get / delete             worker.go:173,190,196 */
    int actions[8];   /* the task's trace                           worker.go:175 */
    int nactions;
} task;

static void record(task *t, int action) { /* trace.RecordAction(...) */
    pthread_mutex_lock(&g_mu);
    if (t->nactions < 8) t->actions[t->nactions] = action;
    t->nactions++;
    pthread_mutex_unlock(&g_mu);
}

/* w.resultChan: WorkerResultWithToken messages on their way to CoordRPCHandler.Result */
typedef struct msg {
    int task;
    int has_secret;
    uint8_t secret[DPOW_MAX_SECRET];
    size_t secret_len;
} msg;
#define MAX_MSGS 4096
static msg g_msgs[MAX_MSGS];
static int g_msg_head, g_msg_tail;

static void results_send(task *t, const uint8_t *secret, size_t len) {
    pthread_mutex_lock(&g_mu);
    msg *m = &g_msgs[g_msg_tail++ % MAX_MSGS];
    m->task = t->id;
    m->has_secret = secret != NULL;
    m->secret_len = secret ? len : 0;
    if (secret) memcpy(m->secret, secret, len);
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
}

static int results_recv(msg *out, double timeout_s) { /* 0, or -1 on timeout */
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    const long ns = (long)(timeout_s * 1e9);
    dl.tv_sec += ns / 1000000000L;
    dl.tv_nsec += ns % 1000000000L;
    if (dl.tv_nsec >= 1000000000L) {
        dl.tv_sec++;
        dl.tv_nsec -= 1000000000L;
    }
    pthread_mutex_lock(&g_mu);
    while (g_msg_head == g_msg_tail)
        if (pthread_cond_timedwait(&g_cv, &g_mu, &dl) != 0 && g_msg_head == g_msg_tail) {
            pthread_mutex_unlock(&g_mu);
            return -1;
        }
    *out = g_msgs[g_msg_head++ % MAX_MSGS];
    pthread_mutex_unlock(&g_mu);
    return 0;
}

/* ------------------------------------- the context pool (ctxPool get/put)
 * Comments of the form "go: <statement>" quote INTEGRATION.md's Go code, in its order;
 * tests/test_option_a.py checks that the two stay line for line the same flow ("..." in a
 * quote stands for the rest of a long Go line). */
static int g_device;
/* gpuBoard: opened by the binding's init() from DPOW_NODE_BOARD; here by the
 * fanout_node scenario (a named board, as the W worker processes of a node would open it). */
static dpow_board *g_board;
static struct {
    dpow_ctx *free[64];
    int n, cap;         /* go: var gpuCtxs = ctxPool{free: make(chan *C.dpow_ctx, gpuPoolSize)} */
    int opens, closes;  /* (the test uses gpuPoolSize = 1: a pooled context is always reused) */
} g_pool = {.cap = 1};

static dpow_ctx *pool_get(void) {                                /* go: func (p ctxPool) get() *C.dpow_ctx { */
    pthread_mutex_lock(&g_mu);                                   /* go: select { */
    if (g_pool.n > 0) {                                          /* go: case ctx := <-p.free: */
        dpow_ctx *ctx = g_pool.free[--g_pool.n];
        pthread_mutex_unlock(&g_mu);
        return ctx;                                              /* go: return ctx */
    }
    g_pool.opens++;                                              /* go: default: */
    pthread_mutex_unlock(&g_mu);
    dpow_ctx *ctx = NULL;                                        /* go: var ctx *C.dpow_ctx */
    if (dpow_open(g_device, &ctx) != 0) {                        /* go: if rc := C.dpow_open(C.int(gpuDevice), &ctx); rc != 0 { */
        fprintf(stderr, "option_a: dpow_open: %s\n", dpow_last_error()); /* go: log.Fatalf("dpow_open: %s", ... */
        exit(1);
    }
    return ctx;                                                  /* go: return ctx */
}

static void pool_put(dpow_ctx *ctx) {                            /* go: func (p ctxPool) put(ctx *C.dpow_ctx) { */
    pthread_mutex_lock(&g_mu);                                   /* go: select { */
    if (g_pool.n < g_pool.cap) {                                 /* go: case p.free <- ctx: */
        g_pool.free[g_pool.n++] = ctx;
        pthread_mutex_unlock(&g_mu);
        return;
    }
    g_pool.closes++;                                             /* go: default: */
    pthread_mutex_unlock(&g_mu);
    dpow_close(ctx);                                             /* go: C.dpow_close(ctx) */
}

/* --------------------------------------------------------- gpuSearch */
/* What gpuSearch's closure shares with its kill goroutine (Go's GC frees it; here the last
 * of its two owners does). */
typedef struct search_state {
    chan_t *kill_chan;          /* killChan (the task's cancelCh) */
    chan_t k;
    pthread_mutex_t mu;
    int searching;
    volatile uint32_t *flag;
#ifdef OPTION_A_R04
    chan_t done;                /* round 4: done := make(chan struct{}) */
#endif
    int refs;
} search_state;

static void state_release(search_state *s) {
    pthread_mutex_lock(&g_mu);
    const int left = --s->refs;
    pthread_mutex_unlock(&g_mu);
    if (left == 0) {
        pthread_mutex_destroy(&s->mu);
        free(s);
    }
}

static void *kill_goroutine(void *arg) {
    search_state *s = arg;
#ifndef OPTION_A_R04
    chan_recv(s->kill_chan);                                  /* go: <-killChan */
    pthread_mutex_lock(&s->mu);                               /* go: mu.Lock() */
#ifdef OPTION_A_NAIVE
    s->searching = 1; /* the naive fix: write the flag whether or not the search still owns ctx */
#endif
    if (s->searching)                                         /* go: if searching { */
        __atomic_store_n(s->flag, 1u, __ATOMIC_SEQ_CST);      /* go: atomic.StoreUint32(flag, 1) */
    pthread_mutex_unlock(&s->mu);                             /* go: mu.Unlock() */
    chan_close(&s->k);                                        /* go: close(k) */
#else
    /* round 4: select { case <-killChan: atomic.StoreUint32(flag, 1); close(k); case <-done: } */
    if (chan_select2(s->kill_chan, &s->done) == 0) {
        __atomic_store_n(s->flag, 1u, __ATOMIC_SEQ_CST);
        chan_close(&s->k);
    }
#endif
    state_release(s);
    return NULL;
}

/* Returns the secret (malloc'd; *len set) or NULL; *killed = the state whose k re-delivers
 * the kill. */
static uint8_t *gpu_search(task *t, size_t *len, search_state **killed) { /* go: func gpuSearch(args WorkerMineArgs, killChan <-chan struct{}) (secret []uint8, killed <-chan struct{}) { */
    dpow_ctx *ctx = pool_get();                                           /* go: ctx := gpuCtxs.get() */
    search_state *s = calloc(1, sizeof *s);
    s->flag = dpow_cancel_flag(ctx);                                      /* go: flag := (*uint32)(unsafe.Pointer(C.dpow_cancel_flag(ctx))) */
    __atomic_store_n(s->flag, 0u, __ATOMIC_SEQ_CST);                      /* go: atomic.StoreUint32(flag, 0) */
    s->kill_chan = &t->kill;
    s->k.cap = 0;                                                         /* go: k := make(chan struct{}) */
    pthread_mutex_init(&s->mu, NULL);                                     /* go: var mu sync.Mutex */
    s->searching = 1;                                                     /* go: searching := true */
    s->refs = 2; /* the goroutine and the miner */
    go(kill_goroutine, s);                                                /* go: go func() { */
    /* (the deferred function is the code at `out:` below)                   go: defer func() { */

    const uint8_t *nonce = t->nonce;                                      /* go: nonce := C.CBytes(args.Nonce) */
    /* (t->nonce is the task's own copy)                                     go: defer C.free(nonce) */
    uint8_t sec[DPOW_MAX_SECRET];                                         /* go: var sec [C.DPOW_MAX_SECRET]C.uint8_t */
    size_t slen = 0;                                                      /* go: var slen C.size_t */
    uint8_t *secret = NULL;
    if (g_board != NULL && t->worker_bits >= 1 && t->worker_bits <= 6 &&
        t->worker_byte < (1u << t->worker_bits)) {                        /* go: if gpuBoard != nil && args.WorkerBits >= 1 && ... */
        uint64_t best = 0;                                                /* go: var best C.uint64_t */
        uint32_t owner = 0;                                               /* go: var owner C.uint32_t */
        const int rc = dpow_board_search(g_board, ctx, nonce, t->nonce_len, t->ntz, t->worker_byte,
                                         t->worker_bits, &best, sec, &slen, &owner); /* go: rc := C.dpow_board_search(gpuBoard, ctx, ... */
                                                                          /* go: switch { */
        if (rc == DPOW_FOUND && owner != 0) {                             /* go: case rc == C.DPOW_FOUND && owner != 0: */
            secret = malloc(slen);                                        /* go: return C.GoBytes(unsafe.Pointer(&sec[0]), C.int(slen)), k */
            memcpy(secret, sec, slen);
            *len = slen;
            goto out;
        }
        if (rc == DPOW_FOUND || rc == DPOW_CANCELLED) {                   /* go: case rc == C.DPOW_FOUND || rc == C.DPOW_CANCELLED: */
            chan_recv(&s->k);                                             /* go: <-k */
            goto out;                                                     /* go: return nil, k */
        }
                                                                          /* go: default: */
        fprintf(stderr, "option_a: dpow_board_search: %d (%s)\n", rc, dpow_last_error());
        abort();                                                          /* go: panic(C.GoString(C.dpow_last_error())) */
    }
    uint64_t window = 1u << 16;                                           /* go: window := uint64(1 << 16) */
    for (uint64_t k_begin = 0; k_begin < DPOW_K_LIMIT;) {                 /* go: for kBegin := uint64(0); kBegin < C.DPOW_K_LIMIT; { */
        uint64_t k_end = k_begin + window;                                /* go: kEnd := kBegin + window */
        if (k_end > DPOW_K_LIMIT)                                         /* go: if kEnd > C.DPOW_K_LIMIT { */
            k_end = DPOW_K_LIMIT;                                         /* go: kEnd = C.DPOW_K_LIMIT */
        uint64_t best = DPOW_NO_HIT;                                      /* go: best := C.uint64_t(C.DPOW_NO_HIT) */
        const int rc = dpow_search(ctx, nonce, t->nonce_len, t->ntz, t->worker_byte, t->worker_bits,
                                   k_begin, k_end, &best, sec, &slen);    /* go: rc := C.dpow_search(ctx, (*C.uint8_t)(nonce), ... */
                                                                          /* go: switch { */
        if (rc == DPOW_FOUND) {                                           /* go: case rc == C.DPOW_FOUND: */
            secret = malloc(slen);                                        /* go: return C.GoBytes(unsafe.Pointer(&sec[0]), C.int(slen)), k */
            memcpy(secret, sec, slen);
            *len = slen;
            goto out;
        }
        if (rc == DPOW_CANCELLED) goto out;                               /* go: case rc == C.DPOW_CANCELLED: */
                                                                          /* go: return nil, k */
        if (rc < 0) {                                                     /* go: case rc < 0: */
            fprintf(stderr, "option_a: dpow_search: %d (%s)\n", rc, dpow_last_error());
            abort();                                                      /* go: panic(C.GoString(C.dpow_last_error())) ... */
        }
        k_begin = k_end;                                                  /* go: kBegin = kEnd */
        if (window < (1u << 24))                                          /* go: if window < 1<<24 { */
            window <<= 4;                                                 /* go: window <<= 4 */
    }
    chan_recv(&s->k);                                                     /* go: <-k */
                                                                          /* go: return nil, k */
out:
#ifndef OPTION_A_R04
    /* the deferred function, on every return path: */
    pthread_mutex_lock(&s->mu);                                           /* go: mu.Lock() */
    s->searching = 0;                                                     /* go: searching = false */
    pthread_mutex_unlock(&s->mu);                                         /* go: mu.Unlock() */
    __atomic_store_n(s->flag, 0u, __ATOMIC_SEQ_CST);                      /* go: atomic.StoreUint32(flag, 0) */
    pool_put(ctx);                                                        /* go: gpuCtxs.put(ctx) */
#else
    chan_close(&s->done); /* round 4: defer close(done) */
    pool_put(ctx);        /* round 4: defer gpuCtxPool.Put(ctx) */
#endif
    *killed = s;
    return secret;
}

/* --------------------------------- the miner's tail (worker.go:301-400) */
static void *miner(void *arg) {
    task *t = arg;
    size_t len = 0;
    search_state *killed = NULL;
    uint8_t *secret = gpu_search(t, &len, &killed);          /* go: secret, killed := gpuSearch(args, killChan) */
    if (secret == NULL) {                                    /* go: if secret == nil { */
        record(t, ACT_CANCEL);                               /* go: trace.RecordAction(WorkerCancel{... */
        results_send(t, NULL, 0);                            /* go: w.resultChan <- WorkerResultWithToken{... Secret: nil, ... */
        results_send(t, NULL, 0);                            /* go: w.resultChan <- WorkerResultWithToken{... Secret: nil, ... */
        state_release(killed);
        return NULL;                                         /* go: return */
    }
    record(t, ACT_RESULT);                                   /* go: trace.RecordAction(WorkerResult{... Secret: secret}) */
    results_send(t, secret, len);                            /* go: w.resultChan <- WorkerResultWithToken{... Secret: secret, ... */
    chan_recv(&killed->k);                                   /* go: <-killed */
    record(t, ACT_CANCEL);                                   /* go: trace.RecordAction(WorkerCancel{... */
    results_send(t, NULL, 0);                                /* go: w.resultChan <- WorkerResultWithToken{... Secret: nil, ... */
    free(secret);
    state_release(killed);
    return NULL;
}

/* ------------------------------------------- the RPC handlers (worker.go:169-232), unchanged */
static void rpc_mine(task *t) { /* WorkerRPCHandler.Mine */
    t->kill.cap = 1;                   /* cancelCh := make(chan struct{}, 1) */
    pthread_mutex_lock(&g_mu);
    t->registered = 1;                 /* w.mineTasks.set(...) */
    pthread_mutex_unlock(&g_mu);
    record(t, ACT_MINE);               /* trace.RecordAction(WorkerMine{...}) */
    go(miner, t);                      /* go miner(w, args, cancelCh, trace) */
}

static int take_task(task *t) { /* w.mineTasks.get(...); ...; w.mineTasks.delete(...) */
    pthread_mutex_lock(&g_mu);
    const int ok = t->registered;
    t->registered = 0;
    pthread_mutex_unlock(&g_mu);
    return ok;
}

static void rpc_found(task *t) { /* WorkerRPCHandler.Found */
    if (take_task(t)) {
        chan_send(&t->kill);           /* cancelChan <- struct{}{} */
    } else {
        record(t, ACT_CANCEL);         /* trace.RecordAction(WorkerCancel{...}) */
        results_send(t, NULL, 0);      /* w.resultChan <- {Secret: nil} */
    }
}

static void rpc_cancel(task *t) { /* WorkerRPCHandler.Cancel */
    if (!take_task(t)) {
        fprintf(stderr, "option_a: Cancel of an unknown task (worker.go:192 log.Fatalf)\n");
        exit(5);
    }
    chan_send(&t->kill);               /* cancelChan <- struct{}{} */
}

/* ----------------------------------------------------------------------- the scenarios */
static double g_timeout_s = 30.0;
static int g_fake;
static int g_next_id = 1;

static task *new_task(const uint8_t *nonce, size_t nlen, uint32_t ntz, uint32_t wb, uint32_t wbits) {
    task *t = calloc(1, sizeof *t);
    t->id = g_next_id++;
    memcpy(t->nonce, nonce, nlen);
    t->nonce_len = nlen;
    t->ntz = ntz;
    t->worker_byte = wb;
    t->worker_bits = wbits;
    return t;
}

static _Noreturn void die(int code, const char *scenario, const char *what) {
    fprintf(stderr, "option_a [%s]: %s\n", scenario, what);
    printf("{\"ok\": false, \"scenario\": \"%s\", \"error\": \"%s\"}\n", scenario, what);
    fflush(stdout);
    _Exit(code); /* threads may be blocked for good (the deadlock being reported) */
}

/* the next message, which must belong to task t */
static msg expect_msg(const char *sc, task *t, const char *what) {
    msg m;
    if (results_recv(&m, g_timeout_s) != 0) die(4, sc, what);
    if (m.task != t->id) die(5, sc, "a message of another task");
    return m;
}

static void expect_quiet(const char *sc, double s) { /* exactly two messages per task */
    msg m;
    if (results_recv(&m, s) == 0) die(5, sc, "a third message for a task");
}

static void expect_trace(const char *sc, task *t, int a0, int a1, int a2) {
    const int want[3] = {a0, a1, a2};
    const int n = a2 ? 3 : 2;
    pthread_mutex_lock(&g_mu);
    int ok = t->nactions == n;
    for (int i = 0; ok && i < n; i++) ok = t->actions[i] == want[i];
    pthread_mutex_unlock(&g_mu);
    if (!ok) die(5, sc, "trace actions out of order");
}

static const uint8_t N1234[4] = {1, 2, 3, 4};

/* secrets of the goldens used below (tests/golden/pow_golden.json first_hits) */
static int is_secret(const msg *m, uint64_t g) {
    uint8_t s[DPOW_MAX_SECRET];
    size_t len = 0;
    dpow_secret_from_index(g, s, &len);
    return m->has_secret && m->secret_len == len && memcmp(m->secret, s, len) == 0;
}

/* A hit, then the coordinator's Found well after it (the miner waits at <-killed):
 * result, nil ACK; WorkerMine, WorkerResult, WorkerCancel. */
static void sc_late_found(void) {
    const char *sc = "late_found";
    const uint32_t n = g_fake ? 4 : 6; /* golden first hits 5236 / 2532284 */
    task *t = new_task(N1234, 4, n, 0, 0);
    rpc_mine(t);
    msg m = expect_msg(sc, t, "no result message");
    if (!is_secret(&m, g_fake ? 5236u : 2532284u)) die(5, sc, "wrong secret");
    sleep_ms(50);
    rpc_found(t);
    m = expect_msg(sc, t, "no nil ACK after the late Found (the miner never got its kill)");
    if (m.has_secret) die(5, sc, "second message carries a secret");
    expect_quiet(sc, 0.1);
    expect_trace(sc, t, ACT_MINE, ACT_RESULT, ACT_CANCEL);
}

/* The Found arrives while the search still runs (before its hit is returned): the search is
 * cancelled mid-launch -> two nil messages, WorkerMine, WorkerCancel.  (If the hit won the
 * race, result + nil ACK; both are the reference's interleavings.) */
static void sc_early_found(int *cancelled) {
    const char *sc = "early_found";
    const uint32_t n = g_fake ? 6 : 8; /* golden first hits 2532284 / 4065377546 */
    task *t = new_task(N1234, 4, n, 0, 0);
    rpc_mine(t);
    sleep_ms(1);
    rpc_found(t);
    msg a = expect_msg(sc, t, "no first message");
    msg b = expect_msg(sc, t, "no second message");
    if (b.has_secret) die(5, sc, "second message carries a secret");
    if (a.has_secret) {
        if (!is_secret(&a, g_fake ? 2532284u : 4065377546u)) die(5, sc, "wrong secret");
        expect_trace(sc, t, ACT_MINE, ACT_RESULT, ACT_CANCEL);
    } else {
        expect_trace(sc, t, ACT_MINE, ACT_CANCEL, 0);
        (*cancelled)++;
    }
    expect_quiet(sc, 0.1);
}

/* Found immediately after Mine on a search that ends at once: the kill lands anywhere
 * between the search's start, its return and the miner's <-killed. */
static void sc_race(int reps, int *results) {
    const char *sc = "race";
    for (int i = 0; i < reps; i++) {
        task *t = new_task(N1234, 4, 3, 0, 0); /* golden first hit 97 */
        rpc_mine(t);
        if (i % 3 == 1) sleep_ms(1);
        rpc_found(t);
        msg a = expect_msg(sc, t, "no first message");
        msg b = expect_msg(sc, t, "no second message");
        if (b.has_secret) die(5, sc, "second message carries a secret");
        if (a.has_secret) {
            if (!is_secret(&a, 97u)) die(5, sc, "wrong secret");
            expect_trace(sc, t, ACT_MINE, ACT_RESULT, ACT_CANCEL);
            (*results)++;
        } else {
            expect_trace(sc, t, ACT_MINE, ACT_CANCEL, 0);
        }
    }
    expect_quiet(sc, 0.1);
}

/* Cancel mid-search of an unreachable search (N = 32): two nil messages. */
static void sc_cancel(double *latency_ms) {
    const char *sc = "cancel";
    task *t = new_task(N1234, 4, 32, 0, 0);
    rpc_mine(t);
    sleep_ms(100);
    const double t0 = now_s();
    rpc_cancel(t);
    msg a = expect_msg(sc, t, "no first nil message after Cancel");
    *latency_ms = (now_s() - t0) * 1e3;
    msg b = expect_msg(sc, t, "no second nil message after Cancel");
    if (a.has_secret || b.has_secret) die(5, sc, "a cancelled search sent a secret");
    expect_quiet(sc, 0.1);
    expect_trace(sc, t, ACT_MINE, ACT_CANCEL, 0);
}

/* A late kill must not reach the context's next search: task A hits and returns its context
 * to the pool (capacity 1); task B takes the same context and searches (N = 32, no hit);
 * A's Found arrives only then.  B must keep running (no message for 300 ms), then end by its
 * own Cancel; a third task C on the same context still finds its golden. */
static void sc_reuse(void) {
    const char *sc = "reuse";
    const int opens0 = g_pool.opens;
    task *a = new_task(N1234, 4, 4, 0, 0);
    rpc_mine(a);
    msg m = expect_msg(sc, a, "no result from A");
    if (!is_secret(&m, 5236u)) die(5, sc, "wrong secret from A");
    sleep_ms(20); /* A's search has returned its context */
    task *b = new_task(N1234, 4, 32, 0, 0);
    rpc_mine(b);
    sleep_ms(50); /* B searches on A's context */
    rpc_found(a); /* the late kill of A */
    if (results_recv(&m, g_timeout_s) != 0) die(4, sc, "no nil ACK from A");
    if (m.task == b->id) die(5, sc, "A's late kill cancelled B's search on the pooled context");
    if (m.task != a->id || m.has_secret) die(5, sc, "A's second message is not its nil ACK");
    msg x;
    if (results_recv(&x, 0.3) == 0)
        die(5, sc, x.task == b->id ? "A's late kill cancelled B's search on the pooled context"
                                   : "unexpected message");
    rpc_cancel(b);
    m = expect_msg(sc, b, "no nil message from B");
    msg m2 = expect_msg(sc, b, "no second nil message from B");
    if (m.has_secret || m2.has_secret) die(5, sc, "B sent a secret");
    task *c = new_task(N1234, 4, 3, 0, 0);
    rpc_mine(c);
    m = expect_msg(sc, c, "no result from C");
    if (!is_secret(&m, 97u)) die(5, sc, "wrong secret from C");
    rpc_found(c);
    m = expect_msg(sc, c, "no nil ACK from C");
    expect_quiet(sc, 0.1);
    expect_trace(sc, a, ACT_MINE, ACT_RESULT, ACT_CANCEL);
    expect_trace(sc, b, ACT_MINE, ACT_CANCEL, 0);
    expect_trace(sc, c, ACT_MINE, ACT_RESULT, ACT_CANCEL);
    if (g_pool.opens != opens0 + (opens0 == 0 ? 1 : 0)) die(5, sc, "the pooled context was not reused");
}

/* coordinator.go:179-248 with W = 4 workers (config 3's fan-out, workerBits = 2): the first
 * result wins, Found goes to every worker, and the coordinator waits for 2W messages. */
static void sc_fanout(int *results) {
    const char *sc = "fanout";
    const int W = 4;
    const uint32_t n = g_fake ? 4 : 7;
    task *t[4];
    for (int i = 0; i < W; i++) t[i] = new_task(N1234, 4, n, (uint32_t)i, 2);
    for (int i = 0; i < W; i++) rpc_mine(t[i]);
    int count[4] = {0}, got = 0;
    msg m;
    if (results_recv(&m, g_timeout_s) != 0) die(4, sc, "no first result");
    if (!m.has_secret) die(5, sc, "first message is not a result");
    if (dpow_verify(N1234, 4, m.secret, m.secret_len, n) != 1) die(5, sc, "first result does not verify");
    count[m.task - t[0]->id]++;
    got = 1;
    for (int i = 0; i < W; i++) rpc_found(t[i]); /* coordinator.go:210-230 */
    while (got < 2 * W) {                         /* coordinator.go:237-248 */
        if (results_recv(&m, g_timeout_s) != 0) die(4, sc, "fewer than 2W messages");
        const int i = m.task - t[0]->id;
        if (i < 0 || i >= W) die(5, sc, "a message of another task");
        if (m.has_secret) {
            if (count[i] != 0) die(5, sc, "a result after a nil message");
            if (dpow_verify(N1234, 4, m.secret, m.secret_len, n) != 1) die(5, sc, "a result does not verify");
            (*results)++;
        }
        count[i]++;
        got++;
    }
    for (int i = 0; i < W; i++)
        if (count[i] != 2) die(5, sc, "a worker did not send exactly 2 messages");
    expect_quiet(sc, 0.1);
    (*results)++; /* the first one */
}

/* The same fan-out with the W workers on a node board (DPOW_NODE_BOARD, dpow.h
 * dpow_board_search): the first result is the node's first hit -- the golden, reported by the
 * owner of its index only -- and the other workers send their two nil messages on the kill. */
static void sc_fanout_node(void) {
    const char *sc = "fanout_node";
    const int W = 4;
    const uint32_t n = g_fake ? 4 : 7;
    const uint64_t golden = g_fake ? 5236u : 231910082u; /* tests/golden/pow_golden.json first_hits */
    const int owner = (int)((golden & 255u) >> 6);
    char name[64];
    snprintf(name, sizeof name, "/dpow_option_a_%ld", (long)getpid());
    if (dpow_board_open(name, &g_board) != 0) die(5, sc, "dpow_board_open");
    task *t[4];
    for (int i = 0; i < W; i++) t[i] = new_task(N1234, 4, n, (uint32_t)i, 2);
    for (int i = 0; i < W; i++) rpc_mine(t[i]);
    msg m;
    if (results_recv(&m, g_timeout_s) != 0) die(4, sc, "no first result");
    if (!m.has_secret) die(5, sc, "first message is not a result");
    if (m.task != t[owner]->id) die(5, sc, "the first result is not the owner's");
    if (!is_secret(&m, golden)) die(5, sc, "the first result is not the node's first hit (the golden)");
    int count[4] = {0}, got = 1;
    count[owner] = 1;
    for (int i = 0; i < W; i++) rpc_found(t[i]); /* coordinator.go:210-230 */
    while (got < 2 * W) {                         /* coordinator.go:237-248 */
        if (results_recv(&m, g_timeout_s) != 0) die(4, sc, "fewer than 2W messages");
        const int i = m.task - t[0]->id;
        if (i < 0 || i >= W) die(5, sc, "a message of another task");
        if (m.has_secret) die(5, sc, "a second result (only the owner reports)");
        count[i]++;
        got++;
    }
    for (int i = 0; i < W; i++) {
        if (count[i] != 2) die(5, sc, "a worker did not send exactly 2 messages");
        if (i == owner) expect_trace(sc, t[i], ACT_MINE, ACT_RESULT, ACT_CANCEL);
        else expect_trace(sc, t[i], ACT_MINE, ACT_CANCEL, 0);
    }
    expect_quiet(sc, 0.1);
    if (dpow_board_tasks(g_board) != 0) die(5, sc, "a rank did not leave the task's board entry");
    dpow_board_close(g_board);
    g_board = NULL;
    dpow_board_unlink(name);
}

int main(int argc, char **argv) {
    if (dpow_abi_version() != DPOW_ABI_VERSION) { /* the binding's init() */
        fprintf(stderr, "option_a: libdpow.so implements ABI %d, built for %d\n", dpow_abi_version(),
                DPOW_ABI_VERSION);
        return 3;
    }
    if (argc < 2 || (strcmp(argv[1], "gpu") != 0 && strcmp(argv[1], "fake") != 0)) {
        fprintf(stderr, "usage: option_a gpu|fake [scenario ...]\n");
        return 2;
    }
    g_fake = strcmp(argv[1], "fake") == 0;
    if (g_fake) g_timeout_s = 60.0;
    const char *to = getenv("OPTION_A_TIMEOUT_S"); /* how long a missing message is waited for */
    if (to && atof(to) > 0) g_timeout_s = atof(to);
    int want[7] = {1, 1, 1, 1, 1, 1, 1};
    static const char *names[7] = {"late_found", "early_found", "race", "cancel", "reuse", "fanout", "fanout_node"};
    if (argc > 2) {
        memset(want, 0, sizeof want);
        for (int a = 2; a < argc; a++)
            for (int i = 0; i < 7; i++)
                if (strcmp(argv[a], names[i]) == 0) want[i] = 1;
    }
    const double t0 = now_s();
    int early_cancelled = 0, race_results = 0, fanout_results = 0;
    double cancel_ms = -1;
    const int race_reps = 24;
    if (want[0]) sc_late_found();
    if (want[1]) sc_early_found(&early_cancelled);
    if (want[2]) sc_race(race_reps, &race_results);
    if (want[3]) sc_cancel(&cancel_ms);
    if (want[4]) sc_reuse();
    if (want[5]) sc_fanout(&fanout_results);
    if (want[6]) sc_fanout_node();
    /* every goroutine has exited: each got its kill (none is left waiting on a killChan) */
    const double dl = now_s() + 10.0;
    pthread_mutex_lock(&g_mu);
    while (g_live > 0 && now_s() < dl) {
        pthread_mutex_unlock(&g_mu);
        sleep_ms(5);
        pthread_mutex_lock(&g_mu);
    }
    const int nth = g_nthreads, live = g_live;
    pthread_mutex_unlock(&g_mu);
    if (live > 0) die(5, "teardown", "a goroutine never exited (leaked)");
    for (int i = 0; i < nth; i++) pthread_join(g_threads[i], NULL);
    /* every context is either pooled or closed: close the pool and count */
    while (g_pool.n > 0) {
        dpow_close(g_pool.free[--g_pool.n]);
        g_pool.closes++;
    }
    if (g_pool.opens != g_pool.closes) die(5, "teardown", "a context leaked");
    printf("{\"ok\": true, \"mode\": \"%s\", \"flow\": \"%s\", \"goroutines\": %d, \"contexts_opened\": %d, "
           "\"contexts_closed\": %d, \"early_found_cancelled\": %d, \"race_reps\": %d, \"race_results\": %d, "
           "\"cancel_latency_ms\": %.3f, \"fanout_results\": %d, \"fanout_node\": %s, \"seconds\": %.3f}\n",
           g_fake ? "fake" : "gpu",
#if defined(OPTION_A_R04)
           "r04",
#elif defined(OPTION_A_NAIVE)
           "naive",
#else
           "r05",
#endif
           nth, g_pool.opens, g_pool.closes, early_cancelled, want[2] ? race_reps : 0, race_results, cancel_ms,
           fanout_results, want[6] ? "true" : "false", now_s() - t0);
    return 0;
}
