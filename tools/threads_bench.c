/*
 * threads_bench.c — SDFS's own calling pattern against the C-ABI, for bench.py and the GPU tests.
 *
 * SDFS flushes write buffers from a pool of Main.writeThreads threads (WritableCacheBuffer.java:
 * 100-104); each flush calls the ONE shared engine's getChunks on one CHUNK_LENGTH buffer and
 * blocks until it returns (SparseDedupFile.java:100,432).  This harness reproduces that from C
 * threads (no interpreter in the measured path): T threads, each calling sdfs_cdc_get_chunks on
 * one buffer at a time, all released together by a start gate; it reports the aggregate rate and
 * the per-call latency distribution, and can keep every buffer's results for a parity check.
 * Test/bench infrastructure: not part of the product library.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/sdfs_cdc.h"

typedef struct sdfs_threads_result {
    double secs;      /* start gate -> last call returned */
    double gibps;     /* bytes of all calls / secs */
    double mean_us, p50_us, p90_us, p99_us, max_us;
    uint64_t calls;
    int first_error;  /* 0 or the first non-zero status */
    double caller_cpu_us; /* CPU time of the calling threads over their calls (CLOCK_THREAD_CPUTIME_ID) */
    double fill_us;       /* wall time the calling threads spent in the fill callback (mode 1) */
} sdfs_threads_result;

typedef struct {
    sdfs_cdc_engine* e;
    int kind; /* 0 = getChunks, 1 = getHash */
    int mode; /* getChunks: 0 = sdfs_cdc_get_chunks, 1 = sdfs_cdc_get_chunks_fill (the JNI glue's
                 entry: the bytes are copied once, by the fill callback, into pinned staging),
                 2 = sdfs_cdc_get_chunks_stream with stream key = buffer index / 16 */
    const uint8_t* data;
    uint64_t nbuf;
    uint32_t buf_len;
    uint32_t cap;
    int nthreads, tid;
    uint64_t total_calls;
    uint32_t* counts;   /* [nbuf] or NULL */
    uint32_t* starts;   /* [nbuf * cap] */
    uint32_t* lens;     /* [nbuf * cap] */
    uint8_t* digests;   /* [nbuf * cap * digest_len] (getHash: [nbuf * 32]) */
    double* lat_us;     /* [total_calls] */
    struct gate* gate;
    int err;
    struct timespec end;
    double cpu_us, fill_us;
} worker_t;

/* start gate: every worker waits until all have been created, then they start together */
struct gate {
    pthread_mutex_t m;
    pthread_cond_t cv;
    int go;
};

static void gate_wait(struct gate* g) {
    pthread_mutex_lock(&g->m);
    while (!g->go) pthread_cond_wait(&g->cv, &g->m);
    pthread_mutex_unlock(&g->m);
}

static double ts_us(const struct timespec* a, const struct timespec* b) {
    return (double)(b->tv_sec - a->tv_sec) * 1e6 + (double)(b->tv_nsec - a->tv_nsec) / 1e3;
}

struct fill_ctx {
    const uint8_t* src;
    double* acc_us;
};

static int copy_fill(void* ctx, uint8_t* dst, uint32_t len) {
    const struct fill_ctx* f = (const struct fill_ctx*)ctx;
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    memcpy(dst, f->src, len);
    clock_gettime(CLOCK_MONOTONIC, &b);
    *f->acc_us += (double)(b.tv_sec - a.tv_sec) * 1e6 + (double)(b.tv_nsec - a.tv_nsec) / 1e3;
    return 0;
}

static void* worker(void* arg) {
    worker_t* w = (worker_t*)arg;
    const int dl = sdfs_cdc_digest_len(w->e);
    uint32_t* st = malloc(sizeof(uint32_t) * w->cap);
    uint32_t* ln = malloc(sizeof(uint32_t) * w->cap);
    uint8_t* dg = malloc((size_t)w->cap * 32);
    gate_wait(w->gate);
    struct timespec c0, c1;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
    for (uint64_t i = (uint64_t)w->tid; i < w->total_calls; i += (uint64_t)w->nthreads) {
        const uint64_t b = i % w->nbuf;
        const uint8_t* buf = w->data + b * w->buf_len;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        int rc;
        if (w->kind == 0) {
            uint32_t n = 0;
            uint32_t* so = w->counts ? w->starts + b * w->cap : st;
            uint32_t* lo = w->counts ? w->lens + b * w->cap : ln;
            uint8_t* dgo = w->counts ? w->digests + b * w->cap * (uint64_t)dl : dg;
            if (w->mode == 1) {
                struct fill_ctx f = {buf, &w->fill_us};
                rc = sdfs_cdc_get_chunks_fill(w->e, SDFS_CDC_NO_STREAM, w->buf_len, copy_fill, &f, so, lo, dgo,
                                              w->cap, &n);
            }
            else if (w->mode == 2)
                rc = sdfs_cdc_get_chunks_stream(w->e, b / 16, buf, w->buf_len, so, lo, dgo, w->cap, &n);
            else
                rc = sdfs_cdc_get_chunks(w->e, buf, w->buf_len, so, lo, dgo, w->cap, &n);
            if (w->counts && rc == 0) w->counts[b] = n;
        } else {
            rc = sdfs_cdc_get_hash(w->e, buf, w->buf_len, w->counts ? w->digests + b * 32 : dg);
        }
        clock_gettime(CLOCK_MONOTONIC, &t1);
        w->lat_us[i] = ts_us(&t0, &t1);
        if (rc && !w->err) w->err = rc;
    }
    clock_gettime(CLOCK_MONOTONIC, &w->end);
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
    w->cpu_us = ts_us(&c0, &c1);
    free(st);
    free(ln);
    free(dg);
    return NULL;
}

static int cmp_d(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : (x > y);
}

static int run(sdfs_cdc_engine* const* hs, int nh, int kind, int mode, int nthreads, const uint8_t* data, uint64_t nbuf,
               uint32_t buf_len, uint64_t total_calls, uint32_t cap, uint32_t* counts, uint32_t* starts,
               uint32_t* lens, uint8_t* digests, sdfs_threads_result* res) {
    if (!hs || nh < 1 || !data || nthreads < 1 || nbuf == 0 || !res || total_calls == 0) return -1;
    res->caller_cpu_us = res->fill_us = 0;
    worker_t* ws = calloc((size_t)nthreads, sizeof(worker_t));
    pthread_t* th = calloc((size_t)nthreads, sizeof(pthread_t));
    double* lat = calloc(total_calls, sizeof(double));
    struct gate g = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0};
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        worker_t* w = &ws[t];
        w->e = hs[t % nh]; /* thread t uses engine handle t mod nh (SDFS: many engine instances) */
        w->kind = kind;
        w->mode = mode;
        w->data = data;
        w->nbuf = nbuf;
        w->buf_len = buf_len;
        w->cap = cap;
        w->nthreads = nthreads;
        w->tid = t;
        w->total_calls = total_calls;
        w->counts = counts;
        w->starts = starts;
        w->lens = lens;
        w->digests = digests;
        w->lat_us = lat;
        w->gate = &g;
        /* small stacks: hundreds of threads like a JVM flush pool */
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setstacksize(&at, 256 * 1024);
        const int ok = pthread_create(&th[t], &at, worker, w) == 0;
        pthread_attr_destroy(&at);
        if (!ok) break;
        started++;
    }
    /* a thread that could not be created leaves its calls undone: the run is reported failed */
    const int rc = started == nthreads ? 0 : -2;
    for (int t = started; t < nthreads; t++) ws[t].err = -2;
    struct timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_mutex_lock(&g.m);
    g.go = 1;
    pthread_cond_broadcast(&g.cv);
    pthread_mutex_unlock(&g.m);
    struct timespec end = t0;
    for (int t = 0; t < nthreads; t++) {
        if (t >= started) {
            if (!res->first_error) res->first_error = -2;
            continue;
        }
        pthread_join(th[t], NULL);
        if (ws[t].end.tv_sec > end.tv_sec || (ws[t].end.tv_sec == end.tv_sec && ws[t].end.tv_nsec > end.tv_nsec))
            end = ws[t].end;
        if (ws[t].err && !res->first_error) res->first_error = ws[t].err;
        res->caller_cpu_us += ws[t].cpu_us;
        res->fill_us += ws[t].fill_us;
    }
    double sum = 0;
    for (uint64_t i = 0; i < total_calls; i++) sum += lat[i];
    qsort(lat, total_calls, sizeof(double), cmp_d);
    res->calls = total_calls;
    res->secs = ts_us(&t0, &end) / 1e6;
    res->gibps = (double)total_calls * buf_len / res->secs / (1024.0 * 1024.0 * 1024.0);
    res->mean_us = sum / (double)total_calls;
    res->p50_us = lat[total_calls / 2];
    res->p90_us = lat[(total_calls * 9) / 10];
    res->p99_us = lat[(total_calls * 99) / 100];
    res->max_us = lat[total_calls - 1];
    free(lat);
    free(th);
    free(ws);
    return rc;
}

/* T threads x getChunks: call i (i < total_calls) takes buffer i % nbuf of data (nbuf buffers of
 * buf_len bytes back to back).  With counts != NULL every buffer's chunk list is kept at
 * starts/lens[b * cap ..], digests[(b * cap + k) * digest_len]. */
int sdfs_threads_getchunks(sdfs_cdc_engine* e, int nthreads, const uint8_t* data, uint64_t nbuf, uint32_t buf_len,
                           uint64_t total_calls, uint32_t cap, uint32_t* counts, uint32_t* starts, uint32_t* lens,
                           uint8_t* digests, sdfs_threads_result* res) {
    if (res) memset(res, 0, sizeof(*res));
    return run(&e, 1, 0, 0, nthreads, data, nbuf, buf_len, total_calls, cap, counts, starts, lens, digests, res);
}

/* The same over nh engine handles (thread t calls through handles[t % nh]) and an entry point
 * (mode: 0 get_chunks, 1 get_chunks_fill, 2 get_chunks_stream). */
int sdfs_threads_getchunks_ex(sdfs_cdc_engine* const* handles, int nh, int mode, int nthreads, const uint8_t* data,
                              uint64_t nbuf, uint32_t buf_len, uint64_t total_calls, uint32_t cap, uint32_t* counts,
                              uint32_t* starts, uint32_t* lens, uint8_t* digests, sdfs_threads_result* res) {
    if (res) memset(res, 0, sizeof(*res));
    return run(handles, nh, 0, mode, nthreads, data, nbuf, buf_len, total_calls, cap, counts, starts, lens, digests,
               res);
}

/* T threads x getHash over the same buffers (digests[b * 32] kept when keep != 0). */
int sdfs_threads_gethash(sdfs_cdc_engine* e, int nthreads, const uint8_t* data, uint64_t nbuf, uint32_t buf_len,
                         uint64_t total_calls, int keep, uint8_t* digests, sdfs_threads_result* res) {
    static uint32_t dummy;
    if (res) memset(res, 0, sizeof(*res));
    return run(&e, 1, 1, 0, nthreads, data, nbuf, buf_len, total_calls, 1, keep ? &dummy : NULL, NULL, NULL, digests,
               res);
}
