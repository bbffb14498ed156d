/*
 * cdc_fast.c — fast CPU form of the oracle, for bench.py's cpu_baseline leg and its own parity
 * test against cdc_ref.c.  TEST INFRASTRUCTURE ONLY (same rules as cdc_ref.h: never linked or
 * called by the product path).
 *
 * Same semantics as cdc_ref_chunk (VariableSha256HashEngine.java:71-86), made
 * representative of what the reference's CPU path would achieve on the GPU box:
 *   - the rolling hash reads the outgoing byte straight from the buffer (b[k-W]) instead of a
 *     FIFO, one 256-entry push and one pop table lookup per byte;
 *   - fingerprints go through OpenSSL's EVP SHA-256 / MD5, which dispatches to the SHA
 *     extensions (SHA-NI) on x86 — what HotSpot's SHA intrinsic uses under Guava
 *     Hashing.sha256() -> MessageDigest (VariableSha256HashEngine.java:45,58-67).
 * It is still a C restatement, not the Java reference (no JDK or jars in this image).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cdc_ref.h"

typedef struct {
    uint64_t push[256], pop[256];
    int shift;
    const EVP_MD* md;
} fast_ctx;

static int ctx_init(fast_ctx* c, const cdc_ref_params* p) {
    uint64_t push[512];
    if (cdc_ref_tables(p->poly, p->window, push, c->pop) != 0) return -1;
    memcpy(c->push, push, sizeof(c->push));  /* fp < 2^d: bit 8 of the push index is always 0 */
    c->shift = cdc_ref_poly_degree(p->poly) - 8;
    c->md = p->hash_algo == CDC_REF_MD5 ? EVP_md5() : EVP_sha256();
    return 0;
}

static void digest(const fast_ctx* c, uint32_t algo, const uint8_t* d, size_t n, uint8_t* out) {
    uint8_t full[EVP_MAX_MD_SIZE];
    EVP_Digest(d, n, full, NULL, c->md, NULL);
    memcpy(out, full, cdc_ref_digest_len(algo));
}

static long chunk_ctx(const fast_ctx* c, const cdc_ref_params* p, const uint8_t* buf, size_t len, uint32_t* starts,
                      uint32_t* lens, uint8_t* digests, size_t cap) {
    const size_t dl = cdc_ref_digest_len(p->hash_algo);
    const size_t W = p->window;
    const size_t first = p->min_cmp == CDC_REF_MIN_GE ? (p->min_len ? p->min_len - 1 : 0) : p->min_len;
    uint64_t fp = 0;
    long count = 0;
    size_t start = 0;
    size_t k = 0;
    while (k < len) {
        /* the chunk starting at `start` can end no earlier than start + first and no later than
         * start + max_len - 1 (or the buffer end); roll through the rest without testing */
        const size_t lo = start + first;
        size_t hi = start + p->max_len - 1;
        if (hi > len - 1) hi = len - 1;
        size_t cut = hi;
        for (; k < len; k++) {
            fp = ((fp << 8) | buf[k]) ^ c->push[(fp >> c->shift) & 0xFF];
            if (k >= W) fp ^= c->pop[buf[k - W]];
            if (k >= lo && cdc_ref_is_boundary(p, fp)) {
                cut = k;
                break;
            }
            if (k == hi) break; /* forced cut at max_len, or the tail chunk */
        }
        if ((size_t)count >= cap) return -1;
        starts[count] = (uint32_t)start;
        lens[count] = (uint32_t)(cut + 1 - start);
        if (digests) digest(c, p->hash_algo, buf + start, cut + 1 - start, digests + (size_t)count * dl);
        count++;
        start = cut + 1;
        k = cut + 1;
    }
    return count;
}

long cdc_fast_chunk(const cdc_ref_params* p, const uint8_t* buf, size_t len, uint32_t* starts, uint32_t* lens,
                    uint8_t* digests, size_t cap) {
    fast_ctx c;
    if (p->max_len == 0 || ctx_init(&c, p) != 0) return -1;
    return chunk_ctx(&c, p, buf, len, starts, lens, digests, cap);
}

typedef struct {
    const cdc_ref_params* p;
    const fast_ctx* c;
    uint64_t seed, stream0;
    uint32_t bps, b0, b1, buf_len;
    double secs;
    uint64_t chunks, bytes;
} job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    uint8_t* buf = (uint8_t*)malloc(j->buf_len);
    const size_t dl = cdc_ref_digest_len(j->p->hash_algo);
    uint32_t shortest = j->p->min_len < j->p->max_len ? j->p->min_len : j->p->max_len;
    if (shortest == 0) shortest = 1;
    const size_t cap = (size_t)j->buf_len / shortest + 2;
    uint32_t* st = (uint32_t*)malloc(cap * 4);
    uint32_t* ln = (uint32_t*)malloc(cap * 4);
    uint8_t* dg = (uint8_t*)malloc(cap * dl);
    j->secs = 0;
    j->chunks = j->bytes = 0;
    for (uint32_t b = j->b0; b < j->b1; b++) {
        const uint64_t stream = j->stream0 + b / j->bps;
        const uint64_t off = (uint64_t)(b % j->bps) * j->buf_len;
        cdc_ref_synth(j->seed, stream, off, buf, j->buf_len); /* generation is not timed */
        const double t0 = now_s();
        const long c = chunk_ctx(j->c, j->p, buf, j->buf_len, st, ln, dg, cap);
        j->secs += now_s() - t0;
        if (c > 0) j->chunks += (uint64_t)c;
        j->bytes += j->buf_len;
    }
    free(buf);
    free(st);
    free(ln);
    free(dg);
    return NULL;
}

/* Same contract as cdc_ref_bench_synth: the slowest thread's summed chunk+hash time. */
double cdc_fast_bench_synth(const cdc_ref_params* p, uint64_t seed, uint64_t stream0, uint32_t buffers_per_stream,
                            uint32_t nbuf, uint32_t buf_len, int nthreads, uint64_t* total_chunks,
                            uint64_t* total_bytes) {
    fast_ctx c;
    if (ctx_init(&c, p) != 0) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 512) nthreads = 512;
    if (buffers_per_stream == 0) buffers_per_stream = 1;
    pthread_t th[512];
    job_t jobs[512];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (job_t){p, &c, seed, stream0, buffers_per_stream, (uint32_t)((uint64_t)nbuf * t / nthreads),
                          (uint32_t)((uint64_t)nbuf * (t + 1) / nthreads), buf_len, 0, 0, 0};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    double worst = 0;
    uint64_t ch = 0, by = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].secs > worst) worst = jobs[t].secs;
        ch += jobs[t].chunks;
        by += jobs[t].bytes;
    }
    if (total_chunks) *total_chunks = ch;
    if (total_bytes) *total_bytes = by;
    return worst;
}
