/*
 * cdc_ref.c — CPU ORACLE (test infrastructure only; see cdc_ref.h for the rules and the
 * reference file:line anchors).  Scalar, byte-at-a-time, written to mirror the Java
 * reference's control flow rather than to be fast: the GPU path is checked against this.
 */
#include "cdc_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void cdc_ref_default_params(cdc_ref_params* p) {
    memset(p, 0, sizeof(*p));
    p->poly = 10923124345206883ULL; /* VariableSha256HashEngine.java:41 */
    p->window = 48;                 /* HashFunctionPool.java:51, VolumeConfigWriter.java:97 */
    p->min_len = 4 * 1024 - 1;      /* Main.java:189, Config.java:145-148 */
    p->max_len = 32 * 1024;         /* VolumeConfigWriter.java:96 -> Config.java:162-166 */
    p->min_cmp = CDC_REF_MIN_GT;    /* SURVEY.md A.3 (inferred from blankBlock = minLen+1) */
    p->pred_mask = 0xFFF;           /* BitmaskBoundaryDetector, 12 bits ... */
    p->pred_value = 0;              /* ... pattern 0 (fp == 0 on zero data -> 4096-B chunks) */
    p->hash_algo = CDC_REF_SHA256;  /* VolumeConfigWriter.java:109 VARIABLE_SHA256 */
}

int cdc_ref_poly_degree(uint64_t poly) {
    if (poly == 0) return -1;
    return 63 - __builtin_clzll(poly);
}

/* (v * x) mod P for deg(v) < d: GF(2) shift-and-reduce. */
static inline uint64_t mulx_mod(uint64_t v, uint64_t poly, int d) {
    v <<= 1;
    if ((v >> d) & 1) v ^= poly;
    return v;
}

/* RabinFingerprintLong.precomputePushTable / RabinFingerprintLongWindowed.precomputePopTable
 * (rabinwindow jar): push[i] = (i*x^d) XOR ((i*x^d) mod P), i < 512;
 * pop[i] = (i*x^(8W)) mod P, i < 256. */
int cdc_ref_tables(uint64_t poly, uint32_t window, uint64_t* push, uint64_t* pop) {
    const int d = cdc_ref_poly_degree(poly);
    if (d < 9 || d > 55) return -1; /* fp<<8 must fit 64 bits and the index must be 9 bits */
    for (uint64_t i = 0; i < 512; i++) {
        uint64_t v = i;
        /* i has degree < 9 <= d, but reduce in steps so every intermediate has degree < d */
        uint64_t r = 0;
        for (int bit = 8; bit >= 0; bit--) {
            r = mulx_mod(r, poly, d);
            if ((v >> bit) & 1) r ^= 1;
        }
        /* r = i mod P (= i when d > 8); now multiply by x^d */
        for (int k = 0; k < d; k++) r = mulx_mod(r, poly, d);
        push[i] = (i << d) ^ r;
    }
    for (uint64_t i = 0; i < 256; i++) {
        uint64_t r = i;
        for (uint32_t k = 0; k < 8 * window; k++) r = mulx_mod(r, poly, d);
        pop[i] = r;
    }
    return 0;
}

/* One engine instance's rolling state: RabinFingerprintLongWindowed (window fp only; the
 * second, whole-chunk fingerprint is passed to visit() but ignored by SDFS,
 * VariableSha256HashEngine.java:74-82, so it is not computed). */
typedef struct {
    uint64_t push[512], pop[256];
    uint64_t fp;
    int shift;
    uint32_t window;
    uint8_t* ring; /* window + 1 byte FIFO (CircularByteQueue(bytesPerWindow + 1)) */
    uint32_t head, count;
} rabin_win;

static int rabin_init(rabin_win* r, uint64_t poly, uint32_t window) {
    if (cdc_ref_tables(poly, window, r->push, r->pop) != 0 || window == 0) return -1;
    r->shift = cdc_ref_poly_degree(poly) - 8;
    r->window = window;
    r->ring = (uint8_t*)calloc(window + 1, 1);
    r->fp = 0;
    r->head = r->count = 0;
    return r->ring ? 0 : -1;
}
static void rabin_free(rabin_win* r) { free(r->ring); }

/* pushByte: fp = ((fp << 8) | b) ^ push[(fp >> shift) & 0x1FF]; byteWindow.add(b);
 * if (byteWindow.isFull()) popByte()  ->  fp ^= pop[oldest]. */
static inline void rabin_push(rabin_win* r, uint8_t b) {
    const uint32_t j = (uint32_t)((r->fp >> r->shift) & 0x1FF);
    r->fp = ((r->fp << 8) | b) ^ r->push[j];
    const uint32_t cap = r->window + 1;
    r->ring[(r->head + r->count) % cap] = b;
    r->count++;
    if (r->count == cap) {
        const uint8_t o = r->ring[r->head];
        r->head = (r->head + 1) % cap;
        r->count--;
        r->fp ^= r->pop[o];
    }
}

int cdc_ref_window_fps(uint64_t poly, uint32_t window, const uint8_t* buf, size_t len, uint64_t* out) {
    rabin_win r;
    if (rabin_init(&r, poly, window) != 0) return -1;
    for (size_t k = 0; k < len; k++) {
        rabin_push(&r, buf[k]);
        out[k] = r.fp;
    }
    rabin_free(&r);
    return 0;
}

/* ---------------- SHA-256 (FIPS 180-4), own code ---------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_compress(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        const uint32_t s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        const uint32_t S1 = ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        const uint32_t S0 = ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void cdc_ref_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) sha256_compress(st, data + i);
    uint8_t tail[128];
    const size_t rem = len - i;
    memset(tail, 0, sizeof(tail));
    memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = (rem < 56) ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha256_compress(st, tail);
    if (tl == 128) sha256_compress(st, tail + 64);
    for (int k = 0; k < 8; k++) {
        out[4 * k] = (uint8_t)(st[k] >> 24);
        out[4 * k + 1] = (uint8_t)(st[k] >> 16);
        out[4 * k + 2] = (uint8_t)(st[k] >> 8);
        out[4 * k + 3] = (uint8_t)st[k];
    }
}

/* ---------------- MD5 (RFC 1321), own code ---------------- */
static const uint32_t KMD5[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const int RMD5[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                             5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                             4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                             6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_compress(uint32_t st[4], const uint8_t blk[64]) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) |
               ((uint32_t)blk[4 * i + 2] << 16) | ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        const uint32_t t = a + f + KMD5[i] + m[g];
        a = d; d = c; c = b;
        b = b + ((t << RMD5[i]) | (t >> (32 - RMD5[i])));
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

void cdc_ref_md5(const uint8_t* data, size_t len, uint8_t out[16]) {
    uint32_t st[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) md5_compress(st, data + i);
    uint8_t tail[128];
    const size_t rem = len - i;
    memset(tail, 0, sizeof(tail));
    memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = (rem < 56) ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; k++) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
    md5_compress(st, tail);
    if (tl == 128) md5_compress(st, tail + 64);
    for (int k = 0; k < 4; k++)
        for (int j = 0; j < 4; j++) out[4 * k + j] = (uint8_t)(st[k] >> (8 * j));
}

size_t cdc_ref_digest_len(uint32_t hash_algo) {
    switch (hash_algo) {
    case CDC_REF_SHA256: return 32;
    case CDC_REF_SHA256_160: return 20; /* VariableSha256HashEngine.java:60-65 */
    case CDC_REF_MD5: return 16;
    default: return 0;
    }
}

void cdc_ref_hash(uint32_t hash_algo, const uint8_t* data, size_t len, uint8_t* out) {
    uint8_t tmp[32];
    switch (hash_algo) {
    case CDC_REF_SHA256: cdc_ref_sha256(data, len, out); break;
    case CDC_REF_SHA256_160: cdc_ref_sha256(data, len, tmp); memcpy(out, tmp, 20); break;
    case CDC_REF_MD5: cdc_ref_md5(data, len, out); break;
    default: break;
    }
}

/* ---------------- chunking loop ---------------- */
long cdc_ref_chunk(const cdc_ref_params* p, const uint8_t* buf, size_t len, uint32_t* starts,
                   uint32_t* lens, uint8_t* digests, size_t cap) {
    const size_t dl = cdc_ref_digest_len(p->hash_algo);
    if (dl == 0 || p->max_len == 0) return -1;
    rabin_win r;
    if (rabin_init(&r, p->poly, p->window) != 0) return -1;
    long count = 0;
    size_t start = 0, n = 0; /* window state is reset once per call, never per cut */
    for (size_t k = 0; k < len; k++) {
        rabin_push(&r, buf[k]);
        n++;
        const int min_ok = (p->min_cmp == CDC_REF_MIN_GE) ? (n >= p->min_len) : (n > p->min_len);
        const int boundary = cdc_ref_is_boundary(p, r.fp);
        if ((min_ok && boundary) || n >= p->max_len) {
            if ((size_t)count >= cap) { rabin_free(&r); return -1; }
            starts[count] = (uint32_t)start;
            lens[count] = (uint32_t)n;
            if (digests) cdc_ref_hash(p->hash_algo, buf + start, n, digests + (size_t)count * dl);
            count++;
            start = k + 1;
            n = 0;
        }
    }
    if (n > 0) { /* final (tail) chunk; a zero-length tail is never emitted (HashLocPair.java:66-68) */
        if ((size_t)count >= cap) { rabin_free(&r); return -1; }
        starts[count] = (uint32_t)start;
        lens[count] = (uint32_t)n;
        if (digests) cdc_ref_hash(p->hash_algo, buf + start, n, digests + (size_t)count * dl);
        count++;
    }
    rabin_free(&r);
    return count;
}

/* ---------------- batch + threads ---------------- */
typedef struct {
    const cdc_ref_params* p;
    const uint8_t* base;
    const uint64_t* offs;
    const uint32_t* lens;
    uint32_t* counts;
    uint32_t* starts;
    uint32_t* lens_out;
    uint8_t* digests;
    uint32_t cap;
    uint32_t b0, b1;
    long total;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    const size_t dl = cdc_ref_digest_len(j->p->hash_algo);
    j->total = 0;
    for (uint32_t b = j->b0; b < j->b1; b++) {
        const size_t slot = (size_t)b * j->cap;
        long c = cdc_ref_chunk(j->p, j->base + j->offs[b], j->lens[b], j->starts + slot,
                               j->lens_out + slot, j->digests ? j->digests + slot * dl : NULL, j->cap);
        if (c < 0) { j->total = -1; return NULL; }
        j->counts[b] = (uint32_t)c;
        j->total += c;
    }
    return NULL;
}

long cdc_ref_chunk_batch(const cdc_ref_params* p, const uint8_t* base, const uint64_t* offs,
                         const uint32_t* lens, uint32_t nbuf, uint32_t* counts, uint32_t* starts,
                         uint32_t* lens_out, uint8_t* digests, uint32_t cap, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > nbuf) nthreads = nbuf ? (int)nbuf : 1;
    pthread_t th[256];
    batch_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (batch_job){p, base, offs, lens, counts, starts, lens_out, digests, cap,
                              (uint32_t)((uint64_t)nbuf * t / nthreads),
                              (uint32_t)((uint64_t)nbuf * (t + 1) / nthreads), 0};
        if (nthreads == 1) batch_worker(&jobs[0]);
        else pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    long total = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].total < 0) total = -1;
        if (total >= 0) total += jobs[t].total;
    }
    return total;
}

/* ---------------- synthetic input ---------------- */
uint64_t cdc_ref_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* byte `o` of stream `s` = little-endian byte (o % 8) of
 * splitmix64(key + o/8), key = splitmix64(seed ^ (s * 0xD1B54A32D192ED03)). */
void cdc_ref_synth(uint64_t seed, uint64_t stream, uint64_t offset, uint8_t* out, size_t n) {
    const uint64_t key = cdc_ref_splitmix64(seed ^ (stream * 0xD1B54A32D192ED03ULL));
    for (size_t i = 0; i < n; i++) {
        const uint64_t o = offset + i;
        const uint64_t w = cdc_ref_splitmix64(key + (o >> 3));
        out[i] = (uint8_t)(w >> (8 * (o & 7)));
    }
}

typedef struct {
    const cdc_ref_params* p;
    uint64_t seed, stream0;
    uint32_t bps, b0, b1, buf_len;
    double secs;
    uint64_t chunks, bytes;
} synth_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* synth_worker(void* arg) {
    synth_job* j = (synth_job*)arg;
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
        cdc_ref_synth(j->seed, stream, off, buf, j->buf_len);
        const double t0 = now_s();
        long c = cdc_ref_chunk(j->p, buf, j->buf_len, st, ln, dg, cap);
        j->secs += now_s() - t0;
        if (c > 0) j->chunks += (uint64_t)c;
        j->bytes += j->buf_len;
    }
    free(buf); free(st); free(ln); free(dg);
    return NULL;
}

double cdc_ref_bench_synth(const cdc_ref_params* p, uint64_t seed, uint64_t stream0,
                           uint32_t buffers_per_stream, uint32_t nbuf, uint32_t buf_len,
                           int nthreads, uint64_t* total_chunks, uint64_t* total_bytes) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (buffers_per_stream == 0) buffers_per_stream = 1;
    pthread_t th[256];
    synth_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (synth_job){p, seed, stream0, buffers_per_stream,
                              (uint32_t)((uint64_t)nbuf * t / nthreads),
                              (uint32_t)((uint64_t)nbuf * (t + 1) / nthreads), buf_len, 0, 0, 0};
        pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
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
    return worst; /* slowest thread's chunking time = the parallel wall time of the work */
}
