/* CPU baseline for the LZ4 row (scripts/lz4_bench.py) — TEST INFRASTRUCTURE ONLY: the image's
 * own liblz4 (1.9.x, dlopen'd; the optimised C codec the reference's lz4-java JNI binding is a
 * build of, HashBlobArchive.java:1283-1289 / 1927-1933) compressing or decoding a batch of
 * chunks on N pthreads.  Never part of the product path. */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdatomic.h>

typedef int (*lz4_fn)(const char* src, char* dst, int n, int cap);

struct sys_job {
    lz4_fn fn;
    const uint8_t* base;
    const uint64_t* offs;
    const uint32_t* lens;
    uint8_t* out;
    const uint64_t* out_offs;
    const uint32_t* out_caps;
    uint32_t* out_lens;
    uint32_t n;
    atomic_uint next;
    atomic_int bad;
};

static void* sys_worker(void* arg) {
    struct sys_job* j = (struct sys_job*)arg;
    for (;;) {
        const uint32_t i = atomic_fetch_add(&j->next, 1u);
        if (i >= j->n) return NULL;
        const int k = j->fn((const char*)j->base + j->offs[i], (char*)j->out + j->out_offs[i], (int)j->lens[i],
                            (int)j->out_caps[i]);
        if (k < 0) atomic_store(&j->bad, 1);
        j->out_lens[i] = (uint32_t)k;
    }
}

/* decompress = 0: LZ4_compress_default (out_caps = room per chunk); 1: LZ4_decompress_safe
 * (out_caps = the decoded length).  Returns 0, -1 without a liblz4, -2 on a codec error. */
long lz4_sys_batch(int decompress, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                   uint8_t* out, const uint64_t* out_offs, const uint32_t* out_caps, uint32_t* out_lens,
                   int nthreads) {
    static void* h = NULL;
    if (!h) h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    lz4_fn fn = (lz4_fn)dlsym(h, decompress ? "LZ4_decompress_safe" : "LZ4_compress_default");
    if (!fn) return -1;
    struct sys_job j = {fn, base, offs, lens, out, out_offs, out_caps, out_lens, n, 0, 0};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    int started = 0;
    for (int t = 0; t < nthreads; t++)
        if (pthread_create(&th[t], NULL, sys_worker, &j) == 0) started++;
    if (!started) sys_worker(&j);
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    return atomic_load(&j.bad) ? -2 : 0;
}
