/*
 * lz4_ref.c — CPU ORACLE for LZ4 block compression of unique chunks.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the benches' CPU-baseline
 * legs may load this library, and only as the checker / the timed CPU baseline.  The product
 * path (sdfs_amd/, libsdfs_cdc.so) never links or calls it.
 *
 * Reference call sites: HashBlobArchive.putChunk (HashBlobArchive.java:1281-1289) stores a new
 * chunk as [int nz = chunk.length, big-endian ByteBuffer.putInt][CompressionUtils.compressLz4(chunk)]
 * when Main.compress is set (on for --backup-volume, VolumeConfigWriter.java:300, and for the
 * cloud stores); the read side is HashBlobArchive.java:1927-1933.  compressLz4 is
 * lz4Compressor.compress(input) (CompressionUtils.java:118-120) with lz4Compressor =
 * LZ4Factory.nativeInstance().fastCompressor() (CompressionUtils.java:52-53): third-party
 * net.jpountz.lz4:lz4:1.3.0 (pom.xml:158-162), ABSENT from /root/reference and from this image.
 * Its native fast compressor is the C LZ4 it bundles (r123): LZ4_compress_limitedOutput(src,
 * dst, n, LZ4_compressBound(n)) = LZ4_compress_generic with a 2^13-entry table of 16-bit
 * positions for n < 64 KiB + 11 and a 2^12-entry table of 32-bit positions above.
 *
 * This file restates that published algorithm (LZ4 block format: token, literal run, 16-bit
 * little-endian offset, match run; MINMATCH 4, MFLIMIT 12, LASTLITERALS 5, skip trigger 6) as a
 * plain byte-serial loop, with the two places where later LZ4 releases changed the emitted bytes
 * as an explicit mode:
 *   LZ4_REF_R123 — lz4-java 1.3.0's bundled r123: the match search stops once the next probe
 *                  position passes iend - MFLIMIT; 32-bit tables hash 4 bytes.
 *   LZ4_REF_V19  — LZ4 1.9.x LZ4_compress_default (acceleration 1): the search may probe one
 *                  position further (mflimitPlusOne); 32-bit tables hash 5 bytes (64-bit hosts).
 * PARITY STATUS: the V19 mode is pinned byte for byte against the system liblz4 (1.9.3) by
 * tests/test_lz4.py; the R123 mode shares every other line with it and differs exactly in the
 * two rules above, restated from the r123 source — no r123 binary or fixture exists here, so
 * those two rules are "parity unpinned".  Both modes' outputs are checked to decode to the input.
 */
#include "lz4_ref.h"

#include <string.h>

#define MINMATCH 4
#define MFLIMIT 12
#define LASTLITERALS 5
#define ML_BITS 4
#define ML_MASK ((1U << ML_BITS) - 1)
#define RUN_MASK ((1U << (8 - ML_BITS)) - 1)
#define SKIP_TRIGGER 6
#define LIMIT_64K (65536 + (MFLIMIT - 1))
#define MAX_DISTANCE 65535

static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

/* Table index of the sequence at p: 16-bit table -> 13 bits of a 4-byte multiplicative hash;
 * 32-bit table -> 12 bits of the 4-byte hash (r123) or of the 5-byte hash (1.9.x, 64-bit). */
static uint32_t hash_at(const uint8_t* p, int u16, int mode) {
    if (u16) return (rd32(p) * 2654435761U) >> (32 - 13);
    if (mode == LZ4_REF_V19) return (uint32_t)(((rd64(p) << 24) * 889523592379ULL) >> (64 - 12));
    return (rd32(p) * 2654435761U) >> (32 - 12);
}

uint32_t lz4_ref_bound(uint32_t n) { return n + n / 255 + 16; }

/* run of `len` as 255-bytes and a remainder byte (length fields past the 4-bit token nibble) */
static uint32_t put_run(uint8_t* dst, uint32_t op, uint32_t len) {
    for (; len >= 255; len -= 255) dst[op++] = 255;
    dst[op++] = (uint8_t)len;
    return op;
}

long lz4_ref_compress(int mode, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap) {
    if (cap < lz4_ref_bound(n)) return -1;
    uint32_t table[1 << 13];
    memset(table, 0, sizeof(table));
    const int u16 = n < LIMIT_64K;
    const uint32_t mflimit = n >= MFLIMIT ? n - MFLIMIT : 0;
    const uint32_t search_end = mode == LZ4_REF_V19 ? mflimit + 1 : mflimit;
    const uint32_t matchlimit = n >= LASTLITERALS ? n - LASTLITERALS : 0;
    uint32_t ip = 0, anchor = 0, op = 0;

    if (n < MFLIMIT + 1) goto last_literals;
    table[hash_at(src, u16, mode)] = 0;
    ip = 1;
    uint32_t fh = hash_at(src + ip, u16, mode);
    for (;;) {
        uint32_t match;
        {   /* find a match: probe ip, ip+1, ... with a step that grows by one every 64 misses */
            uint32_t fip = ip, step = 1, nb = 1u << SKIP_TRIGGER;
            for (;;) {
                const uint32_t h = fh;
                ip = fip;
                fip += step;
                step = nb++ >> SKIP_TRIGGER;
                if (fip > search_end) goto last_literals;
                match = table[h];
                fh = hash_at(src + fip, u16, mode);
                table[h] = ip;
                if (!u16 && match + MAX_DISTANCE < ip) continue;
                if (rd32(src + match) == rd32(src + ip)) break;
            }
        }
        /* catch up: extend the match backwards over equal bytes */
        while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
            ip--;
            match--;
        }
        /* literal run */
        uint32_t token = op++;
        {
            const uint32_t lit = ip - anchor;
            if (lit >= RUN_MASK) {
                dst[token] = (uint8_t)(RUN_MASK << ML_BITS);
                op = put_run(dst, op, lit - RUN_MASK);
            } else {
                dst[token] = (uint8_t)(lit << ML_BITS);
            }
            memcpy(dst + op, src + anchor, lit);
            op += lit;
        }
        for (;;) { /* a match, possibly followed at once by another one */
            const uint32_t off = ip - match;
            dst[op++] = (uint8_t)off;
            dst[op++] = (uint8_t)(off >> 8);
            uint32_t a = ip + MINMATCH, b = match + MINMATCH;
            while (a < matchlimit && src[a] == src[b]) {
                a++;
                b++;
            }
            uint32_t ml = a - (ip + MINMATCH);
            ip = a;
            if (ml >= ML_MASK) {
                dst[token] += ML_MASK;
                op = put_run(dst, op, ml - ML_MASK);
            } else {
                dst[token] += (uint8_t)ml;
            }
            anchor = ip;
            if (ip > mflimit) goto last_literals;
            /* fill the table at ip-2, then test an immediate match at ip */
            table[hash_at(src + ip - 2, u16, mode)] = ip - 2;
            const uint32_t h = hash_at(src + ip, u16, mode);
            match = table[h];
            table[h] = ip;
            if ((u16 || match + MAX_DISTANCE >= ip) && rd32(src + match) == rd32(src + ip)) {
                token = op++;
                dst[token] = 0;
                continue;
            }
            break;
        }
        fh = hash_at(src + ++ip, u16, mode);
    }

last_literals: {
    const uint32_t last = n - anchor;
    if (last >= RUN_MASK) {
        dst[op++] = (uint8_t)(RUN_MASK << ML_BITS);
        op = put_run(dst, op, last - RUN_MASK);
    } else {
        dst[op++] = (uint8_t)(last << ML_BITS);
    }
    memcpy(dst + op, src + anchor, last);
    op += last;
}
    return (long)op;
}

long lz4_ref_decompress(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap) {
    uint32_t ip = 0, op = 0;
    for (;;) {
        if (ip >= n) return -1;
        const uint32_t token = src[ip++];
        uint32_t lit = token >> ML_BITS;
        if (lit == RUN_MASK) {
            uint32_t s;
            do {
                if (ip >= n) return -1;
                s = src[ip++];
                lit += s;
            } while (s == 255);
        }
        if (ip + lit > n || op + lit > cap) return -1;
        memcpy(dst + op, src + ip, lit);
        ip += lit;
        op += lit;
        if (ip == n) return (long)op; /* the last sequence carries literals only */
        if (ip + 2 > n) return -1;
        const uint32_t off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
        ip += 2;
        if (off == 0 || off > op) return -1;
        uint32_t ml = token & ML_MASK;
        if (ml == ML_MASK) {
            uint32_t s;
            do {
                if (ip >= n) return -1;
                s = src[ip++];
                ml += s;
            } while (s == 255);
        }
        ml += MINMATCH;
        if (op + ml > cap) return -1;
        for (uint32_t k = 0; k < ml; k++, op++) dst[op] = dst[op - off]; /* may overlap */
    }
}

long lz4_ref_compress_framed(int mode, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap) {
    if (cap < 4) return -1;
    dst[0] = (uint8_t)(n >> 24);
    dst[1] = (uint8_t)(n >> 16);
    dst[2] = (uint8_t)(n >> 8);
    dst[3] = (uint8_t)n;
    const long k = lz4_ref_compress(mode, src, n, dst + 4, cap - 4);
    return k < 0 ? k : k + 4;
}

/* ---- batch over threads (the timed CPU baseline of scripts/lz4_bench.py) ---- */
#include <pthread.h>

typedef struct {
    int mode;
    const uint8_t* base;
    const uint64_t* offs;
    const uint32_t* lens;
    uint8_t* out;
    const uint64_t* out_offs;
    uint32_t* out_lens;
    uint32_t i0, i1;
    int failed;
} lz4_job;

static void* lz4_worker(void* arg) {
    lz4_job* j = (lz4_job*)arg;
    for (uint32_t i = j->i0; i < j->i1; i++) {
        const long k = lz4_ref_compress_framed(j->mode, j->base + j->offs[i], j->lens[i], j->out + j->out_offs[i],
                                               lz4_ref_bound(j->lens[i]) + 4);
        if (k < 0) j->failed = 1;
        j->out_lens[i] = (uint32_t)(k < 0 ? 0 : k);
    }
    return NULL;
}

long lz4_ref_compress_batch(int mode, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                            uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    lz4_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (lz4_job){mode, base, offs, lens, out, out_offs, out_lens,
                            (uint32_t)((uint64_t)n * t / nthreads), (uint32_t)((uint64_t)n * (t + 1) / nthreads), 0};
        pthread_create(&th[t], NULL, lz4_worker, &jobs[t]);
    }
    long total = 0;
    int failed = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        failed |= jobs[t].failed;
    }
    if (failed) return -1;
    for (uint32_t i = 0; i < n; i++) total += out_lens[i];
    return total;
}
