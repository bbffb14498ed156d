/*
 * cdc_ref.h — CPU ORACLE for the SDFS variable-block CDC + fingerprint path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (sdfs_amd/, libsdfs_cdc.so) never links or calls it.
 *
 * What it restates:
 *   - VariableSha256HashEngine.getChunks        src/org/opendedup/hashing/VariableSha256HashEngine.java:71-86
 *   - VariableSha256HashEngine.getHash          .../VariableSha256HashEngine.java:58-67 (HASH256 / HASH160)
 *   - VariableMD5HashEngine.getHash             .../VariableMD5HashEngine.java:55-58
 *   - EnhancedFingerFactory.getChunkFingerprints + RabinFingerprintLong[Windowed] +
 *     BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR: third-party jar
 *     org.opendedupe:rabinwindow:1.0.2 (pom.xml:92-96), ABSENT from /root/reference and from
 *     this container.  Its published algorithm (upstream org.rabinfingerprint) is restated
 *     from SURVEY.md A.2/A.3; every unverifiable choice is a knob in cdc_ref_params.
 *   - SHA-256 (FIPS 180-4) and MD5 (RFC 1321), which Guava 30.1.1 Hashing.sha256()/md5()
 *     wrap (pom.xml:142-147).  Own implementations; pinned by the standards' vectors.
 *
 * PARITY STATUS: digests pinned (FIPS/RFC vectors + the reference's blank-chunk constants,
 * WritableCacheBuffer.java:93-94, HashStore.java:63-71); rolling-hash arithmetic pinned by
 * the GF(2) definition (tests/test_oracle.py); chunk BOUNDARIES "parity unpinned" — no
 * reference test or fixture pins the jar's predicate constants / min comparison / tail rule.
 */
#ifndef SDFS_CDC_REF_H
#define SDFS_CDC_REF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CDC_REF_SHA256 = 0, CDC_REF_SHA256_160 = 1, CDC_REF_MD5 = 2 };
enum { CDC_REF_MIN_GT = 0, CDC_REF_MIN_GE = 1 };
enum { CDC_REF_PRED_MASK = 0, CDC_REF_PRED_DIV = 1 };

typedef struct cdc_ref_params {
    uint64_t poly;       /* Polynomial.createFromLong(10923124345206883L): bit i = coeff of x^i */
    uint32_t window;     /* HashFunctionPool.bytesPerWindow (48) */
    uint32_t min_len;    /* HashFunctionPool.minLen (4095) */
    uint32_t max_len;    /* HashFunctionPool.maxLen (32768 / 131072 backup) */
    uint32_t min_cmp;    /* CDC_REF_MIN_GT: cut needs n > min_len (default); _GE: n >= min_len */
    uint64_t pred_mask;  /* boundary predicate: (fp & mask) == value  (default 0xFFF, 0) */
    uint64_t pred_value;
    uint32_t hash_algo;  /* CDC_REF_SHA256 / _SHA256_160 / _MD5 */
    uint32_t pred_kind;  /* CDC_REF_PRED_MASK: (fp & pred_mask) == pred_value (default);
                            CDC_REF_PRED_DIV: fp % pred_div == pred_rem (SURVEY.md A.3's other
                            candidate form of BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR) */
    uint64_t pred_div;   /* divisor D >= 1 (CDC_REF_PRED_DIV) */
    uint64_t pred_rem;   /* target remainder R (Java long %: fp >= 0, so R >= D never matches) */
} cdc_ref_params;

/* The boundary predicate on one window fingerprint. */
static inline int cdc_ref_is_boundary(const cdc_ref_params* p, uint64_t fp) {
    return p->pred_kind == CDC_REF_PRED_DIV ? (p->pred_div != 0 && fp % p->pred_div == p->pred_rem)
                                            : (fp & p->pred_mask) == p->pred_value;
}

void cdc_ref_default_params(cdc_ref_params* p);
int cdc_ref_poly_degree(uint64_t poly);
/* push[512], pop[256] exactly as SURVEY.md A.2 defines them. Returns 0, <0 on bad poly. */
int cdc_ref_tables(uint64_t poly, uint32_t window, uint64_t* push, uint64_t* pop);
/* Window fingerprint after each byte of buf (rolling, byte at a time, FIFO of W+1). */
int cdc_ref_window_fps(uint64_t poly, uint32_t window, const uint8_t* buf, size_t len, uint64_t* out);

size_t cdc_ref_digest_len(uint32_t hash_algo);
void cdc_ref_sha256(const uint8_t* data, size_t len, uint8_t out[32]);
void cdc_ref_md5(const uint8_t* data, size_t len, uint8_t out[16]);
void cdc_ref_hash(uint32_t hash_algo, const uint8_t* data, size_t len, uint8_t* out);

/* getChunks on one buffer: fills starts/lens (+ digests, digest_len(algo) bytes each, may be
 * NULL) up to cap entries.  Returns the chunk count, or -1 if cap is too small / bad params. */
long cdc_ref_chunk(const cdc_ref_params* p, const uint8_t* buf, size_t len, uint32_t* starts,
                   uint32_t* lens, uint8_t* digests, size_t cap);

/* Batch of buffers (offsets into base), each chunked from fresh state, nthreads pthreads.
 * Per-buffer slots of `cap` entries; counts[b] = chunk count.  Returns total chunks or -1. */
long cdc_ref_chunk_batch(const cdc_ref_params* p, const uint8_t* base, const uint64_t* offs,
                         const uint32_t* lens, uint32_t nbuf, uint32_t* counts, uint32_t* starts,
                         uint32_t* lens_out, uint8_t* digests, uint32_t cap, int nthreads);

/* CPU-baseline driver: generate+chunk `nbuf` synthetic buffers of buf_len bytes (streams
 * stream0.., seed) on nthreads threads, timing only the chunk+hash work.  Returns seconds of
 * summed per-thread chunking wall time / writes total chunks and bytes. */
double cdc_ref_bench_synth(const cdc_ref_params* p, uint64_t seed, uint64_t stream0,
                           uint32_t buffers_per_stream, uint32_t nbuf, uint32_t buf_len,
                           int nthreads, uint64_t* total_chunks, uint64_t* total_bytes);

/* Counter-based synthetic generator: byte at (seed, stream, offset). */
uint64_t cdc_ref_splitmix64(uint64_t x);
void cdc_ref_synth(uint64_t seed, uint64_t stream, uint64_t offset, uint8_t* out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
