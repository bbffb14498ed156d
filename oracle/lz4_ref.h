/*
 * lz4_ref.h — CPU ORACLE for LZ4 block compression of unique chunks (test infrastructure only;
 * see lz4_ref.c for what it restates and what pins it).
 */
#ifndef SDFS_LZ4_REF_H
#define SDFS_LZ4_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { LZ4_REF_R123 = 0, LZ4_REF_V19 = 1 };

/* LZ4_compressBound / LZ4Compressor.maxCompressedLength: n + n/255 + 16 */
uint32_t lz4_ref_bound(uint32_t n);
/* One LZ4 block of src[0..n) into dst (cap >= lz4_ref_bound(n)); returns its length or -1. */
long lz4_ref_compress(int mode, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap);
/* [big-endian int32 n][block], the record HashBlobArchive.putChunk writes (java:1281-1289). */
long lz4_ref_compress_framed(int mode, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap);
/* Decode one block (independent check of the format); returns the decoded length or -1. */
long lz4_ref_decompress(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap);
/* Framed records of chunks base[offs[i] .. + lens[i]) at out + out_offs[i] (room bound + 4),
 * on nthreads pthreads; returns the total bytes written or -1. */
long lz4_ref_compress_batch(int mode, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                            uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
