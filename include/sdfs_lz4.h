/*
 * sdfs_lz4.h — C-ABI of the MI355X LZ4 block compressor for unique chunks.
 *
 * After the dedup-hit step, SDFS stores every NEW chunk through HashBlobArchive.putChunk
 * (HashBlobArchive.java:1267-1294): when Main.compress is set (always for --backup-volume,
 * VolumeConfigWriter.java:298-300, and for the cloud stores) the stored record is
 *     [int nz = chunk.length, big-endian][CompressionUtils.compressLz4(chunk)]
 * and the read side (HashBlobArchive.java:1927-1933) decompresses when nz > 0.  compressLz4 is
 * lz4Compressor.compress(input) (CompressionUtils.java:118-120) with lz4Compressor =
 * LZ4Factory.nativeInstance().fastCompressor() (CompressionUtils.java:52-53), third-party
 * net.jpountz.lz4:lz4:1.3.0 (pom.xml:158-162): the C LZ4 r123 LZ4_compress_limitedOutput.
 *
 * These entry points compress a whole batch of chunks on the GPU, byte-identical to that
 * greedy LZ4 parse (oracle/lz4_ref.c restates it; mode SDFS_CDC_LZ4_V19 is pinned there against
 * the image's liblz4 1.9.x, mode SDFS_CDC_LZ4_R123 is the reference's r123 rules).  The framed
 * form writes the putChunk record.  Errors, threading and sdfs_cdc_last_error() as in sdfs_cdc.h.
 * Device-path calls may come on different streams: launches that share the compressor's device
 * scratch wait for the previous such launch when it was enqueued on another stream.
 */
#ifndef SDFS_LZ4_H
#define SDFS_LZ4_H

#include <stdint.h>

#include "sdfs_cdc.h"

#ifdef __cplusplus
extern "C" {
#endif

enum sdfs_cdc_lz4_mode {
    SDFS_CDC_LZ4_R123 = 0, /* lz4-java 1.3.0's bundled LZ4 r123 (the reference) */
    SDFS_CDC_LZ4_V19 = 1,  /* LZ4 1.9.x LZ4_compress_default (acceleration 1) */
};

typedef struct sdfs_cdc_lz4 sdfs_cdc_lz4;

/* LZ4Compressor.maxCompressedLength(n) = LZ4_compressBound(n) = n + n/255 + 16 */
uint64_t sdfs_cdc_lz4_bound(uint64_t n);

/* LZ4Factory.nativeInstance().fastCompressor() on HIP device `device` (CompressionUtils.java:52-53). */
int sdfs_cdc_lz4_create(int device, int mode, sdfs_cdc_lz4** out);
int sdfs_cdc_lz4_destroy(sdfs_cdc_lz4* z);

/* Device batch.  Chunk i (i < *d_count when d_count != NULL, else i < n_max) is
 * d_data[d_src_off[i] .. + d_src_len[i]) (each < 2 GiB); its LZ4 block (framed != 0: preceded by
 * the big-endian length, the putChunk record) is written at d_out + d_dst_off[i], which must have
 * room for sdfs_cdc_lz4_bound(len) (+4 when framed) bytes; d_dst_len[i] receives the bytes
 * written.  Enqueued on `stream` (NULL = the HIP null stream). */
int sdfs_cdc_lz4_compress_device(sdfs_cdc_lz4* z, const uint8_t* d_data, const uint64_t* d_src_off,
                                 const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max,
                                 uint8_t* d_out, const uint64_t* d_dst_off, uint32_t* d_dst_len, int framed,
                                 void* stream);

/* Chunk extents of selected fingerprint records (the 48-byte records of sdfs_cdc_dev_out, e.g.
 * the new ones listed by sdfs_cdc_index_put_records: d_sel = d_new_list, d_count = the low word
 * of d_new_count; d_sel NULL = all records).  Record {.., u64 buffer_id, u32 start, u32 len}
 * lives in buffer buffer_id - buffer_id_base at d_buf_offs[b] (or b * uniform_len when
 * d_buf_offs is NULL).  Writes d_src_off / d_src_len and d_dst_off = exclusive prefix of the
 * output room (bound + 4 when framed); *d_total_bytes = total room. */
int sdfs_cdc_lz4_plan_records(sdfs_cdc_lz4* z, const uint8_t* d_records, const uint32_t* d_sel,
                              const uint32_t* d_count, uint64_t n_max, uint64_t buffer_id_base,
                              uint32_t uniform_len, const uint64_t* d_buf_offs, int framed, uint64_t* d_src_off,
                              uint32_t* d_src_len, uint64_t* d_dst_off, uint64_t* d_total_bytes, void* stream);

/* LZ4Compressor.compress(byte[]) on host bytes (one chunk through the GPU); *out_len = block size. */
int sdfs_cdc_lz4_compress(sdfs_cdc_lz4* z, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                          uint32_t* out_len);

/* Host batch: chunk i = base[offs[i] .. + lens[i]) -> out + out_offs[i] (room for bound(+4));
 * out_lens[i] = bytes written.  One H2D, one launch, one D2H. */
int sdfs_cdc_lz4_compress_batch(sdfs_cdc_lz4* z, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                                uint32_t n, uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int framed);

/* Read side (HashBlobArchive.getChunk -> CompressionUtils.decompressLz4(block, nz) =
 * LZ4FastDecompressor.decompress, HashBlobArchive.java:1927-1933, CompressionUtils.java:122-125).
 * Device batch: record i = d_src[d_src_off[i] .. + d_src_len[i]) decoded to d_out + d_dst_off[i]
 * (room d_dst_cap[i]); d_dst_len[i] = decoded length, or UINT32_MAX for a malformed block.
 * framed != 0: records are putChunk records [BE32 nz][payload]: nz > 0 = an LZ4 block that must
 * decode to exactly nz bytes, else the payload is the raw chunk (copied). */
int sdfs_cdc_lz4_decompress_device(sdfs_cdc_lz4* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                   const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max, uint8_t* d_out,
                                   const uint64_t* d_dst_off, const uint32_t* d_dst_cap, uint32_t* d_dst_len,
                                   int framed, void* stream);
/* LZ4FastDecompressor.decompress(src, destLen) on host bytes: SDFS_CDC_EINVAL unless the block
 * decodes to exactly dst_len bytes. */
int sdfs_cdc_lz4_decompress(sdfs_cdc_lz4* z, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t dst_len);

#ifdef __cplusplus
}
#endif
#endif /* SDFS_LZ4_H */
