/*
 * sdfs_meta.h — C-ABI of the device-side metadata emission for flushed write buffers
 * (the per-buffer HashLocPair / SparseDataChunk records).
 *
 * After a write buffer's chunks are fingerprinted and deduplicated, SparseDedupFile.writeCache
 * builds one HashLocPair per chunk (SparseDedupFile.java:535-556: hash = the chunk's digest,
 * hashloc = its fingerprint's position as Longs.toByteArray, len = nlen = chunk length, pos =
 * chunk start, offset = 0, dup = not the inserted copy) into a TreeMap by pos, and
 * LongByteArrayMap.put (LongByteArrayMap.java:547-579) writes SparseDataChunk.getBytes() at the
 * buffer's slot of the file map, fpos = (file position / CHUNK_LENGTH) * slot length
 * (LongByteArrayMap.java:536-539).  For map versions >= 2 (SparseDataChunk.java:295-318) the
 * image is
 *     [u8 flags = 0][BE32 image length][BE32 n][n x HashLocPair.asArray()][BE32 doop]
 * with HashLocPair.asArray() (HashLocPair.java:49-59) =
 *     [hash, hashLength bytes][hashloc, 8 bytes][BE32 len][BE32 pos][BE32 offset][BE32 nlen]
 * (BAL = hashLength + 24 bytes, HashLocPair.java:37-38) and doop = the bytes of duplicate chunks.
 * Slot length = 13 + BAL * 2 * max_hash_cluster (LongByteArrayMap.java:59-60).
 *
 * sdfs_cdc_map_emit writes these images for a whole batch of buffers from the engine's per-buffer
 * chunk slots (sdfs_cdc_dev_out) and the dedup index's per-record outputs
 * (sdfs_cdc_index_put_records: dup, hashloc, in (buffer, chunk) record order).  Errors and
 * threading as in sdfs_cdc.h.
 */
#ifndef SDFS_META_H
#define SDFS_META_H

#include <stdint.h>

#include "sdfs_cdc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* LongByteArrayMap slot length for a version >= 2 map: 13 + (hash_len + 24) * max_elements,
 * max_elements = 2 * (CHUNK_LENGTH / minLen) (LongByteArrayMap.java:59-60). */
uint32_t sdfs_cdc_map_slot_bytes(uint32_t hash_len, uint32_t chunk_length, uint32_t min_len);

/* Buffer b (b < nbuf) of the batch described by `out` (counts, starts, lens, digests, cap; the
 * record table is not needed) gets its SparseDataChunk image at d_map + b * slot_bytes; bytes of
 * the slot past the image are left as they are (LongByteArrayMap.put writes the image only).
 * hash_len: HashFunctionPool.hashLength (32 for VARIABLE_SHA256, 16 for VARIABLE_MD5; 20 is
 * refused: HASH160 digests are 20 bytes while hashLength is 18, which asArray() cannot hold).
 * d_dup / d_hashloc: per record r = (first record of buffer b) + i, as the index wrote them.
 * d_doop (optional, [nbuf]): WritableCacheBuffer.setDoop's value per buffer.  A buffer whose image
 * does not fit its slot (13 + n_b * (hash_len + 24) > slot_bytes; LongByteArrayMap throws
 * "Buffer overflow" there, SparseDataChunk.java:303-307) is not written and sets *d_overflow = 1
 * (device u32, zeroed by the caller; required). */
int sdfs_cdc_map_emit(int device, uint32_t nbuf, const sdfs_cdc_dev_out* out, uint32_t hash_len,
                      const uint8_t* d_dup, const uint64_t* d_hashloc, uint8_t* d_map, uint32_t slot_bytes,
                      uint32_t* d_doop, uint32_t* d_overflow, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SDFS_META_H */
