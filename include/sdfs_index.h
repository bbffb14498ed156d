/*
 * sdfs_index.h — C-ABI of the device-resident dedup-hit index.
 *
 * After getChunks, SDFS dedups a flushed buffer's chunks by fingerprint and hands each distinct
 * one to the hash store: SparseDedupFile.writeCache groups the buffer's Fingers by hash and counts
 * `claims` (SparseDedupFile.java:435-446), calls HCServiceProxy.writeChunk(hash, chunk, claims)
 * for every distinct hash (Finger.java:50-60 -> HashChunkService.writeChunk,
 * HashChunkService.java:98-118 -> AbstractHashesMap.put), and records per chunk whether it was a
 * duplicate and where the data lives (HashLocPair dup/hashloc, SparseDedupFile.java:541-560).
 * The hash store's put (RocksDBMap.put, RocksDBMap.java:785-870) is: present -> refcount +=
 * claims, return InsertRecord(inserted=false, pos); absent -> persist the chunk, insert
 * {pos, refcount = claims}, return InsertRecord(inserted=true, pos).
 *
 * This index keeps that map (fingerprint -> {pos, refcount}) in HBM and applies a whole batch of
 * fingerprint records (the engine's 48-byte records, include/sdfs_cdc.h, in buffer order) in
 * one pass.  Results equal applying the buffers one after another in record order: the first
 * record of a fingerprint that was not yet in the index is the one "inserted"; every other
 * record is a duplicate; every record's hashloc is its fingerprint's pos.  Positions of newly
 * inserted fingerprints are pos_base + their rank among the batch's insertions (in record order):
 * the host persists exactly those chunks (new_list) and owns the pos namespace, as
 * HashBlobArchive does for the reference.
 *
 * Errors, threading and the last-error message follow include/sdfs_cdc.h (sdfs_cdc_last_error).
 * Calls apply in call order whatever streams they are enqueued on (a call on another stream than
 * the previous one waits for it on the device).
 * A full index returns SDFS_CDC_ECAP (HashtableFullException in the reference).
 */
#ifndef SDFS_INDEX_H
#define SDFS_INDEX_H

#include <stdint.h>

#include "sdfs_cdc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sdfs_cdc_index sdfs_cdc_index;

/* A device-resident map with room for `capacity` fingerprints (rounded up to a power of two,
 * filled to at most 7/8) on HIP device `device`.  64 bytes of HBM per slot.
 * (AbstractHashesMap.init, AbstractHashesMap.java: init(maxSize, fileName, fpp)) */
int sdfs_cdc_index_create(int device, uint64_t capacity, sdfs_cdc_index** out);
int sdfs_cdc_index_destroy(sdfs_cdc_index* ix);

/* Apply a batch of fingerprint records (d_records: n_max x SDFS_CDC_RECORD_BYTES on the device,
 * of which the first *d_count are valid when d_count != NULL, else all n_max).  Outputs (device,
 * n_max entries, written for the valid records): d_dup[r] = 1 if record r is a duplicate (its
 * fingerprint was indexed before or appeared earlier in the batch), d_hashloc[r] = pos of its
 * fingerprint; d_new_list[0..k) = indices of the inserted records in record order, *d_new_count
 * = k (u64).  Enqueued on `stream` (NULL = the HIP null stream).
 * (AbstractHashesMap.put(ChunkData) per distinct fingerprint, RocksDBMap.java:785-870, as driven
 * by SparseDedupFile.writeCache, SparseDedupFile.java:435-446,487-564) */
int sdfs_cdc_index_put_records(sdfs_cdc_index* ix, const uint8_t* d_records, uint64_t n_max,
                               const uint32_t* d_count, uint64_t pos_base, uint8_t* d_dup,
                               uint64_t* d_hashloc, uint32_t* d_new_list, uint64_t* d_new_count,
                               void* stream);

/* Look up n fingerprints (d_digests: n x 32 bytes, zero-padded past the digest length):
 * d_pos[i] = pos or UINT64_MAX when absent, d_refcount[i] = reference count or 0 (either output
 * may be NULL).  (AbstractHashesMap.get / containsKey, RocksDBMap.get) */
int sdfs_cdc_index_get(sdfs_cdc_index* ix, const uint8_t* d_digests, uint64_t n, uint64_t* d_pos,
                       uint64_t* d_refcount, void* stream);

/* Drop every fingerprint (AbstractHashesMap.clear / a fresh map), enqueued on `stream`. */
int sdfs_cdc_index_clear(sdfs_cdc_index* ix, void* stream);

/* Fingerprints held (synchronises the index's last stream) and slot capacity.
 * (AbstractHashesMap.getSize / getMaxSize) */
int sdfs_cdc_index_size(sdfs_cdc_index* ix, uint64_t* used, uint64_t* capacity);

/* Test hook: the batch epoch counter (31 bits; the next put_records uses epoch + 1, wrapping to 1).
 * Stamps only mark a batch's own insertions while it runs, so any value is safe. */
int sdfs_cdc_index_set_epoch(sdfs_cdc_index* ix, uint32_t epoch);

#ifdef __cplusplus
}
#endif
#endif /* SDFS_INDEX_H */
