/*
 * sdfs_cdc.h — C-ABI of the MI355X-native variable-block CDC + fingerprint engine.
 *
 * This is the drop-in boundary behind SDFS's hash-engine plugin surface
 * (org.opendedup.hashing.AbstractHashEngine, src/org/opendedup/hashing/AbstractHashEngine.java:24-39).
 * A JNI shim binds a new Java class
 * org.opendedup.hashing.HipVariableSha256HashEngine to these entry points; the Python package
 * sdfs_amd binds them with ctypes.  Plain pointers and sizes only: no torch / HIP types in the
 * signatures (HIP streams and device pointers travel as void* / uint8_t*).
 *
 * Errors: every entry point returns an int status (SDFS_CDC_OK = 0, negative on failure) and
 * records a message readable with sdfs_cdc_last_error() (thread-local).  The JNI shim maps a
 * non-zero status to java.io.IOException, which is what getChunks throws today
 * (SparseDedupFile.java:578-580).  Engine creation failure corresponds to the factory's
 * SDFSLogger.fatal + System.exit(5) (HashFunctionPool.java:116-119); the shim decides.
 *
 * Threading: one engine may be shared by all SDFS flush threads (SparseDedupFile.java:100 is a
 * static singleton; the flush pools are Main.writeThreads wide, WritableCacheBuffer.java:100-104),
 * so every call is re-entrant and thread-safe.  Concurrent sdfs_cdc_get_chunks / sdfs_cdc_get_hash
 * calls are coalesced: each caller copies its bytes into a shared pinned staging slot, one GPU
 * pass serves the whole slot (up to four passes in flight per device), and each caller returns
 * with its own results.  The product library reads no environment variables.
 *
 * Sharing (ABI 2): SDFS makes many engine instances — static singletons (SparseDedupFile.java:100,
 * HashBlobArchive.java:140, FileIOServiceImpl.java:152), one-shot ones (HashStore.java:68) and a
 * pool of one per concurrent write-accelerator caller (HashFunctionPool.java:73-86,
 * WritableCacheBuffer.java:640,779).  sdfs_cdc_create therefore returns a HANDLE to a
 * process-wide engine shared by every handle with the same parameters and device set: all of
 * them feed the same coalescing queue(s).  sdfs_cdc_destroy ends one handle: its calls in
 * progress finish first, later calls on it fail with SDFS_CDC_EINVAL, and the last handle of an
 * engine releases the GPU resources.
 *
 * Devices (ABI 2): an engine spans a DEVICE SET (params.device / params.device_mask), one
 * coalescing queue and lane set per GPU.  Host-buffer calls are spread over the set: a call that
 * names its write stream (sdfs_cdc_get_chunks_stream; getChunks(buf, uuid)) goes to the device
 * its stream key maps to, so one stream stays on one GPU; an unkeyed call goes to the least busy
 * device; a batched call is split into contiguous shares, one per device, run concurrently.
 * Device-resident calls run on the device that holds their data pointer.  The fingerprint tables
 * of the devices are all-gathered in process over RCCL (sdfs_cdc_allgather_records).
 */
#ifndef SDFS_CDC_H
#define SDFS_CDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDFS_CDC_ABI_VERSION 3

enum sdfs_cdc_status {
    SDFS_CDC_OK = 0,
    SDFS_CDC_EINVAL = -1,   /* bad argument / unsupported parameter combination */
    SDFS_CDC_ECAP = -2,     /* caller's output capacity too small */
    SDFS_CDC_EHIP = -3,     /* HIP runtime / kernel error */
    SDFS_CDC_ENOMEM = -4,   /* device or pinned host allocation failed */
    SDFS_CDC_ENODEV = -5,   /* no usable gfx950 device */
};

/* hash-type (Main.hashType, HashFunctionPool.java:36-43,102-121) */
enum sdfs_cdc_hash_algo {
    SDFS_CDC_SHA256 = 0,     /* VARIABLE_SHA256      -> 32-byte SHA-256 */
    SDFS_CDC_SHA256_160 = 1, /* VARIABLE_SHA256_160  -> first 20 bytes of SHA-256 (VariableSha256HashEngine.java:60-65) */
    SDFS_CDC_MD5 = 2,        /* VARIABLE_MD5         -> 16-byte MD5 (VariableMD5HashEngine.java:55-58) */
};

/* minimum-length comparison of the (absent) rabinwindow jar — SURVEY.md A.3 knob */
enum sdfs_cdc_min_cmp { SDFS_CDC_MIN_GT = 0 /* n > min_len (default) */, SDFS_CDC_MIN_GE = 1 };

/* Engine parameters = the numbers SDFS passes to EnhancedFingerFactory
 * (VariableSha256HashEngine.java:50-52) plus the unpinned predicate knobs. */
typedef struct sdfs_cdc_params {
    uint64_t poly;          /* 10923124345206883 = 0x26CE86126EF863 (VariableSha256HashEngine.java:41) */
    uint32_t window;        /* HashFunctionPool.bytesPerWindow = 48 (HashFunctionPool.java:51) */
    uint32_t min_len;       /* HashFunctionPool.minLen = Main.MIN_CHUNK_LENGTH = 4095 (Main.java:189) */
    uint32_t max_len;       /* HashFunctionPool.maxLen = 32768 (131072 backup) (Config.java:162-166) */
    uint32_t chunk_length;  /* Main.CHUNK_LENGTH = 262144 (41943040 backup) (Config.java:158) */
    uint64_t pred_mask;     /* boundary predicate (fp & pred_mask) == pred_value; default 0xFFF / 0 */
    uint64_t pred_value;
    uint32_t min_cmp;       /* enum sdfs_cdc_min_cmp */
    uint32_t hash_algo;     /* enum sdfs_cdc_hash_algo */
    int32_t device;         /* HIP device ordinal; -1 = every gfx950 device (a device set) */
    uint32_t flags;         /* SDFS_CDC_FLAG_*; 0 = defaults */
    uint64_t max_batch_bytes; /* host-batch staging per slot (pinned, two slots); 0 = default 256 MiB */
    uint64_t device_mask;   /* ABI 2: bit i = HIP ordinal i in the device set (0 = use `device`) */
    /* ABI 3: the FORM of the boundary predicate.  BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR
     * (VariableSha256HashEngine.java:42, absent rabinwindow jar) is one of two detector forms
     * (SURVEY.md A.3): a bitmask detector (fp & pred_mask) == pred_value (SDFS_CDC_PRED_MASK, the
     * default) or a divisor detector fp % pred_div == pred_rem (SDFS_CDC_PRED_DIV; Java long
     * remainder of the non-negative window fp).  pred_div >= 1; a power of two runs as the
     * equivalent mask; any other divisor needs deg(poly) <= 53 (the default poly's degree). */
    uint32_t pred_kind;     /* enum sdfs_cdc_pred_kind */
    uint32_t reserved2;     /* 0 */
    uint64_t pred_div;      /* SDFS_CDC_PRED_DIV: divisor D (1 .. 2^32-1) */
    uint64_t pred_rem;      /* SDFS_CDC_PRED_DIV: target remainder R (R >= D never matches) */
} sdfs_cdc_params;

enum sdfs_cdc_pred_kind { SDFS_CDC_PRED_MASK = 0, SDFS_CDC_PRED_DIV = 1 };

/* flags: serve every getChunks / getHash call with its own GPU round trip instead of coalescing
 * concurrent callers (A/B measurements; the results are identical). */
#define SDFS_CDC_FLAG_DIRECT 1u

typedef struct sdfs_cdc_engine sdfs_cdc_engine;

/* Per-buffer output slots on the DEVICE for sdfs_cdc_run_device (all device pointers).
 * Buffer b's chunk i lives at slot b*cap + i, i < counts[b]; chunks are ascending, contiguous
 * and cover [0, len_b) exactly (the List<Finger> contract, SparseDedupFile.java:535-564). */
typedef struct sdfs_cdc_dev_out {
    uint32_t* counts;   /* [nbuf] */
    uint32_t* starts;   /* [nbuf*cap]  Finger.start */
    uint32_t* lens;     /* [nbuf*cap]  Finger.len */
    uint8_t* digests;   /* [nbuf*cap*32] Finger.hash (digest_len bytes used, rest zero) */
    uint32_t cap;       /* slots per buffer, >= sdfs_cdc_slot_cap(engine, max buffer length) */
    uint32_t reserved;
    /* Optional dense fingerprint table (the record set that is RCCL all-gathered across GPUs):
     * record r = {digest[32], u64 buffer_id, u32 start, u32 len} = 48 bytes, ordered by
     * (buffer, chunk).  NULL to skip.  *total receives the record count (device u32). */
    uint8_t* records;
    uint64_t records_cap;
    uint32_t* total;    /* [1] device; required */
} sdfs_cdc_dev_out;

#define SDFS_CDC_RECORD_BYTES 48

/* ---- lifecycle ---- */
int sdfs_cdc_abi_version(void);
/* Fill p with the reference defaults; backup_volume != 0 selects the --backup-volume profile
 * (VolumeConfigWriter.java:298-307: chunk-size 40960 KiB, max segment 128 KiB). */
int sdfs_cdc_params_default(sdfs_cdc_params* p, int backup_volume);
/* new VariableSha256HashEngine(...) / new VariableMD5HashEngine() (HashFunctionPool.java:102-121). */
int sdfs_cdc_create(const sdfs_cdc_params* p, sdfs_cdc_engine** out);
/* AbstractHashEngine.destroy() */
int sdfs_cdc_destroy(sdfs_cdc_engine* e);
const char* sdfs_cdc_last_error(void);

/* The engine's device set: number of devices, and the HIP ordinal of set member i. */
int sdfs_cdc_device_count(const sdfs_cdc_engine* e);
int sdfs_cdc_device_ordinal(const sdfs_cdc_engine* e, int i);
/* Live handles sharing this handle's engine (1 = not shared). */
int sdfs_cdc_share_count(const sdfs_cdc_engine* e);

/* ---- AbstractHashEngine accessors ---- */
int sdfs_cdc_is_variable_length(const sdfs_cdc_engine* e);   /* isVariableLength(): 1 */
int sdfs_cdc_get_max_len(const sdfs_cdc_engine* e);          /* getMaxLen(): Main.CHUNK_LENGTH (VariableSha256HashEngine.java:106-109) */
int sdfs_cdc_get_min_len(const sdfs_cdc_engine* e);          /* getMinLen(): HashFunctionPool.minLen (:111-114) */
int sdfs_cdc_set_seed(sdfs_cdc_engine* e, int seed);         /* setSeed(): no-op (:116-120) */
int sdfs_cdc_digest_len(const sdfs_cdc_engine* e);           /* 32 / 20 / 16 */
/* Output slots a buffer of buf_len bytes can need: ceil-bound on len/shortest-chunk + 2. */
uint32_t sdfs_cdc_slot_cap(const sdfs_cdc_engine* e, uint64_t buf_len);

/* ---- AbstractHashEngine.getHash(byte[]) (VariableSha256HashEngine.java:58-67) ----
 * Host bytes in, digest_len bytes out (computed on the GPU). */
int sdfs_cdc_get_hash(sdfs_cdc_engine* e, const uint8_t* data, uint64_t len, uint8_t* digest);

/* Page-lock caller memory (e.g. the flush buffers a JNI shim allocates as direct ByteBuffers) so
 * sdfs_cdc_get_chunks_batch copies it to the GPU in place instead of through its staging slots
 * (hipHostRegister / hipHostUnregister). */
int sdfs_cdc_host_register(void* p, uint64_t n);
int sdfs_cdc_host_unregister(void* p);

/* ---- getHash in bulk: many chunks fingerprinted in one GPU pass ----
 * The getHash callers that verify or key whole chunks (HashBlobArchive.java:1271-1276 VERIFY_WRITES,
 * :1936-1940 VERIFY_READS; HashStore.java:63-71; WritableCacheBuffer.java:93-97) one call per chunk
 * today.  Host form: chunk i = base[offs[i] .. + lens[i]) (each < 4 GiB), digest_len bytes per
 * chunk written densely to digests.  Device form: chunk i (i < *d_count when d_count != NULL,
 * else i < n_max) = d_data[d_offs[i] .. + d_lens[i]), 32-byte digest slot i of d_digests
 * (digest_len bytes used, zero-padded); chunks are scheduled longest first; enqueued on stream. */
int sdfs_cdc_get_hash_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                            uint32_t n, uint8_t* digests);
int sdfs_cdc_hash_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs, const uint32_t* d_lens,
                         const uint32_t* d_count, uint64_t n_max, uint8_t* d_digests, void* stream);

/* ---- AbstractHashEngine.getChunks(byte[], uuid) (VariableSha256HashEngine.java:71-86) ----
 * One host buffer (1..CHUNK_LENGTH bytes, fresh CDC state).  Writes *count chunks into
 * starts/lens/digests (digest_len bytes each, densely packed), capacity cap entries.
 * Synchronous for the caller; concurrent callers share GPU passes (see "Threading"). */
int sdfs_cdc_get_chunks(sdfs_cdc_engine* e, const uint8_t* buf, uint32_t len, uint32_t* starts,
                        uint32_t* lens, uint8_t* digests, uint32_t cap, uint32_t* count);
/* The same for a buffer of write stream `stream_key` (getChunks(buf, uuid): e.g. a hash of the
 * file GUID the caller passes, SparseDedupFile.java:432): a device set serves every buffer of one
 * stream on one device.  SDFS_CDC_NO_STREAM = no stream (least busy device). */
#define SDFS_CDC_NO_STREAM UINT64_MAX
int sdfs_cdc_get_chunks_stream(sdfs_cdc_engine* e, uint64_t stream_key, const uint8_t* buf, uint32_t len,
                               uint32_t* starts, uint32_t* lens, uint8_t* digests, uint32_t cap, uint32_t* count);
/* The same with the caller writing the buffer's bytes itself: fill(ctx, dst, len) is called once,
 * on the calling thread, with dst = the space reserved for this call in the engine's pinned
 * staging (so a JNI caller copies its byte[] once, GetByteArrayRegion straight into it).  A
 * non-zero return from fill fails the call with SDFS_CDC_EINVAL and sdfs_cdc_last_error()
 * "getChunks: fill callback failed (<rc>)"; *count is 0 and no results are written. */
typedef int (*sdfs_cdc_fill_fn)(void* ctx, uint8_t* dst, uint32_t len);
int sdfs_cdc_get_chunks_fill(sdfs_cdc_engine* e, uint64_t stream_key, uint32_t len, sdfs_cdc_fill_fn fill, void* ctx,
                             uint32_t* starts, uint32_t* lens, uint8_t* digests, uint32_t cap, uint32_t* count);
/* Coalescing statistics since create: GPU passes launched and getChunks/getHash calls they served;
 * mean microseconds per pass spent filling (first call joined -> pass closed), waiting for the
 * callers' copies into pinned staging, and on the device (transfers + kernels). */
int sdfs_cdc_queue_stats(sdfs_cdc_engine* e, uint64_t* batches, uint64_t* requests);
int sdfs_cdc_queue_timing(sdfs_cdc_engine* e, double* fill_us, double* copy_us, double* device_us);
/* getChunks calls answered before the rest of their GPU pass finished: a pass's callers each
 * return once their own buffer's last chunk is fingerprinted, not when the pass's longest chunk
 * is (SparseDedupFile.java:432 callers block on that call).  Cumulative, all devices. */
int sdfs_cdc_queue_early(sdfs_cdc_engine* e, uint64_t* early);

/* Batched getChunks over nbuf independent host buffers at base+offs[b], lens[b] (each chunked
 * from fresh state; SURVEY.md 0 "every call starts from a fresh state").  Per-buffer slots of
 * cap entries (digests packed digest_len bytes per slot).  Pinned staging + H2D + kernels + D2H. */
int sdfs_cdc_get_chunks_batch(sdfs_cdc_engine* e, const uint8_t* base, const uint64_t* offs,
                              const uint32_t* lens, uint32_t nbuf, uint32_t* counts, uint32_t* starts,
                              uint32_t* lens_out, uint8_t* digests, uint32_t cap);

/* ---- device-resident path (bench / multi-GPU) ----
 * d_data: device bytes, 64-byte aligned.  Uniform layout: nbuf buffers of uniform_len bytes
 * (a multiple of 64) at b*uniform_len — the SDFS write-buffer case (every flushed buffer is
 * CHUNK_LENGTH bytes, WritableCacheBuffer.java:115).  buffer_id_base is added to b in the
 * record table.  stream: the hipStream_t to enqueue on (NULL = the HIP null stream, as in every
 * HIP API).  Asynchronous: returns after enqueueing; d_offs/d_lens are ignored (pass NULL).
 * Runs enqueued on different streams proceed concurrently (the engine keeps a ring of device
 * workspaces, each reused behind its previous run): alternating two streams keeps two batches
 * in flight, so one batch's scan fills the tail of the other's fingerprinting. */
int sdfs_cdc_run_device(sdfs_cdc_engine* e, const uint8_t* d_data, const uint64_t* d_offs,
                        const uint32_t* d_lens, uint32_t nbuf, uint32_t uniform_len,
                        uint64_t buffer_id_base, const sdfs_cdc_dev_out* out, void* stream);
/* Ragged layout: buffer b = d_data[d_offs[b] .. d_offs[b]+d_lens[b]) (device arrays), offsets
 * multiples of 64, non-overlapping, all inside the first data_bytes bytes of d_data (the
 * write-accelerator path hands getChunks arbitrary lengths, WritableCacheBuffer.java:641-643). */
int sdfs_cdc_run_device_ragged(sdfs_cdc_engine* e, const uint8_t* d_data, uint64_t data_bytes,
                               const uint64_t* d_offs, const uint32_t* d_lens, uint32_t nbuf,
                               uint64_t buffer_id_base, const sdfs_cdc_dev_out* out, void* stream);
/* Block until the engine's own stream (every device's) has drained. */
int sdfs_cdc_stream_sync(sdfs_cdc_engine* e);

/* ---- multi-GPU exchange: the set's fingerprint tables all-gathered in process
 * over RCCL (xGMI), one communicator per device (ncclCommInitAll over the set).  Per device i of
 * the set (set order): records[i] = its 48-byte records (sdfs_cdc_dev_out.records, room for
 * records_cap[i]), d_totals[i] = their count (device u32, sdfs_cdc_dev_out.total), gathered[i] =
 * the destination on device i (room for gathered_cap records), streams[i] = a hipStream_t of
 * device i (NULL array = null streams).  First the counts are gathered and read back (counts[j],
 * one small device->host copy: the call blocks for it), then every table is gathered padded to
 * the largest count *stride: device j's records land at gathered[i] + j * *stride * 48.  The
 * table gather is enqueued on streams[i] and the call returns.  Errors: ECAP when a table would
 * not fit, ENODEV when RCCL cannot be loaded. */
int sdfs_cdc_allgather_records(sdfs_cdc_engine* e, uint8_t* const* records, const uint64_t* records_cap,
                               const uint32_t* const* d_totals, uint8_t* const* gathered, uint64_t gathered_cap,
                               uint32_t* counts, uint64_t* stride, void* const* streams);

/* Per-kernel timing with HIP events recorded on the launch stream around every kernel of the
 * next runs (a ring of `nruns` event sets; 0 disables).  sdfs_cdc_kernel_times waits for the
 * recorded events and returns, per pipeline stage, the average milliseconds over the last
 * min(nruns, runs since set_timing) runs; returns the number of stages written. */
int sdfs_cdc_set_timing(sdfs_cdc_engine* e, int nruns);
/* The same for a subset of the stages only (bit i = i-th name sdfs_cdc_kernel_times reports:
 * prep, cdc_scan, cdc_resolve, cdc_prefix, cdc_scatter, chunk_hash, pipeline); untimed stages
 * report 0.  Fewer events per run = less event overhead in a timed region. */
int sdfs_cdc_set_timing_mask(sdfs_cdc_engine* e, int nruns, uint32_t stage_mask);
int sdfs_cdc_kernel_times(sdfs_cdc_engine* e, const char** names, float* ms, int n);
/* The same for device set member dev_index (sdfs_cdc_kernel_times = member 0). */
int sdfs_cdc_kernel_times_on(sdfs_cdc_engine* e, int dev_index, const char** names, float* ms, int n);

/* Synthetic input generator, device side: fills d_out[0..n) with byte
 * (offset+i) of stream `stream` (counter-based SplitMix64; same bytes as the CPU definition),
 * enqueued on stream_handle (NULL = the HIP null stream). */
int sdfs_cdc_synth_device(sdfs_cdc_engine* e, uint8_t* d_out, uint64_t n, uint64_t seed,
                          uint64_t stream, uint64_t offset, void* stream_handle);

#ifdef __cplusplus
}
#endif
#endif /* SDFS_CDC_H */
