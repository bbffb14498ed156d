// cdc_internal.h — device-side layout shared by the kernels (cdc_kernels.hip) and the engine
// (cdc_engine.hip).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdfs {

// LDS image of the rolling-hash tables (DESIGN.md "Rabin scan"): C lane-private copies of each
// 256 x 8-byte table; lane l reads copy (l mod C), so with C = 32 every ds_read_b64 of a 32-lane
// group hits 32 distinct bank pairs (conflict-free for random indices), with C = 16 two lanes
// share a bank pair (2-way).  Entry e of the pop table, copy c: byte (e << 8) | (c << 3).
// Push table: C = 32 -> 0x10000 | (e << 8) | (c << 3) (two 64 KiB tables);
//             C = 16 -> (e << 8) | 0x80 | (c << 3) (interleaved with pop in 256-byte rows).
constexpr int scan_lds_bytes(int copies) { return 2 * 256 * copies * 8; }

constexpr int kScanThreads = 1024;  // widest scan workgroup (one per CU: the tables fill 128 KiB of LDS)
constexpr uint32_t kSmallBatchSeg = 512;  // scan segment of batches with fewer buffers than SIMDs
constexpr uint32_t kTinyBatchSeg = 256;   // ... and of batches under 32 MiB (the queue's passes)

struct ScanVariantInfo {
    int copies;      // table copies (image layout)
    int chains;      // segments per lane
    int lds_bytes;   // LDS image size
    int wg_per_cu;   // resident workgroups per CU the variant is built for
    int blk;         // bytes per lane per iteration (segment length must be a multiple)
    int fuse;        // cut walk in the epilogue when one wave = one buffer: 1 = from the bitmap
                     // (sweep only), 2 = from register candidate summaries (production)
    int threads;     // widest workgroup the variant is compiled for
    int mirror;      // bit-reversed rolling state (mirrored LDS tables, one-compare predicate)
    int pop_swap;    // pop-table entries stored high word first (kAblPopSwap: register banks)
};
ScanVariantInfo scan_variant_info(int variant);

constexpr int kMaxBins = 1024;  // SHA work binning by block count (exact counts up to maxLen 64 KiB)
constexpr int kRecordBytes = 48;

struct ResolveArgs {
    const uint32_t* bitmap;
    const uint64_t* offs;
    const uint32_t* lens;
    uint32_t nbuf;
    uint32_t uniform_len;
    uint32_t first_off;  // min_len (n > min) or min_len-1 (n >= min): first cut offset allowed
    uint32_t max_len;
    uint32_t cap;        // slots per buffer
    uint32_t bin_shift;
    uint32_t nbins;
    uint32_t* counts;
    uint32_t* starts;
    uint32_t* clens;
    uint32_t* hist;      // [nbins]
    uint32_t* overflow;  // [1] set when a buffer needs more than cap slots
    uint64_t max_buf_len;  // longest buffer of a ragged batch (selects the resolve kernel)
    // sectioned walk of long buffers (speculate per section, then stitch; engine scratch)
    uint32_t sec_len;      // positions per section (0 = not sectioned)
    uint32_t nsec;         // sections per buffer (of the longest buffer)
    uint32_t spec_cap;     // chunk starts recorded per section
    uint32_t* spec_starts; // [nbuf * nsec * spec_cap]
    uint32_t* spec_cnt;    // [nbuf * nsec]
    uint32_t* spec_next;   // [nbuf * nsec] first chunk start at or past the section end
    // parallel stitch (cdc_resolve_join_kernel / cdc_resolve_place_kernel): per section
    // {first speculative start on the true chain or kJoinUnmerged, extra true starts, ...},
    // then one flag per buffer (1 = the sequential stitch walks it)
    uint32_t* join;        // [nbuf * nsec * kJoinWords]
    uint32_t* join_bad;    // [nbuf]
    // 1: the scan's epilogue walked every section (piece_walk_from_summary: spec_starts and
    // spec_cnt, each section's last chunk open) — no spec kernel; the join kernel writes spec_next.
    // The scan then stores the bitmap sparsely (from a segment's summary overflow on) and every
    // segment's summary in seg_sum (kSegSumWords each, global segment order); the join and
    // stitch kernels search candidates there (find_first_sum) instead of in the bitmap.
    uint32_t spec_from_scan;
    uint32_t* seg_sum;
    uint32_t seg_len;
    uint32_t small_ballot;  // cdc_resolve_small_kernel: 1 = 64-word ballots only, no candidate list
};
constexpr uint32_t kSegSumWords = 8;  // summary u16 x 8 (4 words) | ncand | ovf_off | pad
constexpr uint32_t kJoinExtra = 8;  // true chunk starts a section may take before its chains meet
constexpr uint32_t kJoinWords = 2 + kJoinExtra;
// Section length of the sectioned cut walk for a buffer of `len` bytes (0 = not sectioned).
uint32_t resolve_section_len(uint64_t len, uint32_t max_len, uint32_t sec_log2 = 18);

struct ScanArgs {
    const uint8_t* data;
    const uint64_t* offs;        // general layout (nullptr when uniform)
    const uint32_t* lens;
    const uint64_t* seg_prefix;  // [nbuf+1] segment prefix (general layout)
    uint32_t* bitmap;            // 1 bit per byte position, bit i of word w = position 32w+i
    uint64_t total_segs;
    uint32_t nbuf;
    uint32_t uniform_len;        // != 0 -> uniform layout
    uint32_t seg_len;            // bytes per segment, multiple of 64
    uint32_t jshift;             // bit offset of the push index in the word holding it: deg(P) - 40
                                 // (hi word), mirrored 64 - deg(P) (lo word of bitrev64(fp))
    uint32_t mask_lo, mask_hi, val_lo, val_hi;  // mirrored: bit-reversed, lo = the word of fp bits 0..31
    uint32_t thr;                // predicate kind 2: 2^(32-k) for a zero test of the low k fp bits
    double div_d, div_inv, rem_d;  // predicate kind 3 (divisor detector): D, 1/D, R as f64 (fp < 2^53)
    const uint8_t* tab_image;    // global copy of the LDS image (scan_lds_bytes(copies))
    const uint8_t* zero_page;    // 256 zero bytes (branch-free prefetch of tail blocks)
    // fused cut resolution: when every wave's 64 segments are exactly one buffer (uniform layout,
    // uniform_len == 64 * seg_len, one segment per lane), the wave resolves that buffer's cuts
    // right after scanning it, from its own L2-resident bitmap words (no separate resolve pass)
    uint32_t fuse_resolve;
    ResolveArgs res;
    uint32_t skip_walk;  // measurement only (tuning: SDFS_SKIP_WALK): 1 no epilogue walk, 2/3 list walk without outputs
    uint32_t list_walk;  // fused walk (fuse_resolve 1): the LDS list walk, else the queue walk only
    uint32_t* wave_ctr;  // nullable, zeroed per launch: one-chain scans hand out 64-segment wave items
                         // from this counter instead of a static workgroup stride
};
// Every segment of the batch is a whole number of `blk`-byte blocks (the scan kernel's
// kAblFullBlocks form may run it).
inline bool scan_full_blocks(const ScanArgs& a, uint32_t blk) {
    return a.uniform_len != 0 && a.seg_len % blk == 0 && a.uniform_len % a.seg_len == 0;
}


struct PrefixArgs {
    const uint32_t* counts;
    uint32_t nbuf;
    const uint32_t* hist;
    uint32_t nbins;
    uint32_t* cursor;     // [nbins] exclusive prefix, descending bin order
    uint32_t* rec_base;   // [nbuf] exclusive prefix of counts (+ *base_in)
    uint32_t* total;      // [1] chunks of this (sub-)batch
    const uint32_t* base_in;  // nullable: records of the earlier sub-batches
    uint32_t* base_out;       // nullable: *base_in + total
    uint32_t* grand_total;    // nullable: same as base_out, the caller's total
};

struct ScatterArgs {
    const uint32_t* counts;
    const uint32_t* clens;
    uint32_t nbuf;
    uint32_t cap;
    uint32_t bin_shift;
    uint32_t nbins;
    uint32_t* cursor;
    uint32_t* tasks;
};

// Long chunks (chunk_hash_long_kernel): more than kLongBlocks SHA-256 blocks, i.e. > 32 KiB - 8
// bytes — only a maxLen above the default makes them.  More long chunks than kLongSplitMax fill
// the chip on their own (their chains no longer form a tail) and the latency form's half-idle
// workgroups would cost throughput, so then every chunk takes the lane form.
constexpr uint32_t kLongBlocks = 512;
constexpr uint32_t kLongSplitMax = 64 * 256;

struct HashArgs {
    const uint8_t* data;
    const uint64_t* offs;
    uint32_t uniform_len;
    const uint32_t* tasks;     // slot indices, longest first
    const uint32_t* total;     // [1] number of tasks
    const uint32_t* starts;
    const uint32_t* clens;
    const uint32_t* rec_base;  // may be null when records == null
    uint32_t cap;
    uint8_t* digests;          // [slot*32]
    uint8_t* records;          // optional dense table
    uint64_t records_cap;
    uint64_t buffer_id_base;
    uint32_t algo;             // SDFS_CDC_SHA256 / _SHA256_160 / _MD5
    uint32_t persist_grid;     // workgroups of the persistent variant (0 = not used)
    uint32_t* wave_ctr;        // [1] zeroed task counter of the persistent variant
    const uint8_t* zero_page;  // 256 zero bytes: target of the branch-free next-block load past a chunk's last whole block
    // long-chunk split (chunk_hash_long_kernel): [1] the number of tasks of more than kLongBlocks
    // SHA blocks (they head the longest-first list), and a host bound on it for the grid; null /
    // 0 = one lane per chunk throughout
    const uint32_t* nlong;
    uint32_t max_long;
    // Early completion of a coalescing-queue pass (host_queue.h): `digests` points into the pass's
    // pinned result image; a buffer whose last chunk's digest is stored gets its ready word set to
    // `seq` (after a system-scope fence), so its caller returns before the pass's longest chunk
    // is done.  done_ctr: [nbuf] zeroed per-buffer counters of stored chunks; counts: [nbuf] the
    // buffers' chunk counts (device).  done_ctr == null: off.
    uint32_t* done_ctr;
    const uint32_t* counts;
    uint32_t* ready;
    uint32_t seq;
    // Per-buffer groups of the latency form (chunk_hash_split_packed_kernel): > 0 = workgroup
    // b * bybuf + g takes chunks 32g .. 32g+31 of buffer b in slot order (`counts` required),
    // so a buffer's fingerprints end with its own longest chunk, not the pass's; 0 = groups of
    // the longest-first task list
    uint32_t bybuf;
    uint32_t split_masked;     // tuning A/B only (SDFS_SPLIT_MASKED): latency form with finished lanes masked off
    // measurement only (tuning build, fingerprint variant 50): per wave {wall clock, shader clock}
    // at its start and end, and its HW_ID / XCC_ID, 8 u64 per wave (scripts/hash_stamps.py)
    uint64_t* stamps;
};

// Longest-first order of arbitrary chunk extents (getHash in bulk): tasks[] = extent indices,
// starts[] zeroed, *total = the live count.  hist/cursor: 512 words each (engine scratch).
struct ExtentArgs {
    const uint32_t* lens;
    const uint32_t* count;  // optional device count (else n_max)
    uint64_t n_max;
    uint32_t* starts;
    uint32_t* tasks;
    uint32_t* total;
    uint32_t* hist;
    uint32_t* cursor;
};
constexpr uint32_t kExtentScratchWords = 2 * 512 + 1;

// Record a C-ABI error message (sdfs_cdc_last_error) and return `code`.
int fail_status(int code, const char* fmt, ...);

inline uint64_t splitmix64_host(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// kernel launchers (cdc_kernels.hip); all asynchronous on `stream`
hipError_t launch_seg_prefix(const uint32_t* lens, uint32_t nbuf, uint32_t seg_len, uint64_t* seg_prefix,
                             hipStream_t stream);
// pk: predicate kind (cand_shift): 0 = one 32-bit word, 1 = both words, 2 = low-k zero (mirrored
// variants only), 3 = divisor detector fp % D == R (production variant only)
hipError_t launch_scan(const ScanArgs& a, int window, int pk, int variant, int grid, int block,
                       hipStream_t stream);
// the tiny-batch scan (64-byte blocks, no fused walk) for segments shorter than 256 bytes
hipError_t launch_scan_tiny(const ScanArgs& a, int window, int pk, int grid, int block, hipStream_t stream);
hipError_t launch_resolve(const ResolveArgs& a, hipStream_t stream);
hipError_t launch_prefix(const PrefixArgs& a, hipStream_t stream);
hipError_t launch_scatter(const ScatterArgs& a, hipStream_t stream);
hipError_t launch_hash(const HashArgs& a, uint64_t max_tasks, int variant, hipStream_t stream, bool packed = true);
// latency form for small batches (SHA-256 / SHA-256/160 only): two waves per 64 chunks
hipError_t launch_hash_split(const HashArgs& a, uint64_t max_tasks, hipStream_t stream, bool packed = true,
                             uint32_t lds_pad = 0);
hipError_t launch_extent_order(const ExtentArgs& a, hipStream_t stream);
hipError_t launch_copy_out(const void* src, void* dst, uint64_t bytes, hipStream_t stream);
// Early completion (HashArgs::done_ctr): everything the pinned image's header needs before the
// fingerprint runs -- a kernel that copies [0, bytes) of the device image to pinned memory.
// (launch_copy_out itself, launched before the fingerprint.)
hipError_t launch_prep_zero(uint32_t* small, uint32_t words, uint32_t* flag, hipStream_t stream);
constexpr uint64_t kSmallScatterSlots = 65536;  // chunk slots up to which prefix + scatter run fused
hipError_t launch_prefix_scatter_small(const PrefixArgs& a, const ScatterArgs& c, hipStream_t stream);
hipError_t launch_synth(uint8_t* out, uint64_t n, uint64_t seed, uint64_t stream_id, uint64_t offset,
                        hipStream_t stream);
bool scan_window_supported(int window);

#ifdef SDFS_TUNING
// measurement-only variants (cdc_sweep.hip; tuning library only)
ScanVariantInfo scan_variant_info_sweep(int variant);
// round-3 variants (cdc_sweep_r3.hip: a translation unit of its own, so that a new variant
// compiles in a minute instead of rebuilding every earlier one)
ScanVariantInfo scan_variant_info_sweep_r3(int variant);
hipError_t launch_scan_sweep_r3(const ScanArgs& a, int window, int pk, int variant, int grid, int block,
                                hipStream_t s);
// measurement probe (tuning build, SDFS_FUSED_PROBE): the fused scan + fingerprint kernel over the
// batch's own scan (again: same slots, same values) and its fingerprint tasks
hipError_t launch_fused_probe(const ScanArgs& a, const HashArgs& ha, uint32_t* ctr, int window, int pk, int grid,
                              int form, hipStream_t s);
hipError_t launch_scan_sweep(const ScanArgs& a, int window, int pk, int variant, int grid, int block,
                             hipStream_t stream);
hipError_t launch_hash_sweep(const HashArgs& a, uint64_t max_tasks, int variant, hipStream_t stream);
#endif

}  // namespace sdfs
