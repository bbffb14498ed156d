// dedup_index.hip — device-resident dedup-hit index (include/sdfs_index.h).
//
// The reference's write path, after getChunks, groups a buffer's chunks by fingerprint and counts
// `claims` (SparseDedupFile.java:435-446), then puts every distinct fingerprint into the hash
// store with that claim count (Finger.java:50-60 -> HashChunkService.writeChunk,
// HashChunkService.java:98-118 -> RocksDBMap.put, RocksDBMap.java:785-870: present -> refcount +=
// claims, not inserted; absent -> persist + insert {pos, claims}), and marks each chunk dup /
// not dup with its hashloc (SparseDedupFile.java:541-560).
//
// MI355X form: the map lives in HBM as an open-addressing table of 64-byte slots (one cache line:
// digest[32] | pos | refcount | state), and a whole batch of fingerprint records is applied with
// five small integer kernels and no sort:
//   1. group   — a batch-local table of RECORD INDICES (the keys stay in the immutable record
//                table, so a CAS on a 4-byte slot publishes a fully formed key): equal
//                fingerprints meet in one local slot, which keeps the smallest record index
//                (atomicMin) and counts the group (the claims);
//   2. probe   — one lane per group representative probes the global table: hit -> refcount +=
//                claims; miss -> claim an empty slot with a CAS on its state word, stamped with
//                this batch's epoch (lanes of the same batch skip each other's fresh slots without
//                reading their keys: representatives are distinct fingerprints); the assign step
//                turns every stamp of the batch into the committed state, so no stamp outlives
//                its batch (epochs may wrap);
//   3-4. rank  — block counts + one-block scan of the "inserted" flags in record order;
//   5. assign  — inserted record -> new_list[rank], slot pos = pos_base + rank;
//   6. output  — per record: dup = not inserted, hashloc = its fingerprint's pos.
// The outcome is what applying the batch's buffers one after another gives (the first record of
// a new fingerprint is the inserted one), independent of the GPU's schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>

#include "../../include/sdfs_index.h"
#include "cdc_internal.h"
#include "stream_order.h"

namespace sdfs {
namespace {

struct alignas(64) IndexSlot {
    uint4 key[2];     // digest, zero-padded to 32 bytes
    uint64_t pos;     // where the chunk lives (caller's namespace)
    uint64_t ref;     // reference count
    uint32_t state;   // 0 = empty, kCommitted = holds a fingerprint, (epoch << 1) | 1 (epoch >= 1) =
                      // being inserted by the batch of that epoch
    uint32_t pad[3];
};
static_assert(sizeof(IndexSlot) == 64, "one cache line per slot");

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kCommitted = 1u;  // never a batch stamp: those are >= 3
constexpr int kIxThreads = 256;
constexpr int kRankBlock = 1024;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void load_digest(const uint8_t* records, uint32_t r, uint4& a, uint4& b) {
    const uint4* p = reinterpret_cast<const uint4*>(records + (uint64_t)r * kRecordBytes);
    a = p[0];
    b = p[1];
}

__device__ __forceinline__ bool eq4(const uint4& x, const uint4& y) {
    return ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) == 0;
}

__device__ __forceinline__ uint32_t batch_count(const uint32_t* d_count, uint64_t n_max) {
    return d_count ? (uint32_t)min<uint64_t>(*d_count, n_max) : (uint32_t)n_max;
}

// 1. group equal fingerprints of the batch; ltab holds the smallest record index of each group
__global__ __launch_bounds__(kIxThreads) void ix_group_kernel(const uint8_t* records, const uint32_t* d_count,
                                                              uint64_t n_max, uint32_t* ltab, uint32_t* lcount,
                                                              uint32_t lmask, uint32_t* lslot) {
    const uint32_t n = batch_count(d_count, n_max);
    const uint32_t r = blockIdx.x * kIxThreads + threadIdx.x;
    if (r >= n) return;
    uint4 a, b;
    load_digest(records, r, a, b);
    uint32_t h = (uint32_t)mix64(((uint64_t)a.w << 32 | a.z) ^ 0x5DF50001ull) & lmask;
    for (;;) {  // lmask + 1 >= 2n: an empty slot always exists
        uint32_t v = ltab[h];
        if (v == kEmpty) {
            const uint32_t old = atomicCAS(&ltab[h], kEmpty, r);
            if (old == kEmpty) break;
            v = old;
        }
        uint4 c, d;
        load_digest(records, v, c, d);
        if (eq4(a, c) && eq4(b, d)) {
            atomicMin(&ltab[h], r);
            break;
        }
        h = (h + 1) & lmask;
    }
    atomicAdd(&lcount[h], 1u);
    lslot[r] = h;
}

// 2. representatives probe / insert into the global table
__global__ __launch_bounds__(kIxThreads) void ix_probe_kernel(const uint8_t* records, const uint32_t* d_count,
                                                              uint64_t n_max, const uint32_t* ltab,
                                                              const uint32_t* lcount, const uint32_t* lslot,
                                                              IndexSlot* table, uint64_t cmask, uint32_t stamp,
                                                              uint32_t* gidx, uint32_t* isnew, uint32_t* overflow) {
    const uint32_t n = batch_count(d_count, n_max);
    const uint32_t r = blockIdx.x * kIxThreads + threadIdx.x;
    if (r >= n) return;
    const uint32_t ls = lslot[r];
    if (ltab[ls] != r) {  // not the first record of its fingerprint in this batch
        isnew[r] = 0;
        return;
    }
    const uint32_t claims = lcount[ls];
    uint4 a, b;
    load_digest(records, r, a, b);
    uint64_t h = mix64((uint64_t)a.y << 32 | a.x) & cmask;
    for (uint64_t step = 0; step <= cmask; step++, h = (h + 1) & cmask) {
        IndexSlot& s = table[h];
        uint32_t st = s.state;
        if (st == 0) {
            const uint32_t old = atomicCAS(&s.state, 0u, stamp);
            if (old == 0) {
                s.key[0] = a;
                s.key[1] = b;
                s.ref = claims;
                s.pos = ~0ull;  // assigned in rank order by ix_assign_kernel
                gidx[ls] = (uint32_t)h;
                isnew[r] = 1;
                return;
            }
            st = old;
        }
        if (st == stamp) continue;  // inserted by this batch: a different fingerprint
        if (eq4(s.key[0], a) && eq4(s.key[1], b)) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&s.ref), (unsigned long long)claims);
            gidx[ls] = (uint32_t)h;
            isnew[r] = 0;
            return;
        }
    }
    atomicOr(overflow, 1u);
    gidx[ls] = 0xFFFFFFFFu;
    isnew[r] = 0;
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
    // kRankBlock threads = 16 waves: wave-level inclusive scan, then a scan of the 16 wave sums
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) lds[wv] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint32_t w = threadIdx.x < kRankBlock / 64 ? lds[threadIdx.x] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(w, o);
            if (lane >= (uint32_t)o) w += y;
        }
        if (threadIdx.x < kRankBlock / 64) lds[16 + threadIdx.x] = w;
    }
    __syncthreads();
    total = lds[16 + kRankBlock / 64 - 1];
    const uint32_t before = wv ? lds[16 + wv - 1] : 0;
    const uint32_t res = before + x - v;
    __syncthreads();
    return res;
}

// 3. inserted records per block of kRankBlock records
__global__ __launch_bounds__(kRankBlock) void ix_count_kernel(const uint32_t* d_count, uint64_t n_max,
                                                              const uint32_t* isnew, uint32_t* bsum) {
    __shared__ uint32_t lds[64];
    const uint32_t n = batch_count(d_count, n_max);
    const uint32_t r = blockIdx.x * kRankBlock + threadIdx.x;
    uint32_t total;
    (void)block_exclusive_scan(r < n ? isnew[r] : 0u, lds, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// 4. exclusive scan of the block counts (one block), batch total, running index size
__global__ __launch_bounds__(kRankBlock) void ix_scan_kernel(uint32_t* bsum, uint32_t nblocks, uint64_t* new_count,
                                                             uint64_t* used) {
    __shared__ uint32_t lds[64];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += kRankBlock) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nblocks ? bsum[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, lds, total);
        if (i < nblocks) bsum[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) {
        *new_count = carry;
        *used += carry;
    }
}

// 5. inserted records: rank -> new_list, slot pos
__global__ __launch_bounds__(kRankBlock) void ix_assign_kernel(const uint32_t* d_count, uint64_t n_max,
                                                               const uint32_t* isnew, const uint32_t* bbase,
                                                               const uint32_t* lslot, const uint32_t* gidx,
                                                               IndexSlot* table, uint64_t pos_base,
                                                               uint32_t* new_list) {
    __shared__ uint32_t lds[64];
    const uint32_t n = batch_count(d_count, n_max);
    const uint32_t r = blockIdx.x * kRankBlock + threadIdx.x;
    const uint32_t f = r < n ? isnew[r] : 0u;
    uint32_t total;
    const uint32_t ex = block_exclusive_scan(f, lds, total);
    if (f) {
        const uint32_t rank = bbase[blockIdx.x] + ex;
        if (new_list) new_list[rank] = r;
        IndexSlot& slot = table[gidx[lslot[r]]];
        slot.pos = pos_base + rank;
        slot.state = kCommitted;  // the batch stamp must not survive the batch
    }
}

// 6. per-record dup flag and hashloc
__global__ __launch_bounds__(kIxThreads) void ix_output_kernel(const uint32_t* d_count, uint64_t n_max,
                                                               const uint32_t* isnew, const uint32_t* lslot,
                                                               const uint32_t* gidx, const IndexSlot* table,
                                                               uint8_t* dup, uint64_t* hashloc) {
    const uint32_t n = batch_count(d_count, n_max);
    const uint32_t r = blockIdx.x * kIxThreads + threadIdx.x;
    if (r >= n) return;
    if (dup) dup[r] = isnew[r] ? 0 : 1;
    if (hashloc) {
        const uint32_t g = gidx[lslot[r]];
        hashloc[r] = g == 0xFFFFFFFFu ? ~0ull : table[g].pos;
    }
}

__global__ __launch_bounds__(kIxThreads) void ix_get_kernel(const uint8_t* digests, uint64_t n,
                                                            const IndexSlot* table, uint64_t cmask, uint64_t* pos,
                                                            uint64_t* ref) {
    const uint64_t i = (uint64_t)blockIdx.x * kIxThreads + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(digests + i * 32);
    const uint4 a = p[0], b = p[1];
    uint64_t h = mix64((uint64_t)a.y << 32 | a.x) & cmask;
    uint64_t rp = ~0ull, rr = 0;
    for (uint64_t step = 0; step <= cmask; step++, h = (h + 1) & cmask) {
        const IndexSlot& s = table[h];
        if (s.state == 0) break;
        if (eq4(s.key[0], a) && eq4(s.key[1], b)) {
            rp = s.pos;
            rr = s.ref;
            break;
        }
    }
    if (pos) pos[i] = rp;
    if (ref) ref[i] = rr;
}

template <typename T>
struct IxBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(want, 1) * sizeof(T));
        if (e == hipSuccess) n = std::max<size_t>(want, 1);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace
}  // namespace sdfs

using namespace sdfs;

struct sdfs_cdc_index {
    int device = 0;
    uint64_t slots = 0;     // power of two
    uint64_t max_fill = 0;  // 7/8 of slots
    uint64_t used_ub = 0;   // host-side upper bound of the fingerprints held
    uint32_t epoch = 0;
    IxBuf<IndexSlot> table;
    IxBuf<uint64_t> used;  // [1] device count of fingerprints held
    IxBuf<uint32_t> ltab, lcount, lslot, gidx, isnew, bsum, overflow;
    hipStream_t own = nullptr;   // the index's own non-blocking stream: set-up and readbacks
    hipStream_t last = nullptr;  // the stream of the latest batch (own until one comes)
    StreamOrder order;  // batches apply in call order whatever streams they come on
    std::mutex mu;
};

#define IX_TRY(expr)                                                                                  \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return fail_status(SDFS_CDC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                               __FILE__, __LINE__);                                                   \
    } while (0)

extern "C" {

int sdfs_cdc_index_create(int device, uint64_t capacity, sdfs_cdc_index** out) {
    if (!out) return fail_status(SDFS_CDC_EINVAL, "null output");
    *out = nullptr;
    if (capacity == 0 || capacity > (1ull << 30)) return fail_status(SDFS_CDC_EINVAL, "capacity out of range");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail_status(SDFS_CDC_ENODEV, "no HIP device %d", device);
    IX_TRY(hipSetDevice(device));
    auto* ix = new sdfs_cdc_index();
    ix->device = device;
    if (ix->order.init() != hipSuccess || hipStreamCreateWithFlags(&ix->own, hipStreamNonBlocking) != hipSuccess) {
        ix->order.destroy();
        delete ix;
        return fail_status(SDFS_CDC_EHIP, "event or stream creation failed");
    }
    ix->last = ix->own;
    ix->slots = next_pow2(capacity + capacity / 7 + 1);
    ix->max_fill = ix->slots - ix->slots / 8;
    if (ix->table.ensure(ix->slots) != hipSuccess || ix->used.ensure(1) != hipSuccess ||
        ix->overflow.ensure(1) != hipSuccess) {
        sdfs_cdc_index_destroy(ix);
        return fail_status(SDFS_CDC_ENOMEM, "index allocation (%llu slots) failed",
                           (unsigned long long)ix->slots);
    }
    // Nothing here or below runs on the legacy null stream or synchronises the device: the CDC
    // queue's lanes are blocking streams, and a null-stream operation would wait for their passes.
    if (hipMemsetAsync(ix->table.p, 0, ix->slots * sizeof(IndexSlot), ix->own) != hipSuccess ||
        hipMemsetAsync(ix->used.p, 0, sizeof(uint64_t), ix->own) != hipSuccess ||
        hipMemsetAsync(ix->overflow.p, 0, sizeof(uint32_t), ix->own) != hipSuccess ||
        hipStreamSynchronize(ix->own) != hipSuccess) {
        sdfs_cdc_index_destroy(ix);
        return fail_status(SDFS_CDC_EHIP, "index initialisation failed");
    }
    *out = ix;
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_destroy(sdfs_cdc_index* ix) {
    if (!ix) return SDFS_CDC_OK;
    (void)hipSetDevice(ix->device);
    // batches are chained in call order (StreamOrder), so the latest one's stream finishing means
    // every earlier one has
    if (ix->last) (void)hipStreamSynchronize(ix->last);
    if (ix->own) (void)hipStreamSynchronize(ix->own);
    ix->table.release();
    ix->used.release();
    for (auto* b : {&ix->ltab, &ix->lcount, &ix->lslot, &ix->gidx, &ix->isnew, &ix->bsum, &ix->overflow})
        b->release();
    ix->order.destroy();
    if (ix->own) (void)hipStreamDestroy(ix->own);
    delete ix;
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_put_records(sdfs_cdc_index* ix, const uint8_t* d_records, uint64_t n_max,
                               const uint32_t* d_count, uint64_t pos_base, uint8_t* d_dup, uint64_t* d_hashloc,
                               uint32_t* d_new_list, uint64_t* d_new_count, void* stream) {
    if (!ix) return fail_status(SDFS_CDC_EINVAL, "null index");
    if (!d_new_count) return fail_status(SDFS_CDC_EINVAL, "null new_count");
    if (n_max && !d_records) return fail_status(SDFS_CDC_EINVAL, "null records");
    if (n_max >= (1ull << 31)) return fail_status(SDFS_CDC_EINVAL, "batch too large");
    std::lock_guard<std::mutex> lk(ix->mu);
    IX_TRY(hipSetDevice(ix->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (ix->used_ub + n_max > ix->max_fill) {  // refresh the bound from the device count
        IX_TRY(hipStreamSynchronize(ix->last));
        IX_TRY(hipStreamSynchronize(s));
        uint64_t used = 0;
        uint32_t ovf = 0;
        IX_TRY(hipMemcpyAsync(&used, ix->used.p, sizeof(used), hipMemcpyDeviceToHost, ix->own));
        IX_TRY(hipMemcpyAsync(&ovf, ix->overflow.p, sizeof(ovf), hipMemcpyDeviceToHost, ix->own));
        IX_TRY(hipStreamSynchronize(ix->own));
        if (ovf) return fail_status(SDFS_CDC_ECAP, "index overflowed");
        ix->used_ub = used;
        if (used + n_max > ix->max_fill)
            return fail_status(SDFS_CDC_ECAP, "index full: %llu of %llu fingerprints held, batch of %llu",
                               (unsigned long long)used, (unsigned long long)ix->max_fill,
                               (unsigned long long)n_max);
    }
    IX_TRY(ix->order.acquire(s));
    ix->last = s;
    if (n_max == 0) {
        IX_TRY(hipMemsetAsync(d_new_count, 0, sizeof(uint64_t), s));
        IX_TRY(ix->order.release(s));
        return SDFS_CDC_OK;
    }
    const uint64_t lsize = std::max<uint64_t>(64, next_pow2(2 * n_max));
    const uint32_t nrank = (uint32_t)((n_max + kRankBlock - 1) / kRankBlock);
    if (ix->ltab.ensure(lsize) != hipSuccess || ix->lcount.ensure(lsize) != hipSuccess ||
        ix->gidx.ensure(lsize) != hipSuccess || ix->lslot.ensure(n_max) != hipSuccess ||
        ix->isnew.ensure(n_max) != hipSuccess || ix->bsum.ensure(nrank) != hipSuccess)
        return fail_status(SDFS_CDC_ENOMEM, "index scratch allocation failed");
    ix->epoch = (ix->epoch + 1) & 0x7FFFFFFFu;
    if (ix->epoch == 0) ix->epoch = 1;
    const uint32_t stamp = (ix->epoch << 1) | 1u;
    IX_TRY(hipMemsetAsync(ix->ltab.p, 0xFF, lsize * sizeof(uint32_t), s));
    IX_TRY(hipMemsetAsync(ix->lcount.p, 0, lsize * sizeof(uint32_t), s));
    const uint32_t g = (uint32_t)((n_max + kIxThreads - 1) / kIxThreads);
    const uint64_t cmask = ix->slots - 1;
    hipLaunchKernelGGL(ix_group_kernel, dim3(g), dim3(kIxThreads), 0, s, d_records, d_count, n_max, ix->ltab.p,
                       ix->lcount.p, (uint32_t)(lsize - 1), ix->lslot.p);
    hipLaunchKernelGGL(ix_probe_kernel, dim3(g), dim3(kIxThreads), 0, s, d_records, d_count, n_max, ix->ltab.p,
                       ix->lcount.p, ix->lslot.p, ix->table.p, cmask, stamp, ix->gidx.p, ix->isnew.p,
                       ix->overflow.p);
    hipLaunchKernelGGL(ix_count_kernel, dim3(nrank), dim3(kRankBlock), 0, s, d_count, n_max, ix->isnew.p,
                       ix->bsum.p);
    hipLaunchKernelGGL(ix_scan_kernel, dim3(1), dim3(kRankBlock), 0, s, ix->bsum.p, nrank, d_new_count, ix->used.p);
    hipLaunchKernelGGL(ix_assign_kernel, dim3(nrank), dim3(kRankBlock), 0, s, d_count, n_max, ix->isnew.p,
                       ix->bsum.p, ix->lslot.p, ix->gidx.p, ix->table.p, pos_base, d_new_list);
    hipLaunchKernelGGL(ix_output_kernel, dim3(g), dim3(kIxThreads), 0, s, d_count, n_max, ix->isnew.p, ix->lslot.p,
                       ix->gidx.p, ix->table.p, d_dup, d_hashloc);
    IX_TRY(hipGetLastError());
    IX_TRY(ix->order.release(s));
    ix->used_ub += n_max;
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_get(sdfs_cdc_index* ix, const uint8_t* d_digests, uint64_t n, uint64_t* d_pos,
                       uint64_t* d_refcount, void* stream) {
    if (!ix) return fail_status(SDFS_CDC_EINVAL, "null index");
    if (n && !d_digests) return fail_status(SDFS_CDC_EINVAL, "null digests");
    if (n == 0) return SDFS_CDC_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    IX_TRY(hipSetDevice(ix->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    IX_TRY(ix->order.acquire(s));
    ix->last = s;
    const uint64_t g = (n + kIxThreads - 1) / kIxThreads;
    hipLaunchKernelGGL(ix_get_kernel, dim3((uint32_t)g), dim3(kIxThreads), 0, s, d_digests, n, ix->table.p,
                       ix->slots - 1, d_pos, d_refcount);
    IX_TRY(hipGetLastError());
    IX_TRY(ix->order.release(s));
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_clear(sdfs_cdc_index* ix, void* stream) {
    if (!ix) return fail_status(SDFS_CDC_EINVAL, "null index");
    std::lock_guard<std::mutex> lk(ix->mu);
    IX_TRY(hipSetDevice(ix->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    IX_TRY(ix->order.acquire(s));
    IX_TRY(hipMemsetAsync(ix->table.p, 0, ix->slots * sizeof(IndexSlot), s));
    IX_TRY(hipMemsetAsync(ix->used.p, 0, sizeof(uint64_t), s));
    IX_TRY(hipMemsetAsync(ix->overflow.p, 0, sizeof(uint32_t), s));
    IX_TRY(ix->order.release(s));
    ix->used_ub = 0;
    ix->last = s;
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_set_epoch(sdfs_cdc_index* ix, uint32_t epoch) {
    if (!ix) return fail_status(SDFS_CDC_EINVAL, "null index");
    std::lock_guard<std::mutex> lk(ix->mu);
    ix->epoch = epoch & 0x7FFFFFFFu;  // the next batch uses epoch + 1 (wrapping to 1)
    return SDFS_CDC_OK;
}

int sdfs_cdc_index_size(sdfs_cdc_index* ix, uint64_t* used, uint64_t* capacity) {
    if (!ix) return fail_status(SDFS_CDC_EINVAL, "null index");
    std::lock_guard<std::mutex> lk(ix->mu);
    IX_TRY(hipSetDevice(ix->device));
    IX_TRY(hipStreamSynchronize(ix->last));
    uint64_t u = 0;
    IX_TRY(hipMemcpyAsync(&u, ix->used.p, sizeof(u), hipMemcpyDeviceToHost, ix->own));
    IX_TRY(hipStreamSynchronize(ix->own));
    ix->used_ub = u;
    if (used) *used = u;
    if (capacity) *capacity = ix->max_fill;
    return SDFS_CDC_OK;
}

}  // extern "C"
