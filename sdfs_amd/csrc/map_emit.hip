// map_emit.hip — SparseDataChunk / HashLocPair images of flushed write buffers on the device
// (include/sdfs_meta.h).
//
// Reference: SparseDedupFile.writeCache builds one HashLocPair per chunk
// (SparseDedupFile.java:535-556) and LongByteArrayMap.put writes SparseDataChunk.getBytes()
// (SparseDataChunk.java:295-318, HashLocPair.asArray HashLocPair.java:49-59) into the buffer's
// slot of the file map (LongByteArrayMap.java:536-579).  Two kernels: a one-block prefix of the
// per-buffer chunk counts (first record of each buffer), then one wave per buffer writing its
// image — lane i the i-th record (big-endian fields, byte stores: records start at odd offsets),
// a wave reduction for doop, lane 0 the header and trailer.  Pure byte formatting: ~1/4700 of
// the data volume, HBM-write bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/sdfs_meta.h"
#include "cdc_internal.h"

namespace sdfs {
namespace {

struct MapArgs {
    uint32_t nbuf;
    const uint32_t* counts;
    const uint32_t* starts;
    const uint32_t* lens;
    const uint8_t* digests;
    uint32_t cap;
    uint32_t hash_len;
    const uint8_t* dup;
    const uint64_t* hashloc;
    const uint32_t* first;  // [nbuf] first record of each buffer
    uint8_t* map;
    uint32_t slot_bytes;
    uint32_t* doop;
    uint32_t* overflow;
};

__device__ __forceinline__ void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

// first[b] = sum of counts[0..b) (one block; 16 Ki buffers = 16 per thread)
__global__ __launch_bounds__(1024) void map_prefix_kernel(const uint32_t* counts, uint32_t nbuf, uint32_t* first) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nbuf + 1023) / 1024;
    const uint32_t b0 = min(t * per, nbuf), b1 = min(b0 + per, nbuf);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += counts[b];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t b = b0; b < b1; b++) {
        first[b] = run;
        run += counts[b];
    }
}

__global__ __launch_bounds__(256) void map_emit_kernel(MapArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= a.nbuf) return;
    const uint32_t n = a.counts[b];
    const uint32_t bal = a.hash_len + 24;
    const uint64_t need = 13ull + (uint64_t)n * bal;
    if (need > a.slot_bytes) {
        if (lane == 0) atomicOr(a.overflow, 1u);
        return;
    }
    uint8_t* img = a.map + (uint64_t)b * a.slot_bytes;
    const uint32_t r0 = a.first[b];
    uint32_t doop = 0;
    for (uint32_t i = lane; i < n; i += 64) {
        const uint64_t slot = (uint64_t)b * a.cap + i;
        const uint32_t st = a.starts[slot], ln = a.lens[slot];
        const uint64_t r = (uint64_t)r0 + i;
        const uint64_t hl = a.hashloc[r];
        uint8_t* p = img + 9 + (uint64_t)i * bal;
        const uint8_t* d = a.digests + slot * 32;
        for (uint32_t k = 0; k < a.hash_len; k++) p[k] = d[k];
        p += a.hash_len;
        put_be32(p, (uint32_t)(hl >> 32));  // hashloc = Longs.toByteArray(pos)
        put_be32(p + 4, (uint32_t)hl);
        put_be32(p + 8, ln);                // len
        put_be32(p + 12, st);               // pos
        put_be32(p + 16, 0);                // offset
        put_be32(p + 20, ln);               // nlen
        if (a.dup[r]) doop += ln;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) doop += __shfl_xor(doop, o);
    if (lane == 0) {
        img[0] = 0;                    // flags (not RECONSTRUCTED)
        put_be32(img + 1, (uint32_t)need);  // buf.capacity()
        put_be32(img + 5, n);          // ar.size()
        put_be32(img + 9 + (uint64_t)n * bal, doop);
        if (a.doop) a.doop[b] = doop;
    }
}

}  // namespace
}  // namespace sdfs

using namespace sdfs;

extern "C" {

uint32_t sdfs_cdc_map_slot_bytes(uint32_t hash_len, uint32_t chunk_length, uint32_t min_len) {
    const uint32_t max_cluster = min_len ? chunk_length / min_len : 0;  // HashFunctionPool.java:66
    return 13 + (hash_len + 24) * 2 * max_cluster;
}

int sdfs_cdc_map_emit(int device, uint32_t nbuf, const sdfs_cdc_dev_out* out, uint32_t hash_len,
                      const uint8_t* d_dup, const uint64_t* d_hashloc, uint8_t* d_map, uint32_t slot_bytes,
                      uint32_t* d_doop, uint32_t* d_overflow, void* stream) {
    if (!out || !out->counts || !out->starts || !out->lens || !out->digests)
        return fail_status(SDFS_CDC_EINVAL, "incomplete sdfs_cdc_dev_out");
    if (hash_len != 32 && hash_len != 16)
        return fail_status(SDFS_CDC_EINVAL, "hash_len %u: HashLocPair holds 32 (SHA-256) or 16 (MD5) bytes", hash_len);
    if (nbuf && (!d_dup || !d_hashloc || !d_map || !d_overflow)) return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (nbuf == 0) return SDFS_CDC_OK;
    if (slot_bytes < 13) return fail_status(SDFS_CDC_EINVAL, "slot_bytes %u < 13", slot_bytes);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail_status(SDFS_CDC_ENODEV, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // per-call scratch for the buffers' first records, released once the stream reaches it
    uint32_t* first = nullptr;
    e = hipMallocAsync(reinterpret_cast<void**>(&first), (size_t)nbuf * 4, s);
    if (e != hipSuccess) return fail_status(SDFS_CDC_ENOMEM, "hipMallocAsync: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(map_prefix_kernel, dim3(1), dim3(1024), 0, s, out->counts, nbuf, first);
    MapArgs a{nbuf,     out->counts, out->starts, out->lens, out->digests, out->cap, hash_len, d_dup,
              d_hashloc, first,      d_map,       slot_bytes, d_doop,      d_overflow};
    hipLaunchKernelGGL(map_emit_kernel, dim3((nbuf + 3) / 4), dim3(256), 0, s, a);
    e = hipGetLastError();
    const hipError_t ef = hipFreeAsync(first, s);
    if (e != hipSuccess) return fail_status(SDFS_CDC_EHIP, "map_emit launch: %s", hipGetErrorString(e));
    if (ef != hipSuccess) return fail_status(SDFS_CDC_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return SDFS_CDC_OK;
}

}  // extern "C"
