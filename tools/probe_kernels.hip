// probe_kernels.hip — measurement-only kernels that bench.py runs beside the product library
// (tools/libsdfs_probe.so; never linked into libsdfs_cdc.so).
//
// sdfs_probe_sha256_ceiling: the VALU issue ceiling of the fingerprint.  chunk_hash (cdc_device.h
// hash_task) spends its time in sha256_compress, one 64-byte block per lane per call, and the
// compression is issue-bound (scripts/valu_issue_mb.hip: the production round sequence runs at the
// issue rate of its own instruction mix; no order, register assignment or ILP form of the round
// beats it).  This kernel runs the SAME sha256_compress on register-resident data on every CU at
// `waves_per_simd` waves per SIMD (the rest of the CU's LDS reserved so exactly that many 256-thread
// workgroups fit), so bytes compressed per second here = the most chunk_hash can reach on this box
// at this clock; bench.py reports chunk_hash's compressed bytes per second against it.
//
// sdfs_probe_exchange_proxy_launch: a one-GPU stand-in for what the 8-rank fingerprint-table
// all-gather costs the step (bench.py --exchange-proxy).  RCCL's all-gather kernel holds a fixed
// number of workgroups (its channels) for as long as xGMI takes to deliver the peers' tables, and
// writes those bytes into this GPU's HBM.  This kernel does the same with local bytes: `wgs`
// workgroups of 256 threads copy `nbytes`, each paced by the wall clock so the copy lasts
// nbytes / gbps (the assumed xGMI receive rate), i.e. the same CU footprint for the same time.
#include <hip/hip_runtime.h>

#include <vector>

#include "../sdfs_amd/csrc/cdc_device.h"

using namespace sdfs;

__global__ __launch_bounds__(256) void probe_sha256_kernel(uint32_t* sink, int blocks_per_lane) {
    extern __shared__ uint32_t pad[];
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < blocks_per_lane; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = st[j & 7] + seed + j;
        sha256_compress(st, w);
    }
    if (threadIdx.x == 0xFFFFu) pad[0] = st[0];  // keeps the dynamic LDS (occupancy governor) allocated
    sink[blockIdx.x * 256 + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3] ^ st[4] ^ st[5] ^ st[6] ^ st[7];
}

// Paced copy: workgroup g copies its contiguous share in 32 KiB pieces (256 lanes x 8 x 16 B, all
// loads of a piece in flight before its stores), and before each piece waits until the wall clock
// (s_memrealtime) reaches its own start + bytes done / the per-workgroup rate.
__global__ __launch_bounds__(256) void exchange_proxy_kernel(uint4* dst, const uint4* src, uint64_t n16,
                                                             double bytes_per_tick) {
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per;
    const uint64_t hi = lo + per < n16 ? lo + per : n16;
    const uint64_t t0 = wall_clock64();
    for (uint64_t base = lo; base < hi; base += 2048) {
        const uint64_t due = t0 + (uint64_t)((double)(base - lo) * 16.0 / bytes_per_tick);
        while (wall_clock64() < due) __builtin_amdgcn_s_sleep(8);
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t i = base + k * 256 + threadIdx.x;
            v[k] = i < hi ? src[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t i = base + k * 256 + threadIdx.x;
            if (i < hi) dst[i] = v[k];
        }
    }
}

// The same loop with its waves' shader-clock and wall-clock spans (first lane of each wave):
// the clock the register-only compression runs at (scripts/hash_stamps.py).
__global__ __launch_bounds__(256) void probe_sha256_clock_kernel(uint32_t* sink, int blocks_per_lane, uint64_t* spans) {
    extern __shared__ uint32_t pad[];
    const uint64_t r0 = wall_clock64(), c0 = clock64();
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < blocks_per_lane; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = st[j & 7] + seed + j;
        sha256_compress(st, w);
    }
    if (threadIdx.x == 0xFFFFu) pad[0] = st[0];
    sink[blockIdx.x * 256 + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3] ^ st[4] ^ st[5] ^ st[6] ^ st[7];
    const uint64_t c1 = clock64(), r1 = wall_clock64();
    if ((threadIdx.x & 63) == 0) {
        uint64_t* q = spans + 2ull * ((blockIdx.x * 256 + threadIdx.x) >> 6);
        q[0] = c1 - c0;
        q[1] = r1 - r0;
    }
}

extern "C" {

// Mean shader clock (MHz) of the register-only compression at waves_per_simd waves per SIMD on
// every CU: sum of the waves' shader-clock spans over their wall-clock spans.
int sdfs_probe_sha256_clock(int device, int waves_per_simd, int blocks_per_lane, double* mhz) {
    if (waves_per_simd < 1 || waves_per_simd > 8 || blocks_per_lane < 1 || !mhz) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    hipDeviceProp_t p;
    int khz = 0;
    if (hipGetDeviceProperties(&p, device) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
        return -2;
    const int blocks = p.multiProcessorCount * waves_per_simd;
    const size_t lds = (size_t)(160 * 1024) / waves_per_simd - 1024;
    const size_t nw = (size_t)blocks * 4;
    uint32_t* sink = nullptr;
    uint64_t* spans = nullptr;
    int rc = 0;
    std::vector<uint64_t> h(2 * nw);
    if (hipMalloc(&sink, 4ull * blocks * 256) != hipSuccess || hipMalloc(&spans, 16 * nw) != hipSuccess) {
        rc = -3;
    } else {
        for (int r = 0; r < 2 && rc == 0; r++) {  // the first launch warms the clock
            hipLaunchKernelGGL(probe_sha256_clock_kernel, dim3(blocks), dim3(256), lds, 0, sink, blocks_per_lane, spans);
            if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -4;
        }
        if (rc == 0 && hipMemcpy(h.data(), spans, 16 * nw, hipMemcpyDeviceToHost) != hipSuccess) rc = -4;
        if (rc == 0) {
            double c = 0, w = 0;
            for (size_t i = 0; i < nw; i++) {
                c += (double)h[2 * i];
                w += (double)h[2 * i + 1];
            }
            *mhz = w > 0 ? c / w * (khz / 1000.0) : 0;
        }
    }
    if (sink) (void)hipFree(sink);
    if (spans) (void)hipFree(spans);
    return rc;
}

// Launches the paced copy on `stream` (a hipStream_t, 0 = the null stream): `nbytes` (a multiple of
// 16) from src to dst in `wgs` workgroups at `gbps` GB/s in total.  Returns 0 or a negative value.
int sdfs_probe_exchange_proxy_launch(void* dst, const void* src, uint64_t nbytes, int wgs, double gbps, void* stream) {
    if (!dst || !src || nbytes % 16 || wgs < 1 || gbps <= 0) return -1;
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        return -2;
    // bytes one workgroup moves per wall-clock tick
    const double per_tick = gbps * 1e9 / wgs / ((double)khz * 1e3);
    hipLaunchKernelGGL(exchange_proxy_kernel, dim3(wgs), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), nbytes / 16, per_tick);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Compressed input bytes per second (GB/s) of the register-only SHA-256 loop at waves_per_simd
// (1..8) waves per SIMD on every CU of `device`, best of `reps` timed launches (HIP events).
// Returns 0, or a negative value on a HIP error.
int sdfs_probe_sha256_ceiling(int device, int waves_per_simd, int blocks_per_lane, int reps, double* gbps,
                              double* ms_out) {
    if (waves_per_simd < 1 || waves_per_simd > 8 || blocks_per_lane < 1 || reps < 1 || !gbps) return -1;
    if (hipSetDevice(device) != hipSuccess) return -2;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return -2;
    const int blocks = p.multiProcessorCount * waves_per_simd;
    const size_t lds = (size_t)(160 * 1024) / waves_per_simd - 1024;  // gfx950: 160 KiB of LDS per CU
    uint32_t* sink = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    int rc = 0;
    if (hipMalloc(&sink, 4ull * blocks * 256) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        rc = -3;
    } else {
        hipLaunchKernelGGL(probe_sha256_kernel, dim3(blocks), dim3(256), lds, s, sink, blocks_per_lane);  // warm
        float best = 0;
        for (int r = 0; r < reps && rc == 0; r++) {
            float ms = 0;
            if (hipEventRecord(a, s) != hipSuccess) rc = -4;
            hipLaunchKernelGGL(probe_sha256_kernel, dim3(blocks), dim3(256), lds, s, sink, blocks_per_lane);
            if (hipGetLastError() != hipSuccess || hipEventRecord(b, s) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                hipEventElapsedTime(&ms, a, b) != hipSuccess)
                rc = -4;
            if (rc == 0 && (best == 0 || ms < best)) best = ms;
        }
        if (rc == 0) {
            *gbps = (double)blocks * 256 * blocks_per_lane * 64 / (best * 1e-3) / 1e9;
            if (ms_out) *ms_out = best;
        }
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (s) (void)hipStreamDestroy(s);
    if (sink) (void)hipFree(sink);
    return rc;
}

}  // extern "C"
