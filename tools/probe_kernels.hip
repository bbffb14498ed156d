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
#include <hip/hip_runtime.h>

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

extern "C" {

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
