// sha_occupancy_mb.hip — throughput of the production SHA-256 compression (cdc_kernels.hip) on
// register-resident data vs waves per SIMD (occupancy capped with dynamic LDS), gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/sha_occupancy_mb.hip -o build/sha_mb
#include "../sdfs_amd/csrc/cdc_kernels.hip"

#include <cstdio>

using namespace sdfs;

__global__ __launch_bounds__(256) void ksha(uint32_t* out, int blocks_per_lane) {
    extern __shared__ uint32_t pad[];
    uint32_t s[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int b = 0; b < blocks_per_lane; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = s[j & 7] + seed + j;
        sha256_compress(s, w);
    }
    if (threadIdx.x == 1023) pad[0] = s[0];
    out[blockIdx.x * 256 + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3] ^ s[4] ^ s[5] ^ s[6] ^ s[7];
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    (void)hipMalloc(&out, 64 << 20);
    const int bpl = 200;
    for (int wps = 1; wps <= 8; wps++) {
        const size_t lds = (160 * 1024) / wps - 1024;  // at most wps 256-thread blocks per CU
        const int blocks = cus * wps * 4;              // 4 rounds of full occupancy
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        hipLaunchKernelGGL(ksha, dim3(blocks), dim3(256), lds, 0, out, bpl);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(ksha, dim3(blocks), dim3(256), lds, 0, out, bpl);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double bytes = (double)blocks * 256 * bpl * 64;
        printf("waves/SIMD %d: %.3f ms  %.1f GB/s of SHA-256 input (register data)\n", wps, ms, bytes / ms / 1e6);
    }
    return 0;
}
