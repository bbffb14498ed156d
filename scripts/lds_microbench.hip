// lds_microbench.hip — LDS read throughput on gfx950 for the scan's table-lookup patterns.
// 8 independent ds_read_b64 per iteration from addresses held in registers (rotated by a
// scalar xor each iteration, 1 cheap VALU per read), 8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/lds_microbench.hip -o build/lds_mb
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE, int BYTES>
__global__ __launch_bounds__(256) void klds(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[65536];
    for (int i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<uint32_t*>(tab)[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t addr[8];
    uint32_t x = threadIdx.x * 0x9E3779B9u + 12345u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint32_t row = (x >> 8) & 255;
        if (MODE == 0) addr[k] = (row << 8) | ((lane & 31) << 3);        // 32 lane-private copies
        if (MODE == 1) addr[k] = (row << 8) | ((lane & 15) << 3);        // 16 copies (2-way)
        if (MODE == 2) addr[k] = ((x >> 16) & 0xFFF8);                   // random 8-byte entries
        if (MODE == 3) addr[k] = (row << 8) | ((lane & 7) << 3);         // 8 copies (4-way)
    }
    uint32_t a0 = 0, a1 = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t flip = (uint32_t)(i & 255) << 8;  // scalar: next row, same bank
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t ad = addr[k] ^ flip;
            if constexpr (BYTES == 8) {
                const uint2 v = *reinterpret_cast<const uint2*>(tab + ad);
                a0 ^= v.x; a1 ^= v.y;
            } else {
                a0 ^= *reinterpret_cast<const uint32_t*>(tab + ad);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1;
}

template <typename K>
float run(K k, int blocks, int iters, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    (void)hipMalloc(&out, 64 << 20);
    const int iters = 4000;
    const double ghz = 2.1;  // approximate; ratios between modes are what matters
    const char* names[] = {"b64 32 lane-private copies", "b64 16 copies (2-way)", "b64 random", "b64 8 copies (4-way)",
                           "b32 32 copies", "b32 random"};
    for (int wps = 2; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;  // 256-thread blocks: wps blocks per CU = wps waves per SIMD
        float ms[6] = {run(klds<0, 8>, blocks, iters, out), run(klds<1, 8>, blocks, iters, out),
                       run(klds<2, 8>, blocks, iters, out), run(klds<3, 8>, blocks, iters, out),
                       run(klds<0, 4>, blocks, iters, out), run(klds<2, 4>, blocks, iters, out)};
        for (int m = 0; m < 6; m++) {
            const double reads_per_cu = (double)wps * 4 * iters * 8;  // wave-level reads per CU
            printf("waves/SIMD %d  %-28s %7.3f ms  %5.2f cycles per wave-read per CU (@%.1f GHz)\n", wps, names[m],
                   ms[m], ms[m] * 1e-3 * ghz * 1e9 / reads_per_cu, ghz);
        }
    }
    return 0;
}
