// sdwa_microbench.hip — issue cost on gfx950 of the SDWA (sub-dword addressing) forms the scan's
// per-byte step could use instead of v_perm / v_alignbit / shift + v_bitop3:
//   v_lshrrev_b32_sdwa dst_sel:BYTE_1 UNUSED_PRESERVE   (push address: (lo >> s) & 0xFF into byte 1)
//   v_mov_b32_sdwa     dst_sel:BYTE_1 UNUSED_PRESERVE   (pop address: any data byte into byte 1)
//   v_mov_b32_sdwa     dst_sel:BYTE_3 UNUSED_PRESERVE   (insert the incoming byte on top)
//   v_lshrrev_b64                                          (shift the 64-bit state by 8 in one op)
// Throughput: cycles per wave64 instruction per SIMD (8 waves per SIMD, 8 independent
// accumulators per lane), calibrated on v_xor_b32 = 2 cycles so the clock drops out.
// Latency: one dependent chain per lane, one wave per SIMD, in v_xor_b32 units.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probes/sdwa_microbench.hip -o build/sdwa_mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define OPS(A, B, C)                                                                                                    \
    if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(A) : "v"(B));                                    \
    if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(A) : "v"(B), "v"(C));                        \
    if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %1, %0, 8" : "+v"(A) : "v"(B));                             \
    if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(A) : "v"(B), "v"(C));          \
    if constexpr (OP == 4)                                                                                              \
        asm volatile("v_lshrrev_b32_sdwa %0, 11, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "          \
                     "src1_sel:DWORD" : "+v"(A) : "v"(B));                                                              \
    if constexpr (OP == 5)                                                                                              \
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(A) : "v"(B)); \
    if constexpr (OP == 6)                                                                                              \
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(A) : "v"(B)); \
    if constexpr (OP == 7) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(A));                                          \
    if constexpr (OP == 8)                                                                                              \
        asm volatile("v_lshrrev_b32_sdwa %0, 11, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "          \
                     "src1_sel:DWORD" : "+v"(A));                                                                       \
    if constexpr (OP == 9)                                                                                              \
        asm volatile("v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 "             \
                     "src1_sel:BYTE_3" : "+v"(A) : "v"(B));                                                             \
    if constexpr (OP == 10)                                                                                             \
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(A) : "v"(B)); \
    if constexpr (OP == 11)                                                                                             \
        asm volatile("v_lshrrev_b32_sdwa %0, 11, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:DWORD "               \
                     "src1_sel:DWORD" : "=v"(A) : "v"(B));

constexpr int kNops = 12;
const char* kNames[kNops] = {"v_xor_b32",
                             "v_perm_b32",
                             "v_alignbit_b32",
                             "v_bitop3_b32",
                             "v_lshrrev_b32_sdwa BYTE_1 preserve (src != dst)",
                             "v_mov_b32_sdwa BYTE_1<-BYTE_2 preserve",
                             "v_mov_b32_sdwa BYTE_3<-BYTE_0 preserve",
                             "v_lshrrev_b32",
                             "v_lshrrev_b32_sdwa BYTE_1 preserve (src == dst)",
                             "v_xor_b32_sdwa BYTE_3 preserve",
                             "v_mov_b32_sdwa BYTE_1<-BYTE_2 pad",
                             "v_lshrrev_b32_sdwa BYTE_1 pad"};

template <int OP>
__global__ __launch_bounds__(256) void kthr(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5A5A5A5Au;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#define OPX(k) OPS(a##k, b, c)
            R8(OPX)
#undef OPX
            b += a0;  // keep (b, c) live and varying across iterations
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b;
}

template <int OP>
__global__ __launch_bounds__(256) void klat(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed;
    const uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5A5A5A5Au;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 64; u++) {
            if constexpr (OP == 10 || OP == 11) {
                uint32_t t;
                OPS(t, a, c)
                a = t ^ b;  // keep it a chain: the padded forms do not read their destination
            } else {
                OPS(a, b, c)
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

template <typename K>
float time_kernel(K kern, int blocks, int iters, uint32_t* out) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 2u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

template <int OP>
void run(int cus, uint32_t* out, float* thr, float* lat) {
    thr[OP] = time_kernel(kthr<OP>, cus * 8, 2000, out);
    lat[OP] = time_kernel(klat<OP>, cus, 2000, out);
    if constexpr (OP + 1 < kNops) run<OP + 1>(cus, out, thr, lat);
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    CHECK(hipMalloc(&out, cus * 8 * 256 * 4));
    float thr[kNops], lat[kNops];
    run<0>(cus, out, thr, lat);
    // throughput kernel: per SIMD 8 waves x 2000 x 16 x 8 instructions (+16 v_add per iter)
    printf("{\"cus\": %d, \"ops\": [\n", cus);
    for (int i = 0; i < kNops; i++)
        printf("  {\"op\": \"%s\", \"thr_cycles\": %.2f, \"lat_cycles\": %.2f}%s\n", kNames[i], 2.0 * thr[i] / thr[0],
               2.0 * lat[i] / lat[0], i + 1 < kNops ? "," : "");
    printf("], \"note\": \"thr: cycles per wave64 instruction per SIMD at 8 waves/SIMD (v_xor_b32 = 2); lat: dependent "
           "chain, 1 wave/SIMD, in units where v_xor_b32 = 2 (x_lat/x_xor * 2)\"}\n");
    return 0;
}
