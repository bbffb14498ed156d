// isa_microbench.hip — issue throughput of the VALU/LDS instructions the CDC + SHA kernels are
// built from, on gfx950 (cycles per wave64 instruction per SIMD, 8 waves per SIMD, 8 independent
// accumulators per lane).  Calibrated against v_add_u32 (expected 2 cycles on a SIMD-32) so the
// clock drops out.  Build: hipcc --offload-arch=gfx950 -O3 scripts/isa_microbench.hip -o build/isa_mb
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

template <int OP>
__global__ __launch_bounds__(256) void kvalu(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5A5A5A5Au;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#define OPX(k)                                                                                              \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));                      \
    if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "v"(c));          \
    if constexpr (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a##k) : "v"(b));               \
    if constexpr (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##k) : "v"(b), "v"(c)); \
    if constexpr (OP == 4) asm volatile("v_bfe_u32 %0, %0, 5, 8" : "+v"(a##k));                             \
    if constexpr (OP == 5) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a##k) : "v"(b));                \
    if constexpr (OP == 6) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "v"(c));          \
    if constexpr (OP == 7) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##k) : "v"(b));                       \
    if constexpr (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a##k));                       \
    if constexpr (OP == 9) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "s"(0x06050400u));          \
    if constexpr (OP == 10) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##k) : "v"(a0), "v"(a1)); \
    if constexpr (OP == 11) asm volatile("v_and_b32 %0, 0xfff, %0" : "+v"(a##k));                            \
    if constexpr (OP == 12) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a##k));                           \
    if constexpr (OP == 13) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a##k) : "v"(b));              \
    if constexpr (OP == 14) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a##k) : "v"(b));              \
    if constexpr (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##k) : "v"(b));             \
    if constexpr (OP == 16) asm volatile("v_mov_b32 %0, %1" : "=v"(a##k) : "v"(b));                           \
    if constexpr (OP == 17) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##k) : "v"(b));                  \
    if constexpr (OP == 18) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "v"(c));          \
    if constexpr (OP == 19) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a##k) : "v"(b), "v"(c));

            R8(OPX)
#undef OPX
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 64-bit shifts on register pairs: v_lshrrev_b64 / v_lshlrev_b64 / v_lshl_add_u64 / v_mov_b64
template <int OP>
__global__ __launch_bounds__(256) void kvalu64(uint32_t* out, int iters, uint32_t seed) {
    uint64_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint64_t b = seed * 0x9E3779B97F4A7C15ull + threadIdx.x;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
#define OPX(k)                                                                                     \
    if constexpr (OP == 0) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a##k));                  \
    if constexpr (OP == 1) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(a##k));                  \
    if constexpr (OP == 2) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(a##k) : "v"(b));    \
    if constexpr (OP == 3) asm volatile("v_mov_b64 %0, %1" : "=v"(a##k) : "v"(b));
            R8(OPX)
#undef OPX
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

// candidate chain: v_and + v_cmp(vcc) + v_addc(vcc) per step, 4 independent chains
__global__ __launch_bounds__(256) void kcand(uint32_t* out, int iters, uint32_t seed) {
    uint32_t l0 = threadIdx.x ^ seed, l1 = l0 * 3, l2 = l0 * 5, l3 = l0 * 7;
    uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, t;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 32; u++) {
#define CX(k)                                                                                   \
    asm volatile("v_and_b32 %1, 0xfff, %2\n\tv_cmp_eq_u32 vcc, 0, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" \
                 : "+v"(b##k), "=&v"(t) : "v"(l##k) : "vcc");
            CX(0) CX(1) CX(2) CX(3)
#undef CX
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = b0 ^ b1 ^ b2 ^ b3 ^ t;
}

// LDS: ds_read_b64, lane-private 8-byte slots (conflict-free) or random rows, 8 in flight
template <int MODE>
__global__ __launch_bounds__(256) void klds(uint32_t* out, int iters, uint32_t seed) {
    __shared__ uint2 tab[8192];  // 64 KiB
    for (int i = threadIdx.x; i < 8192; i += 256) tab[i] = make_uint2(i * 2654435761u, i);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x = threadIdx.x * 0x9E3779B9u ^ seed;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        uint32_t addr[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            x = x * 1664525u + 1013904223u;
            const uint32_t row = (x >> 20) & 255;
            addr[k] = MODE == 0 ? ((row << 8) | ((lane & 31) << 3)) : ((row << 8) | ((x >> 8) & 0xF8));
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(tab) + addr[k]);
            acc ^= v.x + v.y;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// dependent-chain latency: ONE accumulator per lane, one wave per SIMD
template <int OP>
__global__ __launch_bounds__(256) void klat(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed;
    const uint32_t b = seed * 0x9E3779B9u + threadIdx.x, c = b ^ 0x5A5A5A5Au;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 64; u++) {
            if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
            if constexpr (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
            if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
            if constexpr (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
            if constexpr (OP == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a));
            if constexpr (OP == 5) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
            if constexpr (OP == 6) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

// dependent LDS round trip: address from the previous load's value
__global__ __launch_bounds__(256) void klatlds(uint32_t* out, int iters, uint32_t seed) {
    __shared__ uint2 tab[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) tab[i] = make_uint2((i * 8 + 8) & 0xFFF8, i);
    __syncthreads();
    uint32_t a = (threadIdx.x & 31) << 3;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(tab) + a);
            a = v.x;
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

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;  // 8 x 256 threads = 32 waves per CU = 8 per SIMD
    uint32_t* out;
    CHECK(hipMalloc(&out, blocks * 256 * 4));
    const int iters = 2000;
    const double simds = cus * 4.0;
    const double wave_instr_valu = (double)blocks * 4 * iters * 16 * 8;  // per kernel
    const char* names[] = {"v_add_u32", "v_perm_b32(vvv)", "v_alignbit_b32(vv,imm)", "v_bitop3_b32(vvv)",
                           "v_bfe_u32(v,imm,imm)", "v_lshl_or_b32(v,imm,v)", "v_add3_u32(vvv)", "v_xor_b32",
                           "v_alignbit_b32 rot(x,x)", "v_perm_b32(vv,sgpr)", "v_bitop3(a,a0,a1)", "v_and_b32 lit",
                           "v_lshrrev_b32", "v_alignbyte_b32", "v_lshl_add_u32", "v_cndmask_b32 vcc", "v_mov_b32",
                           "v_mul_u32_u24", "v_or3_b32", "v_and_or_b32"};
    constexpr int NOPS = 20;
    float ms[NOPS];
    ms[0] = time_kernel(kvalu<0>, blocks, iters, out);
    ms[1] = time_kernel(kvalu<1>, blocks, iters, out);
    ms[2] = time_kernel(kvalu<2>, blocks, iters, out);
    ms[3] = time_kernel(kvalu<3>, blocks, iters, out);
    ms[4] = time_kernel(kvalu<4>, blocks, iters, out);
    ms[5] = time_kernel(kvalu<5>, blocks, iters, out);
    ms[6] = time_kernel(kvalu<6>, blocks, iters, out);
    ms[7] = time_kernel(kvalu<7>, blocks, iters, out);
    ms[8] = time_kernel(kvalu<8>, blocks, iters, out);
    ms[9] = time_kernel(kvalu<9>, blocks, iters, out);
    ms[10] = time_kernel(kvalu<10>, blocks, iters, out);
    ms[11] = time_kernel(kvalu<11>, blocks, iters, out);
    ms[12] = time_kernel(kvalu<12>, blocks, iters, out);
    ms[13] = time_kernel(kvalu<13>, blocks, iters, out);
    ms[14] = time_kernel(kvalu<14>, blocks, iters, out);
    ms[15] = time_kernel(kvalu<15>, blocks, iters, out);
    ms[16] = time_kernel(kvalu<16>, blocks, iters, out);
    ms[17] = time_kernel(kvalu<17>, blocks, iters, out);
    ms[18] = time_kernel(kvalu<18>, blocks, iters, out);
    ms[19] = time_kernel(kvalu<19>, blocks, iters, out);
    const float xor_ms = ms[7];  // calibration: a plain 2-operand VALU op = 2 cycles per wave64 on SIMD-32
    const double ghz = wave_instr_valu * 2.0 / simds / (xor_ms * 1e-3) / 1e9;
    printf("effective clock if v_xor_b32 = 2 cyc/wave-instr: %.2f GHz\n", ghz);
    for (int i = 0; i < NOPS; i++)
        printf("%-28s %8.3f ms  %5.2f cyc/wave-instr/SIMD\n", names[i], ms[i], 2.0 * ms[i] / xor_ms);
    const char* n64[] = {"v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_mov_b64"};
    float m64[4] = {time_kernel(kvalu64<0>, blocks, iters, out), time_kernel(kvalu64<1>, blocks, iters, out),
                    time_kernel(kvalu64<2>, blocks, iters, out), time_kernel(kvalu64<3>, blocks, iters, out)};
    for (int i = 0; i < 4; i++)
        printf("%-28s %8.3f ms  %5.2f cyc/wave-instr/SIMD\n", n64[i], m64[i], 2.0 * m64[i] / xor_ms);
    {
        const char* ln[] = {"v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_perm_b32", "v_lshrrev_b32",
                            "v_add3_u32", "v_add_u32"};
        const int lb = cus;  // one 256-thread block per CU = one wave per SIMD
        const int li = 200;
        float lm[7] = {time_kernel(klat<0>, lb, li, out), time_kernel(klat<1>, lb, li, out),
                       time_kernel(klat<2>, lb, li, out), time_kernel(klat<3>, lb, li, out),
                       time_kernel(klat<4>, lb, li, out), time_kernel(klat<5>, lb, li, out),
                       time_kernel(klat<6>, lb, li, out)};
        for (int i = 0; i < 7; i++)
            printf("dependent %-18s %6.1f cycles/instr (1 wave/SIMD)\n", ln[i], lm[i] * 1e-3 * ghz * 1e9 / (li * 64.0));
        float ll = time_kernel(klatlds, lb, li, out);
        printf("dependent ds_read_b64 round trip %6.1f cycles\n", ll * 1e-3 * ghz * 1e9 / (li * 16.0));
    }
    float mc = time_kernel(kcand, blocks, iters, out);
    const double wi_c = (double)blocks * 4 * iters * 32 * 4 * 3;
    printf("%-28s %8.3f ms  %5.2f cyc/wave-instr (3 instr/step)\n", "and+cmp(vcc)+addc chain", mc,
           mc * 1e-3 * ghz * 1e9 * simds / wi_c);
    for (int mode = 0; mode < 2; mode++) {
        float ml = mode == 0 ? time_kernel(klds<0>, blocks, iters, out) : time_kernel(klds<1>, blocks, iters, out);
        const double reads = (double)blocks * 4 * iters * 8;  // wave-level ds_read_b64
        printf("ds_read_b64 %-16s %8.3f ms  %5.2f LDS cyc per wave-read per CU\n",
               mode == 0 ? "lane-private" : "random", ml, ml * 1e-3 * ghz * 1e9 * cus / reads);
    }
    return 0;
}
