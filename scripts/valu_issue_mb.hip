// valu_issue_mb.hip — what one SIMD of gfx950 issues per cycle, measured with the shader clock.
//
// The clock: every wave reads s_memtime (core-clock cycles) and s_memrealtime (100 MHz) around its
// loop, which gives the clock the kernel actually ran at (the round-1 isa_microbench.hip assumed
// v_xor_b32 = 2 cycles to derive one).  The cost: the kernel's event time x that clock x 4 SIMDs x
// CUs / all waves' instructions = REAL cycles per wave64 instruction per SIMD ("wall_cycles_...").
// W waves per SIMD (one 256-thread block per CU per W, the rest of the CU's LDS reserved so exactly
// W blocks fit).  The per-wave figure (cycles / (W x instructions per wave), "cycles_...") is printed
// too but reads too low once W > 1: the SIMD does not interleave its waves evenly, so early waves
// finish first and each wave's own span is shorter than the kernel's.
//
// Forms (SHA-256 compression of chunk_hash, DESIGN.md §5, VERDICT r4 "what's weak" 2):
//   single ops, 8 independent accumulators      the issue cost of each op type
//   mix: the compression's op mix, independent  (a) the mix's issue ceiling
//   sha_prod: cdc_device.h sha256_compress      (b) the production round sequence
//   sha_roll: the schedule W[t+16] computed in round t (no per-16 batching)   (c)
//   add3 / bitop3 with three sources in one VGPR bank vs three banks           (d)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/valu_issue_mb.hip -o scripts/bin/valu_issue
#include "../sdfs_amd/csrc/cdc_device.h"

#include <cstdio>
#include <vector>

using namespace sdfs;

struct Rec {
    unsigned long long cyc, rt, r0;
};

#define TIMED_BEGIN                                           \
    __builtin_amdgcn_s_waitcnt(0);                            \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();  \
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#define TIMED_END(acc)                                                            \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                    \
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();                \
    if ((threadIdx.x & 63) == 0) {                                                 \
        const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);     \
        rec[w].cyc = t1 - t0;                                                      \
        rec[w].rt = r1 - r0;                                                       \
        rec[w].r0 = r0;                                                            \
    }                                                                              \
    sink[blockIdx.x * blockDim.x + threadIdx.x] = (acc);

// 8 independent accumulators, 8 ops each per iteration (64 VALU per iteration)
#define OP8(stmt)                                                                          \
    stmt(x0); stmt(x1); stmt(x2); stmt(x3); stmt(x4); stmt(x5); stmt(x6); stmt(x7);

template <int OP>
__global__ __launch_bounds__(256) void k_single(Rec* rec, uint32_t* sink, int iters, uint32_t s) {
    extern __shared__ uint32_t pad[];
    uint32_t x0 = threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 ^ 9, x5 = x0 + 11, x6 = x0 + 13,
             x7 = x0 + 17;
    const uint32_t y = s * threadIdx.x, z = s ^ threadIdx.x;
    TIMED_BEGIN
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if constexpr (OP == 0) { OP8([&](uint32_t& v) { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v) : "v"(y)); }) }
            if constexpr (OP == 1) { OP8([&](uint32_t& v) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(y)); }) }
            if constexpr (OP == 2) { OP8([&](uint32_t& v) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(y), "v"(z)); }) }
            if constexpr (OP == 3) { OP8([&](uint32_t& v) { asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(v)); }) }
            if constexpr (OP == 4) { OP8([&](uint32_t& v) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "v"(z)); }) }
            if constexpr (OP == 5) { OP8([&](uint32_t& v) { asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "v"(z)); }) }
            if constexpr (OP == 6) { OP8([&](uint32_t& v) { asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v)); }) }
            if constexpr (OP == 7) { OP8([&](uint32_t& v) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "s"(s)); }) }
            if constexpr (OP == 8) { OP8([&](uint32_t& v) { asm volatile("v_lshrrev_b32_sdwa %0, %1, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(v) : "s"(s)); }) }
            if constexpr (OP == 9) { OP8([&](uint32_t& v) { asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(v) : "v"(y)); }) }
            if constexpr (OP == 10) { OP8([&](uint32_t& v) { asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "v"(z)); }) }
            if constexpr (OP == 11) { OP8([&](uint32_t& v) { asm volatile("v_bfrev_b32 %0, %0" : "+v"(v)); }) }
        }
    }
    TIMED_END(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7)
    if (threadIdx.x == 100000) pad[0] = 0;
}

// (a) the compression's mix per 64 instructions, all independent: 26 alignbit, 16 bitop3,
// 11 add3, 6 add, 5 shift (576 / 352 / 241 / 118 / 96 per 64-byte block)
__global__ __launch_bounds__(256) void k_mix(Rec* rec, uint32_t* sink, int iters, uint32_t s) {
    extern __shared__ uint32_t pad[];
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * (2 * i + 1);
    const uint32_t y = s * threadIdx.x, z = s ^ threadIdx.x;
    TIMED_BEGIN
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 64; k++) {
            uint32_t& v = x[k & 7];
            const int m = (k * 37) % 64;  // spread the kinds through the group
            if (m < 26) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(v));
            else if (m < 42) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(y), "v"(z));
            else if (m < 53) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v) : "v"(y), "v"(z));
            else if (m < 59) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(y));
            else asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v));
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= x[i];
    TIMED_END(acc)
    if (threadIdx.x == 100000) pad[0] = 0;
}

// (c) message schedule rolled into the rounds: W[t+16] is computed in round t
__device__ __forceinline__ void sha256_compress_roll(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const uint32_t wi = w[i & 15];
        if (i < 48) {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            w[i & 15] = w[i & 15] + xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3) + w[(i + 9) & 15] +
                        xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        }
        const uint32_t t1 = h + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + __builtin_amdgcn_bitop3_b32(e, f, g, 0xE4) +
                            kSha256K[i] + wi;
        const uint32_t t2 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj3(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

template <int FORM>
__global__ __launch_bounds__(256) void k_sha(Rec* rec, uint32_t* sink, int iters, uint32_t s) {
    extern __shared__ uint32_t pad[];
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const uint32_t seed = blockIdx.x * 256 + threadIdx.x + s;
    TIMED_BEGIN
    for (int it = 0; it < iters; it++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = st[j & 7] + seed + j;
        if constexpr (FORM == 0) sha256_compress(st, w);
        else sha256_compress_roll(st, w);
    }
    TIMED_END(st[0] ^ st[1] ^ st[2] ^ st[3] ^ st[4] ^ st[5] ^ st[6] ^ st[7])
    if (threadIdx.x == 100000) pad[0] = 0;
}

// (d) three-source ops whose sources share one VGPR bank (v8, v12, v16: bank 0) or not
// (v9, v10, v11), eight destinations; fixed registers through the clobber list
template <int KIND>
__global__ __launch_bounds__(256) void k_bank(Rec* rec, uint32_t* sink, int iters, uint32_t s) {
    extern __shared__ uint32_t pad[];
    TIMED_BEGIN
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if constexpr (KIND == 0)
                asm volatile(
                    "v_add3_u32 v20, v8, v12, v16\n v_add3_u32 v21, v8, v12, v16\n v_add3_u32 v22, v8, v12, v16\n"
                    "v_add3_u32 v23, v8, v12, v16\n v_add3_u32 v24, v8, v12, v16\n v_add3_u32 v25, v8, v12, v16\n"
                    "v_add3_u32 v26, v8, v12, v16\n v_add3_u32 v27, v8, v12, v16" ::: "v8", "v12", "v16", "v20", "v21",
                    "v22", "v23", "v24", "v25", "v26", "v27");
            else if constexpr (KIND == 1)
                asm volatile(
                    "v_add3_u32 v20, v9, v10, v11\n v_add3_u32 v21, v9, v10, v11\n v_add3_u32 v22, v9, v10, v11\n"
                    "v_add3_u32 v23, v9, v10, v11\n v_add3_u32 v24, v9, v10, v11\n v_add3_u32 v25, v9, v10, v11\n"
                    "v_add3_u32 v26, v9, v10, v11\n v_add3_u32 v27, v9, v10, v11" ::: "v9", "v10", "v11", "v20", "v21",
                    "v22", "v23", "v24", "v25", "v26", "v27");
            else if constexpr (KIND == 2)
                asm volatile(
                    "v_add3_u32 v20, v8, v12, s4\n v_add3_u32 v21, v8, v12, s4\n v_add3_u32 v22, v8, v12, s4\n"
                    "v_add3_u32 v23, v8, v12, s4\n v_add3_u32 v24, v8, v12, s4\n v_add3_u32 v25, v8, v12, s4\n"
                    "v_add3_u32 v26, v8, v12, s4\n v_add3_u32 v27, v8, v12, s4" ::: "v8", "v12", "s4", "v20", "v21",
                    "v22", "v23", "v24", "v25", "v26", "v27");
            else if constexpr (KIND == 3)
                asm volatile(
                    "v_add3_u32 v20, v9, v10, s4\n v_add3_u32 v21, v9, v10, s4\n v_add3_u32 v22, v9, v10, s4\n"
                    "v_add3_u32 v23, v9, v10, s4\n v_add3_u32 v24, v9, v10, s4\n v_add3_u32 v25, v9, v10, s4\n"
                    "v_add3_u32 v26, v9, v10, s4\n v_add3_u32 v27, v9, v10, s4" ::: "v9", "v10", "s4", "v20", "v21",
                    "v22", "v23", "v24", "v25", "v26", "v27");
            else if constexpr (KIND == 4)
                asm volatile(
                    "v_alignbit_b32 v20, v8, v8, 7\n v_alignbit_b32 v21, v12, v12, 7\n v_alignbit_b32 v22, v16, v16, 7\n"
                    "v_alignbit_b32 v23, v8, v8, 9\n v_alignbit_b32 v24, v12, v12, 9\n v_alignbit_b32 v25, v16, v16, 9\n"
                    "v_alignbit_b32 v26, v8, v8, 11\n v_alignbit_b32 v27, v12, v12, 11" ::: "v8", "v12", "v16", "v20",
                    "v21", "v22", "v23", "v24", "v25", "v26", "v27");
            else
                asm volatile(
                    "v_bitop3_b32 v20, v8, v12, v16 bitop3:0x96\n v_bitop3_b32 v21, v8, v12, v16 bitop3:0x96\n"
                    "v_bitop3_b32 v22, v8, v12, v16 bitop3:0x96\n v_bitop3_b32 v23, v8, v12, v16 bitop3:0x96\n"
                    "v_bitop3_b32 v24, v9, v10, v11 bitop3:0x96\n v_bitop3_b32 v25, v9, v10, v11 bitop3:0x96\n"
                    "v_bitop3_b32 v26, v9, v10, v11 bitop3:0x96\n v_bitop3_b32 v27, v9, v10, v11 bitop3:0x96" ::: "v8",
                    "v9", "v10", "v11", "v12", "v16", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27");
        }
    }
    TIMED_END(s)
    if (threadIdx.x == 100000) pad[0] = 0;
}

typedef void (*kfn)(Rec*, uint32_t*, int, uint32_t);

static void measure(const char* name, kfn f, double instr_per_iter, int iters, int cus, Rec* d_rec, uint32_t* sink,
                    const char* unit = "instr") {
    for (int W : {1, 2, 4, 8}) {
        const size_t lds = (160 * 1024) / W - 1024;
        const int blocks = cus * W;
        hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d_rec, sink, iters / 4, 1u);
        (void)hipDeviceSynchronize();
        hipEvent_t ea, eb;
        (void)hipEventCreate(&ea);
        (void)hipEventCreate(&eb);
        (void)hipEventRecord(ea);
        hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d_rec, sink, iters, 1u);
        (void)hipEventRecord(eb);
        (void)hipEventSynchronize(eb);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ea, eb);
        const int nw = blocks * 4;
        std::vector<Rec> r(nw);
        (void)hipMemcpy(r.data(), d_rec, sizeof(Rec) * nw, hipMemcpyDeviceToHost);
        double cyc = 0, rt = 0;
        unsigned long long smin = ~0ull, smax = 0;
        for (auto& x : r) {
            cyc += (double)x.cyc;
            rt += (double)x.rt;
            smin = x.r0 < smin ? x.r0 : smin;
            smax = x.r0 > smax ? x.r0 : smax;
        }
        cyc /= nw;
        rt /= nw;
        const double ghz = cyc / (rt * 10.0);  // s_memrealtime ticks at 100 MHz
        const double per = cyc / (W * instr_per_iter * iters);
        // wall-clock cross-check: every wave's instructions over the kernel's event time, per SIMD
        // (4 SIMDs per CU), at the clock the waves saw; start_spread = latest wave start - earliest,
        // as a fraction of a wave's run (near 0: the W waves per SIMD really ran together)
        const double wall_per = (double)ms * 1e-3 * ghz * 1e9 * 4 * cus / ((double)nw * instr_per_iter * iters);
        printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_%s_per_simd\": %.3f, \"clock_ghz\": %.3f, "
               "\"wall_cycles_per_%s_per_simd\": %.3f, \"kernel_ms\": %.4f, \"start_spread\": %.3f}\n",
               name, W, unit, per, ghz, unit, wall_per, ms, (double)(smax - smin) / rt);
        fflush(stdout);
    }
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    Rec* d_rec;
    uint32_t* sink;
    (void)hipMalloc(&d_rec, sizeof(Rec) * cus * 8 * 4);
    (void)hipMalloc(&sink, 4ull * cus * 8 * 256);
    const int it = 2000;
    measure("v_xor_b32", k_single<0>, 64, it, cus, d_rec, sink);
    measure("v_add_u32", k_single<1>, 64, it, cus, d_rec, sink);
    measure("v_bitop3_b32", k_single<2>, 64, it, cus, d_rec, sink);
    measure("v_alignbit_b32", k_single<3>, 64, it, cus, d_rec, sink);
    measure("v_add3_u32(vvv)", k_single<4>, 64, it, cus, d_rec, sink);
    measure("v_add3_u32(vvs)", k_single<7>, 64, it, cus, d_rec, sink);
    measure("v_perm_b32", k_single<5>, 64, it, cus, d_rec, sink);
    measure("v_lshrrev_b32", k_single<6>, 64, it, cus, d_rec, sink);
    measure("v_lshrrev_b32_sdwa", k_single<8>, 64, it, cus, d_rec, sink);
    measure("v_mov_b32_sdwa", k_single<9>, 64, it, cus, d_rec, sink);
    measure("v_min3_u32", k_single<10>, 64, it, cus, d_rec, sink);
    measure("v_bfrev_b32", k_single<11>, 64, it, cus, d_rec, sink);
    measure("mix(a)", k_mix, 64, it, cus, d_rec, sink);
    measure("add3 same-bank vvv", k_bank<0>, 64, it, cus, d_rec, sink);
    measure("add3 3-bank vvv", k_bank<1>, 64, it, cus, d_rec, sink);
    measure("add3 same-bank vvs", k_bank<2>, 64, it, cus, d_rec, sink);
    measure("add3 2-bank vvs", k_bank<3>, 64, it, cus, d_rec, sink);
    measure("alignbit x,x", k_bank<4>, 64, it, cus, d_rec, sink);
    measure("bitop3 half same-bank", k_bank<5>, 64, it, cus, d_rec, sink);
    measure("sha_prod(b)", k_sha<0>, 1, 200, cus, d_rec, sink, "block");
    measure("sha_roll(c)", k_sha<1>, 1, 200, cus, d_rec, sink, "block");
    return 0;
}
