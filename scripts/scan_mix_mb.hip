// scan_mix_mb.hip — what bounds the scan's byte loop on gfx950 (SQ_WAIT_ANY 0.53,
// 1.21 ms per 4 GiB = ~40 wall cycles per wave-byte per SIMD at 4 waves/SIMD).
//
// One 1024-thread workgroup per CU with the production LDS tables (32 lane-private copies of the
// push and pop tables, 128 KiB), every lane rolling over 64 bytes of register-resident data per
// iteration (no global loads), the production per-byte sequence (cdc_device.h roll_step, mirrored
// state, SDWA addresses, pop entries high word first) and the group-of-8 candidate minimum:
//   chain   production: the push address comes from the rolling state (SDWA of lo), so every
//           byte waits for the previous byte's LDS read (address -> ds_read -> xor3 -> address)
//   free    the same instructions, but the push address is taken from a data dword: the LDS
//           reads no longer sit on the loop-carried chain (only the VALU shift/xor chain does)
//   valu    chain without the two LDS reads (register stand-ins, ABL 1|2: one extra shift each)
// Wall cycles per wave-byte per SIMD = kernel time x clock x 4 SIMDs x CUs / (waves x bytes).
// If `free` runs near `chain`, the loop is bound by issue + LDS throughput (no ILP will help); if
// it runs much faster, the chain's latency is what costs.  (An LDS-only form was dropped: hipcc
// hoisted its reads into 128 VGPRs and the number measured that, not the LDS.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/scan_mix_mb.hip -o scripts/bin/scan_mix_mb
#include "../sdfs_amd/csrc/cdc_device.h"

#include <cstdio>
#include <vector>

using namespace sdfs;

constexpr int kProdAbl = kAblMirror | kAblSdwa | kAblSdwaPop | kAblPopSwap;

// FORM 1: roll_step with the push address from data dword `ad` instead of the state
template <int P, int Q>
__device__ __forceinline__ void roll_free(uint32_t& lo, uint32_t& hi, uint32_t dw, uint32_t odw, uint32_t ad,
                                          uint32_t& c8, uint32_t& push_base, uint32_t jshift, const uint8_t* tab) {
    asm("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : "+v"(push_base)
        : "v"(ad), "s"(jshift));
    const uint32_t pa = push_base;
    sdwa_byte_to_b1<3 - Q>(c8, odw);
    const uint32_t qa = c8;
    const uint2 pv = *reinterpret_cast<const uint2*>(tab + pa);
    const uint2 qv = *reinterpret_cast<const uint2*>(tab + qa);
    const uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, 8);
    const uint32_t nhi = __builtin_amdgcn_perm(hi, dw, 0x00070605u | ((3u - P) << 24));
    lo = xor3(nlo, pv.x, qv.y);
    hi = xor3(nhi, pv.y, qv.x);
}

template <int O, int FORM>
__device__ __forceinline__ void steps(uint32_t& lo, uint32_t& hi, uint32_t& bits, const uint32_t (&cur)[16],
                                      const uint32_t (&prev)[16], uint32_t& c8, uint32_t& pb, uint32_t jshift,
                                      const uint8_t* tab, uint32_t (&hv)[8], uint32_t thr) {
    if constexpr (O < 64) {
        constexpr int OLD = O - 48;
        constexpr int OI = OLD >= 0 ? OLD : OLD + 64;
        const uint32_t odw = OLD >= 0 ? cur[OI >> 2] : prev[OI >> 2];
        if constexpr (FORM == 0)
            roll_step<(O & 3), (OI & 3), kProdAbl>(lo, hi, cur[O >> 2], odw, c8, pb, jshift, tab);
        else if constexpr (FORM == 1)
            roll_free<(O & 3), (OI & 3)>(lo, hi, cur[O >> 2], odw, cur[(O * 5 + 3) & 15], c8, pb, jshift, tab);
        else
            roll_step<(O & 3), (OI & 3), kProdAbl | 1 | 2>(lo, hi, cur[O >> 2], odw, c8, pb, jshift, tab);
        hv[O & 7] = hi;
        if constexpr ((O & 7) == 7) {
            uint32_t m = min(min(hv[0], hv[1]), hv[2]);
            m = min(min(m, hv[3]), hv[4]);
            m = min(min(m, hv[5]), hv[6]);
            m = min(m, hv[7]);
            if (__builtin_expect(__any(m < thr), 0))
                bits ^= m;
            else
                bits <<= 8;
        }
        if constexpr ((O & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        steps<O + 1, FORM>(lo, hi, bits, cur, prev, c8, pb, jshift, tab, hv, thr);
    }
}

struct Rec {
    unsigned long long cyc, rt;
};

template <int FORM>
__global__ __launch_bounds__(1024, 1) void k_scan(Rec* rec, uint32_t* sink, int iters, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[128 * 1024];
    for (int i = threadIdx.x; i < 128 * 1024 / 4; i += 1024)
        reinterpret_cast<uint32_t*>(tab)[i] = (uint32_t)i * 2654435761u ^ seed;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t c8 = (lane & 31) << 3;
    uint32_t pb = 0x10000u | c8;
    const uint32_t jshift = 11;
    uint32_t cur[16], prev[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        cur[j] = __builtin_bitreverse32((threadIdx.x + 1) * 0x9E3779B9u * (j + 3) ^ seed);
        prev[j] = __builtin_bitreverse32((threadIdx.x + 7) * 0x85EBCA6Bu * (j + 5) ^ seed);
    }
    uint32_t lo = threadIdx.x, hi = seed, bits = 0, hv[8];
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        steps<0, FORM>(lo, hi, bits, cur, prev, c8, pb, jshift, tab, hv, 0u);
        // next 64 bytes: one VALU per data dword (the production loop's bfrev of the loaded block)
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] ^= (uint32_t)it;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        const uint32_t w = blockIdx.x * 16 + (threadIdx.x >> 6);
        rec[w].cyc = t1 - t0;
        rec[w].rt = r1 - r0;
    }
    sink[blockIdx.x * 1024 + threadIdx.x] = lo ^ hi ^ bits;
}

typedef void (*kfn)(Rec*, uint32_t*, int, uint32_t);

static void measure(const char* name, kfn f, int iters, int cus, Rec* d_rec, uint32_t* sink) {
    hipLaunchKernelGGL(f, dim3(cus), dim3(1024), 0, 0, d_rec, sink, iters / 4, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t ea, eb;
    (void)hipEventCreate(&ea);
    (void)hipEventCreate(&eb);
    float best = 1e30f;
    double ghz = 0;
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(ea);
        hipLaunchKernelGGL(f, dim3(cus), dim3(1024), 0, 0, d_rec, sink, iters, 1u + rep);
        (void)hipEventRecord(eb);
        (void)hipEventSynchronize(eb);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ea, eb);
        if (ms < best) {
            best = ms;
            const int nw = cus * 16;
            std::vector<Rec> r(nw);
            (void)hipMemcpy(r.data(), d_rec, sizeof(Rec) * nw, hipMemcpyDeviceToHost);
            double cyc = 0, rt = 0;
            for (auto& x : r) {
                cyc += (double)x.cyc;
                rt += (double)x.rt;
            }
            ghz = cyc / (rt * 10.0);
        }
    }
    // 16 waves per CU = 4 per SIMD; each wave-iteration is 64 wave-bytes
    const double wave_bytes_per_simd = 4.0 * 64.0 * iters;
    const double wall = (double)best * 1e-3 * ghz * 1e9 / wave_bytes_per_simd;
    const double ms_4g = (double)best * (4294967296.0 / ((double)cus * 1024 * 64 * iters));
    printf("{\"form\": \"%s\", \"wall_cycles_per_wave_byte_per_simd\": %.2f, \"clock_ghz\": %.3f, \"kernel_ms\": %.4f, "
           "\"ms_per_4GiB_equiv\": %.3f}\n",
           name, wall, ghz, best, ms_4g);
    fflush(stdout);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    Rec* d_rec;
    uint32_t* sink;
    (void)hipMalloc(&d_rec, sizeof(Rec) * cus * 16);
    (void)hipMalloc(&sink, 4ull * cus * 1024);
    const int it = 2048;
    measure("chain (production)", k_scan<0>, it, cus, d_rec, sink);
    measure("free (push address from data)", k_scan<1>, it, cus, d_rec, sink);
    measure("valu (no LDS reads)", k_scan<2>, it, cus, d_rec, sink);
    return 0;
}
