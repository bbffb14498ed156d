// cdc_sweep.hip — measurement-only kernel variants (scan layouts, ablations, fingerprint-kernel
// forms) for the A/B sweeps behind DESIGN.md §7-8 (scripts/sweep_scan.py, scripts/ab.py).
// Built only into the tuning library (`make tuning` -> sdfs_amd/libsdfs_cdc_tuning.so, compiled
// with -DSDFS_TUNING); the product library libsdfs_cdc.so contains none of these kernels and
// ignores every SDFS_* tuning variable.
#include <algorithm>

#include "cdc_device.h"

namespace sdfs {

// scan variants: ScanCfg<copies, chains, prefetch, waves/SIMD, ablation, block bytes, fuse>
using ScanV21 = ScanCfg<32, 1, false, 4, 0, 256, 2>;  // register-summary resolve without the split body
using ScanV20 = ScanCfg<32, 1, false, 4, 0, 256>;    // production before the fused resolve
using ScanV16 = ScanCfg<32, 2, false, 4>;  // round-1 first version: 64-byte loads, 2 chains
using ScanV17 = ScanCfg<32, 2, true, 4, 0, 128>;
using ScanV1 = ScanCfg<32, 2, true, 4>;
using ScanV2 = ScanCfg<32, 1, true, 4>;
using ScanV3 = ScanCfg<16, 1, true, 8>;
using ScanV4 = ScanCfg<16, 1, false, 8>;
using ScanV5 = ScanCfg<16, 2, false, 4>;
using ScanV6 = ScanCfg<32, 2, false, 4, 0, 128>;
using ScanV7 = ScanCfg<32, 1, false, 4, 0, 128>;
using ScanV8 = ScanCfg<16, 1, false, 8, 0, 128>;
using ScanV9 = ScanCfg<32, 1, true, 4, 0, 128>;
using ScanV10 = ScanCfg<32, 1, false, 4, 0, 256>;
using ScanV15 = ScanCfg<32, 2, false, 4, 0, 256>;
using ScanV19 = ScanCfg<32, 1, false, 4, 0, 128, 1>;  // 128-B blocks + bitmap-walk resolve in the epilogue
// more independent rolling chains per SIMD at the same 128 KiB of tables: several segments per
// lane, fewer waves, the register budget that frees (fused walk of every chain's buffer)
using ScanV22 = ScanCfg<32, 2, false, 3, 16, 128, 2, 768>;  // 2 chains x 3 waves/SIMD, 168 VGPRs
using ScanV26 = ScanCfg<32, 3, false, 2, 16, 128, 2, 512>;  // 3 chains x 2 waves/SIMD, 256 VGPRs
using ScanV27 = ScanCfg<32, 4, false, 2, 16, 128, 2, 512>;  // 4 chains x 2 waves/SIMD
using ScanV28 = ScanCfg<32, 2, false, 2, 16, 256, 2, 512>;  // 2 chains x 2 waves/SIMD, 256-B blocks
// ablations (ids 11..25): 1 = no pop read, 2 = no push read, 4 = no candidate test, 8 = no
// global loads; the skipped values are replaced by register values that keep the rest live
// production before / with the bit-reversed (mirrored) rolling state
using ScanV29 = ScanCfg<32, 1, false, 4, 16, 256, 2>;
using ScanV30 = ScanCfg<32, 1, false, 4, 16, 256, 2, kScanThreads, true>;
// production with the round-2 cut walk (a min over the 8 summary slots per cut, ABL bit 128)
using ScanV31 = ScanCfg<32, 1, false, 4, 16 | 128, 256, 2, kScanThreads, true>;
// production with the candidate bits built from per-position SGPR masks (kAblSgprPred)
using ScanV32 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred, 256, 2, kScanThreads, true>;
// ablations of the production kernel (round 3): no pop read / no push read / neither
using ScanV33 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | 1, 256, 2, kScanThreads, true>;
using ScanV34 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | 2, 256, 2, kScanThreads, true>;
using ScanV35 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | 3, 256, 2, kScanThreads, true>;
// production for batches of whole blocks only: no guarded load path in the block loop (kAblFullBlocks)
using ScanV36 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | kAblFullBlocks, 256, 2, kScanThreads, true>;
// two rolling chains per lane (more independent LDS round trips in flight per SIMD), 128-byte
// blocks: 2 chains x 4 waves/SIMD (128 VGPRs) / 2 chains x 3 waves/SIMD (150 VGPRs)
using ScanV37 = ScanCfg<32, 2, false, 4, 16 | kAblSgprPred | kAblFullBlocks, 128, 2, 1024, true>;
using ScanV38 = ScanCfg<32, 2, false, 3, 16 | kAblSgprPred | kAblFullBlocks, 128, 2, 768, true>;
// more ablations of the production kernel (round 3): 4 = no candidate test (one v_xor per byte
// instead of the SGPR-mask compare and its scalar OR / group branch), 8 = no global loads (block
// words synthesized from registers; the guarded body), and their combinations with the LDS reads
using ScanV39 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | kAblFullBlocks | 4, 256, 2, kScanThreads, true>;
using ScanV40 = ScanCfg<32, 1, false, 4, kAblSgprPred | 8, 256, 2, kScanThreads, true>;
using ScanV41 = ScanCfg<32, 1, false, 4, kAblSgprPred | 4 | 8, 256, 2, kScanThreads, true>;
using ScanV42 = ScanCfg<32, 1, false, 4, kAblSgprPred | 3 | 4 | 8, 256, 2, kScanThreads, true>;
using ScanA1 = ScanCfg<32, 1, false, 4, 1, 128>;
using ScanA2 = ScanCfg<32, 1, false, 4, 2, 128>;
using ScanA3 = ScanCfg<32, 1, false, 4, 3, 128>;
using ScanA4 = ScanCfg<32, 1, false, 4, 4, 128>;
using ScanA8 = ScanCfg<32, 1, false, 4, 8, 128>;
using ScanA15 = ScanCfg<32, 1, false, 4, 15, 128>;

template <class CFG>
constexpr ScanVariantInfo sweep_info() {
    return {CFG::kCopies, CFG::kChains, CFG::kLds, std::max(1, CFG::kWavesPerSimd * 256 / CFG::kThreads), CFG::kBlk,
            CFG::kFuse, CFG::kThreads, CFG::kMirror};
}

ScanVariantInfo scan_variant_info_sweep(int v) {
    switch (v) {
    case 1: return sweep_info<ScanV1>();
    case 2: return sweep_info<ScanV2>();
    case 3: return sweep_info<ScanV3>();
    case 4: return sweep_info<ScanV4>();
    case 5: return sweep_info<ScanV5>();
    case 6: return sweep_info<ScanV6>();
    case 7: return sweep_info<ScanV7>();
    case 8: return sweep_info<ScanV8>();
    case 9: return sweep_info<ScanV9>();
    case 10: return sweep_info<ScanV10>();
    case 15: return sweep_info<ScanV15>();
    case 16: return sweep_info<ScanV16>();
    case 17: return sweep_info<ScanV17>();
    case 19: return sweep_info<ScanV19>();
    case 20: return sweep_info<ScanV20>();
    case 21: return sweep_info<ScanV21>();
    case 11: return sweep_info<ScanA1>();
    case 12: return sweep_info<ScanA2>();
    case 13: return sweep_info<ScanA3>();
    case 14: return sweep_info<ScanA4>();
    case 18: return sweep_info<ScanA8>();
    case 25: return sweep_info<ScanA15>();
    case 22: return sweep_info<ScanV22>();
    case 26: return sweep_info<ScanV26>();
    case 27: return sweep_info<ScanV27>();
    case 28: return sweep_info<ScanV28>();
    case 29: return sweep_info<ScanV29>();
    case 30: return sweep_info<ScanV30>();
    case 31: return sweep_info<ScanV31>();
    case 32: return sweep_info<ScanV32>();
    case 33: return sweep_info<ScanV33>();
    case 34: return sweep_info<ScanV34>();
    case 35: return sweep_info<ScanV35>();
    case 36: return sweep_info<ScanV36>();
    case 37: return sweep_info<ScanV37>();
    case 38: return sweep_info<ScanV38>();
    case 39: return sweep_info<ScanV39>();
    case 40: return sweep_info<ScanV40>();
    case 41: return sweep_info<ScanV41>();
    case 42: return sweep_info<ScanV42>();
    default: return scan_variant_info_sweep_r3(v);
    }
}

template <class T>
static hipError_t sweep_launch(const ScanArgs& a, int pk, int grid, int block, hipStream_t s) {
    if ((T::kAbl & kAblFullBlocks) != 0 && !scan_full_blocks(a, T::kBlk)) return hipErrorInvalidValue;
    if (pk == 1)
        hipLaunchKernelGGL((cdc_scan_kernel<48, 1, T>), dim3(grid), dim3(block), 0, s, a);
    else if (pk == 2 && T::kMirror)
        hipLaunchKernelGGL((cdc_scan_kernel<48, T::kMirror ? 2 : 0, T>), dim3(grid), dim3(block), 0, s, a);
    else
        hipLaunchKernelGGL((cdc_scan_kernel<48, 0, T>), dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_scan_sweep(const ScanArgs& a, int window, int pk, int variant, int grid, int block, hipStream_t s) {
    if (window != 48) return hipErrorInvalidValue;  // variants are built for the reference window only
    switch (variant) {
#define SWEEP_CASE(id, T) \
    case id: return sweep_launch<T>(a, pk, grid, block, s);
    SWEEP_CASE(1, ScanV1) SWEEP_CASE(2, ScanV2) SWEEP_CASE(3, ScanV3) SWEEP_CASE(4, ScanV4)
    SWEEP_CASE(5, ScanV5) SWEEP_CASE(6, ScanV6) SWEEP_CASE(7, ScanV7) SWEEP_CASE(8, ScanV8)
    SWEEP_CASE(9, ScanV9) SWEEP_CASE(10, ScanV10) SWEEP_CASE(15, ScanV15) SWEEP_CASE(16, ScanV16)
    SWEEP_CASE(17, ScanV17) SWEEP_CASE(19, ScanV19) SWEEP_CASE(20, ScanV20) SWEEP_CASE(21, ScanV21)
    SWEEP_CASE(11, ScanA1) SWEEP_CASE(12, ScanA2) SWEEP_CASE(13, ScanA3) SWEEP_CASE(14, ScanA4)
    SWEEP_CASE(18, ScanA8) SWEEP_CASE(25, ScanA15) SWEEP_CASE(22, ScanV22) SWEEP_CASE(26, ScanV26)
    SWEEP_CASE(27, ScanV27) SWEEP_CASE(28, ScanV28) SWEEP_CASE(29, ScanV29) SWEEP_CASE(30, ScanV30)
    SWEEP_CASE(31, ScanV31) SWEEP_CASE(32, ScanV32) SWEEP_CASE(33, ScanV33) SWEEP_CASE(34, ScanV34)
    SWEEP_CASE(35, ScanV35) SWEEP_CASE(36, ScanV36) SWEEP_CASE(37, ScanV37)
    SWEEP_CASE(38, ScanV38) SWEEP_CASE(39, ScanV39) SWEEP_CASE(40, ScanV40) SWEEP_CASE(41, ScanV41)
    SWEEP_CASE(42, ScanV42)
#undef SWEEP_CASE
    default: return launch_scan_sweep_r3(a, window, pk, variant, grid, block, s);
    }
}

// ---- two chunks per lane (variant 40/41): two independent SHA-256 chains interleaved round by
// round in one lane, for twice the instruction-level parallelism per wave at ~1.5x the VGPRs.
// Lane l of workgroup g takes tasks 2(256g+l) and 2(256g+l)+1: adjacent in the longest-first
// list, so (binned by exact block count) their block counts are equal or differ by one.
__device__ __forceinline__ void sha_round_pair(uint32_t (&x)[8], uint32_t (&y)[8], uint32_t k, uint32_t wx, uint32_t wy) {
    {
        const uint32_t S1 = xor3(rotr(x[4], 6), rotr(x[4], 11), rotr(x[4], 25));
        const uint32_t ch = (x[4] & x[5]) | (~x[4] & x[6]);
        const uint32_t t1 = x[7] + S1 + ch + k + wx;
        const uint32_t S0 = xor3(rotr(x[0], 2), rotr(x[0], 13), rotr(x[0], 22));
        const uint32_t mj = maj3(x[0], x[1], x[2]);
        x[7] = x[6]; x[6] = x[5]; x[5] = x[4]; x[4] = x[3] + t1; x[3] = x[2]; x[2] = x[1]; x[1] = x[0]; x[0] = t1 + S0 + mj;
    }
    {
        const uint32_t S1 = xor3(rotr(y[4], 6), rotr(y[4], 11), rotr(y[4], 25));
        const uint32_t ch = (y[4] & y[5]) | (~y[4] & y[6]);
        const uint32_t t1 = y[7] + S1 + ch + k + wy;
        const uint32_t S0 = xor3(rotr(y[0], 2), rotr(y[0], 13), rotr(y[0], 22));
        const uint32_t mj = maj3(y[0], y[1], y[2]);
        y[7] = y[6]; y[6] = y[5]; y[5] = y[4]; y[4] = y[3] + t1; y[3] = y[2]; y[2] = y[1]; y[1] = y[0]; y[0] = t1 + S0 + mj;
    }
}

__device__ __forceinline__ void sha_sched16(uint32_t (&w)[16]) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
    }
}

// One 64-byte block of one chunk as 16 big-endian words: data block, tail block(s), or zeros.
__device__ __forceinline__ void pair_block_words(uint32_t (&w)[16], const uint4 (&v)[4], uint32_t blk, uint32_t nfull,
                                                 uint32_t nblocks, const uint8_t* p, uint32_t len) {
    if (blk < nfull) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            w[4 * q] = __builtin_bswap32(v[q].x);
            w[4 * q + 1] = __builtin_bswap32(v[q].y);
            w[4 * q + 2] = __builtin_bswap32(v[q].z);
            w[4 * q + 3] = __builtin_bswap32(v[q].w);
        }
    } else {
        if (blk == nfull) {
            tail_words<true>(w, p + 64 * nfull, len & 63);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = 0;
        }
        if (blk == nblocks - 1) {
            const uint64_t bits = (uint64_t)len * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    }
}

template <bool PRIO, int WPE = 3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void chunk_hash_pair_kernel(HashArgs a) {
    const uint32_t total = *a.total;
    const uint32_t i0 = 2 * (blockIdx.x * 256 + threadIdx.x);
    if (i0 >= total) return;
    const bool has1 = i0 + 1 < total;
    uint32_t slot[2], b[2], k[2], cs[2], len[2], nfull[2], nblocks[2];
    const uint8_t* p[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const uint32_t i = c == 0 || has1 ? i0 + c : i0;  // a missing second task repeats the first
        slot[c] = a.tasks[i];
        b[c] = slot[c] / a.cap;
        k[c] = slot[c] - b[c] * a.cap;
        const uint64_t boff = a.uniform_len ? (uint64_t)b[c] * a.uniform_len : a.offs[b[c]];
        cs[c] = a.starts[slot[c]];
        len[c] = a.clens[slot[c]];
        p[c] = a.data + boff + cs[c];
        nfull[c] = len[c] >> 6;
        nblocks[c] = (len[c] + 8) / 64 + 1;
    }
    if constexpr (PRIO) {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(nblocks[0]);
        if (nb > 1024) __builtin_amdgcn_s_setprio(3);
        else if (nb > 512) __builtin_amdgcn_s_setprio(2);
        else if (nb > 256) __builtin_amdgcn_s_setprio(1);
    }
    uint32_t x[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t y[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const uint32_t nbmax = nblocks[0] > nblocks[1] ? nblocks[0] : nblocks[1];
    for (uint32_t blk = 0; blk < nbmax; blk++) {
        uint4 v0[4], v1[4];
        load_block64(v0, blk < nfull[0] ? p[0] + 64 * blk : a.zero_page);
        load_block64(v1, blk < nfull[1] ? p[1] + 64 * blk : a.zero_page);
        uint32_t w0[16], w1[16];
        pair_block_words(w0, v0, blk, nfull[0], nblocks[0], p[0], len[0]);
        pair_block_words(w1, v1, blk, nfull[1], nblocks[1], p[1], len[1]);
        uint32_t u[8], z[8];
#pragma unroll
        for (int j = 0; j < 8; j++) { u[j] = x[j]; z[j] = y[j]; }
#pragma clang loop unroll(full)
        for (int r = 0; r < 64; r++) {
            if (r >= 16 && (r & 15) == 0) {
                asm("" : "+v"(w0[0]), "+v"(w0[1]), "+v"(w0[2]), "+v"(w0[3]), "+v"(w0[4]), "+v"(w0[5]), "+v"(w0[6]),
                    "+v"(w0[7]), "+v"(w0[8]), "+v"(w0[9]), "+v"(w0[10]), "+v"(w0[11]), "+v"(w0[12]), "+v"(w0[13]),
                    "+v"(w0[14]), "+v"(w0[15]) : "v"(u[0]));
                sha_sched16(w0);
                asm("" : "+v"(w1[0]), "+v"(w1[1]), "+v"(w1[2]), "+v"(w1[3]), "+v"(w1[4]), "+v"(w1[5]), "+v"(w1[6]),
                    "+v"(w1[7]), "+v"(w1[8]), "+v"(w1[9]), "+v"(w1[10]), "+v"(w1[11]), "+v"(w1[12]), "+v"(w1[13]),
                    "+v"(w1[14]), "+v"(w1[15]) : "v"(z[0]));
                sha_sched16(w1);
            }
            sha_round_pair(u, z, kSha256K[r], w0[r & 15], w1[r & 15]);
        }
        const bool live0 = blk < nblocks[0], live1 = blk < nblocks[1];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            x[j] = live0 ? x[j] + u[j] : x[j];
            y[j] = live1 ? y[j] + z[j] : y[j];
        }
    }
    store_digest<0>(a, slot[0], b[0], k[0], cs[0], len[0], x);
    if (has1) store_digest<0>(a, slot[1], b[1], k[1], cs[1], len[1], y);
}

// fingerprint-kernel variants (SHA-256 only)
hipError_t launch_hash_sweep(const HashArgs& a, uint64_t max_tasks, int variant, hipStream_t s) {
    const uint32_t blocks = (uint32_t)((max_tasks + 255) / 256);
    if (blocks == 0) return hipSuccess;
    if (a.algo != 0) return hipErrorInvalidValue;
    const uint32_t b64 = (uint32_t)((max_tasks + 63) / 64);
    switch (variant) {
    case 1: hipLaunchKernelGGL((chunk_hash_kernel<0, 1>), dim3(blocks), dim3(256), 0, s, a); break;    // no loads
    case 2: hipLaunchKernelGGL((chunk_hash_kernel<0, 2>), dim3(blocks), dim3(256), 0, s, a); break;    // no compression
    case 3: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 64, false>), dim3(b64), dim3(64), 0, s, a); break;
    case 4: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, false>), dim3(blocks), dim3(256), 0, s, a); break;
    case 5: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 64, true>), dim3(b64), dim3(64), 0, s, a); break;
    case 6:
        if (!a.wave_ctr || !a.persist_grid) return hipErrorInvalidValue;
        hipLaunchKernelGGL((chunk_hash_persistent_kernel<0, true>), dim3(a.persist_grid), dim3(256), 0, s, a);
        break;
    case 7:
        if (!a.wave_ctr || !a.persist_grid) return hipErrorInvalidValue;
        hipLaunchKernelGGL((chunk_hash_persistent_kernel<0, false>), dim3(a.persist_grid), dim3(256), 0, s, a);
        break;
    case 8: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 9: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, true, false>), dim3(blocks), dim3(256), 0, s, a); break;
    case 11: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, false, true, 5>), dim3(blocks), dim3(256), 0, s, a); break;
    case 12: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, false, true, 6>), dim3(blocks), dim3(256), 0, s, a); break;
    case 13: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, true, true, 5>), dim3(blocks), dim3(256), 0, s, a); break;
    case 14: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, false, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 15: hipLaunchKernelGGL((chunk_hash_kernel<0, 8, 256, true, true, 5>), dim3(blocks), dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL((chunk_hash_kernel<0, 8, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 10: hipLaunchKernelGGL((chunk_hash_kernel<0, 4, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 45:  // production kernel without its data loads (ABL bit 1: message words from the state;
              // wrong digests): the clock of the same VALU work without the HBM traffic
        hipLaunchKernelGGL((chunk_hash_kernel<0, 16 | 1, 256, true, true>), dim3(blocks), dim3(256), 0, s, a);
        break;
    case 50:  // production kernel + per-wave clock stamps (HashArgs::stamps; scripts/hash_stamps.py)
        hipLaunchKernelGGL((chunk_hash_kernel<0, 16 | 128, 256, true, true>), dim3(blocks), dim3(256), 0, s, a);
        break;
    case 31:  // production kernel without the issue priority for waves of long chunks
        hipLaunchKernelGGL((chunk_hash_kernel<0, 16, 256, true, false>), dim3(blocks), dim3(256), 0, s, a);
        break;
    case 30:  // production kernel + 15 KiB of LDS per workgroup: co-resides 2 waves/SIMD with a 512-thread scan
        hipLaunchKernelGGL((chunk_hash_kernel<0, 16 | 64, 256, true, true>), dim3(blocks), dim3(256), 0, s, a);
        break;
    case 21:  // persistent grid with the production task body (true next-block prefetch)
        if (!a.wave_ctr || !a.persist_grid) return hipErrorInvalidValue;
        hipLaunchKernelGGL((chunk_hash_persistent_kernel<0, true, 16>), dim3(a.persist_grid), dim3(256), 0, s, a);
        break;
    // LDS-DMA prefetch (ABL bit 32): no VGPRs for the next block, five waves per SIMD
    case 22: hipLaunchKernelGGL((chunk_hash_kernel<0, 48, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 23: hipLaunchKernelGGL((chunk_hash_kernel<0, 48, 256, true, true, 5>), dim3(blocks), dim3(256), 0, s, a); break;
    case 24: hipLaunchKernelGGL((chunk_hash_kernel<0, 48, 256, true, true, 6>), dim3(blocks), dim3(256), 0, s, a); break;
    // two chunks per lane (twice the ILP per wave), without / with the long-chunk issue priority
    case 40: hipLaunchKernelGGL((chunk_hash_pair_kernel<false>), dim3((blocks + 1) / 2), dim3(256), 0, s, a); break;
    case 41: hipLaunchKernelGGL((chunk_hash_pair_kernel<true>), dim3((blocks + 1) / 2), dim3(256), 0, s, a); break;
    case 42: hipLaunchKernelGGL((chunk_hash_pair_kernel<true, 2>), dim3((blocks + 1) / 2), dim3(256), 0, s, a); break;
    // the prefetch before ABL bit 16 (its copy at the data/tail merge waited for the load)
    case 20: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sdfs
