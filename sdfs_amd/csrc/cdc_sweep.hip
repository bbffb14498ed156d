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
    default: return {0, 0, 0, 0, 0, 0, 0};
    }
}

template <class T>
static hipError_t sweep_launch(const ScanArgs& a, int pk, int grid, int block, hipStream_t s) {
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
    SWEEP_CASE(31, ScanV31) SWEEP_CASE(32, ScanV32)
#undef SWEEP_CASE
    default: return hipErrorInvalidValue;
    }
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
    // the prefetch before ABL bit 16 (its copy at the data/tail merge waited for the load)
    case 20: hipLaunchKernelGGL((chunk_hash_kernel<0, 0, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sdfs
