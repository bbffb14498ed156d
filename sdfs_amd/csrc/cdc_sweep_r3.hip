// cdc_sweep_r3.hip — round-3 measurement-only scan variants (tuning library only, -DSDFS_TUNING;
// see cdc_sweep.hip).  Kept in a translation unit of their own so that a new variant builds in
// about a minute.  Only the one-compare predicate (PK 2: the reference's low-k-bit zero test) is
// instantiated; any other predicate is refused (hipErrorInvalidValue) so a sweep cannot silently
// measure something else.
#include <algorithm>

#include "cdc_device.h"

namespace sdfs {

// 43: the push address as one SDWA shift into byte 1 of a base register (kAblSdwa); 44: plus
// the pop address as one SDWA byte move (kAblSdwaPop); 45: 43 on whole-block batches.
using ScanV43 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | kAblSdwa, 256, 2, kScanThreads, true>;
using ScanV44 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | kAblSdwa | kAblSdwaPop, 256, 2, kScanThreads, true>;
using ScanV45 = ScanCfg<32, 1, false, 4, 16 | kAblSgprPred | kAblSdwa | kAblFullBlocks, 256, 2, kScanThreads, true>;
// 46 / 47: 16 table copies (2-way bank conflicts, 64 KiB) so that two workgroups share a CU —
// six (46: 768-thread workgroups, <= 80 VGPRs) or five (47: 640 threads, <= 96 VGPRs) waves per
// SIMD instead of four — with 128-byte blocks to fit the register budget; SDWA push address.
using ScanV46 = ScanCfg<16, 1, false, 6, 16 | kAblSgprPred | kAblSdwa, 128, 2, 768, true>;
using ScanV47 = ScanCfg<16, 1, false, 5, 16 | kAblSgprPred | kAblSdwa, 128, 2, 640, true>;
// 48 / 49: production (SDWA push + pop addresses) with the candidate bits from each group's
// minimum predicate word, groups of 4 (48) or 8 (49) positions, instead of per-position SGPR masks
constexpr int kProdR3 = 16 | kAblSdwa | kAblSdwaPop;
using ScanV48 = ScanCfg<32, 1, false, 4, kProdR3 | kAblMinGroup, 256, 2, kScanThreads, true>;
using ScanV49 = ScanCfg<32, 1, false, 4, kProdR3 | kAblMinGroup | kAblMinGroup8, 256, 2, kScanThreads, true>;
// 50: production with the pop entries stored high word first (kAblPopSwap: no three-way register
// bank conflict in the low-word xor3); 51: 50 with the groups-of-8 minimum candidate bits (49)
using ScanV50 = ScanCfg<32, 1, false, 4, kProdR3 | kAblSgprPred | kAblPopSwap, 256, 2, kScanThreads, true>;
using ScanV51 = ScanCfg<32, 1, false, 4, kProdR3 | kAblMinGroup | kAblMinGroup8 | kAblPopSwap, 256, 2, kScanThreads, true>;
// 52: 51 with the bit-select pop address for the byte already in place (kAblPopMux); 53: 50 + mux
using ScanV52 = ScanCfg<32, 1, false, 4, kProdR3 | kAblMinGroup | kAblMinGroup8 | kAblPopSwap | kAblPopMux, 256, 2,
                        kScanThreads, true>;
using ScanV53 = ScanCfg<32, 1, false, 4, kProdR3 | kAblSgprPred | kAblPopSwap | kAblPopMux, 256, 2, kScanThreads, true>;

template <class CFG>
constexpr ScanVariantInfo info_r3() {
    return {CFG::kCopies, CFG::kChains, CFG::kLds, std::max(1, CFG::kWavesPerSimd * 256 / CFG::kThreads), CFG::kBlk,
            CFG::kFuse, CFG::kThreads, CFG::kMirror, CFG::kPopSwap};
}

ScanVariantInfo scan_variant_info_sweep_r3(int v) {
    switch (v) {
    case 43: return info_r3<ScanV43>();
    case 44: return info_r3<ScanV44>();
    case 45: return info_r3<ScanV45>();
    case 46: return info_r3<ScanV46>();
    case 47: return info_r3<ScanV47>();
    case 48: return info_r3<ScanV48>();
    case 49: return info_r3<ScanV49>();
    case 50: return info_r3<ScanV50>();
    case 51: return info_r3<ScanV51>();
    case 52: return info_r3<ScanV52>();
    case 53: return info_r3<ScanV53>();
    default: return {0, 0, 0, 0, 0, 0, 0, 0};
    }
}

template <class T>
static hipError_t launch_r3(const ScanArgs& a, int pk, int grid, int block, hipStream_t s) {
    static_assert(T::kMirror, "round-3 variants are mirrored-state forms");
    if ((T::kAbl & kAblFullBlocks) != 0 && !scan_full_blocks(a, T::kBlk)) return hipErrorInvalidValue;
    if (pk != 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL((cdc_scan_kernel<48, 2, T>), dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_scan_sweep_r3(const ScanArgs& a, int window, int pk, int variant, int grid, int block,
                                hipStream_t s) {
    if (window != 48) return hipErrorInvalidValue;
    switch (variant) {
    case 43: return launch_r3<ScanV43>(a, pk, grid, block, s);
    case 44: return launch_r3<ScanV44>(a, pk, grid, block, s);
    case 45: return launch_r3<ScanV45>(a, pk, grid, block, s);
    case 46: return launch_r3<ScanV46>(a, pk, grid, block, s);
    case 47: return launch_r3<ScanV47>(a, pk, grid, block, s);
    case 48: return launch_r3<ScanV48>(a, pk, grid, block, s);
    case 49: return launch_r3<ScanV49>(a, pk, grid, block, s);
    case 50: return launch_r3<ScanV50>(a, pk, grid, block, s);
    case 51: return launch_r3<ScanV51>(a, pk, grid, block, s);
    case 52: return launch_r3<ScanV52>(a, pk, grid, block, s);
    case 53: return launch_r3<ScanV53>(a, pk, grid, block, s);
    default: return hipErrorInvalidValue;
    }
}

template <int NS, int SP = 0>
static void fused_launch(const ScanArgs& a, const HashArgs& ha, uint32_t* ctr, int grid, hipStream_t s) {
    using Prod = ScanV51;  // the production scan form
    if (ha.algo == 2)
        hipLaunchKernelGGL((cdc_fused_kernel<48, 2, Prod, 2, NS, SP>), dim3(grid), dim3(1024), 0, s, a, ha, ctr);
    else
        hipLaunchKernelGGL((cdc_fused_kernel<48, 2, Prod, 0, NS, SP>), dim3(grid), dim3(1024), 0, s, a, ha, ctr);
}

// form 1: two scan-first waves per SIMD (interleaved); 2 / 3 / 4: one / two / three scan-first
// waves per SIMD (the first k waves of each SIMD)
hipError_t launch_fused_probe(const ScanArgs& a, const HashArgs& ha, uint32_t* ctr, int window, int pk, int grid,
                              int form, hipStream_t s) {
    if (window != 48 || pk != 2 || !a.uniform_len || !a.fuse_resolve) return hipErrorInvalidValue;
    switch (form) {
    case 1: fused_launch<0>(a, ha, ctr, grid, s); break;
    case 2: fused_launch<1>(a, ha, ctr, grid, s); break;
    case 3: fused_launch<2>(a, ha, ctr, grid, s); break;
    case 4: fused_launch<3>(a, ha, ctr, grid, s); break;
    case 5: fused_launch<1, 2>(a, ha, ctr, grid, s); break;  // 5-7: scan items at issue priority 2
    case 6: fused_launch<0, 2>(a, ha, ctr, grid, s); break;
    case 7: fused_launch<3, 2>(a, ha, ctr, grid, s); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sdfs
