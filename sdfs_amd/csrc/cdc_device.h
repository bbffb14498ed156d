// cdc_device.h — device-side building blocks shared by the production kernels (cdc_kernels.hip)
// and the measurement-only variant build (cdc_sweep.hip): the rolling-hash scan kernel template,
// the greedy cut walk, and the per-chunk SHA-256 / MD5 fingerprint task.
//
// Reference semantics: VariableSha256HashEngine.getChunks (VariableSha256HashEngine.java:71-86)
// driving the rabinwindow EnhancedFingerFactory loop; getHash (:58-67).
#pragma once

#include "cdc_internal.h"

namespace sdfs {

// gfx950 has no v_xor3_b32, but it has v_bitop3_b32 (any 3-input boolean function, truth table
// 0x96 = a^b^c, 0xE8 = majority); hipcc does not form it for xor chains on its own.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
// (a & b) | c.  v_bitop3 truth-table bit index is (A << 2) | (B << 1) | C (the encoding hipcc
// itself emits for Ch, bitop3:0xE4 = C ? A : B).
__device__ __forceinline__ uint32_t bitop3_and_or(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xEA);
}

// ------------------------------------------------------------------------------------------
// 1. candidate scan
// ------------------------------------------------------------------------------------------
// One rolling step for byte `inb` (taken from byte p of dword `dw`), popping the byte that left
// the window (byte q of dword `odw`).  fp = hi:lo (deg < 56).  Equivalent to the jar's
// pushByte/popByte pair:
//   j = (fp >> (d-8)) & 0xFF;  fp = ((fp << 8) | b) ^ push[j];  fp ^= pop[o]
// push[j] carries j*x^d, which cancels the 8 bits shifted above deg-1.
// Ablation bits (scan sweeps only): 1 = no pop LDS read, 2 = no push LDS read, 4 = no candidate
// test, 8 = no global loads.  The skipped values are replaced by register values that keep every
// remaining instruction live.  Bit 16 is not an ablation but a code layout (production): whole
// blocks are loaded and scanned in a branch of their own (see the scan kernel's block loop).
//
// Mirrored state (ABL bit kAblMirror, ScanCfg MIRROR): the same recurrence on R = bitrev64(fp),
// held as hi:lo = R >> 32 : R.  fp << 8 becomes R >> 8, the incoming byte lands bit-reversed in
// R's top byte, and fp bits 0..31 (the predicate's field) are hi bits 31..0 — so a low-k-bit
// zero predicate is ONE compare (hi < 2^(32-k)) instead of v_and + v_cmp.  The data dwords are
// bit-reversed in registers once, before their first position (block_words; byte p of a dword
// becomes byte 3-p, bits reversed), the
// push index rev8(j) sits at lo bits [64-d, 72-d) (jshift = 64 - d), and the LDS tables hold
// bitrev64(push[rev8(x)]) / bitrev64(pop[rev8(x)]) at entry x (build_table_image, mirror).
constexpr int kAblMirror = 64;
// ABL bit kAblSgprPred (mirrored state, low-k zero predicate only): each position's compare goes
// to an SGPR pair of its own (v_cmp_*_e64), eight positions are OR-ed on the scalar unit, and
// only a group with a candidate in some lane shifts its eight bits in with v_addc (carry-in from
// the SGPR pair); a group without one is a single v_lshlrev.  1 -> ~0.25 VALU per byte for the
// candidate bits at a 12-bit predicate.
constexpr int kAblSgprPred = 256;
// ABL bit kAblFullBlocks (scan kernel only): the batch is uniform and every segment is a whole
// number of blocks (uniform_len % seg_len == 0, seg_len % BLK == 0), so the block loop has no
// guarded path: its loads are unconditional and hipcc waits for them per 64 bytes scanned
// instead of for the whole block at a control-flow merge.  Lanes past the batch's last segment
// (nblk == 0) read the batch's first block and discard what they compute.
constexpr int kAblFullBlocks = 512;

// ABL bit kAblSdwa (mirrored state): the push address is ONE v_lshrrev_b32_sdwa writing
// (lo >> jshift) & 0xFF into byte 1 of a register that keeps push_base in its other bytes
// (dst_unused:UNUSED_PRESERVE), instead of v_lshrrev + v_bitop3: one VALU less per byte, and one
// dependent instruction less in the per-byte chain (index -> LDS read -> xor3 -> index).
// kAblSdwaPop: the pop address the same way (v_mov_b32_sdwa of the outgoing byte into byte 1 of a
// register holding c8) instead of v_perm / v_bitop3.
constexpr int kAblSdwa = 1024;
constexpr int kAblSdwaPop = 2048;
// kAblMinGroup (mirrored state, low-k zero predicate; sweep only): candidate bits per group of 4
// positions (kAblMinGroup8: 8) from the group's minimum predicate word, VALU only — no per-position
// SGPR mask and no scalar OR chain (see byte_step).
constexpr int kAblMinGroup = 4096;
constexpr int kAblMinGroup8 = 8192;
// kAblPopSwap (mirrored state): the pop-table entries are stored high word first, so the low-word
// xor3 takes its pop operand from the ODD register of the ds_read_b64 destination pair.  VGPR
// tuples are even-aligned on gfx950 and hipcc keeps handing both lookups' pairs and the shifted
// low word registers of one bank (v54, v58, v62): a v_bitop3 whose three sources share a bank
// issues in ~3.5 instead of ~2.2 cycles (scripts/vgpr_bank_microbench.hip).
constexpr int kAblPopSwap = 16384;
// kAblPopMux (with kAblSdwaPop): for the one byte in four whose bit-reversed copy already sits in
// byte 1 of its dword, the pop address is a full-rate v_bitop3 bit-select instead of the SDWA move.
constexpr int kAblPopMux = 32768;

template <int B>
__device__ __forceinline__ void sdwa_byte_to_b1(uint32_t& d, uint32_t src) {
    static_assert(B >= 0 && B < 4, "byte select");
    if constexpr (B == 0)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(d) : "v"(src));
    else if constexpr (B == 1)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(d) : "v"(src));
    else if constexpr (B == 2)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(d) : "v"(src));
    else
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(d) : "v"(src));
}

template <int P, int Q, int ABL = 0>
__device__ __forceinline__ void roll_step(uint32_t& lo, uint32_t& hi, uint32_t dw, uint32_t odw, uint32_t& c8,
                                          uint32_t& push_base, uint32_t jshift, const uint8_t* tab) {
    if constexpr ((ABL & kAblMirror) != 0) {
        uint32_t pa, qa;
        if constexpr ((ABL & kAblSdwa) != 0) {
            asm("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                : "+v"(push_base)
                : "v"(lo), "s"(jshift));
            pa = push_base;
        } else {
            pa = bitop3_and_or(lo >> (jshift - 8), 0xFF00u, push_base);
        }
        if constexpr ((ABL & kAblSdwaPop) != 0 && (ABL & kAblPopMux) != 0 && Q == 2) {
            // the outgoing byte already sits in byte 1: one full-rate bit-select (B ? A : C)
            // takes byte 1 from it and the rest (base, lane offset) from the address register
            qa = __builtin_amdgcn_bitop3_b32(odw, 0xFF00u, c8, 0xE2);
        } else if constexpr ((ABL & kAblSdwaPop) != 0) {
            sdwa_byte_to_b1<3 - Q>(c8, odw);
            qa = c8;
        } else {
            // (rev8(o) << 8) | c8; a byte already at bits 8..15 needs only the full-rate v_bitop3
            qa = Q == 2 ? bitop3_and_or(odw, 0xFF00u, c8)
                        : __builtin_amdgcn_perm(odw, c8, 0x0C0C0000u | ((4u + 3 - Q) << 8));
        }
        const uint2 pv = (ABL & 2) ? make_uint2(pa, pa >> 3) : *reinterpret_cast<const uint2*>(tab + pa);
        const uint2 qv = (ABL & 1) ? make_uint2(qa, qa >> 3) : *reinterpret_cast<const uint2*>(tab + qa);
        const uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, 8);                      // R >> 8, low word
        const uint32_t nhi = __builtin_amdgcn_perm(hi, dw, 0x00070605u | ((3u - P) << 24));  // (hi >> 8) | rev8(b) << 24
        if constexpr ((ABL & kAblPopSwap) != 0) {
            lo = xor3(nlo, pv.x, qv.y);
            hi = xor3(nhi, pv.y, qv.x);
        } else {
            lo = xor3(nlo, pv.x, qv.x);
            hi = xor3(nhi, pv.y, qv.y);
        }
        return;
    }
    // push[j] address (j << 8) | push_base with j = (fp >> (d-8)) & 0xFF = hi bits [jshift, jshift+8):
    // one full-rate shift + one v_bitop3 ((A & B) | C, table 0xEA) instead of v_bfe + v_lshl_or
    // (both half-rate on gfx950, scripts/isa_microbench.hip).
    const uint32_t pa = bitop3_and_or(hi >> (jshift - 8), 0xFF00u, push_base);
    const uint32_t qa = __builtin_amdgcn_perm(odw, c8, 0x0C0C0000u | ((4u + Q) << 8));  // (o << 8) | c8
    const uint2 pv = (ABL & 2) ? make_uint2(pa, pa >> 3) : *reinterpret_cast<const uint2*>(tab + pa);
    const uint2 qv = (ABL & 1) ? make_uint2(qa, qa >> 3) : *reinterpret_cast<const uint2*>(tab + qa);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);             // (fp << 8) >> 32
    const uint32_t nlo = __builtin_amdgcn_perm(lo, dw, 0x06050400u | P);     // (lo << 8) | b
    lo = xor3(nlo, pv.x, qv.x);
    hi = xor3(nhi, pv.y, qv.y);
}

// push-only step (window warm-up from the zero state; no byte leaves the window yet)
template <int P, bool M = false>
__device__ __forceinline__ void push_step(uint32_t& lo, uint32_t& hi, uint32_t dw, uint32_t push_base,
                                          uint32_t jshift, const uint8_t* tab) {
    if constexpr (M) {
        const uint2 pv = *reinterpret_cast<const uint2*>(tab + bitop3_and_or(lo >> (jshift - 8), 0xFF00u, push_base));
        const uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, 8);
        const uint32_t nhi = __builtin_amdgcn_perm(hi, dw, 0x00070605u | ((3u - P) << 24));
        lo = nlo ^ pv.x;
        hi = nhi ^ pv.y;
        return;
    }
    const uint2 pv = *reinterpret_cast<const uint2*>(tab + bitop3_and_or(hi >> (jshift - 8), 0xFF00u, push_base));
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 24);
    const uint32_t nlo = __builtin_amdgcn_perm(lo, dw, 0x06050400u | P);
    lo = nlo ^ pv.x;
    hi = nhi ^ pv.y;
}

// Shift the candidate flag of the current position into `bits` (first position ends in the MSB,
// bit-reversed once per 32 positions).  Written as one v_and/v_cmp/v_addc sequence: in plain C
// hipcc reassociates the 32 per-byte tests of a word into an OR tree at the end of the word,
// keeping all 32 fingerprints live (scratch spills on every byte).
// Predicate kinds PK: 0 = (lo & mask) == val on one word, 1 = both words, 2 (mirrored state
// only) = the low k fp bits all zero, i.e. `lo` (here the mirrored hi word) < a.thr = 2^(32-k).
// `lo` is the word holding fp bits 0..31 (mirrored: R's hi word, masks bit-reversed by the host).
// PK 3 (mirrored state only) is the divisor detector fp % D == R: fp = bitrev64(R) < 2^53 is exact
// in f64, q = floor(fp * (1/D)) is within one of floor(fp / D) (for D >= 3 — the host runs powers
// of two as masks — the two roundings leave an absolute error <= fp/D * 2^-52 < 2^53/3 * 2^-52 < 1),
// so r = fp - q*D (one exact fma) is the remainder t or t -/+ D, and exactly one of r, r + D, r - D
// lies in [0, D): the test is true iff t == R (the host passes R >= D as NaN: never true).
template <int PK>
__device__ __forceinline__ void cand_shift(uint32_t& bits, uint32_t lo, uint32_t hi, const ScanArgs& a) {
    if constexpr (PK == 3) {
        const uint32_t flo = __builtin_bitreverse32(lo), fhi = __builtin_bitreverse32(hi);
        const double f = __builtin_fma((double)fhi, 4294967296.0, (double)flo);
        const double q = __builtin_floor(f * a.div_inv);
        const double r = __builtin_fma(-q, a.div_d, f);
        const uint32_t h = (r == a.rem_d) | (r + a.div_d == a.rem_d) | (r - a.div_d == a.rem_d);
        asm("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(bits) : "v"(h));
    } else if constexpr (PK == 2) {
        asm("v_cmp_gt_u32 vcc, %2, %1\n\t"
            "v_addc_co_u32 %0, vcc, %0, %0, vcc"
            : "+v"(bits)
            : "v"(lo), "s"(a.thr)
            : "vcc");
    } else if constexpr (PK == 1) {
        uint32_t t, t2;
        asm("v_and_b32 %1, %4, %3\n\t"
            "v_xor_b32 %1, %5, %1\n\t"
            "v_and_b32 %2, %7, %6\n\t"
            "v_xor_b32 %2, %8, %2\n\t"
            "v_or_b32 %1, %1, %2\n\t"
            "v_cmp_eq_u32 vcc, 0, %1\n\t"
            "v_addc_co_u32 %0, vcc, %0, %0, vcc"
            : "+v"(bits), "=&v"(t), "=&v"(t2)
            : "v"(lo), "s"(a.mask_lo), "s"(a.val_lo), "v"(hi), "s"(a.mask_hi), "s"(a.val_hi)
            : "vcc");
    } else {
        uint32_t t;
        asm("v_and_b32 %1, %3, %2\n\t"
            "v_cmp_eq_u32 vcc, %4, %1\n\t"
            "v_addc_co_u32 %0, vcc, %0, %0, vcc"
            : "+v"(bits), "=&v"(t)
            : "v"(lo), "s"(a.mask_lo), "s"(a.val_lo)
            : "vcc");
    }
}

// Byte O of the current block (BLKW dwords), with the byte that leaves the window at O - W: in
// this block when O >= W, otherwise in `prev` (the previous block's last 64 bytes).
template <int W, int PK, int O, int ABL, int BLKW>
__device__ __forceinline__ void byte_step(uint32_t& lo, uint32_t& hi, uint32_t& bits, const uint32_t (&cur)[BLKW],
                                          const uint32_t (&prev)[16], uint32_t& c8, uint32_t& push_base,
                                          const uint8_t* tab, const ScanArgs& a, uint64_t (&gm)[8], uint32_t (&hv)[8]) {
    constexpr int OLD = O - W;  // may be negative -> previous block
    constexpr int OI = OLD >= 0 ? OLD : OLD + 64;
    const uint32_t odw = OLD >= 0 ? cur[OI >> 2] : prev[OI >> 2];
    roll_step<(O & 3), (OI & 3), ABL>(lo, hi, cur[O >> 2], odw, c8, push_base, a.jshift, tab);
    if constexpr ((ABL & 4) != 0 && (ABL & kAblSgprPred) != 0) {
        asm volatile("" ::"v"(hi));  // round-3 form: the state stays live, no candidates at all
    } else if constexpr (ABL & 4) {
        bits ^= lo;
    } else if constexpr ((ABL & kAblMinGroup) != 0 && (ABL & kAblMirror) != 0 && PK == 2) {
        // groups of G positions: the group's minimum predicate word decides (one v_min3 per two
        // positions, one compare per group); only a group in which some lane has a candidate
        // shifts its G exact bits in (v_cmp/v_addc), every other group is one shift by G
        constexpr int G = (ABL & kAblMinGroup8) != 0 ? 8 : 4;
        hv[O & (G - 1)] = hi;
        if constexpr ((O & (G - 1)) == G - 1) {
            uint32_t m = min(min(hv[0], hv[1]), hv[2]);
            m = min(m, hv[3]);
            if constexpr (G == 8) {
                m = min(min(m, hv[4]), hv[5]);
                m = min(min(m, hv[6]), hv[7]);
            }
            if (__builtin_expect(__any(m < a.thr), 0)) {
#pragma unroll
                for (int p = 0; p < G; p++) cand_shift<2>(bits, hv[p], 0u, a);
            } else {
                bits <<= G;
            }
        }
    } else if constexpr ((ABL & kAblSgprPred) != 0 && (ABL & kAblMirror) != 0 && PK == 2) {
        asm("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(gm[O & 7]) : "s"(a.thr), "v"(hi));
        if constexpr ((O & 7) == 7) {
            const uint64_t any = (gm[0] | gm[1]) | (gm[2] | gm[3]) | (gm[4] | gm[5]) | (gm[6] | gm[7]);
            if (__builtin_expect(any != 0, 0)) {
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    uint64_t co;
                    asm volatile("v_addc_co_u32_e64 %0, %1, %0, %0, %2" : "+v"(bits), "=s"(co) : "s"(gm[p]));
                }
            } else {
                bits <<= 8;
            }
        }
    } else if constexpr ((ABL & kAblMirror) != 0)
        cand_shift<PK>(bits, hi, lo, a);
    else
        cand_shift<PK>(bits, lo, hi, a);
}

// Byte O of every chain at once (NCH > 1): all chains' lookup addresses and their 2 x NCH LDS
// reads first, then each chain's update, so the chains' lookup latencies overlap (hipcc's
// waitcnt pass then waits lgkmcnt(2 x later chains) before each chain's update).  The reads are
// volatile so that they stay in issue order ahead of the updates: left alone, hipcc reuses one
// destination pair for every chain and waits lgkmcnt(0) per chain.
template <int W, int PK, int O, int NCH, int BLKW>
__device__ __forceinline__ void bytes_multi(uint32_t (&lo)[NCH], uint32_t (&hi)[NCH], uint32_t (&bits)[NCH],
                                            const uint32_t (&cur)[NCH][BLKW], const uint32_t (&prev)[NCH][16],
                                            uint32_t c8, uint32_t push_base, const uint8_t* tab, const ScanArgs& a) {
    constexpr int OLD = O - W;
    constexpr int OI = OLD >= 0 ? OLD : OLD + 64;
    constexpr int Q = OI & 3;
    uint2 pv[NCH], qv[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const uint32_t odw = OLD >= 0 ? cur[c][OI >> 2] : prev[c][OI >> 2];
        const uint32_t pa = bitop3_and_or(hi[c] >> (a.jshift - 8), 0xFF00u, push_base);
        const uint32_t qa = __builtin_amdgcn_perm(odw, c8, 0x0C0C0000u | ((4u + Q) << 8));
        typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
        const __attribute__((address_space(3))) uint8_t* lt = (const __attribute__((address_space(3))) uint8_t*)tab;
        const uint64_t pw = *(lds_u64*)(lt + pa);
        const uint64_t qw = *(lds_u64*)(lt + qa);
        pv[c] = make_uint2((uint32_t)pw, (uint32_t)(pw >> 32));
        qv[c] = make_uint2((uint32_t)qw, (uint32_t)(qw >> 32));
    }
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const uint32_t nhi = __builtin_amdgcn_alignbit(hi[c], lo[c], 24);
        const uint32_t nlo = __builtin_amdgcn_perm(lo[c], cur[c][O >> 2], 0x06050400u | (O & 3));
        lo[c] = xor3(nlo, pv[c].x, qv[c].x);
        hi[c] = xor3(nhi, pv[c].y, qv[c].y);
        cand_shift<PK>(bits[c], lo[c], hi[c], a);
    }
}

#ifndef SDFS_SCAN_SCHED_GROUP
#define SDFS_SCAN_SCHED_GROUP 4
#endif
constexpr int kSchedGroup = SDFS_SCAN_SCHED_GROUP;  // bytes per scheduling region

// Positions O .. O0+31 of one candidate word, all chains interleaved (independent rolling chains
// give the ILP that hides the LDS latency of the push lookups).
template <int W, int PK, int O0, int O, int NCH, int ABL, int BLKW>
__device__ __forceinline__ void word_steps(uint32_t (&lo)[NCH], uint32_t (&hi)[NCH], uint32_t (&bits)[NCH],
                                           const uint32_t (&cur)[NCH][BLKW], const uint32_t (&prev)[NCH][16],
                                           uint32_t& c8, uint32_t& push_base, const uint8_t* tab, const ScanArgs& a,
                                           uint64_t (&gm)[NCH][8], uint32_t (&hv)[NCH][8]) {
    if constexpr (O < O0 + 32) {
        if constexpr (NCH > 1 && ABL == 0) {
            bytes_multi<W, PK, O, NCH, BLKW>(lo, hi, bits, cur, prev, c8, push_base, tab, a);
        } else {
#pragma unroll
            for (int c = 0; c < NCH; c++)
                byte_step<W, PK, O, ABL, BLKW>(lo[c], hi[c], bits[c], cur[c], prev[c], c8, push_base, tab, a, gm[c], hv[c]);
        }
        if constexpr ((O & (kSchedGroup - 1)) == kSchedGroup - 1) {
            // keep the scheduler from hoisting every (chain-independent) pop read of the block
            // ahead of the rolling chain: that costs ~2 VGPRs per byte and spills.
            __builtin_amdgcn_sched_barrier(0);
        }
        word_steps<W, PK, O0, O + 1, NCH, ABL, BLKW>(lo, hi, bits, cur, prev, c8, push_base, tab, a, gm, hv);
    }
}

template <int W, int O, bool M = false>
__device__ __forceinline__ void warm_from(uint32_t& lo, uint32_t& hi, const uint32_t (&prev)[16], uint32_t push_base,
                                          uint32_t jshift, const uint8_t* tab) {
    if constexpr (O < 64) {
        push_step<(O & 3), M>(lo, hi, prev[O >> 2], push_base, jshift, tab);
        warm_from<W, O + 1, M>(lo, hi, prev, push_base, jshift, tab);
    }
}

// Load N dwords at byte address `addr` if readable up to `lim`; dwords that hold no byte below
// `lim` read as zero (only a buffer's last block takes the guarded path).
template <int N>
__device__ __forceinline__ void load_block(uint32_t (&d)[N], const uint8_t* data, uint64_t addr, uint64_t lim) {
    const bool full = addr + 4 * N <= lim;
    if (__all(full)) {
        const uint4* p = reinterpret_cast<const uint4*>(data + addr);
#pragma unroll
        for (int i = 0; i < N / 4; i++) {
            const uint4 v = p[i];
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
    } else {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(data + addr);
#pragma unroll
        for (int i = 0; i < N; i++) d[i] = (addr + 4 * i < lim) ? p[i] : 0u;
    }
}

// All candidate words of one block: word WI covers positions 32*WI .. 32*WI+31.
// Mirrored state: each word's 8 data dwords are bit-reversed in place right before its first
// position (not at the load: hipcc then hoists all 64 reversals above the first byte and waits for
// every load of the block there, and keeps raw and reversed copies live).
template <int W, int PK, int WI, int NW, int NCH, int ABL, int BLKW>
__device__ __forceinline__ void block_words(uint32_t (&words)[NCH][NW], uint32_t (&lo)[NCH], uint32_t (&hi)[NCH],
                                            uint32_t (&cur)[NCH][BLKW], const uint32_t (&prev)[NCH][16],
                                            uint32_t& c8, uint32_t& push_base, const uint8_t* tab, const ScanArgs& a) {
    if constexpr (WI < NW) {
        if constexpr ((ABL & kAblMirror) != 0) {
#pragma unroll
            for (int c = 0; c < NCH; c++)
#pragma unroll
                for (int i = 8 * WI; i < 8 * WI + 8; i++) cur[c][i] = __builtin_bitreverse32(cur[c][i]);
        }
        uint32_t bits[NCH];
        uint64_t gm[NCH][8];  // kAblSgprPred: the group's per-position compare masks (SGPR pairs)
        uint32_t hv[NCH][8];  // kAblMinGroup: the group's predicate words (mirrored hi)
#pragma unroll
        for (int c = 0; c < NCH; c++) bits[c] = 0;
        word_steps<W, PK, 32 * WI, 32 * WI, NCH, ABL, BLKW>(lo, hi, bits, cur, prev, c8, push_base, tab, a, gm, hv);
#pragma unroll
        for (int c = 0; c < NCH; c++) words[c][WI] = __builtin_bitreverse32(bits[c]);
        block_words<W, PK, WI + 1, NW, NCH, ABL, BLKW>(words, lo, hi, cur, prev, c8, push_base, tab, a);
    }
}

// Branch-free block load for software prefetch: a block that is not wholly readable (buffer tail,
// or no block at all) is fetched from the 128-byte device zero page instead, so no control flow
// separates the load from its use one iteration later (hipcc puts an s_waitcnt vmcnt(0) at
// every control-flow merge after a load).  `full` records whether the fast load was valid;
// tail blocks are re-read by fix_block when they become current.
template <int N>
__device__ __forceinline__ bool load_block_nb(uint32_t (&d)[N], const uint8_t* data, const uint8_t* zero_page,
                                              uint64_t addr, uint64_t lim) {
    const bool full = addr + 4 * N <= lim;
    const uint4* p = reinterpret_cast<const uint4*>(full ? data + addr : zero_page);
#pragma unroll
    for (int i = 0; i < N / 4; i++) {
        const uint4 v = p[i];
        d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
    }
    return full;
}

template <int N>
__device__ __forceinline__ void fix_block(uint32_t (&d)[N], bool full, const uint8_t* data, uint64_t addr,
                                          uint64_t lim) {
    if (!__all(full)) {  // rare: some lane's block is a buffer tail
        if (!full) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(data + addr);
#pragma unroll
            for (int i = 0; i < N; i++) d[i] = (addr + 4 * i < lim) ? p[i] : 0u;
        }
    }
}

// First candidate position in [lo, hi] (buffer-relative), or -1.
__device__ __forceinline__ int64_t find_first(const uint32_t* bm, uint64_t word0, uint64_t lo, uint64_t hi,
                                              uint32_t lane) {
    const uint64_t wlo = lo >> 5, whi = hi >> 5;
    for (uint64_t wb = wlo; wb <= whi; wb += 64) {
        const uint64_t w = wb + lane;
        uint32_t bits = 0;
        if (w <= whi) {
            bits = bm[word0 + w];
            if (w == wlo) bits &= ~0u << (lo & 31);
            if (w == whi) bits &= (hi & 31) == 31 ? ~0u : ((2u << (hi & 31)) - 1u);
        }
        const uint64_t m = __ballot(bits != 0);
        if (m) {
            const uint32_t l = __builtin_ctzll(m);
            const uint32_t b = __shfl(bits, l);
            return (int64_t)((wb + l) * 32 + __builtin_ctz(b));
        }
    }
    return -1;
}

// First candidate in [lo, hi] from the global bitmap, each lane testing 8 consecutive words
// (a wave covers 16 Ki positions per coalesced 2 KiB load).
__device__ __forceinline__ int64_t find_first_wide(const uint32_t* bm, uint64_t word0, uint32_t lo, uint32_t hi,
                                                   uint32_t lane) {
    const uint32_t lo_w = lo >> 5, hi_w = hi >> 5, lo_b = lo & 31, hi_b = hi & 31;
    for (uint32_t wb = lo_w; wb <= hi_w; wb += 512) {
        const uint32_t w0 = wb + 8 * lane;
        uint32_t bits[8];
        uint32_t any = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t w = w0 + j;
            uint32_t v = 0;
            if (w <= hi_w) {
                v = bm[word0 + w];
                if (w == lo_w) v &= ~0u << lo_b;
                if (w == hi_w) v &= hi_b == 31 ? ~0u : ((2u << hi_b) - 1u);
            }
            bits[j] = v;
            any |= v;
        }
        const uint64_t m = __ballot(any != 0);
        if (m) {
            const uint32_t l = __builtin_ctzll(m);
            uint32_t jj = 0, bb = 0;
#pragma unroll
            for (int j = 7; j >= 0; j--)
                if (bits[j]) { jj = j; bb = bits[j]; }
            const uint32_t pos_in = jj * 32 + (bb ? __builtin_ctz(bb) : 0);
            const uint32_t p = __shfl(pos_in, l);
            return (int64_t)(wb + 8 * l) * 32 + p;
        }
    }
    return -1;
}

__device__ __forceinline__ uint32_t sha_blocks(uint32_t len) { return (len + 8) / 64 + 1; }

// Greedy cut walk over one buffer's candidate bits (one wave, wave-uniform control flow):
// SURVEY.md A.3 — cut at the first candidate with n past min_len, or at max_len, tail last.
__device__ __forceinline__ void resolve_buffer(const ResolveArgs& a, uint32_t b, uint32_t lane, uint32_t* lhist) {
    {
        const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        const uint64_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint64_t word0 = off >> 5;
        uint64_t start = 0;
        uint32_t cnt = 0;
        while (start < len) {
            const uint64_t lo = start + a.first_off;
            const uint64_t forced = start + a.max_len - 1;
            const uint64_t hi = forced < len - 1 ? forced : len - 1;
            int64_t k = -1;
            // 64 words per probe: with thousands of short buffers this kernel is throughput-bound and
            // the 8-word-per-lane search (find_first_wide) measured 2.5x slower here
            if (lo <= hi) k = find_first(a.bitmap, word0, lo, hi, lane);
            if (k < 0) k = (int64_t)hi;  // forced cut at max_len, or the tail chunk
            const uint32_t clen = (uint32_t)(k + 1 - start);
            if (cnt < a.cap) {
                if (lane == 0) {
                    const uint64_t slot = (uint64_t)b * a.cap + cnt;
                    a.starts[slot] = (uint32_t)start;
                    a.clens[slot] = clen;
                    uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                    bin = bin < a.nbins ? bin : a.nbins - 1;
                    atomicAdd(&lhist[bin], 1u);
                }
            } else if (lane == 0) {
                atomicOr(a.overflow, 1u);
            }
            cnt++;
            start = (uint64_t)k + 1;
        }
        if (lane == 0) a.counts[b] = cnt < a.cap ? cnt : a.cap;
    }
}

// Candidate summary of one scan segment: the first kSumCands candidate offsets (segment-relative,
// u16) shifted into a 128-bit register quadruple, newest in the low half of s[0]; unused slots
// hold 0xFFFF.  ncand counts every candidate of the segment (> kSumCands = overflow).
constexpr uint32_t kSumCands = 8;

__device__ __forceinline__ void sum_push(uint32_t (&s)[4], uint32_t& ncand, uint32_t off) {
    if (ncand < kSumCands) {
        s[3] = __builtin_amdgcn_alignbit(s[3], s[2], 16);
        s[2] = __builtin_amdgcn_alignbit(s[2], s[1], 16);
        s[1] = __builtin_amdgcn_alignbit(s[1], s[0], 16);
        s[0] = (s[0] << 16) | off;
    }
    ncand++;
}

// Greedy cut walk of buffer b (one wave; lane l scanned segment l of it, seg_len bytes) from
// the lanes' candidate summaries: the first candidate in [lo, hi] is the smallest candidate of
// the first lane whose segment holds one there.  A step whose range touches an overflowed
// segment searches the bitmap instead (same answer; the bitmap is complete).
// QW (production): per-lane ascending candidate queue, one compare per cut; !QW (sweep variant
// 31, the round-2 form): a min over the 8 summary slots per cut.
template <bool QW = true>
__device__ __forceinline__ void resolve_from_summary(const ResolveArgs& a, uint32_t b, uint32_t lane,
                                                     const uint32_t (&sm)[4], uint32_t ncand, uint32_t ovf_off,
                                                     uint32_t seg_len, uint32_t* lhist) {
    const uint32_t len = a.uniform_len;
    const uint64_t word0 = ((uint64_t)b * len) >> 5;
    const uint32_t my_base = lane * seg_len;
    // The lane's candidates as an ascending queue, smallest in the top slot: the summary holds the
    // n = min(ncand, 8) candidates newest-lowest, so shift it up by 8 - n slots (0xFFFF fill).
    // `head` is the smallest candidate not yet passed by the walk (cuts only move forward, so
    // each candidate is popped once): per cut one compare instead of a min over all 8 slots.
    uint32_t q0 = sm[0], q1 = sm[1], q2 = sm[2], q3 = sm[3];
    {
        const uint32_t sh = kSumCands - (ncand < kSumCands ? ncand : kSumCands);
        if (sh & 4) { q3 = q1; q2 = q0; q1 = 0xFFFFFFFFu; q0 = 0xFFFFFFFFu; }
        if (sh & 2) { q3 = q2; q2 = q1; q1 = q0; q0 = 0xFFFFFFFFu; }
        if (sh & 1) {
            q3 = __builtin_amdgcn_alignbit(q3, q2, 16);
            q2 = __builtin_amdgcn_alignbit(q2, q1, 16);
            q1 = __builtin_amdgcn_alignbit(q1, q0, 16);
            q0 = (q0 << 16) | 0xFFFFu;
        }
    }
    auto head_of = [&](uint32_t top) { return (top >> 16) == 0xFFFFu ? 0xFFFFFFFFu : my_base + (top >> 16); };
    uint32_t head = head_of(q3);
    const bool ovf = ncand > kSumCands;
    uint32_t start = 0, cnt = 0;
    while (start < len) {
        const uint32_t lo = start + a.first_off;
        const uint32_t forced = start + a.max_len - 1;
        const uint32_t hi = forced < len - 1 ? forced : len - 1;
        int64_t k = -1;
        if (lo <= hi) {
            uint32_t best = 0xFFFFFFFFu;
            bool search;
            if constexpr (QW) {
                for (;;) {  // drop every candidate the walk has passed
                    const bool adv = head < lo;
                    if (__ballot(adv) == 0) break;
                    if (adv) {
                        q3 = __builtin_amdgcn_alignbit(q3, q2, 16);
                        q2 = __builtin_amdgcn_alignbit(q2, q1, 16);
                        q1 = __builtin_amdgcn_alignbit(q1, q0, 16);
                        q0 = (q0 << 16) | 0xFFFFu;
                        head = head_of(q3);
                    }
                }
                best = head <= hi ? head : 0xFFFFFFFFu;
                search = ovf && head == 0xFFFFFFFFu;
            } else {
#pragma unroll
                for (uint32_t j = 0; j < kSumCands; j++) {
                    const uint32_t v = (sm[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                    const uint32_t c = v == 0xFFFFu ? 0xFFFFFFFFu : my_base + v;
                    if (c >= lo && c <= hi && c < best) best = c;
                }
                search = ovf && best == 0xFFFFFFFFu;
            }
            // an overflowed segment's later candidates (after its 8th) are in the bitmap words
            // the scan stored from block ovf_off on; they follow every summary candidate, so they
            // matter only once the summary has none left in range
            if (search) {
                uint32_t x = my_base + ovf_off > lo ? my_base + ovf_off : lo;
                const uint32_t seg_hi = my_base + seg_len - 1;
                const uint32_t to = seg_hi < hi ? seg_hi : hi;
                while (x <= to) {
                    uint32_t w = a.bitmap[word0 + (x >> 5)] >> (x & 31);
                    const uint32_t span = to - x;  // positions x .. to, at most 32 of them in this word
                    if (span < 31) w &= (2u << span) - 1u;
                    if (w) { best = x + __builtin_ctz(w); break; }
                    x = (x | 31u) + 1u;
                }
            }
            const uint64_t m = __ballot(best != 0xFFFFFFFFu);
            if (m) k = (int64_t)__builtin_amdgcn_readlane(best, (int)__builtin_ctzll(m));
        }
        if (k < 0) k = (int64_t)hi;  // forced cut at max_len, or the tail chunk
        const uint32_t clen = (uint32_t)(k + 1 - start);
        if (cnt < a.cap) {
            if (lane == 0) {
                const uint64_t slot = (uint64_t)b * a.cap + cnt;
                a.starts[slot] = start;
                a.clens[slot] = clen;
                uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                bin = bin < a.nbins ? bin : a.nbins - 1;
                atomicAdd(&lhist[bin], 1u);
            }
        } else if (lane == 0) {
            atomicOr(a.overflow, 1u);
        }
        cnt++;
        start = (uint32_t)k + 1;
    }
    if (lane == 0) a.counts[b] = cnt < a.cap ? cnt : a.cap;
}

// Cross-lane scans on the DPP network (VALU only: no trip through the LDS unit, whose queue the
// scan's table lookups keep long).  Inclusive sum / max over the wave; wave_shr1: lane i gets
// lane i - 1's value, lane 0 gets 0.
#define SDFS_DPP(x, ctrl, rm) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), (ctrl), (rm), 0xf, false))
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += SDFS_DPP(x, 0x111, 0xf);  // row_shr:1
    x += SDFS_DPP(x, 0x112, 0xf);  // row_shr:2
    x += SDFS_DPP(x, 0x114, 0xf);  // row_shr:4
    x += SDFS_DPP(x, 0x118, 0xf);  // row_shr:8
    x += SDFS_DPP(x, 0x142, 0xa);  // row_bcast:15 into rows 1 and 3
    x += SDFS_DPP(x, 0x143, 0xc);  // row_bcast:31 into rows 2 and 3
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    auto mx = [](uint32_t u, uint32_t v) { return u > v ? u : v; };
    x = mx(x, SDFS_DPP(x, 0x111, 0xf));
    x = mx(x, SDFS_DPP(x, 0x112, 0xf));
    x = mx(x, SDFS_DPP(x, 0x114, 0xf));
    x = mx(x, SDFS_DPP(x, 0x118, 0xf));
    x = mx(x, SDFS_DPP(x, 0x142, 0xa));
    x = mx(x, SDFS_DPP(x, 0x143, 0xc));
    return x;
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) { return SDFS_DPP(x, 0x138, 0xf); }
#undef SDFS_DPP

// List walk (production since round 4): the greedy cut walk of buffer b from the lanes' candidate
// summaries with only four trips through the LDS unit, so it does not queue behind the other
// waves' table lookups once per cut as the queue walk's lane-0 work and an LDS pointer chase
// would (scripts/probes/probe_r4_walk_pmc.sh, probe_r4_list_walk.sh):
//   1. the lanes' candidates, ascending, go to the wave's LDS list at the (DPP) prefix of their
//      counts; entry e (page e / 64) is then read back by lane e % 64;
//   2. each entry's next-cut pointer — the first entry >= pos + 1 + first_off, if within the
//      chunk's max_len — from the segment lane T holding pos + 1 + first_off: its list base and
//      count (one bpermute) and its <= 8 entries plus the one after (one round of reads);
//   3. the chain from the first cut follows the pointers with v_readlane (registers only) and
//      marks the cut entries in per-page SGPR masks;
//   4. every lane writes the chunk of its marked entry (rank from the masks, start = the previous
//      cut + 1 by a DPP max-scan) and lane 0 the tail chunk.
// It declines (false, nothing written) when a summary overflowed, the list would exceed kListCap,
// seg_len is not a power of two, or a forced cut (a max_len chunk ending at a non-candidate)
// occurs before the tail; the queue walk (resolve_from_summary) then resolves the buffer.
constexpr uint32_t kListCap = 256;

__device__ __forceinline__ bool resolve_from_list(const ResolveArgs& a, uint32_t b, uint32_t lane,
                                                  const uint32_t (&sm)[4], uint32_t ncand, uint32_t seg_len,
                                                  uint32_t* lhist, uint32_t* wl, uint32_t probe = 0) {
    // probe (measurement only, tuning: SDFS_SKIP_WALK=2/3): 2 = no outputs at all, 3 = chunk
    // stores and LDS histogram but no counts (the pipeline then sees no chunks)
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const uint32_t len = a.uniform_len;
    if (__ballot(ncand > kSumCands) || len > (1u << 22) || (seg_len & (seg_len - 1)) != 0) return false;
    const uint32_t n = ncand;
    const uint32_t incl = wave_incl_sum(n);
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
    if (total > kListCap) return false;
    const uint32_t base = incl - n;
    const uint32_t sh = __builtin_ctz(seg_len);
    // 1. the sorted list (summary slot j, j = 0 the newest = largest, goes to base + n - 1 - j)
#pragma unroll
    for (uint32_t j = 0; j < kSumCands; j++)
        if (j < n) wl[base + n - 1 - j] = (lane << sh) + ((sm[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr uint32_t NP = kListCap / 64;
    uint32_t pos[NP], np[NP];
#pragma unroll
    for (uint32_t k = 0; k < NP; k++) pos[k] = lane + 64 * k < total ? wl[lane + 64 * k] : kNone;
    // 2. next pointers: entries of lane T's segment sit at [base_T, base_T + n_T); the first entry
    //    >= lo is base_T + (those < lo), and it is the one read at j = that count (entries of later
    //    segments all exceed lo)
    const uint32_t bn = base | (n << 16);
#pragma unroll
    for (uint32_t k = 0; k < NP; k++) {
        np[k] = kNone;
        if (64 * k < total) {
            const uint32_t p = pos[k];
            const uint32_t lo = p + 1 + a.first_off;
            const uint32_t hi = p + a.max_len < len - 1 ? p + a.max_len : len - 1;
            const bool act = p != kNone && lo <= hi;
            const uint32_t t = act ? lo >> sh : 0u;
            const uint32_t tb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(t << 2), (int)bn);
            const uint32_t tbase = tb & 0xFFFFu, tn = tb >> 16;
            uint32_t less = 0, q = kNone;
#pragma unroll
            for (uint32_t j = 0; j <= kSumCands; j++) {
                const uint32_t e = tbase + j;
                const uint32_t v = act && j <= tn && e < total ? wl[e] : kNone;
                less += v < lo ? 1u : 0u;
                q = v >= lo && v < q ? v : q;
            }
            if (act && q <= hi) np[k] = tbase + less;
        }
    }
    // 3. the chain (wave-uniform): the first cut is the first entry >= first_off, if within max_len
    uint32_t first = 0;
#pragma unroll
    for (uint32_t k = 0; k < NP; k++) first += (uint32_t)__builtin_popcountll(__ballot(pos[k] < a.first_off));
    uint32_t idx = kNone;
    if (first < total) {
        uint32_t fp = kNone;
#pragma unroll
        for (uint32_t k = 0; k < NP; k++)
            if ((first >> 6) == k) fp = __builtin_amdgcn_readlane(pos[k], first & 63);
        const uint32_t hi0 = a.max_len - 1 < len - 1 ? a.max_len - 1 : len - 1;
        if (fp <= hi0) idx = first;
    }
    uint64_t cut[NP];
    uint32_t cnt = 0, start = 0;
#pragma unroll
    for (uint32_t k = 0; k < NP; k++) {
        cut[k] = 0;
        uint32_t last = kNone;
        while (idx != kNone && (idx >> 6) == k) {
            cut[k] |= 1ull << (idx & 63);
            last = idx & 63;
            cnt++;
            idx = __builtin_amdgcn_readlane(np[k], last);
        }
        if (last != kNone) start = __builtin_amdgcn_readlane(pos[k], last) + 1;
    }
    // no candidate in the next chunk's range: the tail chunk if that range reaches the buffer end,
    // else a forced cut — declined
    if (start < len && start + a.max_len - 1 < len - 1) return false;
    // 4. the chunks, wave-parallel
    uint32_t carry_rank = 0, carry_pos = 0;  // cuts of the earlier pages, the last cut's end + 1
#pragma unroll
    for (uint32_t k = 0; k < NP; k++) {
        if (cut[k] == 0) continue;
        const bool c = (cut[k] >> lane) & 1;
        const uint32_t rank = carry_rank + __builtin_amdgcn_mbcnt_hi((uint32_t)(cut[k] >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)cut[k], 0u));
        const uint32_t end1 = c ? pos[k] + 1 : 0u;
        uint32_t prev = wave_incl_max(wave_shr1(end1));
        prev = prev > carry_pos ? prev : carry_pos;
        if (c && probe != 2) {
            if (rank < a.cap) {
                const uint64_t slot = (uint64_t)b * a.cap + rank;
                const uint32_t clen = end1 - prev;
                a.starts[slot] = prev;
                a.clens[slot] = clen;
                uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                bin = bin < a.nbins ? bin : a.nbins - 1;
                atomicAdd(&lhist[bin], 1u);
            } else {
                atomicOr(a.overflow, 1u);
            }
        }
        carry_rank += (uint32_t)__builtin_popcountll(cut[k]);
        const uint32_t mx = __builtin_amdgcn_readlane(wave_incl_max(end1), 63);
        carry_pos = mx > carry_pos ? mx : carry_pos;
    }
    if (lane == 0 && probe) {
        a.counts[b] = 0;
    } else if (lane == 0) {
        const uint32_t nchunks = cnt + (start < len ? 1u : 0u);
        if (start < len) {  // the tail chunk
            if (cnt < a.cap) {
                const uint64_t slot = (uint64_t)b * a.cap + cnt;
                a.starts[slot] = start;
                a.clens[slot] = len - start;
                uint32_t bin = sha_blocks(len - start) >> a.bin_shift;
                bin = bin < a.nbins ? bin : a.nbins - 1;
                atomicAdd(&lhist[bin], 1u);
            } else {
                atomicOr(a.overflow, 1u);
            }
        }
        a.counts[b] = nchunks < a.cap ? nchunks : a.cap;
    }
    return true;
}

// First candidate position in [lo, hi] of uniform buffer b (buffer-relative), or -1, from the
// scan's stored segment summaries (piece mode, ResolveArgs::seg_sum): lane l takes segment
// lo / seg_len + l — its candidates are the summary's (the segment's first kSumCands) and, past
// them, the sparse bitmap words the scan stored from the summary's overflow on.  One round covers
// 64 segments (256 KiB at 4 KiB segments; a search spans at most max_len).
__device__ __forceinline__ int64_t find_first_sum(const ResolveArgs& a, uint32_t b, uint32_t lo, uint32_t hi,
                                                  uint32_t lane) {
    const uint32_t sl = a.seg_len;
    const uint64_t spb = a.uniform_len / sl;
    const uint64_t word0 = ((uint64_t)b * a.uniform_len) >> 5;
    for (uint32_t s0 = lo / sl; s0 <= hi / sl; s0 += 64) {
        const uint32_t sj = s0 + lane;
        uint32_t best = 0xFFFFFFFFu;
        if (sj <= hi / sl) {
            const uint32_t* ss = a.seg_sum + ((uint64_t)b * spb + sj) * kSegSumWords;
            const uint4 q = *reinterpret_cast<const uint4*>(ss);
            const uint32_t nc = ss[4], ovf = ss[5];
            const uint32_t base = sj * sl;
            const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t v = (qw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                const uint32_t c = base + v;
                if (v != 0xFFFFu && c >= lo && c <= hi && c < best) best = c;
            }
            if (best == 0xFFFFFFFFu && nc > kSumCands) {
                // the segment's later candidates, in the bitmap words stored from ovf on
                uint32_t x = base + ovf > lo ? base + ovf : lo;
                const uint32_t seg_hi = base + sl - 1;
                const uint32_t to = seg_hi < hi ? seg_hi : hi;
                while (x <= to) {
                    uint32_t w = a.bitmap[word0 + (x >> 5)] >> (x & 31);
                    const uint32_t span = to - x;
                    if (span < 31) w &= (2u << span) - 1u;
                    if (w) { best = x + __builtin_ctz(w); break; }
                    x = (x | 31u) + 1u;
                }
            }
        }
        const uint64_t m = __ballot(best != 0xFFFFFFFFu);
        if (m) return (int64_t)__builtin_amdgcn_readlane(best, (int)__builtin_ctzll(m));
    }
    return -1;
}

// Speculative walk of one 64-segment piece of a long buffer (the sectioned cut walk with
// sections of 64 x seg_len bytes: one wave scanned exactly this piece), from the lanes' candidate
// summaries instead of bitmap searches: chunk starts from an assumed start at the piece start,
// each cut found inside the piece (or forced inside it); the walk stops at the first chunk whose
// cut lies past the piece end — cdc_resolve_join_kernel finds that one in the complete bitmap and
// writes spec_next.  Replaces cdc_resolve_spec_kernel's per-chunk bitmap round trips.
__device__ __forceinline__ void piece_walk_from_summary(const ResolveArgs& a, uint32_t item, uint32_t r0, uint32_t lane,
                                                        const uint32_t (&sm)[4], uint32_t ncand, uint32_t ovf_off,
                                                        uint32_t seg_len, uint64_t word0) {
    const uint32_t len = a.uniform_len;
    const uint32_t r1 = r0 + 64 * seg_len < len ? r0 + 64 * seg_len : len;
    const uint32_t my_base = r0 + lane * seg_len;
    uint32_t q0 = sm[0], q1 = sm[1], q2 = sm[2], q3 = sm[3];
    {
        const uint32_t sh = kSumCands - (ncand < kSumCands ? ncand : kSumCands);
        if (sh & 4) { q3 = q1; q2 = q0; q1 = 0xFFFFFFFFu; q0 = 0xFFFFFFFFu; }
        if (sh & 2) { q3 = q2; q2 = q1; q1 = q0; q0 = 0xFFFFFFFFu; }
        if (sh & 1) {
            q3 = __builtin_amdgcn_alignbit(q3, q2, 16);
            q2 = __builtin_amdgcn_alignbit(q2, q1, 16);
            q1 = __builtin_amdgcn_alignbit(q1, q0, 16);
            q0 = (q0 << 16) | 0xFFFFu;
        }
    }
    auto head_of = [&](uint32_t top) { return (top >> 16) == 0xFFFFu ? 0xFFFFFFFFu : my_base + (top >> 16); };
    uint32_t head = head_of(q3);
    const bool ovf = ncand > kSumCands;
    uint32_t* sp = a.spec_starts + (uint64_t)item * a.spec_cap;
    uint32_t start = r0, cnt = 0;
    while (start < r1) {
        if (lane == 0 && cnt < a.spec_cap) sp[cnt] = start;
        cnt++;
        const uint32_t lo = start + a.first_off;
        const uint32_t forced = start + a.max_len - 1;
        const uint32_t hi = forced < len - 1 ? forced : len - 1;
        const uint32_t hp = hi < r1 - 1 ? hi : r1 - 1;  // this piece's part of the search
        int64_t k = -1;
        if (lo <= hp) {
            for (;;) {  // drop every candidate the walk has passed
                const bool adv = head < lo;
                if (__ballot(adv) == 0) break;
                if (adv) {
                    q3 = __builtin_amdgcn_alignbit(q3, q2, 16);
                    q2 = __builtin_amdgcn_alignbit(q2, q1, 16);
                    q1 = __builtin_amdgcn_alignbit(q1, q0, 16);
                    q0 = (q0 << 16) | 0xFFFFu;
                    head = head_of(q3);
                }
            }
            uint32_t best = head <= hp ? head : 0xFFFFFFFFu;
            if (ovf && head == 0xFFFFFFFFu) {
                uint32_t x = my_base + ovf_off > lo ? my_base + ovf_off : lo;
                const uint32_t seg_hi = my_base + seg_len - 1;
                const uint32_t to = seg_hi < hp ? seg_hi : hp;
                while (x <= to) {
                    uint32_t w = a.bitmap[word0 + (x >> 5)] >> (x & 31);
                    const uint32_t span = to - x;
                    if (span < 31) w &= (2u << span) - 1u;
                    if (w) { best = x + __builtin_ctz(w); break; }
                    x = (x | 31u) + 1u;
                }
            }
            const uint64_t m = __ballot(best != 0xFFFFFFFFu);
            if (m) k = (int64_t)__builtin_amdgcn_readlane(best, (int)__builtin_ctzll(m));
        }
        if (k < 0) {
            if (hi > r1 - 1) break;  // the cut lies past the piece: the join kernel finds it
            k = (int64_t)hi;         // forced cut, or the buffer's tail chunk, inside the piece
        }
        start = (uint32_t)k + 1;
    }
    if (lane == 0) a.spec_cnt[item] = cnt < a.spec_cap ? cnt : a.spec_cap;
}

// Scan variants (DESIGN.md "Rabin scan"): C lane-private table copies (32: conflict-free,
// 128 KiB, one 1024-thread workgroup per CU; 16: 2-way, 64 KiB, two workgroups per CU), NCH
// independent segments per lane, BLK bytes per lane per iteration (128 = one whole cache line
// per lane per load, so no line is fetched twice), PF = prefetch the next block.
// FUSE: 0 = separate resolve kernel; 1 = each wave walks its buffer's bitmap in the epilogue
// (sweep only, measured slower); 2 = each lane keeps its segment's first kSumCands candidate
// offsets in registers while it scans, and the wave resolves its buffer from them in the epilogue
// (no bitmap reads unless a segment overflows: DESIGN.md §4).
// THREADS: the widest workgroup the variant is launched with (the register budget follows from
// THREADS and WPS: 512 / waves-per-SIMD VGPRs, so 768 threads at 3 waves/SIMD allow 168).
// With FUSE 2 and two chains, chain c of a wave covers segments base + c * blockDim.x + 64w ..
// + 63, i.e. its own buffer, and the epilogue walks both buffers.
template <int C, int NCH, bool PF, int WPS, int ABL = 0, int BLK = 64, int FUSE = 0, int THREADS = kScanThreads,
          bool MIRROR = false>
struct ScanCfg {
    static constexpr bool kMirror = MIRROR;  // bit-reversed rolling state (roll_step, kAblMirror)
    static constexpr bool kPopSwap = MIRROR && (ABL & kAblPopSwap) != 0;  // pop entries high word first
    static constexpr int kFuse = NCH == 1 ? FUSE : (FUSE == 2 ? 2 : 0);  // resolve each wave's buffer(s) in the epilogue
    static constexpr int kThreads = THREADS;
    static constexpr int kAbl = ABL;
    static constexpr int kCopies = C;
    static constexpr int kChains = NCH;
    static constexpr bool kPrefetch = PF;
    static constexpr int kWavesPerSimd = WPS;  // __launch_bounds__ occupancy request
    static constexpr int kLds = scan_lds_bytes(C);
    static constexpr uint32_t kPushOff = C == 32 ? 0x10000u : 0x80u;
    static constexpr int kBlk = BLK;
    // the list walk's per-wave LDS list (1 KiB per wave): one chain, the 32-copy tables
    static constexpr bool kListWalk = kFuse == 2 && NCH == 1 && C == 32;
};

// One pass of the scan over the segments base + c * bdim + tid (c < chains) — one lane's share of
// one iteration of the persistent scan kernel below; the fused scan + fingerprint kernel calls it
// per wave with (buffer * 64, lane, 64).  With the fused cut walk, the wave's 64 segments are
// buffer (base + (tid & ~63)) / 64.
template <int W, int PK, class CFG>
__device__ __forceinline__ void scan_iter(const ScanArgs& a, const uint8_t* tab, uint32_t* lhist, uint64_t base,
                                          uint32_t tid, uint32_t bdim, uint64_t total, uint32_t lane, uint32_t c8,
                                          uint32_t push_base, uint32_t& pa_reg, uint32_t& qa_reg,
                                          uint32_t* wlist = nullptr) {
    constexpr int MB =
        (CFG::kMirror ? kAblMirror : 0) | (CFG::kAbl & (kAblSgprPred | kAblSdwa | kAblSdwaPop | kAblMinGroup | kAblMinGroup8 | kAblPopSwap | kAblPopMux));
    constexpr int NCH = CFG::kChains;
    constexpr int BLK = CFG::kBlk;
    constexpr int BLKW = BLK / 4;
    uint64_t start[NCH], end[NCH];
    uint32_t nblk[NCH];
    bool first[NCH];
    uint32_t maxblk = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const uint64_t seg = base + (uint64_t)c * bdim + tid;
        start[c] = end[c] = 0;
        nblk[c] = 0;
        first[c] = true;
        if (seg < total) {
            uint64_t bstart, blen, sidx;
            if (a.uniform_len) {
                const uint64_t spb = (a.uniform_len + a.seg_len - 1) / a.seg_len;
                const uint64_t b = seg / spb;
                sidx = seg - b * spb;
                bstart = b * a.uniform_len;
                blen = a.uniform_len;
            } else {
                uint32_t lo_b = 0, hi_b = a.nbuf;  // last b with seg_prefix[b] <= seg
                while (hi_b - lo_b > 1) {
                    const uint32_t mid = (lo_b + hi_b) >> 1;
                    if (a.seg_prefix[mid] <= seg) lo_b = mid; else hi_b = mid;
                }
                sidx = seg - a.seg_prefix[lo_b];
                bstart = a.offs[lo_b];
                blen = a.lens[lo_b];
            }
            start[c] = bstart + sidx * a.seg_len;
            const uint64_t bend = bstart + blen;
            end[c] = start[c] + a.seg_len < bend ? start[c] + a.seg_len : bend;
            nblk[c] = (uint32_t)((end[c] - start[c] + BLK - 1) / BLK);
            // window warm-up reads the previous 64 bytes unless this is the buffer's first segment
            first[c] = start[c] == bstart;
        }
        maxblk = nblk[c] > maxblk ? nblk[c] : maxblk;
    }

    uint32_t lo[NCH], hi[NCH];
    uint32_t prev[NCH][16], cur[NCH][BLKW];
    bool cur_full[NCH];
    uint32_t sm[NCH][4];  // FUSE == 2: candidate summary per chain
    uint32_t ncand[NCH];
    uint32_t ovf_off[NCH];  // FUSE == 2: segment offset of the first stored bitmap block
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        sm[c][0] = sm[c][1] = sm[c][2] = sm[c][3] = 0xFFFFFFFFu;
        ncand[c] = 0;
        ovf_off[c] = 0xFFFFFFFFu;
    }
    // FUSE == 2 with the fused resolve: bitmap words are stored only once a lane's summary has
    // overflowed (> kSumCands candidates), from that block on; resolve_from_summary reads them
    // only there.  Saves the 0.5 GB of bitmap writes per 4 GiB.
    const bool sparse_bm = CFG::kFuse == 2 && a.fuse_resolve != 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        if (nblk[c] != 0 && !first[c]) {
            load_block<16>(prev[c], a.data, start[c] - 64, start[c]);
            if constexpr (CFG::kMirror)
#pragma unroll
                for (int i = 0; i < 16; i++) prev[c][i] = __builtin_bitreverse32(prev[c][i]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) prev[c][i] = 0;  // bytes before the buffer are empty
        }
        lo[c] = hi[c] = 0;
        warm_from<W, 64 - W, CFG::kMirror>(lo[c], hi[c], prev[c], push_base, a.jshift, tab);
        if constexpr (CFG::kPrefetch) {
            const bool act = nblk[c] != 0;
            cur_full[c] = load_block_nb<BLKW>(cur[c], a.data, a.zero_page, act ? start[c] : 0, act ? end[c] : 0);
        }
    }

    for (uint32_t blk = 0; blk < maxblk; blk++) {
        uint32_t nxt[NCH][CFG::kPrefetch ? BLKW : 1];
        bool nxt_full[NCH];
        uint32_t words[NCH][BLK / 32];
        bool split_fast = false;
        if constexpr ((CFG::kAbl & kAblFullBlocks) != 0) {
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const uint4* p = reinterpret_cast<const uint4*>(a.data + start[c] + (uint64_t)BLK * blk);
#pragma unroll
                for (int i = 0; i < BLKW / 4; i++) {
                    const uint4 v = p[i];
                    cur[c][4 * i] = v.x; cur[c][4 * i + 1] = v.y; cur[c][4 * i + 2] = v.z; cur[c][4 * i + 3] = v.w;
                }
            }
            block_words<W, PK, 0, BLK / 32, NCH, (CFG::kAbl & 7) | MB, BLKW>(words, lo, hi, cur, prev, qa_reg, pa_reg,
                                                                             tab, a);
            split_fast = true;
        } else if constexpr (CFG::kAbl & 16) {
            // split body: when every lane's block is whole, a branch of its own loads and
            // scans it, so no control-flow merge sits between the loads and their uses (hipcc
            // waits for all 16 loads at such a merge; here it waits per 64 bytes scanned).
            // Interleaved A/B: 1.59 -> 1.52 ms per 4 GiB (profiles/r01/probes/scan_split_body_ab.jsonl)
            bool full = true;
#pragma unroll
            for (int c = 0; c < NCH; c++)
                full = full && blk < nblk[c] && start[c] + (uint64_t)BLK * (blk + 1) <= end[c];
            split_fast = __all(full);
            if (split_fast) {
#pragma unroll
                for (int c = 0; c < NCH; c++) {
                    const uint4* p = reinterpret_cast<const uint4*>(a.data + start[c] + (uint64_t)BLK * blk);
#pragma unroll
                    for (int i = 0; i < BLKW / 4; i++) {
                        const uint4 v = p[i];
                        cur[c][4 * i] = v.x; cur[c][4 * i + 1] = v.y; cur[c][4 * i + 2] = v.z; cur[c][4 * i + 3] = v.w;
                    }
                }
                block_words<W, PK, 0, BLK / 32, NCH, (CFG::kAbl & 3) | MB, BLKW>(words, lo, hi, cur, prev, qa_reg, pa_reg,
                                                                                 tab, a);
            }
        }
        if (!split_fast) {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if constexpr (CFG::kPrefetch) {
                fix_block<BLKW>(cur[c], cur_full[c], a.data, start[c] + (uint64_t)BLK * blk, end[c]);
                const bool act = blk + 1 < nblk[c];
                nxt_full[c] = load_block_nb<BLKW>(nxt[c], a.data, a.zero_page,
                                                  act ? start[c] + (uint64_t)BLK * (blk + 1) : 0, act ? end[c] : 0);
            } else if constexpr (CFG::kAbl & 8) {
#pragma unroll
                for (int i = 0; i < BLKW; i++) cur[c][i] = prev[c][i & 15] * 0x9E3779B1u + blk;
            } else {
                const bool act = blk < nblk[c];
                load_block<BLKW>(cur[c], a.data, act ? start[c] + (uint64_t)BLK * blk : 0, act ? end[c] : 0);
            }
        }
        block_words<W, PK, 0, BLK / 32, NCH, (CFG::kAbl & 15) | MB, BLKW>(words, lo, hi, cur, prev, qa_reg, pa_reg, tab, a);
        }
        if constexpr (CFG::kFuse == 2) {
            // candidates are rare (~1 per 4 KiB): a divergent, seldom-taken append
#pragma unroll
            for (int c = 0; c < NCH; c++)
#pragma unroll
                for (int w = 0; w < BLK / 32; w++) {
                    uint32_t bits = blk < nblk[c] ? words[c][w] : 0u;
                    while (bits) {
                        const uint32_t off = blk * BLK + 32 * w + __builtin_ctz(bits);
                        bits &= bits - 1;
                        if (start[c] + off < end[c]) sum_push(sm[c], ncand[c], off);
                    }
                }
        }
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if constexpr (CFG::kFuse == 2)
                if (ncand[c] > kSumCands && ovf_off[c] == 0xFFFFFFFFu) ovf_off[c] = blk * BLK;
            if (blk < nblk[c] && (!sparse_bm || ncand[c] > kSumCands)) {
                const uint64_t pos = start[c] + (uint64_t)BLK * blk;
                uint32_t* bm = a.bitmap + (pos >> 5);
                if (pos + BLK <= end[c]) {
                    if constexpr (BLK >= 128) {
#pragma unroll
                        for (int w = 0; w < BLK / 32; w += 4)
                            *reinterpret_cast<uint4*>(bm + w) =
                                make_uint4(words[c][w], words[c][w + 1], words[c][w + 2], words[c][w + 3]);
                    } else {
                        *reinterpret_cast<uint2*>(bm) = make_uint2(words[c][0], words[c][1]);
                    }
                } else {
                    // buffer tail: words past the buffer end may belong to the next buffer
#pragma unroll
                    for (int w = 0; w < BLK / 32; w++)
                        if (pos + 32 * w < end[c]) bm[w] = words[c][w];
                }
            }
#pragma unroll
            for (int i = 0; i < 16; i++) prev[c][i] = cur[c][BLKW - 16 + i];
            if constexpr (CFG::kPrefetch) {
#pragma unroll
                for (int i = 0; i < BLKW; i++) cur[c][i] = nxt[c][i];
                cur_full[c] = nxt_full[c];
            }
        }
    }
    if constexpr (CFG::kFuse != 0) {
        if (a.fuse_resolve && a.skip_walk != 1) {
            // this wave's 64 segments are buffer seg0 / 64: make the lanes' bitmap stores
            // visible to the whole wave (same CU, so no L1 staleness), then walk its cuts
            const uint64_t seg0 = base + (tid & ~63u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if constexpr (CFG::kFuse == 2) {
                if (a.fuse_resolve == 2) {
                    // piece mode (one chain only; the engine selects it for the production scan):
                    // the wave's 64 segments are piece (seg0 mod spb) / 64 of buffer seg0 / spb (a
                    // long uniform buffer, sections of 64 segments)
                    if constexpr (NCH == 1) {
                        if (base + tid < total) {  // this lane's segment summary, for the join / stitch
                            uint32_t* ss = a.res.seg_sum + (base + tid) * kSegSumWords;
                            *reinterpret_cast<uint4*>(ss) = make_uint4(sm[0][0], sm[0][1], sm[0][2], sm[0][3]);
                            *reinterpret_cast<uint2*>(ss + 4) = make_uint2(ncand[0], ovf_off[0]);
                        }
                        const uint64_t spb = a.uniform_len / a.seg_len;
                        const uint64_t b = seg0 / spb;
                        const uint32_t piece = (uint32_t)((seg0 - b * spb) >> 6);
                        if (seg0 < total)
                            piece_walk_from_summary(a.res, (uint32_t)b * a.res.nsec + piece, piece * 64 * a.seg_len,
                                                    lane, sm[0], ncand[0], ovf_off[0], a.seg_len,
                                                    (b * a.uniform_len) >> 5);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < NCH; c++) {
                        const uint64_t sc = seg0 + (uint64_t)c * bdim;
                        if (sc < total) {
                            bool done = false;
                            if constexpr (CFG::kListWalk)
                                if (wlist && a.list_walk)
                                    done = resolve_from_list(a.res, (uint32_t)(sc >> 6), lane, sm[c], ncand[c], a.seg_len,
                                                             lhist, wlist, a.skip_walk);
                            if (!done && a.skip_walk > 1) {
                                if (lane == 0) a.res.counts[(uint32_t)(sc >> 6)] = 0;
                            } else if (!done)
                                resolve_from_summary<(CFG::kAbl & 128) == 0>(a.res, (uint32_t)(sc >> 6), lane, sm[c],
                                                                             ncand[c], ovf_off[c], a.seg_len, lhist);
                        }
                    }
                }
            } else {
                if (seg0 < total) resolve_buffer(a.res, (uint32_t)(seg0 >> 6), lane, lhist);
            }
        }
    }
}

template <int W, int PK, class CFG>
__global__ __launch_bounds__(CFG::kThreads, CFG::kWavesPerSimd) void cdc_scan_kernel(ScanArgs a) {
    static_assert(!CFG::kMirror || !CFG::kPrefetch, "mirrored state: no prefetch");
    static_assert(CFG::kMirror || PK < 2, "the one-compare and divisor predicates need the mirrored state");
    constexpr int NCH = CFG::kChains;
    constexpr int C = CFG::kCopies;
    __shared__ __attribute__((aligned(16))) uint8_t tab[CFG::kLds];
    __shared__ uint32_t lhist[CFG::kFuse ? kMaxBins : 1];  // fused resolve: chunk-length histogram
    __shared__ uint32_t wlist[CFG::kListWalk ? CFG::kThreads / 64 * kListCap : 1];  // list walk: per wave
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.tab_image);
        uint4* dst = reinterpret_cast<uint4*>(tab);
        for (int i = threadIdx.x; i < CFG::kLds / 16; i += blockDim.x) dst[i] = src[i];
        if constexpr (CFG::kFuse != 0)
            for (uint32_t i = threadIdx.x; i < kMaxBins; i += blockDim.x) lhist[i] = 0;
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c8 = (lane & (C - 1)) << 3;
    const uint32_t push_base = CFG::kPushOff | c8;
    // the block loop's address registers: the SDWA forms (kAblSdwa, kAblSdwaPop) rewrite byte 1
    // of these in place, every other form only reads them
    uint32_t pa_reg = push_base, qa_reg = c8;
    const uint64_t total = a.uniform_len ? a.total_segs : a.seg_prefix[a.nbuf];
    // workgroups of 64..1024 threads (a multiple of 64: a wave never straddles two buffers of the
    // fused walk); small batches launch narrow workgroups so their waves do not share SIMDs
    const uint64_t per_iter = (uint64_t)blockDim.x * NCH;

    uint32_t* const wl = CFG::kListWalk ? wlist + (threadIdx.x >> 6) * kListCap : nullptr;
    // Work queue (tuning only, SDFS_SCAN_DYN=1; one-chain forms with a counter): each wave takes
    // the next 64 segments (one 256 KiB buffer of the fused walk) from a per-launch counter, so
    // waves that start late — their CU still running the other batch's fingerprint workgroups or
    // an RCCL kernel — would take fewer items instead of stretching the launch; every wave leaves
    // once the counter passes the last item.  Measured no faster at N = 1 and 2-5 % slower for
    // the scan alone, so production keeps the static workgroup stride.  One call
    // site, so the byte loop is compiled once.
    bool dyn = false;
    if constexpr (NCH == 1) dyn = a.wave_ctr != nullptr;
    const uint32_t items = (uint32_t)((total + 63) >> 6);
    uint64_t sbase = (uint64_t)blockIdx.x * per_iter;
    for (;;) {
        uint64_t base;
        uint32_t tid, bdim;
        if (dyn) {
            uint32_t it = 0;
            if (lane == 0) it = atomicAdd(a.wave_ctr, 1u);
            it = __builtin_amdgcn_readfirstlane(it);
            if (it >= items) break;
            base = (uint64_t)it * 64;
            tid = lane;
            bdim = 64;
        } else {
            if (sbase >= total) break;
            base = sbase;
            tid = threadIdx.x;
            bdim = blockDim.x;
            sbase += (uint64_t)gridDim.x * per_iter;
        }
        scan_iter<W, PK, CFG>(a, tab, lhist, base, tid, bdim, total, lane, c8, push_base, pa_reg, qa_reg, wl);
    }
    if constexpr (CFG::kFuse != 0) {
        if (a.fuse_resolve && a.skip_walk < 2) {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < a.res.nbins; i += blockDim.x)
                if (lhist[i]) atomicAdd(&a.res.hist[i], lhist[i]);
        }
    }
}

// ------------------------------------------------------------------------------------------
// 5. per-chunk fingerprint: one lane per chunk (tasks are sorted longest-first so the lanes of
//    a wave carry near-equal block counts)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }

constexpr uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

// SHA-256 compression (FIPS 180-4 6.2.2) on 16 big-endian message words; rotations map to
// v_alignbit_b32, the Sigma xors and Ch/Maj to v_bitop3_b32, the three-input sums to v_add3_u32.
// SB (sweep builds): a scheduling barrier after every round, so hipcc cannot overlap rounds
// (lower register pressure, less ILP).
template <bool SB = false>
__device__ __forceinline__ void sha256_compress(uint32_t (&s)[8], uint32_t (&w)[16]) {
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma clang loop unroll(full)
    for (int i = 0; i < 64; i++) {
        if (i >= 16 && (i & 15) == 0) {
            // Message schedule for rounds i..i+15, in place over the 16-word window.  The empty
            // asm ties the window to the round state so hipcc cannot hoist all of W[16..63]
            // above the rounds (48 live VGPRs, occupancy 3); it emits no instruction and, since
            // the old window is dead afterwards, no copies.
            asm("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                "+v"(w[7]), "+v"(w[8]), "+v"(w[9]), "+v"(w[10]), "+v"(w[11]), "+v"(w[12]), "+v"(w[13]),
                "+v"(w[14]), "+v"(w[15]) : "v"(a));
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
            }
        }
        const uint32_t wi = w[i & 15];
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) | (~e & g);
        const uint32_t t1 = h + S1 + ch + kSha256K[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = maj3(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

// MD5 compression (RFC 1321 3.4) on 16 little-endian words.
__device__ __forceinline__ void md5_compress(uint32_t (&s)[4], const uint32_t (&m)[16]) {
    constexpr uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    constexpr int R[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = xor3(b, c, d); g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        const uint32_t t = a + f + K[i] + m[g];
        a = d; d = c; c = b;
        b = b + rotl(t, R[(i >> 4) * 4 + (i & 3)]);
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d;
}

// The chunk's final 1-2 blocks: bytes [0, rem) from `t`, the 0x80 terminator, zero fill and the
// 64-bit bit length (big-endian for SHA-256, little-endian for MD5).  Only aligned dwords that
// hold at least one chunk byte are read.
template <bool SHA>
__device__ __forceinline__ void tail_words(uint32_t (&m)[16], const uint8_t* t, uint32_t rem) {
    const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(t) & 3);
    // pointer arithmetic (not an integer round trip) keeps the global address space: global_load,
    // not flat_load
    const uint32_t* q = reinterpret_cast<const uint32_t*>(t - r);
    const uint32_t nd = (r + rem + 3) >> 2;
    uint32_t d[17];
#pragma unroll
    for (int j = 0; j < 17; j++) d[j] = (uint32_t)j < nd ? q[j] : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t v = __builtin_amdgcn_alignbyte(d[j + 1], d[j], r);  // little-endian bytes t[4j..4j+3]
        const int k = (int)rem - 4 * j;
        if (k <= 0) v = 0;
        else if (k < 4) v &= (1u << (8 * k)) - 1u;
        if (k >= 0 && k < 4) v |= 0x80u << (8 * k);
        m[j] = SHA ? __builtin_bswap32(v) : v;
    }
}

__device__ __forceinline__ void load_block64(uint4 (&v)[4], const uint8_t* q) {
#pragma unroll
    for (int j = 0; j < 4; j++) __builtin_memcpy(&v[j], q + 16 * j, 16);  // unaligned global_load_dwordx4
}

// The chunk's digest into its slot and, when the caller keeps a dense fingerprint table, its
// 48-byte record {digest[32], u64 buffer id, u32 start, u32 len} at rec_base[b] + k.
template <int ALGO>
__device__ __forceinline__ void store_digest(const HashArgs& a, uint32_t slot, uint32_t b, uint32_t k, uint32_t cs,
                                             uint32_t len, const uint32_t (&s)[8]) {
    constexpr bool SHA = ALGO != 2;
    uint32_t dig[8];
    if constexpr (SHA) {
#pragma unroll
        for (int j = 0; j < 8; j++) dig[j] = __builtin_bswap32(s[j]);
        if constexpr (ALGO == 1) dig[5] = dig[6] = dig[7] = 0;  // VARIABLE_SHA256_160: first 20 bytes
    } else {
        dig[0] = s[0]; dig[1] = s[1]; dig[2] = s[2]; dig[3] = s[3];
        dig[4] = dig[5] = dig[6] = dig[7] = 0;
    }
    uint4* out = reinterpret_cast<uint4*>(a.digests + (uint64_t)slot * 32);
    const uint4 d0 = make_uint4(dig[0], dig[1], dig[2], dig[3]);
    const uint4 d1 = make_uint4(dig[4], dig[5], dig[6], dig[7]);
    out[0] = d0;
    out[1] = d1;
    if (a.done_ctr) {
        // a queue pass: the digest went to the pinned image; the buffer's last chunk publishes
        // the buffer (its header was copied to the image before this kernel started).  The
        // release fence (system scope, no acquire half: nothing here reads what others wrote)
        // makes this lane's digest visible to the host before its count; the finisher's count
        // saw every other lane's fenced digest, so its ready word follows all of them.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        const uint32_t c = a.counts[b];
        if (atomicAdd(a.done_ctr + b, 1u) + 1u == c)
            __hip_atomic_store(a.ready + b, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (a.records) {
        const uint64_t r = (uint64_t)a.rec_base[b] + k;
        if (r < a.records_cap) {
            uint4* rec = reinterpret_cast<uint4*>(a.records + r * kRecordBytes);
            const uint64_t id = a.buffer_id_base + b;
            rec[0] = d0;
            rec[1] = d1;
            rec[2] = make_uint4((uint32_t)id, (uint32_t)(id >> 32), cs, len);
        }
    }
}

// ABL (sweep builds only): 1 = synthesize the message words instead of loading them, 2 = skip the
// compression (fold the loaded words instead), 4 = read from the chunk start rounded down to 128 B
// (wrong digests; every line is fetched once: the cost of the unaligned-line re-fetch).
// Production ABL = 0.
// BS = threads per workgroup; PF = load data block blk+1 while block blk is compressed.
// ABL bit 32 (LDS-DMA prefetch): the next block goes straight to LDS (global_load_lds_dwordx4,
// four per block: lane l's 16 bytes of quarter q land at q * 1024 + 16 l of its wave's 4 KiB),
// so the prefetch holds no VGPRs (90 instead of 120: five waves per SIMD instead of four).
typedef __attribute__((address_space(3))) uint8_t lds_u8;

__device__ __forceinline__ void dma_block64(lds_u8* wave_lds, const uint8_t* q) {
#pragma unroll
    for (int j = 0; j < 4; j++)
        __builtin_amdgcn_global_load_lds(q + 16 * j, (__attribute__((address_space(3))) void*)(wave_lds + 1024 * j), 16, 0,
                                         0);
}

template <int ALGO, int ABL, bool PF>
__device__ __forceinline__ void hash_task(const HashArgs& a, uint32_t i, lds_u8* wave_lds = nullptr) {
    constexpr bool SHA = ALGO != 2;
    const uint32_t slot = a.tasks[i];
    const uint32_t b = slot / a.cap;
    const uint32_t k = slot - b * a.cap;
    const uint64_t boff = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
    const uint32_t cs = a.starts[slot];
    const uint32_t len = a.clens[slot];
    const uint8_t* p = a.data + boff + cs;
    if constexpr ((ABL & 4) != 0) p = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(127));
    const uint32_t nfull = len >> 6;           // whole 64-byte data blocks
    const uint32_t nblocks = (len + 8) / 64 + 1;  // + terminator/length block(s)
    const uint64_t bits = (uint64_t)len * 8;
    uint32_t s[8];
    if constexpr (SHA) {
        s[0] = 0x6a09e667; s[1] = 0xbb67ae85; s[2] = 0x3c6ef372; s[3] = 0xa54ff53a;
        s[4] = 0x510e527f; s[5] = 0x9b05688c; s[6] = 0x1f83d9ab; s[7] = 0x5be0cd19;
    } else {
        s[0] = 0x67452301; s[1] = 0xefcdab89; s[2] = 0x98badcfe; s[3] = 0x10325476;
        s[4] = s[5] = s[6] = s[7] = 0;
    }
    // One compression per block; lanes of a wave hold chunks of near-equal block count
    // (longest-first binning), so the data/tail branch below is wave-uniform almost always.
    // ABL bit 16 (with PF): the next block's load is unconditional (the zero page past the last
    // whole block), so the loop-carried registers need no copy at the data/tail merge; with the
    // load inside the branch, hipcc copied the new block into place before the compression and
    // so waited for it there (s_waitcnt vmcnt right after issuing: no prefetch at all).
    constexpr bool kPF2 = PF && (ABL & 16);
    constexpr bool kDMA = PF && (ABL & 32);
    const uint32_t lane = threadIdx.x & 63;
    uint4 nx[4];
    if constexpr (kDMA) {
        dma_block64(wave_lds, nfull ? p : a.zero_page);
    } else if constexpr (kPF2) {
        load_block64(nx, nfull ? p : a.zero_page);
    } else if constexpr (PF) {
        if (nfull) load_block64(nx, p);  // block 0 (a chunk shorter than 64 B has none to read)
    }
    for (uint32_t blk = 0; blk < nblocks; blk++) {
        uint32_t w[16];
        uint4 pf_cur[4];
        if constexpr (kDMA) {
            __builtin_amdgcn_s_waitcnt(0);  // this block's DMA has landed
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(wave_lds + 1024 * q + 16 * lane);
                pf_cur[q] = make_uint4(v.x, v.y, v.z, v.w);
            }
            __builtin_amdgcn_s_waitcnt(0);  // read out before the next DMA overwrites it
            dma_block64(wave_lds, blk + 1 < nfull ? p + 64 * (blk + 1) : a.zero_page);
        } else if constexpr (kPF2) {
#pragma unroll
            for (int q = 0; q < 4; q++) pf_cur[q] = nx[q];
            load_block64(nx, blk + 1 < nfull ? p + 64 * (blk + 1) : a.zero_page);
        }
        if (blk < nfull) {
            uint4 cur[4];
            if constexpr (kPF2 || kDMA) {
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = pf_cur[q];
            } else if constexpr (PF) {
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                // next block, clamped to the last full one so the load stays branch-free and in bounds
                const uint32_t nb = blk + 1 < nfull ? blk + 1 : blk;
                load_block64(nx, p + 64 * nb);
            } else if constexpr (!(ABL & 1)) {
                load_block64(cur, p + 64 * blk);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint4 v;
                if constexpr (ABL & 1)
                    v = make_uint4(s[q] + blk, s[q + 4] ^ blk, s[q] * 3u, s[q + 4] + q);
                else
                    v = cur[q];
                w[4 * q] = SHA ? __builtin_bswap32(v.x) : v.x;
                w[4 * q + 1] = SHA ? __builtin_bswap32(v.y) : v.y;
                w[4 * q + 2] = SHA ? __builtin_bswap32(v.z) : v.z;
                w[4 * q + 3] = SHA ? __builtin_bswap32(v.w) : v.w;
            }
        } else {
            if (blk == nfull) {
                tail_words<SHA>(w, p + 64 * nfull, len & 63);
            } else {
#pragma unroll
                for (int j = 0; j < 16; j++) w[j] = 0;
            }
            if (blk == nblocks - 1) {
                w[14] = SHA ? (uint32_t)(bits >> 32) : (uint32_t)bits;
                w[15] = SHA ? (uint32_t)bits : (uint32_t)(bits >> 32);
            }
        }
        if constexpr (ABL & 2) {
#pragma unroll
            for (int j = 0; j < 16; j++) s[j & 7] ^= w[j];
        } else if constexpr (SHA) {
            sha256_compress<(ABL & 8) != 0>(s, w);
        } else {
            uint32_t m4[4] = {s[0], s[1], s[2], s[3]};
            md5_compress(m4, w);
            s[0] = m4[0]; s[1] = m4[1]; s[2] = m4[2]; s[3] = m4[3];
        }
    }
    if constexpr (kDMA) __builtin_amdgcn_s_waitcnt(0);  // no DMA into LDS outlives the task
    store_digest<ALGO>(a, slot, b, k, cs, len, s);
}

// PRIO: a wave whose chunks are long raises its issue priority.  A chunk's SHA-256 is a serial
// chain of ~1.4 k VALU instructions per 64-byte block (~2 us per block at full issue rate), so
// the longest chunk of a batch (up to 2049 blocks with the backup profile's 128 KiB maxLen)
// sets a floor under the kernel unless its wave is not slowed by the waves sharing its SIMD.
// WPE: minimum waves per SIMD the register allocation must allow (0 = compiler's choice).
template <int ALGO, int ABL = 0, int BS = 256, bool PF = false, bool PRIO = false, int WPE = 0>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1, 8)))
void chunk_hash_kernel(HashArgs a) {
    const uint32_t i = blockIdx.x * BS + threadIdx.x;
    if constexpr ((ABL & 64) != 0) {
        // LDS as an occupancy governor (sweep): 15 KiB per workgroup, never read.  Alone on a CU the
        // VGPRs still allow four waves per SIMD; next to a 512-thread scan workgroup (130 KiB) only
        // two of these workgroups fit, i.e. two fingerprint waves per SIMD beside two scan waves.
        __shared__ uint8_t lds_pad[15 * 1024];
        if (i == 0xFFFFFFFFu) reinterpret_cast<volatile uint8_t*>(lds_pad)[threadIdx.x] = 0;
    }
    if (i >= *a.total) return;
    if constexpr (PRIO) {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(sha_blocks(a.clens[a.tasks[i]]));
        if (nb > 1024)
            __builtin_amdgcn_s_setprio(3);
        else if (nb > 512)
            __builtin_amdgcn_s_setprio(2);
        else if (nb > 256)
            __builtin_amdgcn_s_setprio(1);
    }
    lds_u8* wave_lds = nullptr;
    if constexpr ((ABL & 32) != 0) {  // LDS only in the DMA-prefetch form
        __shared__ __attribute__((aligned(16))) uint8_t pf_lds[BS / 64 * 4096];
        wave_lds = (lds_u8*)pf_lds + 4096 * __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    }
    if constexpr ((ABL & 128) != 0) {
        // measurement (sweep variant 50): the wave's wall-clock and shader-clock span and where it
        // ran (HW_ID: wave/SIMD/CU/SE; XCC_ID), written by its first lane
        const uint64_t r0 = wall_clock64(), c0 = clock64();
        hash_task<ALGO, ABL & ~128, PF>(a, i, wave_lds);
        const uint64_t c1 = clock64(), r1 = wall_clock64();
        if ((threadIdx.x & 63) == 0 && a.stamps) {
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
            uint64_t* st = a.stamps + 8ull * (i >> 6);
            st[0] = r0;
            st[1] = c0;
            st[2] = r1;
            st[3] = c1;
            st[4] = (uint64_t)xcc << 32 | hw;
            st[5] = sha_blocks(a.clens[a.tasks[i]]);
        }
        return;
    }
    hash_task<ALGO, ABL, PF>(a, i, wave_lds);
}

// Persistent form: a fixed grid (a.persist_grid workgroups) whose waves take the next 64 tasks
// of the longest-first list from a counter until it runs dry.  A capped grid leaves register
// room on every CU for a concurrently running scan (a.wave_ctr is zeroed by the caller).
template <int ALGO, bool PF, int ABL = 0>
__global__ __launch_bounds__(256) void chunk_hash_persistent_kernel(HashArgs a) {
    const uint32_t total = *a.total;
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(a.wave_ctr, 64u);
        base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
        if (base >= total) break;
        if (base + lane < total) hash_task<ALGO, ABL, PF>(a, base + lane);
    }
}

// ------------------------------------------------------------------------------------------
// 5a. scan and fingerprint of two different batches in ONE persistent kernel (round 3)
//     The scan is latency-bound (its waves wait on the LDS-read chain half the time, VALU ~60 %
//     busy) and the fingerprint issue-bound (VALU ~75 %, waves waiting for issue slots): run on
//     the same SIMDs they fill each other's gaps, which two kernels on two streams do not do —
//     whole-CU scan workgroups and the fingerprint kernel's VGPRs keep them on separate CUs.
//     Each wave takes work items from two queues: a scan item is one whole write buffer (64
//     segments, the fused cut walk included), a fingerprint item is 64 consecutive tasks of the
//     OTHER (previous) batch's longest-first task list.  Waves 4k..4k+3 of a workgroup sit on the
//     four SIMDs; waves with bit 2 of their index clear prefer the scan queue, the others the
//     fingerprint queue, and a wave whose queue is empty takes from the other, so both kinds
//     share every SIMD until one queue runs dry.  ctr[0] / ctr[1]: zeroed item counters.
//     Uniform batches whose buffers are exactly 64 segments (the fused cut walk) only.
// ------------------------------------------------------------------------------------------
// NS: scan-first waves per SIMD (0: the k-th waves of each SIMD with k even, i.e. two of four).
// SP > 0: scan items run at issue priority SP and fingerprint items at 0 (the scan's latency-bound
// chain issues first, the fingerprint's independent VALU work fills the rest)
template <int W, int PK, class CFG, int ALGO, int NS = 0, int SP = 0>
__global__ __launch_bounds__(1024, 1) void cdc_fused_kernel(ScanArgs a, HashArgs ha, uint32_t* ctr) {
    static_assert(CFG::kFuse == 2 && CFG::kChains == 1, "fused form: one chain, register-summary cut walk");
    constexpr int C = CFG::kCopies;
    __shared__ __attribute__((aligned(16))) uint8_t tab[CFG::kLds];
    __shared__ uint32_t lhist[kMaxBins];
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.tab_image);
        uint4* dst = reinterpret_cast<uint4*>(tab);
        for (int i = threadIdx.x; i < CFG::kLds / 16; i += blockDim.x) dst[i] = src[i];
        for (uint32_t i = threadIdx.x; i < kMaxBins; i += blockDim.x) lhist[i] = 0;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c8 = (lane & (C - 1)) << 3;
    const uint32_t push_base = CFG::kPushOff | c8;
    uint32_t pa_reg = push_base, qa_reg = c8;
    const uint64_t total = a.total_segs;
    const uint32_t nscan = a.fuse_resolve ? (uint32_t)(total >> 6) : 0u;
    const uint32_t htotal = ha.total ? *ha.total : 0u;
    const bool scan_first = NS == 0 ? ((threadIdx.x >> 8) & 1) == 0 : (int)(threadIdx.x >> 8) < NS;
    bool scan_left = nscan != 0, hash_left = htotal != 0;
    while (scan_left || hash_left) {
        const bool do_scan = scan_left && (scan_first || !hash_left);
        uint32_t it = 0;
        if (lane == 0) it = atomicAdd(&ctr[do_scan ? 0 : 1], 1u);
        it = __builtin_amdgcn_readfirstlane(__shfl(it, 0));
        if (do_scan) {
            if (it >= nscan) {
                scan_left = false;
                continue;
            }
            if constexpr (SP > 0) __builtin_amdgcn_s_setprio(SP);
            scan_iter<W, PK, CFG>(a, tab, lhist, (uint64_t)it * 64, lane, 64, total, lane, c8, push_base, pa_reg, qa_reg);
            if constexpr (SP > 0) __builtin_amdgcn_s_setprio(0);
        } else {
            const uint32_t i0 = it * 64;
            if (i0 >= htotal) {
                hash_left = false;
                continue;
            }
            if constexpr (SP > 0) {
                if (i0 + lane < htotal) hash_task<ALGO, 16, true>(ha, i0 + lane);
                continue;
            }
            // issue priority for waves of long chunks, as in chunk_hash_kernel (task i0 is the
            // wave's longest: the list is longest-first)
            const uint32_t nb = __builtin_amdgcn_readfirstlane(sha_blocks(ha.clens[ha.tasks[i0]]));
            if (nb > 1024)
                __builtin_amdgcn_s_setprio(3);
            else if (nb > 512)
                __builtin_amdgcn_s_setprio(2);
            else if (nb > 256)
                __builtin_amdgcn_s_setprio(1);
            if (i0 + lane < htotal) hash_task<ALGO, 16, true>(ha, i0 + lane);
            __builtin_amdgcn_s_setprio(0);
        }
    }
    __syncthreads();
    if (nscan)
        for (uint32_t i = threadIdx.x; i < a.res.nbins; i += blockDim.x)
            if (lhist[i]) atomicAdd(&a.res.hist[i], lhist[i]);
}

// ------------------------------------------------------------------------------------------
// 5b. latency form of the fingerprint (small batches: a coalescing-queue pass costs its longest
//     chunk's serial SHA-256 chain).  A 128-thread workgroup takes 64 chunks
//     (longest first, as above); wave 0 builds each 64-byte block's message schedule W[t] + K[t]
//     into LDS one block ahead of wave 1, which runs only the 64 rounds.  A wave alone on its
//     SIMD issues one VALU instruction per ~4 cycles, so the chain's wave issues ~920 instead of
//     ~1 423 instructions per block.  Same digests as chunk_hash_kernel (SHA-256 / SHA-256/160).
// ------------------------------------------------------------------------------------------
constexpr int kSplitTasks = 64;  // chunks per workgroup (one per lane of each wave)

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t x = __shfl_xor(v, o);
        v = x > v ? x : v;
    }
    return v;
}

// One 64-chunk group of the latency form: tasks base .. base + 63 (those below ntask).  Wave 0 of
// the workgroup produces, wave 1 consumes; any further waves (the long-chunk groups of the
// throughput kernel below run in its 256-thread workgroups) only take part in the barriers.
template <int ALGO>
__device__ __forceinline__ void hash_split_group(const HashArgs& a, uint32_t base, uint32_t ntask, uint32_t wave,
                                                 uint4 (&wk)[2][16][kSplitTasks]) {
    static_assert(ALGO != 2, "MD5 has no split form");
    const uint32_t lane = threadIdx.x & 63;
    const bool producer = wave == 0, consumer = wave == 1;
    const uint32_t i = base + lane;
    uint32_t slot = 0, b = 0, k = 0, cs = 0, len = 0, nfull = 0, nblocks = 0;
    const uint8_t* p = a.zero_page;
    if (i < ntask) {
        slot = a.tasks[i];
        b = slot / a.cap;
        k = slot - b * a.cap;
        const uint64_t boff = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        cs = a.starts[slot];
        len = a.clens[slot];
        p = a.data + boff + cs;
        nfull = len >> 6;
        nblocks = (len + 8) / 64 + 1;
    }
    const uint32_t maxnb = wave_max_u32(nblocks);  // identical in every wave (same 64 tasks)
    uint32_t s[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint4 nx[4];
    if (producer) load_block64(nx, nfull ? p : a.zero_page);
    for (uint32_t it = 0; it <= maxnb; it++) {
        if (producer) {
            if (it < maxnb) {
                const uint32_t blk = it;
                uint4 cur[4];
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                load_block64(nx, blk + 1 < nfull ? p + 64 * (blk + 1) : a.zero_page);
                if (blk < nblocks) {
                    uint32_t w[16];
                    if (blk < nfull) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            w[4 * q] = __builtin_bswap32(cur[q].x);
                            w[4 * q + 1] = __builtin_bswap32(cur[q].y);
                            w[4 * q + 2] = __builtin_bswap32(cur[q].z);
                            w[4 * q + 3] = __builtin_bswap32(cur[q].w);
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
                    uint4(*dst)[kSplitTasks] = wk[blk & 1];
#pragma unroll
                    for (int g = 0; g < 16; g++) {
                        if (g >= 4 && (g & 3) == 0) {
                            // W[16g' .. 16g'+15] in place over the 16-word window
#pragma unroll
                            for (int j = 0; j < 16; j++) {
                                const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
                                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                                w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
                            }
                        }
                        const int t = 4 * g;
                        dst[g][lane] = make_uint4(w[t & 15] + kSha256K[t], w[(t + 1) & 15] + kSha256K[t + 1],
                                                  w[(t + 2) & 15] + kSha256K[t + 2], w[(t + 3) & 15] + kSha256K[t + 3]);
                    }
                }
            }
        } else if (consumer && it >= 1) {
            const uint32_t blk = it - 1;
            if (blk < nblocks) {
                const uint4(*src)[kSplitTasks] = wk[blk & 1];
                uint32_t a0 = s[0], b0 = s[1], c0 = s[2], d0 = s[3], e0 = s[4], f0 = s[5], g0 = s[6], h0 = s[7];
#pragma unroll
                for (int g = 0; g < 16; g++) {
                    const uint4 q = src[g][lane];
                    const uint32_t wkv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t S1 = xor3(rotr(e0, 6), rotr(e0, 11), rotr(e0, 25));
                        const uint32_t ch = (e0 & f0) | (~e0 & g0);
                        const uint32_t t1 = h0 + S1 + ch + wkv[r];
                        const uint32_t S0 = xor3(rotr(a0, 2), rotr(a0, 13), rotr(a0, 22));
                        const uint32_t mj = maj3(a0, b0, c0);
                        h0 = g0; g0 = f0; f0 = e0; e0 = d0 + t1; d0 = c0; c0 = b0; b0 = a0; a0 = t1 + S0 + mj;
                    }
                }
                s[0] += a0; s[1] += b0; s[2] += c0; s[3] += d0; s[4] += e0; s[5] += f0; s[6] += g0; s[7] += h0;
            }
        }
        __syncthreads();
    }
    if (consumer && i < ntask) store_digest<ALGO>(a, slot, b, k, cs, len, s);
}

template <int ALGO>
__global__ __launch_bounds__(128) void chunk_hash_split_kernel(HashArgs a) {
    __shared__ uint4 wk[2][16][kSplitTasks];  // [buffer][t / 4][lane] = W[t..t+3] + K[t..t+3]
    const uint32_t ntask = *a.total;
    if (blockIdx.x * kSplitTasks >= ntask) return;  // whole workgroup past the end (uniform)
    hash_split_group<ALGO>(a, blockIdx.x * kSplitTasks, ntask, threadIdx.x >> 6, wk);
}

// ------------------------------------------------------------------------------------------
// 5b'. packed latency form: the consumer wave runs each chunk's rounds on TWO lanes.  A lone wave
//     issues one instruction per ~5 cycles whatever the instruction, so a chunk's chain costs its
//     instruction count; the round's two halves are the same instructions on different data:
//       even lane ("A")  holds a, b, c, d      odd lane ("E")  holds e, f, g, h
//       Sigma0(a) / Sigma1(e): three v_alignbit with per-lane rotation counts + one xor3
//       Maj(a,b,c) = (a^c) ? b : c  /  Ch(e,f,g) = e ? f : g: one bit-select after one v_bitop3
//       T = Sigma + Maj/Ch + H with H = 0 on A, h + W[t] + K[t] on E:  A gets T2, E gets T1
//       a' = T1 + T2 on A, e' = d + T1 on E: ONE v_add_u32 with DPP quad_perm [1,0,3,2] on
//       Z = (E ? T : d), i.e. each lane adds its partner's Z to its own T
//     11 instructions per round instead of 14 (the single-lane round), the state rotation is
//     register renaming on both halves.  32 chunks per group: wave 0 builds W[t] + K[t] for them
//     (lanes 0..31) into the odd slots of the LDS rows, whose even slots stay zero (the A lanes'
//     W + K), wave 1 runs the rounds.  Same digests as hash_split_group.
// ------------------------------------------------------------------------------------------
constexpr int kSplitTasksPacked = 32;

// the partner lane's value: DPP quad_perm [1,0,3,2] (lanes 2k and 2k+1 exchange)
__device__ __forceinline__ uint32_t pair_swap(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);
}

// BYBUF: base = the group's first chunk index within buffer `bb`, ntask = that buffer's count,
// and the chunks are taken in slot order (no task list)
template <int ALGO, bool BYBUF = false>
__device__ __forceinline__ void hash_split_group_packed(const HashArgs& a, uint32_t base, uint32_t ntask,
                                                        uint32_t wave, uint4 (&wk)[2][16][64], uint32_t bb = 0) {
    static_assert(ALGO != 2, "MD5 has no split form");
    const uint32_t lane = threadIdx.x & 63;
    const bool producer = wave == 0, consumer = wave == 1;
    // the producer's lane k and the consumer's lanes 2k, 2k+1 hold chunk base + k
    const uint32_t k = producer ? lane : lane >> 1;
    const uint32_t i = base + k;
    const bool valid = k < (uint32_t)kSplitTasksPacked && i < ntask;
    uint32_t slot = 0, b = 0, kk = 0, cs = 0, len = 0, nfull = 0, nblocks = 0;
    const uint8_t* p = a.zero_page;
    if (valid) {
        if constexpr (BYBUF) {
            b = bb;
            kk = i;
            slot = bb * a.cap + i;
        } else {
            slot = a.tasks[i];
            b = slot / a.cap;
            kk = slot - b * a.cap;
        }
        const uint64_t boff = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        cs = a.starts[slot];
        len = a.clens[slot];
        p = a.data + boff + cs;
        nfull = len >> 6;
        nblocks = (len + 8) / 64 + 1;
    }
    const uint32_t maxnb = wave_max_u32(nblocks);  // identical in both waves (same 32 tasks)
#ifdef SDFS_TUNING
    const bool masked = a.split_masked != 0;  // A/B: the round-6 form, finished lanes masked off
#else
    constexpr bool masked = false;
#endif
    if (producer) {
        // the A lanes' W + K: zero, once for both buffers
#pragma unroll
        for (int g = 0; g < 16; g++) {
            if (lane < 32) {
                wk[0][g][2 * lane] = make_uint4(0, 0, 0, 0);
                wk[1][g][2 * lane] = make_uint4(0, 0, 0, 0);
            }
        }
    }
    // consumer lane constants: rotation counts, the Maj/Ch mask, the H mask, the E-lane mask
    const bool elane = (lane & 1) != 0;
    const uint32_t R1 = elane ? 6u : 2u, R2 = elane ? 11u : 13u, R3 = elane ? 25u : 22u;
    const uint32_t MA = elane ? 0u : ~0u;
    const uint32_t ME = ~MA;
    uint32_t x0 = elane ? 0x510e527fu : 0x6a09e667u, x1 = elane ? 0x9b05688cu : 0xbb67ae85u,
             x2 = elane ? 0x1f83d9abu : 0x3c6ef372u, x3 = elane ? 0x5be0cd19u : 0xa54ff53au;
    uint4 nx[4];
    if (producer) load_block64(nx, nfull ? p : a.zero_page);
#ifdef SDFS_TUNING
    // measurement (scripts/split_stamps.py): shader clock at start and end, the cycles this wave
    // spent in the per-block barrier, and where it ran
    const uint64_t st_c0 = clock64(), st_r0 = wall_clock64();
    uint64_t st_wait = 0, st_mid = 0;
#endif
    for (uint32_t it = 0; it <= maxnb; it++) {
        if (producer) {
            if (it < maxnb) {
                const uint32_t blk = it;
                uint4 cur[4];
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                load_block64(nx, blk + 1 < nfull ? p + 64 * (blk + 1) : a.zero_page);
                // every producer lane with a chunk slot runs the schedule (a finished or empty
                // slot on zeros: its consumer lanes discard the block), see the consumer below
                if (k < (uint32_t)kSplitTasksPacked && (!masked || (valid && blk < nblocks))) {
                    uint32_t w[16];
                    if (blk < nfull) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            w[4 * q] = __builtin_bswap32(cur[q].x);
                            w[4 * q + 1] = __builtin_bswap32(cur[q].y);
                            w[4 * q + 2] = __builtin_bswap32(cur[q].z);
                            w[4 * q + 3] = __builtin_bswap32(cur[q].w);
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
                    uint4(*dst)[64] = wk[blk & 1];
#pragma unroll
                    for (int g = 0; g < 16; g++) {
                        if (g >= 4 && (g & 3) == 0) {
#pragma unroll
                            for (int j = 0; j < 16; j++) {
                                const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
                                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                                w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
                            }
                        }
                        const int t = 4 * g;
                        dst[g][2 * lane + 1] = make_uint4(w[t & 15] + kSha256K[t], w[(t + 1) & 15] + kSha256K[t + 1],
                                                          w[(t + 2) & 15] + kSha256K[t + 2],
                                                          w[(t + 3) & 15] + kSha256K[t + 3]);
                    }
                }
            }
        } else if (consumer && it >= 1) {
            const uint32_t blk = it - 1;
            // Every lane runs every block and a lane whose chunk is done (or that has none) keeps
            // its state: a wave with lanes masked off ran its blocks up to 1.6x slower (stamps,
            // scripts/split_stamps.py), which put a pass's longest chunk on its slowest path.
            const bool act = valid && blk < nblocks;  // the same for both lanes of a chunk
            if (act || !masked) {
                const uint4(*src)[64] = wk[blk & 1];
                const uint32_t s0 = x0, s1 = x1, s2 = x2, s3 = x3;
                uint4 q = src[0][lane];
                uint32_t H = (x3 & ME) + q.x;
#pragma unroll
                for (int g = 0; g < 16; g++) {
                    const uint4 qn = g < 15 ? src[g + 1][lane] : make_uint4(0, 0, 0, 0);
                    const uint32_t wkv[5] = {q.x, q.y, q.z, q.w, qn.x};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t S = xor3(__builtin_amdgcn_alignbit(x0, x0, R1), __builtin_amdgcn_alignbit(x0, x0, R2),
                                                __builtin_amdgcn_alignbit(x0, x0, R3));
                        const uint32_t Y = __builtin_amdgcn_bitop3_b32(x0, x2, MA, 0x78);   // x0 ^ (x2 & MA)
                        const uint32_t CM = __builtin_amdgcn_bitop3_b32(Y, x1, x2, 0xCA);  // Y ? x1 : x2
                        const uint32_t T = S + CM + H;
                        const uint32_t Z = elane ? T : x3;
                        // next round's H from the next round's h (x2 now), then the partner add
                        H = (x2 & ME) + wkv[r + 1];
                        const uint32_t N = pair_swap(Z) + T;
                        x3 = x2;
                        x2 = x1;
                        x1 = x0;
                        x0 = N;
                    }
                    q = qn;
                }
                const uint32_t m = act ? ~0u : 0u;
                x0 = s0 + (x0 & m);
                x1 = s1 + (x1 & m);
                x2 = s2 + (x2 & m);
                x3 = s3 + (x3 & m);
            }
        }
#ifdef SDFS_TUNING
        const uint64_t st_b = clock64();
        __syncthreads();
        st_wait += clock64() - st_b;
        if (it == 32) st_mid = clock64();
#else
        __syncthreads();
#endif
    }
#ifdef SDFS_TUNING
    if (a.stamps && lane == 0) {
        const uint64_t c1 = clock64(), r1 = wall_clock64();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
        uint64_t* st = a.stamps + 8ull * (2 * blockIdx.x + wave);
        st[0] = st_r0;
        st[1] = st_c0;
        st[2] = r1;
        st[3] = c1;
        st[4] = (uint64_t)xcc << 32 | hw;
        st[5] = maxnb | (uint64_t)(1 + wave) << 32;
        st[6] = st_wait;
        st[7] = st_mid;
    }
#endif
    // e..h from the E lane, stored by the A lane
    const uint32_t e4 = pair_swap(x0), e5 = pair_swap(x1), e6 = pair_swap(x2), e7 = pair_swap(x3);
    if (consumer && valid && !elane) {
        const uint32_t s[8] = {x0, x1, x2, x3, e4, e5, e6, e7};
        store_digest<ALGO>(a, slot, b, kk, cs, len, s);
    }
}

template <int ALGO>
__global__ __launch_bounds__(128) void chunk_hash_split_packed_kernel(HashArgs a) {
    __shared__ uint4 wk[2][16][64];  // [buffer][t / 4][consumer lane]: odd = W[t..t+3] + K[t..t+3], even = 0
    if (a.bybuf) {
        // workgroup b * bybuf + g: chunks 32g .. 32g+31 of buffer b (all groups of a pass run at
        // once, so each buffer is done after its own longest chunk)
        const uint32_t b = blockIdx.x / a.bybuf, base = (blockIdx.x - b * a.bybuf) * kSplitTasksPacked;
        const uint32_t n = min(a.counts[b], a.cap);
        if (base >= n) return;  // uniform
        hash_split_group_packed<ALGO, true>(a, base, n, threadIdx.x >> 6, wk, b);
        return;
    }
    const uint32_t ntask = *a.total;
    if (blockIdx.x * kSplitTasksPacked >= ntask) return;  // whole workgroup past the end (uniform)
    hash_split_group_packed<ALGO>(a, blockIdx.x * kSplitTasksPacked, ntask, threadIdx.x >> 6, wk);
}

// ------------------------------------------------------------------------------------------
// 5c. throughput form with the longest chunks in the latency form (backup profile: maxLen
//     128 KiB).  A chunk's SHA-256 is one serial chain, so a batch's longest chunk sets a floor
//     under chunk_hash_kernel (a 55 KB chunk: 869 blocks x ~2.8 us with the GPU otherwise idle at
//     the end, 3.50 vs 3.03 ms per 4 GiB with every chunk clipped to 32 KiB,
//     scripts/backup_tail_probe.py).  Tasks 0 .. *nlong-1 (the chunks of more than kLongBlocks
//     blocks, at the head of the longest-first list) go to the first workgroups in producer/
//     consumer groups: PACKED (production) the two-lane form of section 5b' (32 chunks per group,
//     ~710 instructions per block on the chain), else the one-lane form of 5b (64 chunks, ~905);
//     the rest run one lane per chunk as in chunk_hash_kernel.
// ------------------------------------------------------------------------------------------
template <int ALGO, bool PACKED = true>
__global__ __launch_bounds__(256) void chunk_hash_long_kernel(HashArgs a) {
    __shared__ uint4 wk[2][16][64];
    constexpr uint32_t G = PACKED ? kSplitTasksPacked : kSplitTasks;
    uint32_t nl = __builtin_amdgcn_readfirstlane(*a.nlong);
    if (nl > kLongSplitMax) nl = 0;
    const uint32_t lg = (nl + G - 1) / G;  // long-chunk workgroups
    if (blockIdx.x < lg) {
        if constexpr (PACKED)
            hash_split_group_packed<ALGO>(a, blockIdx.x * G, nl, threadIdx.x >> 6, wk);
        else
            hash_split_group<ALGO>(a, blockIdx.x * G, nl, threadIdx.x >> 6, wk);
        return;
    }
    const uint32_t i = nl + (blockIdx.x - lg) * 256 + threadIdx.x;
    if (i >= *a.total) return;
    const uint32_t nb = __builtin_amdgcn_readfirstlane(sha_blocks(a.clens[a.tasks[i]]));
    if (nb > 256) __builtin_amdgcn_s_setprio(1);
    hash_task<ALGO, 16, true>(a, i);
}

}  // namespace sdfs
