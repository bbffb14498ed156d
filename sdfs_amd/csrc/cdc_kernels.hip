// cdc_kernels.hip — hand-written CDNA4 (gfx950) kernels for SDFS variable-block CDC + fingerprint.
//
// Pipeline per batch of write buffers (DESIGN.md "Kernels"):
//   1. cdc_scan     windowed Rabin rolling hash over every byte -> candidate bitmap (1 bit/byte)
//   2. cdc_resolve  greedy cut resolution per buffer (min/max rules) -> (start,len) slots;
//                   long buffers: LDS-staged walk, very long ones: speculative sections + stitch
//   3. cdc_prefix   bin cursors (longest-first) + per-buffer record bases + total
//   4. cdc_scatter  chunk slots -> task list sorted by SHA block count (load balance)
//   5. chunk_hash   one lane per chunk: SHA-256 / MD5 over the chunk bytes -> digests, records
//
// Reference semantics: VariableSha256HashEngine.getChunks (VariableSha256HashEngine.java:71-86)
// driving the rabinwindow EnhancedFingerFactory loop; getHash (:58-67).
// Integer/bit work only: no MFMA (DESIGN.md explains the VALU roofline).
// This file holds the production configurations only; measured alternatives live in
// cdc_sweep.hip, which is built into the measurement library (make tuning) and never into
// libsdfs_cdc.so.
#include <algorithm>

#include "cdc_device.h"

namespace sdfs {

// Production scan configuration: 32 conflict-free lane-private table copies (128 KiB of LDS,
// one 1024-thread workgroup per CU), one 4 KiB segment per lane, 256-byte blocks (two whole
// 128-byte lines per lane per iteration, so no line is fetched twice), the split fast-path
// body (ABL bit 16) and the cut walk fused into the epilogue from register summaries (FUSE 2).
// Bit-reversed (mirrored) rolling state (cdc_device.h roll_step): a low-k-bit zero predicate is
// one compare, and each position's compare lands in an SGPR pair of its own so that only
// 8-position groups with a candidate pay for shifting their bits in (kAblSgprPred): ~8.6 instead
// of 10.1 VALU per byte.  Interleaved A/B on MI355X against the alternatives is in DESIGN.md
// §7-8 (sweep variants 29 = plain state, 30 = mirrored without the SGPR masks).
// Since round 3 both LDS addresses are single SDWA instructions writing byte 1 of a register that
// keeps the table base and lane offset in its other bytes (kAblSdwa, kAblSdwaPop): the push
// address one v_lshrrev_b32_sdwa instead of v_lshrrev + v_bitop3 (one VALU less per byte and
// one dependent instruction less in the rolling chain), the pop address one v_mov_b32_sdwa
// instead of v_perm.  Interleaved A/B, identical records: 1.368 -> 1.245 ms per 4 GiB at the
// 4 KiB-mean mix, 1.282 -> 1.162 at the reference default (sweep variant 32 = the form before).
// Also since round 3: the candidate bits of the one-compare predicate come from each 8-position
// group's minimum predicate word (kAblMinGroup8: three v_min3 + one v_min + one compare per group,
// exact bits only in groups where some lane has a candidate) instead of a per-position compare
// into an SGPR pair and a scalar OR chain, and the pop entries are stored high word first
// (kAblPopSwap) so the low-word xor3 never reads three registers of one bank.  Interleaved A/B,
// identical records: 1.258 -> 1.235 ms (4 KiB-mean mix), 1.157 -> 1.134 (default), sweep
// variant 51 = this form, 44 = the SDWA form before it.
using ScanProd = ScanCfg<32, 1, false, 4, 16 | kAblSdwa | kAblSdwaPop | kAblMinGroup | kAblMinGroup8 | kAblPopSwap, 256,
                         2, kScanThreads, true>;

// Tiny batches (a lone queue pass: a few 256 KiB buffers, segments shorter than ScanProd's
// 256-byte block): the same byte loop over 64-byte blocks and no fused walk (the separate
// small-batch walk resolves them).  A lane alone on its SIMD waits out the LDS round trip of every
// byte, so a lone buffer's scan time is its lanes' chain length: 64-byte segments (+ the 48-byte
// window warm-up) instead of 256 (ScanProd with a short segment still scans its whole block).
using ScanTiny = ScanCfg<32, 1, false, 4, 16 | kAblSdwa | kAblSdwaPop | kAblMinGroup | kAblMinGroup8 | kAblPopSwap, 64,
                         0, kScanThreads, true>;

template <class CFG>
constexpr ScanVariantInfo info_of() {
    return {CFG::kCopies, CFG::kChains, CFG::kLds, std::max(1, CFG::kWavesPerSimd * 256 / CFG::kThreads), CFG::kBlk,
            CFG::kFuse, CFG::kThreads, CFG::kMirror, CFG::kPopSwap};
}

ScanVariantInfo scan_variant_info(int v) {
    if (v == 0) return info_of<ScanProd>();
#ifdef SDFS_TUNING
    return scan_variant_info_sweep(v);
#else
    return {0, 0, 0, 0, 0, 0, 0};
#endif
}

bool scan_window_supported(int window) {
    return window == 16 || window == 32 || window == 48 || window == 64;
}

template <int W, class CFG>
static hipError_t launch_scan_wc(const ScanArgs& a, int pk, int grid, int block, hipStream_t s) {
    static_assert(CFG::kMirror, "the production scan rolls the mirrored state");
    if (pk == 1)
        hipLaunchKernelGGL((cdc_scan_kernel<W, 1, CFG>), dim3(grid), dim3(block), 0, s, a);
    else if (pk == 2)
        hipLaunchKernelGGL((cdc_scan_kernel<W, 2, CFG>), dim3(grid), dim3(block), 0, s, a);
    else if (pk == 3)
        hipLaunchKernelGGL((cdc_scan_kernel<W, 3, CFG>), dim3(grid), dim3(block), 0, s, a);
    else
        hipLaunchKernelGGL((cdc_scan_kernel<W, 0, CFG>), dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_scan(const ScanArgs& a, int window, int pk, int variant, int grid, int block, hipStream_t s) {
    if (variant != 0) {
#ifdef SDFS_TUNING
        return launch_scan_sweep(a, window, pk, variant, grid, block, s);
#else
        return hipErrorInvalidValue;
#endif
    }
    switch (window) {
    case 16: return launch_scan_wc<16, ScanProd>(a, pk, grid, block, s);
    case 32: return launch_scan_wc<32, ScanProd>(a, pk, grid, block, s);
    case 48: return launch_scan_wc<48, ScanProd>(a, pk, grid, block, s);
    case 64: return launch_scan_wc<64, ScanProd>(a, pk, grid, block, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scan_tiny(const ScanArgs& a, int window, int pk, int grid, int block, hipStream_t s) {
    if (a.fuse_resolve) return hipErrorInvalidValue;  // the tiny form has no fused walk
    switch (window) {
    case 16: return launch_scan_wc<16, ScanTiny>(a, pk, grid, block, s);
    case 32: return launch_scan_wc<32, ScanTiny>(a, pk, grid, block, s);
    case 48: return launch_scan_wc<48, ScanTiny>(a, pk, grid, block, s);
    case 64: return launch_scan_wc<64, ScanTiny>(a, pk, grid, block, s);
    default: return hipErrorInvalidValue;
    }
}

// segment prefix for the general (ragged) layout: seg_prefix[b] = sum_{b'<b} ceil(len/seg_len)
__global__ __launch_bounds__(1024) void seg_prefix_kernel(const uint32_t* lens, uint32_t nbuf, uint32_t seg_len,
                                                          uint64_t* seg_prefix) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nbuf + 1023) / 1024;
    const uint32_t b0 = t * per, b1 = (b0 + per < nbuf) ? b0 + per : nbuf;
    uint64_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += (lens[b] + seg_len - 1) / seg_len;
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t b = b0; b < b1; b++) {
        seg_prefix[b] = run;
        run += (lens[b] + seg_len - 1) / seg_len;
    }
    if (t == 1023) seg_prefix[nbuf] = part[1023];
}

hipError_t launch_seg_prefix(const uint32_t* lens, uint32_t nbuf, uint32_t seg_len, uint64_t* seg_prefix,
                             hipStream_t s) {
    hipLaunchKernelGGL(seg_prefix_kernel, dim3(1), dim3(1024), 0, s, lens, nbuf, seg_len, seg_prefix);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// 2. cut resolution: one wave per buffer, ballot search over 64 bitmap words (2048 positions)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cdc_resolve_kernel(ResolveArgs a) {
    __shared__ uint32_t lhist[kMaxBins];
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256) lhist[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < a.nbuf; b += nw) resolve_buffer(a, b, lane, lhist);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256)
        if (lhist[i]) atomicAdd(&a.hist[i], lhist[i]);
}

// LDS-staged cut walk for long buffers (the BACKUP_VOLUME profile's 40 MiB write buffers).
// One 256-thread workgroup per buffer.  Window n holds bitmap words [n*kResStride,
// n*kResStride + 2*kResStride) of the buffer in one of two LDS slots; wave 0 walks the cuts of
// window n from LDS (each lane tests 8 consecutive words, so one ballot covers 16 Ki positions:
// about one iteration per chunk at a 4 KiB candidate spacing) while waves 1-3 stage window n+1
// into the other slot.  The walk leaves window n at the first chunk whose search range ends past
// it; with kResStride > max_len/32 + 1 words that range lies inside window n+1 (its start is at
// least max_len before its end, its end at most max_len past window n's end), so the window
// schedule is fixed and the staging never waits on the walk.
constexpr uint32_t kResStride = 6144;          // words (196 608 positions)
constexpr uint32_t kResWin = 2 * kResStride;   // words per window (48 KiB of LDS)
constexpr uint32_t kResStage = kResWin / 2 / 192;  // uint2 loads per staging thread (waves 1-3)

__device__ __forceinline__ int64_t find_first_lds(const uint32_t* win, uint32_t wbase, uint32_t lo_w, uint32_t lo_b,
                                                  uint32_t hi_w, uint32_t hi_b, uint32_t lane) {
    // words are buffer-relative; win[w - wbase]
    for (uint32_t wb = lo_w; wb <= hi_w; wb += 512) {
        const uint32_t w0 = wb + 8 * lane;
        uint32_t bits[8];
        uint32_t any = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t w = w0 + j;
            uint32_t v = 0;
            if (w <= hi_w) {
                v = win[w - wbase];
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

__device__ __forceinline__ void stage_window(uint32_t* slot, const uint32_t* bm, uint64_t word0, uint64_t wbase,
                                             uint64_t nwords, uint32_t t, uint32_t nthreads_div) {
    // thread t of the staging group loads kResWin/2/nthreads_div uint2 (all issued before any store)
    const uint2* src = reinterpret_cast<const uint2*>(bm + word0 + wbase);
    uint2* dst = reinterpret_cast<uint2*>(slot);
    const uint64_t avail = nwords > wbase ? nwords - wbase : 0;
    uint2 v[kResStage];
#pragma unroll
    for (uint32_t k = 0; k < kResStage; k++) {
        const uint32_t i = t + k * nthreads_div;
        v[k] = 2ull * i < avail ? src[i] : make_uint2(0, 0);
    }
#pragma unroll
    for (uint32_t k = 0; k < kResStage; k++) dst[t + k * nthreads_div] = v[k];
}

// SPEC = false: item = buffer, the walk covers the whole buffer and writes the final chunk slots.
// SPEC = true: item = (buffer, section); the walk starts a chunk at the section start, runs until
// the next chunk start reaches the section end and records the starts for the stitch pass.
template <bool SPEC>
__global__ __launch_bounds__(256) void cdc_resolve_lds_kernel(ResolveArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t win[2][kResWin];
    __shared__ uint32_t lhist[SPEC ? 1 : kMaxBins];
    __shared__ uint32_t s_done[2];  // by window parity: the walker may write window n+1's flag
                                    // before every thread has read window n's
    if constexpr (!SPEC)
        for (uint32_t i = threadIdx.x; i < a.nbins; i += 256) lhist[i] = 0;
    const uint32_t lane = threadIdx.x & 63;
    const bool walker = threadIdx.x < 64;
    const uint32_t nitems = SPEC ? a.nbuf * a.nsec : a.nbuf;
    for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
        const uint32_t b = SPEC ? item / a.nsec : item;
        const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint32_t r0 = SPEC ? (item - b * a.nsec) * a.sec_len : 0;
        if (r0 >= len) {  // workgroup-uniform: section past this buffer's end (or an empty buffer)
            if (threadIdx.x == 0) {
                if constexpr (SPEC) {
                    a.spec_cnt[item] = 0;
                    a.spec_next[item] = len;
                } else {
                    a.counts[b] = 0;
                }
            }
            continue;
        }
        const uint32_t r1 = SPEC ? min(r0 + a.sec_len, len) : len;
        const uint64_t word0 = off >> 5;  // even: buffers start 64-byte aligned
        const uint64_t nwords = ((uint64_t)len + 31) >> 5;
        const uint32_t wb0 = (r0 >> 5) & ~1u;
        uint32_t start = r0;  // walker state (wave 0 registers)
        uint32_t cnt = 0;
        __syncthreads();  // the previous item's walk is done with both slots
        if (threadIdx.x >= 64) stage_window(win[0], a.bitmap, word0, wb0, nwords, threadIdx.x - 64, 192);
        __syncthreads();
        for (uint32_t n = 0;; n++) {
            const uint32_t wbase = wb0 + n * kResStride;
            if (!walker) {
                stage_window(win[(n + 1) & 1], a.bitmap, word0, (uint64_t)wbase + kResStride, nwords,
                             threadIdx.x - 64, 192);
            } else {
                const uint32_t* w = win[n & 1];
                const uint64_t wend = (uint64_t)wbase + kResWin;  // first word past the window
                while (start < r1) {
                    const uint32_t lo = start + a.first_off;
                    const uint32_t forced = start + a.max_len - 1;
                    const uint32_t hi = forced < len - 1 ? forced : len - 1;
                    if (lo <= hi && (uint64_t)(hi >> 5) >= wend) break;  // continues in window n+1
                    int64_t k = -1;
                    if (lo <= hi) k = find_first_lds(w, wbase, lo >> 5, lo & 31, hi >> 5, hi & 31, lane);
                    if (k < 0) k = (int64_t)hi;
                    if constexpr (SPEC) {
                        if (lane == 0 && cnt < a.spec_cap) a.spec_starts[(uint64_t)item * a.spec_cap + cnt] = start;
                    } else {
                        const uint32_t clen = (uint32_t)k + 1 - start;
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
                    }
                    cnt++;
                    start = (uint32_t)k + 1;
                }
                if (lane == 0) {
                    s_done[n & 1] = start >= r1;
                    if (start >= r1) {
                        if constexpr (SPEC) {
                            a.spec_cnt[item] = cnt < a.spec_cap ? cnt : a.spec_cap;
                            a.spec_next[item] = start;
                            if (cnt > a.spec_cap) atomicOr(a.overflow, 2u);  // engine bug guard
                        } else {
                            a.counts[b] = cnt < a.cap ? cnt : a.cap;
                        }
                    }
                }
            }
            __syncthreads();  // window n+1 staged, walk of window n finished
            if (s_done[n & 1]) break;
        }
    }
    if constexpr (!SPEC) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < a.nbins; i += 256)
            if (lhist[i]) atomicAdd(&a.hist[i], lhist[i]);
    }
}

// Small batches (a coalescing-queue pass: a few CHUNK_LENGTH buffers): one workgroup per buffer
// copies the buffer's whole candidate bitmap into LDS with every thread at once (8 KiB words for
// 256 KiB, one round of 8-byte loads).  The global walk of cdc_resolve_kernel pays one dependent
// bitmap load per cut (~0.7 us: ~45 us for a 256 KiB buffer at the 4 KiB mix), and a lone pass's
// latency is what a synchronous getChunks caller waits for.  From LDS:
//   1. the candidates in one ascending list (per-thread popcounts, a block prefix, each thread
//      writes its words' positions) — up to kSmallListCap of them, else step 3 alone;
//   2. every candidate's successor, in parallel: the first candidate at or past its position + 1 +
//      first_off (binary search of the list), i.e. the cut the greedy walk takes next when no
//      forced cut intervenes;
//   3. wave 0 follows the successors (one LDS read per cut); a forced cut (max_len) or the tail
//      starts the chain again from a binary search.  A buffer with more candidates than the list
//      holds (zero runs: every position a candidate) is walked by 64-word ballots instead.
// The cuts are the greedy loop's exactly: each one is the first candidate in
// [start + first_off, start + max_len - 1], else the forced/tail position.
constexpr uint32_t kSmallWalkWords = 16384;  // buffers up to 512 KiB
constexpr uint32_t kSmallWalkMaxBufs = 1024;  // beyond: the global walk, several buffers per wave
constexpr uint32_t kSmallListCap = 2048;      // candidates of one buffer in the list form

// first index i in list[0, n) with list[i].x >= target (n if none)
__device__ __forceinline__ uint32_t list_lower_bound(const uint2* list, uint32_t n, uint32_t target) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (list[mid].x < target)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void cdc_resolve_small_kernel(ResolveArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t win[kSmallWalkWords];
    __shared__ uint2 list[kSmallListCap];  // {position, index of its successor}
    __shared__ uint32_t lhist[kMaxBins];
    __shared__ uint32_t scan[256];
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256) lhist[i] = 0;
    const uint32_t b = blockIdx.x;
    const uint32_t t = threadIdx.x;
    const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
    const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
    const uint32_t nwords = (len + 31) >> 5;
    {
        // bitmap words [off/32, off/32 + nwords): buffers start 64-byte aligned, so the first word
        // is 8-byte aligned; uint2 loads, all issued before any store
        const uint2* src = reinterpret_cast<const uint2*>(a.bitmap + (off >> 5));
        uint2* dst = reinterpret_cast<uint2*>(win);
        const uint32_t n2 = (nwords + 1) >> 1;
        constexpr uint32_t kPer = kSmallWalkWords / 2 / 256;
        uint2 v[kPer];
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = t + k * 256;
            v[k] = i < n2 ? src[i] : make_uint2(0, 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; k++) {
            const uint32_t i = t + k * 256;
            if (i < n2) dst[i] = v[k];
        }
    }
    __syncthreads();
    // 1. the candidate list: thread t owns words [w0, w1); positions past len are not candidates
    const uint32_t per = (nwords + 255) / 256;
    const uint32_t w0 = min(t * per, nwords), w1 = min(w0 + per, nwords);
    const uint32_t tail_mask = (len & 31) ? (1u << (len & 31)) - 1u : ~0u;
    uint32_t mine = 0;
    for (uint32_t w = w0; w < w1; w++) mine += __builtin_popcount(w + 1 == nwords ? win[w] & tail_mask : win[w]);
    scan[t] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? scan[t - o] : 0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const uint32_t total = scan[255];
    const bool listed = total <= kSmallListCap && !a.small_ballot;
    if (listed) {
        uint32_t at = scan[t] - mine;
        for (uint32_t w = w0; w < w1; w++) {
            uint32_t bits = w + 1 == nwords ? win[w] & tail_mask : win[w];
            while (bits) {
                list[at++].x = w * 32 + __builtin_ctz(bits);
                bits &= bits - 1;
            }
        }
    }
    __syncthreads();
    // 2. successors
    if (listed)
        for (uint32_t i = t; i < total; i += 256) list[i].y = list_lower_bound(list, total, list[i].x + 1 + a.first_off);
    __syncthreads();
    if (t < 64) {
        const uint32_t lane = t;
        uint32_t start = 0, cnt = 0, my_s = 0, my_e = 0;
        uint32_t j = listed ? list_lower_bound(list, total, a.first_off) : 0;  // first candidate >= lo
        while (start < len) {
            const uint32_t lo = start + a.first_off;
            const uint32_t forced = start + a.max_len - 1;
            const uint32_t hi = forced < len - 1 ? forced : len - 1;
            int64_t k = -1;
            if (listed) {
                // list[j] is the first candidate >= lo: a cut when it is <= hi.  Position and
                // successor in one ds_read_b64, issued before the tests (read separately, the
                // successor costs a second LDS round trip per cut)
                const uint2 e = list[j < kSmallListCap ? j : kSmallListCap - 1];
                if (lo <= hi && j < total) {
                    if (e.x <= hi) {
                        k = e.x;
                        j = e.y;  // the successor: first candidate >= k + 1 + first_off
                    }
                }
            } else if (lo <= hi) {
                // first candidate in [lo, hi]: 64 words (2048 positions) per ballot
                const uint32_t wlo = lo >> 5, whi = hi >> 5;
                for (uint32_t wb = wlo; wb <= whi; wb += 64) {
                    const uint32_t w = wb + lane;
                    uint32_t bits = 0;
                    if (w <= whi) {
                        bits = win[w];
                        if (w == wlo) bits &= ~0u << (lo & 31);
                        if (w == whi) bits &= (hi & 31) == 31 ? ~0u : ((2u << (hi & 31)) - 1u);
                    }
                    const uint64_t m = __ballot(bits != 0);
                    if (m) {
                        // the lane index is wave-uniform: v_readlane, not an LDS round trip
                        const uint32_t l = __builtin_ctzll(m);
                        const uint32_t bb = __builtin_amdgcn_readlane(bits, l);
                        k = (int64_t)(wb + l) * 32 + __builtin_ctz(bb);
                        break;
                    }
                }
            }
            const bool at_candidate = k >= 0;
            if (k < 0) k = (int64_t)hi;  // forced cut at max_len, or the tail chunk
            // lane (cnt & 63) keeps this cut; every 64 cuts (and at the end) the wave records them
            // together, so the serial loop carries no global stores or histogram atomics
            const uint32_t held = cnt & 63;
            my_s = lane == held ? start : my_s;
            my_e = lane == held ? (uint32_t)k : my_e;
            cnt++;
            start = (uint32_t)k + 1;
            if (held == 63 || start >= len) {
                const uint32_t idx = cnt - 1 - held + lane;
                if (lane <= held) {
                    if (idx < a.cap) {
                        const uint64_t slot = (uint64_t)b * a.cap + idx;
                        const uint32_t clen = my_e + 1 - my_s;
                        a.starts[slot] = my_s;
                        a.clens[slot] = clen;
                        uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                        bin = bin < a.nbins ? bin : a.nbins - 1;
                        atomicAdd(&lhist[bin], 1u);
                    } else {
                        atomicOr(a.overflow, 1u);
                    }
                }
            }
            // a chain through a non-candidate cut restarts from a search
            if (listed && !at_candidate && start < len) j = list_lower_bound(list, total, start + a.first_off);
        }
        if (lane == 0) a.counts[b] = cnt < a.cap ? cnt : a.cap;
    }
    __syncthreads();
    for (uint32_t i = t; i < a.nbins; i += 256)
        if (lhist[i]) atomicAdd(&a.hist[i], lhist[i]);
}

// Speculative walk, one wave per (buffer, section): a chunk starts at the section start; record
// chunk starts until the next start reaches the section end.
__global__ __launch_bounds__(256) void cdc_resolve_spec_kernel(ResolveArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nitems = a.nbuf * a.nsec;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t item = blockIdx.x * 4 + (threadIdx.x >> 6); item < nitems; item += nw) {
        const uint32_t b = item / a.nsec;
        const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint32_t r0 = (item - b * a.nsec) * a.sec_len;
        if (r0 >= len) {
            if (lane == 0) {
                a.spec_cnt[item] = 0;
                a.spec_next[item] = len;
            }
            continue;
        }
        const uint32_t r1 = min(r0 + a.sec_len, len);
        const uint64_t word0 = off >> 5;
        uint32_t start = r0, cnt = 0;
        uint32_t* sp = a.spec_starts + (uint64_t)item * a.spec_cap;
        while (start < r1) {
            const uint32_t lo = start + a.first_off;
            const uint32_t forced = start + a.max_len - 1;
            const uint32_t hi = forced < len - 1 ? forced : len - 1;
            int64_t k = -1;
            if (lo <= hi) k = find_first_wide(a.bitmap, word0, lo, hi, lane);
            if (k < 0) k = (int64_t)hi;
            if (lane == 0 && cnt < a.spec_cap) sp[cnt] = start;
            cnt++;
            start = (uint32_t)k + 1;
        }
        if (lane == 0) {
            a.spec_cnt[item] = cnt < a.spec_cap ? cnt : a.spec_cap;
            a.spec_next[item] = start;
            if (cnt > a.spec_cap) atomicOr(a.overflow, 2u);  // capacity is sized so this cannot happen
        }
    }
}

// Parallel stitch, step 1 (join): one wave per (buffer, section j >= 1).  The true chain enters
// section j at spec_next[j - 1], the first start the chain of section j - 1 reaches past its end
// (that chain is the true one once section j - 1 has joined, by induction from section 0, whose
// speculative walk starts where the buffer does).  From there the wave takes true steps until it
// lands on one of section j's speculative starts — from that start on the two chains are one.
// join[item] = {index of that start (cnt when the true chain only passes through, or
// kJoinUnmerged: more than kJoinExtra steps, or it leaves the section elsewhere than
// spec_next[j]), number of extra true starts, the extra starts}.  On random data the chains meet
// within a chunk or two; a buffer with any unmerged section is left to the sequential stitch.
constexpr uint32_t kJoinUnmerged = 0xFFFFFFFFu;

__global__ __launch_bounds__(256) void cdc_resolve_join_kernel(ResolveArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nitems = a.nbuf * a.nsec;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t item = blockIdx.x * 4 + (threadIdx.x >> 6); item < nitems; item += nw) {
        const uint32_t b = item / a.nsec, j = item - b * a.nsec;
        const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint32_t r0 = j * a.sec_len;
        uint32_t* jo = a.join + (uint64_t)item * kJoinWords;
        uint32_t m = 0, nx = 0;
        const uint64_t word0 = off >> 5;
        // one true step from chunk start p (the next chunk's start)
        auto step = [&](uint32_t p) -> uint32_t {
            const uint32_t lo = p + a.first_off;
            const uint32_t forced = p + a.max_len - 1;
            const uint32_t hi = forced < len - 1 ? forced : len - 1;
            int64_t k = -1;
            if (lo <= hi) k = a.seg_sum ? find_first_sum(a, b, lo, hi, lane) : find_first_wide(a.bitmap, word0, lo, hi, lane);
            if (k < 0) k = (int64_t)hi;
            return (uint32_t)k + 1;
        };
        // the scan's piece walk left every section's last chunk open: close this section's
        // (spec_next) and recompute the previous section's from its last start — the same value
        // that section's own wave writes, so no ordering between the waves is needed
        uint32_t own_next = 0, prev_next = 0;
        if (a.spec_from_scan) {
            const uint32_t cm = a.spec_cnt[item];
            own_next = r0 >= len || cm == 0 ? len : step(a.spec_starts[(uint64_t)item * a.spec_cap + cm - 1]);
            if (lane == 0) a.spec_next[item] = own_next;
            if (j > 0 && r0 < len) {
                const uint32_t cp = a.spec_cnt[item - 1];
                prev_next = cp == 0 ? len : step(a.spec_starts[(uint64_t)(item - 1) * a.spec_cap + cp - 1]);
            }
        }
        if (j > 0 && r0 < len) {
            const uint32_t r1 = min(r0 + a.sec_len, len);
            const uint32_t cm = a.spec_cnt[item];
            const uint32_t* sp = a.spec_starts + (uint64_t)item * a.spec_cap;
            const uint32_t snext = a.spec_from_scan ? own_next : a.spec_next[item];
            uint32_t p = a.spec_from_scan ? prev_next : a.spec_next[item - 1];
            if (p >= len) {
                m = cm;  // the chain ended before this section: none of its speculative starts is a cut
            } else {
                for (;;) {
                    if (p >= r1) {  // passed through without meeting: fine if it leaves where they do
                        m = p == snext ? cm : kJoinUnmerged;
                        break;
                    }
                    int32_t found = -1;
                    for (uint32_t j0 = 0; j0 < cm; j0 += 64) {
                        const uint32_t e = j0 + lane < cm ? sp[j0 + lane] : 0xFFFFFFFFu;
                        const uint64_t hit = __ballot(e == p);
                        if (hit) {
                            found = (int32_t)(j0 + __builtin_ctzll(hit));
                            break;
                        }
                        if (__ballot(e > p)) break;  // sorted: p is not a speculative start
                    }
                    if (found >= 0) {
                        m = (uint32_t)found;
                        break;
                    }
                    if (nx == kJoinExtra) {
                        m = kJoinUnmerged;
                        break;
                    }
                    if (lane == 0) jo[2 + nx] = p;
                    nx++;
                    p = step(p);
                }
            }
        }
        if (lane == 0) {
            jo[0] = m;
            jo[1] = nx;
        }
    }
}

// Parallel stitch, step 2 (place): one wave per (buffer, section) of a buffer whose sections all
// joined: the section's chunks are its extra true starts, then its speculative starts from the
// joining one on, each ending where the next begins (the last at spec_next: the section's chain is
// the true one).  The slot offset is the sum of the earlier sections' chunk counts.
__global__ __launch_bounds__(256) void cdc_resolve_place_kernel(ResolveArgs a) {
    __shared__ uint32_t lhist[kMaxBins];
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256) lhist[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nitems = a.nbuf * a.nsec;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t item = blockIdx.x * 4 + (threadIdx.x >> 6); item < nitems; item += nw) {
        const uint32_t b = item / a.nsec, j = item - b * a.nsec;
        const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint32_t nsb = (len + a.sec_len - 1) / a.sec_len;  // sections of this buffer
        if (j >= nsb) {
            // an empty buffer (nsb = 0) has no section of its own: its first item settles it here,
            // so the stitch kernel skips it and no stale flag or count of an earlier batch survives
            if (nsb == 0 && j == 0 && lane == 0) {
                a.join_bad[b] = 0u;
                a.counts[b] = 0u;
            }
            continue;
        }
        const uint32_t* jb = a.join + (uint64_t)b * a.nsec * kJoinWords;
        const uint32_t* cb = a.spec_cnt + (uint64_t)b * a.nsec;
        // every section joined?  chunks before this section, and in the whole buffer
        bool bad = false;
        uint32_t before = 0, all = 0;
        for (uint32_t s0 = 0; s0 < nsb; s0 += 64) {
            const uint32_t sj = s0 + lane;
            uint32_t n = 0;
            if (sj < nsb) {
                const uint32_t mj = jb[(uint64_t)sj * kJoinWords];
                if (mj == kJoinUnmerged) bad = true;
                else n = jb[(uint64_t)sj * kJoinWords + 1] + cb[sj] - mj;
            }
            if (__ballot(bad)) {
                bad = true;
                break;
            }
            uint32_t nb = sj < j ? n : 0;
            for (int o = 32; o >= 1; o >>= 1) {
                nb += __shfl_xor(nb, o);
                n += __shfl_xor(n, o);
            }
            before += nb;
            all += n;
        }
        if (bad) {
            if (j == 0 && lane == 0) a.join_bad[b] = 1u;
            continue;
        }
        if (j == 0 && lane == 0) {
            a.join_bad[b] = 0u;
            a.counts[b] = all < a.cap ? all : a.cap;
            if (all > a.cap) atomicOr(a.overflow, 1u);
        }
        const uint32_t* jo = jb + (uint64_t)j * kJoinWords;
        const uint32_t m = jo[0], nx = jo[1], cm = cb[j];
        const uint32_t* sp = a.spec_starts + (uint64_t)item * a.spec_cap;
        const uint32_t n = nx + cm - m;
        const uint32_t nxt = a.spec_next[item];
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t st = i < nx ? jo[2 + i] : sp[m + i - nx];
            const uint32_t en = i + 1 < nx ? jo[3 + i] : (i + 1 < n ? sp[m + i + 1 - nx] : nxt);
            const uint32_t c = before + i;
            if (c < a.cap) {
                const uint64_t slot = (uint64_t)b * a.cap + c;
                a.starts[slot] = st;
                a.clens[slot] = en - st;
                uint32_t bin = sha_blocks(en - st) >> a.bin_shift;
                bin = bin < a.nbins ? bin : a.nbins - 1;
                atomicAdd(&lhist[bin], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256)
        if (lhist[i]) atomicAdd(&a.hist[i], lhist[i]);
}

// Stitch: one wave per buffer follows the true cut chain.  Where it lands on a section's
// speculative chunk start the two chains coincide from there on (same greedy rule, same bits),
// so the rest of that section's list is copied wave-parallel; otherwise it takes one true step
// (bitmap search) and tries again.  On random data the chains meet within a chunk or two.
__global__ __launch_bounds__(256) void cdc_resolve_stitch_kernel(ResolveArgs a) {
    __shared__ uint32_t lhist[kMaxBins];
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256) lhist[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6); b < a.nbuf; b += nw) {
        if (a.join_bad && !a.join_bad[b]) continue;  // placed by cdc_resolve_place_kernel
        const uint64_t off = a.uniform_len ? (uint64_t)b * a.uniform_len : a.offs[b];
        const uint32_t len = a.uniform_len ? a.uniform_len : a.lens[b];
        const uint64_t word0 = off >> 5;
        uint32_t p = 0, cnt = 0;
        while (p < len) {
            const uint32_t item = b * a.nsec + p / a.sec_len;
            const uint32_t cm = a.spec_cnt[item];
            const uint32_t* sp = a.spec_starts + (uint64_t)item * a.spec_cap;
            int32_t found = -1;
            for (uint32_t j0 = 0; j0 < cm; j0 += 64) {
                const uint32_t e = j0 + lane < cm ? sp[j0 + lane] : 0xFFFFFFFFu;
                const uint64_t hit = __ballot(e == p);
                if (hit) {
                    found = (int32_t)(j0 + __builtin_ctzll(hit));
                    break;
                }
                if (__ballot(e > p)) break;  // sorted: p is not a speculative start
            }
            if (found >= 0) {
                const uint32_t nxt = a.spec_next[item];
                for (uint32_t j0 = (uint32_t)found; j0 < cm; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    if (j < cm) {
                        const uint32_t st = sp[j];
                        const uint32_t en = j + 1 < cm ? sp[j + 1] : nxt;
                        const uint32_t clen = en - st;
                        const uint32_t c = cnt + (j - (uint32_t)found);
                        if (c < a.cap) {
                            const uint64_t slot = (uint64_t)b * a.cap + c;
                            a.starts[slot] = st;
                            a.clens[slot] = clen;
                            uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                            bin = bin < a.nbins ? bin : a.nbins - 1;
                            atomicAdd(&lhist[bin], 1u);
                        } else {
                            atomicOr(a.overflow, 1u);
                        }
                    }
                }
                cnt += cm - (uint32_t)found;
                p = nxt;
            } else {
                const uint32_t lo = p + a.first_off;
                const uint32_t forced = p + a.max_len - 1;
                const uint32_t hi = forced < len - 1 ? forced : len - 1;
                int64_t k = -1;
                if (lo <= hi)
                    k = a.seg_sum ? find_first_sum(a, b, lo, hi, lane) : find_first_wide(a.bitmap, word0, lo, hi, lane);
                if (k < 0) k = (int64_t)hi;
                const uint32_t clen = (uint32_t)k + 1 - p;
                if (cnt < a.cap) {
                    if (lane == 0) {
                        const uint64_t slot = (uint64_t)b * a.cap + cnt;
                        a.starts[slot] = p;
                        a.clens[slot] = clen;
                        uint32_t bin = sha_blocks(clen) >> a.bin_shift;
                        bin = bin < a.nbins ? bin : a.nbins - 1;
                        atomicAdd(&lhist[bin], 1u);
                    }
                } else if (lane == 0) {
                    atomicOr(a.overflow, 1u);
                }
                cnt++;
                p = (uint32_t)k + 1;
            }
        }
        if (lane == 0) a.counts[b] = cnt < a.cap ? cnt : a.cap;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.nbins; i += 256)
        if (lhist[i]) atomicAdd(&a.hist[i], lhist[i]);
}

uint32_t resolve_section_len(uint64_t len, uint32_t max_len, uint32_t sec_log2) {
    // sections of 2^sec_log2 positions for buffers of 4 MiB and more (40 MiB backup buffers at the
    // engine's default 2^18: 160 sections); a section must hold two chunks of max_len, so a larger
    // max_len grows the section to the next power of two instead of giving up the sectioned walk
    if (len < (4ull << 20) || len >= (1ull << 31) || (uint64_t)max_len + 64 >= 32ull * kResStride) return 0;
    uint64_t sec = 1ull << sec_log2;
    while (sec < 2ull * max_len) sec <<= 1;
    return (uint32_t)sec;
}

hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s) {
    const uint64_t len = a.uniform_len ? a.uniform_len : a.max_buf_len;
    if (a.sec_len && a.spec_starts && a.nbuf) {
        // very long buffers: speculative walk per section (one workgroup each), then stitch
        const uint64_t items = (uint64_t)a.nbuf * a.nsec;
        const uint32_t g = (uint32_t)std::min<uint64_t>((items + 3) / 4, 1u << 20);
        if (!a.spec_from_scan) hipLaunchKernelGGL(cdc_resolve_spec_kernel, dim3(g), dim3(256), 0, s, a);
        if (a.join && a.join_bad) {
            hipLaunchKernelGGL(cdc_resolve_join_kernel, dim3(g), dim3(256), 0, s, a);
            hipLaunchKernelGGL(cdc_resolve_place_kernel, dim3(g), dim3(256), 0, s, a);
        }
        hipLaunchKernelGGL(cdc_resolve_stitch_kernel, dim3((a.nbuf + 3) / 4), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (len > 32ull * kResWin && a.max_len + 64ull < 32ull * kResStride && len < (1ull << 31)) {
        // long buffers: LDS-staged walk, one workgroup per buffer
        hipLaunchKernelGGL(cdc_resolve_lds_kernel<false>, dim3(a.nbuf ? a.nbuf : 1), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (a.nbuf && a.nbuf <= kSmallWalkMaxBufs && len <= 32ull * kSmallWalkWords) {
        // a few buffers (a coalescing-queue pass): LDS-staged walk, one workgroup per buffer
        hipLaunchKernelGGL(cdc_resolve_small_kernel, dim3(a.nbuf), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    uint32_t blocks = (a.nbuf + 3) / 4;
    // large batches: a few buffers per wave so the per-block histogram flush is amortised; small
    // ones (a queue pass) one buffer per wave, since each walk is a serial chain of bitmap loads
    if (a.nbuf > 4096) blocks = (blocks + 3) / 4;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(cdc_resolve_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// 3. prefix: bin cursors (descending bins = longest chunks first) and record bases
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void cdc_prefix_kernel(PrefixArgs a) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    // bins: cursor[b] = sum_{b' > b} hist[b']
    part[t] = t < a.nbins ? a.hist[a.nbins - 1 - t] : 0;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    if (t < a.nbins) a.cursor[a.nbins - 1 - t] = part[t] - a.hist[a.nbins - 1 - t];
    __syncthreads();
    // record bases: exclusive prefix of counts
    const uint32_t per = (a.nbuf + 1023) / 1024;
    const uint32_t b0 = t * per, b1 = (b0 + per < a.nbuf) ? b0 + per : a.nbuf;
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += a.counts[b];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const uint32_t base = a.base_in ? *a.base_in : 0u;
    uint32_t run = base + part[t] - sum;
    if (a.rec_base)
        for (uint32_t b = b0; b < b1; b++) {
            a.rec_base[b] = run;
            run += a.counts[b];
        }
    if (t == 1023) {
        *a.total = part[1023];
        if (a.base_out) *a.base_out = base + part[1023];
        if (a.grand_total) *a.grand_total = base + part[1023];
    }
}

hipError_t launch_prefix(const PrefixArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(cdc_prefix_kernel, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// 4. scatter: slot -> position in the longest-first task list (block-aggregated atomics)
// ------------------------------------------------------------------------------------------
constexpr int kScatterThreads = 256;
constexpr int kScatterPer = 8;

__global__ __launch_bounds__(kScatterThreads) void cdc_scatter_kernel(ScatterArgs a) {
    __shared__ uint32_t lcount[kMaxBins], lbase[kMaxBins];
    for (uint32_t i = threadIdx.x; i < a.nbins; i += kScatterThreads) lcount[i] = 0;
    __syncthreads();
    const uint64_t nslots = (uint64_t)a.nbuf * a.cap;
    const uint64_t s0 = (uint64_t)blockIdx.x * kScatterThreads * kScatterPer;
    uint32_t bin[kScatterPer], loc[kScatterPer];
#pragma unroll
    for (int k = 0; k < kScatterPer; k++) {
        const uint64_t slot = s0 + (uint64_t)k * kScatterThreads + threadIdx.x;
        bin[k] = 0xFFFFFFFFu;
        if (slot < nslots) {
            const uint32_t b = (uint32_t)(slot / a.cap);
            const uint32_t i = (uint32_t)(slot - (uint64_t)b * a.cap);
            if (i < a.counts[b]) {
                uint32_t bb = sha_blocks(a.clens[slot]) >> a.bin_shift;
                bb = bb < a.nbins ? bb : a.nbins - 1;
                bin[k] = bb;
                loc[k] = atomicAdd(&lcount[bb], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.nbins; i += kScatterThreads)
        if (lcount[i]) lbase[i] = atomicAdd(&a.cursor[i], lcount[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScatterPer; k++)
        if (bin[k] != 0xFFFFFFFFu)
            a.tasks[lbase[bin[k]] + loc[k]] = (uint32_t)(s0 + (uint64_t)k * kScatterThreads + threadIdx.x);
}

// Small batches (a queue pass: at most kSmallScatterSlots chunk slots): prefix and scatter in ONE
// 1024-thread workgroup, the bin cursors in LDS (one launch instead of two on the pass's critical
// path).  Same outputs: cursor (advanced past each bin's tasks, as the scatter leaves it), rec_base,
// total, and the task list grouped by bin, longest first (the order inside a bin is free).
__global__ __launch_bounds__(1024) void cdc_prefix_scatter_small_kernel(PrefixArgs a, ScatterArgs c) {
    __shared__ uint32_t part[1024];
    __shared__ uint32_t lcur[kMaxBins];
    const uint32_t t = threadIdx.x;
    part[t] = t < a.nbins ? a.hist[a.nbins - 1 - t] : 0;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    if (t < a.nbins) lcur[a.nbins - 1 - t] = part[t] - a.hist[a.nbins - 1 - t];
    __syncthreads();
    const uint32_t per = (a.nbuf + 1023) / 1024;
    const uint32_t b0 = t * per, b1 = (b0 + per < a.nbuf) ? b0 + per : a.nbuf;
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) sum += a.counts[b];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const uint32_t base = a.base_in ? *a.base_in : 0u;
    uint32_t run = base + part[t] - sum;
    if (a.rec_base)
        for (uint32_t b = b0; b < b1; b++) {
            a.rec_base[b] = run;
            run += a.counts[b];
        }
    if (t == 1023) {
        *a.total = part[1023];
        if (a.base_out) *a.base_out = base + part[1023];
        if (a.grand_total) *a.grand_total = base + part[1023];
    }
    const uint32_t nslots = c.nbuf * c.cap;
    for (uint32_t slot = t; slot < nslots; slot += 1024) {
        const uint32_t b = slot / c.cap, i = slot - b * c.cap;
        if (i < c.counts[b]) {
            uint32_t bb = sha_blocks(c.clens[slot]) >> c.bin_shift;
            bb = bb < c.nbins ? bb : c.nbins - 1;
            c.tasks[atomicAdd(&lcur[bb], 1u)] = slot;
        }
    }
    __syncthreads();
    if (t < a.nbins) c.cursor[t] = lcur[t];
}

hipError_t launch_prefix_scatter_small(const PrefixArgs& a, const ScatterArgs& c, hipStream_t s) {
    if ((uint64_t)c.nbuf * c.cap > kSmallScatterSlots || a.nbins > 1024 || c.cursor != a.cursor) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cdc_prefix_scatter_small_kernel, dim3(1), dim3(1024), 0, s, a, c);
    return hipGetLastError();
}

hipError_t launch_scatter(const ScatterArgs& a, hipStream_t s) {
    const uint64_t nslots = (uint64_t)a.nbuf * a.cap;
    const uint64_t per_block = (uint64_t)kScatterThreads * kScatterPer;
    const uint32_t blocks = (uint32_t)((nslots + per_block - 1) / per_block);
    hipLaunchKernelGGL(cdc_scatter_kernel, dim3(blocks ? blocks : 1), dim3(kScatterThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_hash_split(const HashArgs& a, uint64_t max_tasks, hipStream_t s, bool packed, uint32_t lds_pad) {
    if (packed) {
        // production: two lanes per chunk on the chain (11 instead of 14 instructions per round).
        // lds_pad: dynamic LDS no lane touches, so that at most one such workgroup fits a CU and
        // its chain wave does not share a SIMD with another pass's (the caller decides when)
        // bybuf: max_tasks = nbuf * cap, one group per 32 slots of each buffer
        const uint32_t blocks = a.bybuf ? (uint32_t)(max_tasks / a.cap) * a.bybuf
                                        : (uint32_t)((max_tasks + kSplitTasksPacked - 1) / kSplitTasksPacked);
        if (blocks == 0) return hipSuccess;
        switch (a.algo) {
        case 0: hipLaunchKernelGGL((chunk_hash_split_packed_kernel<0>), dim3(blocks), dim3(128), lds_pad, s, a); break;
        case 1: hipLaunchKernelGGL((chunk_hash_split_packed_kernel<1>), dim3(blocks), dim3(128), lds_pad, s, a); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    const uint32_t blocks = (uint32_t)((max_tasks + kSplitTasks - 1) / kSplitTasks);
    if (blocks == 0) return hipSuccess;
    switch (a.algo) {
    case 0: hipLaunchKernelGGL((chunk_hash_split_kernel<0>), dim3(blocks), dim3(128), 0, s, a); break;
    case 1: hipLaunchKernelGGL((chunk_hash_split_kernel<1>), dim3(blocks), dim3(128), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_hash(const HashArgs& a, uint64_t max_tasks, int variant, hipStream_t s, bool packed) {
    const uint32_t blocks = (uint32_t)((max_tasks + 255) / 256);
    if (blocks == 0) return hipSuccess;
    if (variant != 0) {
#ifdef SDFS_TUNING
        return launch_hash_sweep(a, max_tasks, variant, s);
#else
        return hipErrorInvalidValue;
#endif
    }
    if (a.nlong && a.algo != 2) {
        // long chunks possible (maxLen above 32 KiB): they take the latency form (chunk_hash_long_kernel)
        const uint64_t g = packed ? kSplitTasksPacked : kSplitTasks;
        const uint32_t lg = (uint32_t)(((uint64_t)std::min<uint64_t>(a.max_long, kLongSplitMax) + g - 1) / g);
        if (packed) {
            if (a.algo == 0)
                hipLaunchKernelGGL((chunk_hash_long_kernel<0, true>), dim3(blocks + lg), dim3(256), 0, s, a);
            else
                hipLaunchKernelGGL((chunk_hash_long_kernel<1, true>), dim3(blocks + lg), dim3(256), 0, s, a);
        } else {
            if (a.algo == 0)
                hipLaunchKernelGGL((chunk_hash_long_kernel<0, false>), dim3(blocks + lg), dim3(256), 0, s, a);
            else
                hipLaunchKernelGGL((chunk_hash_long_kernel<1, false>), dim3(blocks + lg), dim3(256), 0, s, a);
        }
        return hipGetLastError();
    }
    // production: next-block prefetch issued unconditionally (ABL bit 16; interleaved A/B 2.762 ->
    // 2.744 ms median, profiles/r01/probes/hash_true_prefetch_ab.jsonl) and issue priority for
    // waves of long chunks (2.75 vs 2.81 ms per 4 GiB, profiles/r01/probes/hash_prio_ab.jsonl)
    switch (a.algo) {
    case 0: hipLaunchKernelGGL((chunk_hash_kernel<0, 16, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL((chunk_hash_kernel<1, 16, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((chunk_hash_kernel<2, 16, 256, true, true>), dim3(blocks), dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// synthetic input: byte o of stream s = byte (o%8) of splitmix64(key + o/8)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(uint8_t* out, uint64_t n, uint64_t key, uint64_t offset) {
    const uint64_t nw = ((offset + n + 7) >> 3) - (offset >> 3);
    const bool fast = ((offset & 7) == 0) && ((reinterpret_cast<uintptr_t>(out) & 7) == 0);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256) {
        const uint64_t wi = (offset >> 3) + i;
        const uint64_t v = splitmix64(key + wi);
        const uint64_t b0 = wi * 8;  // stream byte offset of this word
        if (fast && b0 + 8 <= offset + n) {
            *reinterpret_cast<uint64_t*>(out + (b0 - offset)) = v;
        } else {
            for (int k = 0; k < 8; k++) {
                const uint64_t o = b0 + k;
                if (o >= offset && o < offset + n) out[o - offset] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// a batch's prep: its small scratch (histogram, cursors, totals) and its overflow flag zeroed in
// one launch (two memsets were two fill kernels on the pass's critical path)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_zero_kernel(uint4* small16, uint32_t n16, uint32_t* flag) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) small16[i] = make_uint4(0, 0, 0, 0);
    if (flag && blockIdx.x == 0 && threadIdx.x == 0) *flag = 0;
}

hipError_t launch_prep_zero(uint32_t* small, uint32_t words, uint32_t* flag, hipStream_t s) {
    if ((words & 3) || (reinterpret_cast<uintptr_t>(small) & 15)) return hipErrorInvalidValue;
    const uint32_t n16 = words / 4;
    hipLaunchKernelGGL(prep_zero_kernel, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n16 + 255) / 256, 8))), dim3(256), 0,
                       s, reinterpret_cast<uint4*>(small), n16, flag);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// result image -> pinned host memory, written by the GPU itself in stream order (the coalescing
// queue's passes): no DMA-engine copy behind the kernels and no host round trip to issue one.
// `dst` is device-accessible pinned host memory; n16 = bytes / 16.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void copy_out_kernel(const uint4* src, uint4* dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_copy_out(const void* src, void* dst, uint64_t bytes, hipStream_t s) {
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return hipErrorInvalidValue;
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return hipSuccess;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 1024);
    hipLaunchKernelGGL(copy_out_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(src),
                       reinterpret_cast<uint4*>(dst), n16);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// 6. fingerprints of given extents (getHash in bulk): longest-first order of n chunk lengths
// ------------------------------------------------------------------------------------------
// bin = sha_blocks(len) >> 2, capped: 4-block bins up to 2048 blocks (128 KiB), then one bin.
constexpr uint32_t kExtBins = 512, kExtShift = 2;

__device__ __forceinline__ uint32_t ext_count(const uint32_t* count, uint64_t n_max) {
    return count ? (uint32_t)min<uint64_t>(*count, n_max) : (uint32_t)n_max;
}
__device__ __forceinline__ uint32_t ext_bin(uint32_t len) {
    const uint32_t b = sha_blocks(len) >> kExtShift;
    return b < kExtBins ? b : kExtBins - 1;
}

__global__ __launch_bounds__(256) void ext_hist_kernel(ExtentArgs a) {
    __shared__ uint32_t lh[kExtBins];
    for (uint32_t k = threadIdx.x; k < kExtBins; k += 256) lh[k] = 0;
    __syncthreads();
    const uint32_t n = ext_count(a.count, a.n_max);
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        atomicAdd(&lh[ext_bin(a.lens[i])], 1u);
        a.starts[i] = 0;  // every extent is its own "buffer" with one slot at offset 0
    }
    if (i == 0) *a.total = n;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kExtBins; k += 256)
        if (lh[k]) atomicAdd(&a.hist[k], lh[k]);
}

__global__ __launch_bounds__(kExtBins) void ext_cursor_kernel(ExtentArgs a) {
    __shared__ uint32_t part[kExtBins];
    const uint32_t t = threadIdx.x;
    part[t] = a.hist[kExtBins - 1 - t];  // longest bin first
    __syncthreads();
    for (uint32_t d = 1; d < kExtBins; d <<= 1) {
        const uint32_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    a.cursor[kExtBins - 1 - t] = part[t] - a.hist[kExtBins - 1 - t];
}

__global__ __launch_bounds__(256) void ext_scatter_kernel(ExtentArgs a) {
    __shared__ uint32_t lc[kExtBins], lb[kExtBins];
    for (uint32_t k = threadIdx.x; k < kExtBins; k += 256) lc[k] = 0;
    __syncthreads();
    const uint32_t n = ext_count(a.count, a.n_max);
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t bin = 0, rank = 0;
    if (i < n) {
        bin = ext_bin(a.lens[i]);
        rank = atomicAdd(&lc[bin], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kExtBins; k += 256)
        if (lc[k]) lb[k] = atomicAdd(&a.cursor[k], lc[k]);
    __syncthreads();
    if (i < n) a.tasks[lb[bin] + rank] = (uint32_t)i;
}

hipError_t launch_extent_order(const ExtentArgs& a, hipStream_t s) {
    if (a.n_max == 0) return hipSuccess;
    const uint32_t g = (uint32_t)((a.n_max + 255) / 256);
    hipError_t e = hipMemsetAsync(a.hist, 0, kExtBins * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ext_hist_kernel, dim3(g), dim3(256), 0, s, a);
    hipLaunchKernelGGL(ext_cursor_kernel, dim3(1), dim3(kExtBins), 0, s, a);
    hipLaunchKernelGGL(ext_scatter_kernel, dim3(g), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* out, uint64_t n, uint64_t seed, uint64_t stream_id, uint64_t offset,
                        hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t key = splitmix64_host(seed ^ (stream_id * 0xD1B54A32D192ED03ull));
    const uint64_t nw = ((offset + n + 7) >> 3) - (offset >> 3);
    uint64_t blocks = (nw + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, out, n, key, offset);
    return hipGetLastError();
}

}  // namespace sdfs
