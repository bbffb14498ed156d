// lz4_kernels.hip — LZ4 block compression of unique chunks on the MI355X (include/sdfs_lz4.h;
// SURVEY.md §8(f) row 2).
//
// Reference: HashBlobArchive.putChunk (HashBlobArchive.java:1281-1289) stores a new chunk as
// [int nz = chunk.length, big-endian][CompressionUtils.compressLz4(chunk)]; compressLz4 is
// lz4-java 1.3.0's native fastCompressor (CompressionUtils.java:52-53,118-120), i.e. the bundled
// C LZ4 r123 greedy parse.  The bytes emitted here are exactly that parse (oracle/lz4_ref.c
// restates it; mode V19 = LZ4 1.9.x, pinned there against the image's liblz4).
//
// MI355X form: one wave per chunk, its hash table in LDS (2^13 x u16 below 64 KiB + 11 bytes,
// 2^12 x u32 above: 16 KiB either way).  LZ4's match search probes ip, ip+1, ... with a step that
// grows by one every 64 misses, so the next 64 probe positions are known in closed form until one
// of them matches: the wave probes 64 at once (one lane each).  A probe must see the table as the
// serial loop would — the latest EARLIER probe with the same hash, else the table — so probes
// of one round that share an entry are found through a 1 KiB LDS scratch (write lane id, read it
// back) and resolved in lane order; the first lane whose candidate matches is the serial loop's
// match, and only the probes up to it enter the table.  Match extension (64 x 4 bytes per step),
// the backward catch-up, literal copies (16 B per lane) and the 255-runs of long lengths are
// wave-parallel; the per-sequence bookkeeping is wave-uniform scalar work.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/sdfs_lz4.h"
#include "cdc_internal.h"
#include "stream_order.h"

namespace sdfs {
namespace {

constexpr uint32_t kMinMatch = 4, kMfLimit = 12, kLastLiterals = 5, kMlMask = 15, kRunMask = 15;
constexpr uint32_t kLimit64K = 65536 + kMfLimit - 1;  // below: 16-bit position table
constexpr uint32_t kMaxDistance = 65535;
constexpr uint32_t kScrBuckets = 1024;  // same-entry detection among one round's 64 probes
constexpr int kLz4WgPerCu = 9;          // 17 KiB of LDS per one-wave workgroup: 9 fit in 160 KiB
                                        // (latency-bound: throughput ~ waves in flight, scripts/probes/lz4_grid_sweep.sh)

struct Lz4Args {
    const uint8_t* data;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint32_t* d_count;
    uint64_t n_max;
    uint8_t* out;
    const uint64_t* dst_off;
    uint32_t* dst_len;
    uint32_t framed;
    uint32_t* gtab;  // GTAB kernels: 16 KiB hash table per workgroup in global memory;
                     // LANE kernel: 2^13 tagged u32 entries per lane
    uint32_t* ltag;  // LANE kernel: per-lane table generation
    const uint32_t* idx;   // item i is chunk idx[i] (wave kernel: the lane pass's bailed chunks;
                           // LANE kernel: chunks longest first)
    uint32_t* bail;        // LANE kernel (hybrid): bail[0] = count, bail[1 + k] = chunk index
    uint32_t bail_misses;  // LANE kernel (hybrid): hand a chunk to the wave pass after this many
                           // consecutive search misses in its first quarter (0 = never)
};

// LDS byte scratch accessed as volatile LDS (ds_write_b8 / ds_read_u8, ordered per wave): a
// volatile GENERIC pointer would become flat accesses with system-scope bits and vmcnt(0) waits.
typedef __attribute__((address_space(3))) volatile uint8_t lds_vu8;
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;

template <typename P>
__device__ __forceinline__ uint32_t ld32(P p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
template <typename P>
__device__ __forceinline__ uint64_t ld64(P p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// LDS source (STAGE kernels): unaligned words from two aligned dword reads and a v_alignbyte (a
// plain unaligned 4-byte read from LDS compiles to four ds_read_u8).  The stage has 16 spare bytes
// so the dword after the chunk's last byte is still inside it.
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
__device__ __forceinline__ uint32_t ld32(lds_cu8* p) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    lds_cu32* q = (lds_cu32*)(p - (a & 3));
    return __builtin_amdgcn_alignbyte(q[1], q[0], a & 3);
}
__device__ __forceinline__ uint64_t ld64(lds_cu8* p) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    lds_cu32* q = (lds_cu32*)(p - (a & 3));
    const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, a & 3) << 32 | __builtin_amdgcn_alignbyte(w1, w0, a & 3);
}

// unaligned global words (one dword / dwordx2 load)
__device__ __forceinline__ uint32_t g32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ uint64_t g64(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// table index of the sequence at p (lz4_ref.c hash_at)
template <int MODE, typename P>
__device__ __forceinline__ uint32_t lz4_hash(P p, bool u16) {
    if (u16) return (ld32(p) * 2654435761u) >> 19;
    if constexpr (MODE == SDFS_CDC_LZ4_V19) return (uint32_t)(((ld64(p) << 24) * 889523592379ull) >> 52);
    return (ld32(p) * 2654435761u) >> 20;
}

// Offset of probe i from the search start: steps of 1 for the first 65 probes, then the step
// grows by one every 64 probes (step_i = (63 + i) >> 6 for i >= 1, step_0 = 1).
__device__ __forceinline__ uint32_t probe_off(uint32_t i) {
    if (i == 0) return 0;
    const uint32_t m = i - 1, q = m >> 6, r = m & 63;
    return 1 + 32 * q * (q + 1) + r * (q + 1);
}

__device__ __forceinline__ uint32_t tab_get(const uint32_t* t, uint32_t h, bool u16) {
    return u16 ? (uint32_t) reinterpret_cast<const uint16_t*>(t)[h] : t[h];
}
__device__ __forceinline__ void tab_put(uint32_t* t, uint32_t h, uint32_t v, bool u16) {
    if (u16)
        reinterpret_cast<uint16_t*>(t)[h] = (uint16_t)v;
    else
        t[h] = v;
}

// a length field past the token nibble: len/255 bytes of 255 and the remainder
__device__ __forceinline__ uint32_t put_run(uint8_t* dst, uint32_t op, uint32_t len, uint32_t lane) {
    const uint32_t nff = len / 255;
    for (uint32_t k = lane; k < nff; k += 64) dst[op + k] = 255;
    if (lane == 0) dst[op + nff] = (uint8_t)(len - nff * 255);
    return op + nff + 1;
}

// n bytes src -> dst (disjoint), 16 bytes per lane per step, four steps in flight.  SrcPtr: a
// global or an LDS (address_space(3)) byte pointer.
template <typename SrcPtr>
__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ dst, SrcPtr __restrict__ src, uint32_t n,
                                           uint32_t lane) {
    const uint32_t nv = n >> 4;
    uint32_t k = lane;
    for (; k + 192 < nv; k += 256) {
        uint4 v0, v1, v2, v3;
        __builtin_memcpy(&v0, src + 16 * k, 16);
        __builtin_memcpy(&v1, src + 16 * (k + 64), 16);
        __builtin_memcpy(&v2, src + 16 * (k + 128), 16);
        __builtin_memcpy(&v3, src + 16 * (k + 192), 16);
        __builtin_memcpy(dst + 16 * k, &v0, 16);
        __builtin_memcpy(dst + 16 * (k + 64), &v1, 16);
        __builtin_memcpy(dst + 16 * (k + 128), &v2, 16);
        __builtin_memcpy(dst + 16 * (k + 192), &v3, 16);
    }
    for (; k < nv; k += 64) {
        uint4 v;
        __builtin_memcpy(&v, src + 16 * k, 16);
        __builtin_memcpy(dst + 16 * k, &v, 16);
    }
    for (uint32_t b = (nv << 4) + lane; b < n; b += 64) dst[b] = src[b];
}

// LDS source: the byte offset within a dword is the same for every lane (16 B per lane), so each
// lane reads five aligned dwords and realigns them
__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ dst, lds_cu8* __restrict__ src, uint32_t n,
                                           uint32_t lane) {
    const uint32_t a = (uint32_t)(uintptr_t)src, sh = a & 3;
    lds_cu32* q = (lds_cu32*)(src - sh);
    const uint32_t nv = n >> 4;
    for (uint32_t k = lane; k < nv; k += 64) {
        const uint32_t w0 = q[4 * k], w1 = q[4 * k + 1], w2 = q[4 * k + 2], w3 = q[4 * k + 3], w4 = q[4 * k + 4];
        const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                   __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
        __builtin_memcpy(dst + 16 * k, &v, 16);
    }
    for (uint32_t b = (nv << 4) + lane; b < n; b += 64) dst[b] = src[b];
}

// number of equal bytes src[a0+k] == src[b0+k] with a0+k < lim (LZ4_count), 256 per step
template <typename SrcPtr>
__device__ __forceinline__ uint32_t match_count(SrcPtr src, uint32_t a0, uint32_t b0, uint32_t lim,
                                                uint32_t lane) {
    if (a0 >= lim) return 0;
    const uint32_t total = lim - a0;
    for (uint32_t base = 0; base < total; base += 256) {
        const uint32_t k = base + 4 * lane;
        uint32_t d;
        if (k + 4 <= total) {
            d = ld32(src + a0 + k) ^ ld32(src + b0 + k);
        } else if (k < total) {
            d = 0;
            for (uint32_t t = 0; t < 4; t++)
                if (k + t >= total || src[a0 + k + t] != src[b0 + k + t]) d |= 0xFFu << (8 * t);
        } else {
            d = 0xFFFFFFFFu;
        }
        const uint64_t mm = __ballot(d != 0);
        if (mm) {
            const uint32_t l = (uint32_t)__builtin_ctzll(mm);
            const uint32_t dl = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)l);
            return base + 4 * l + ((uint32_t)__builtin_ctz(dl) >> 3);
        }
    }
    return total;
}

// One chunk, one wave (all lanes run the same scalar control flow).  Returns the block length.
template <int MODE, typename SrcPtr>
__device__ uint32_t compress_chunk(SrcPtr __restrict__ src, uint32_t n, uint8_t* __restrict__ dst,
                                   uint32_t* tab, lds_vu8* scr, uint32_t lane) {
    {
        uint4* t4 = reinterpret_cast<uint4*>(tab);
        for (uint32_t i = lane; i < 1024; i += 64) t4[i] = make_uint4(0, 0, 0, 0);
    }
    asm volatile("" ::: "memory");  // the cleared table before any 16/32-bit entry access
    const bool u16 = n < kLimit64K;
    const uint32_t mflimit = n >= kMfLimit ? n - kMfLimit : 0;
    const uint32_t search_end = MODE == SDFS_CDC_LZ4_V19 ? mflimit + 1 : mflimit;
    const uint32_t matchlimit = n >= kLastLiterals ? n - kLastLiterals : 0;
    uint32_t ip = 0, anchor = 0, op = 0;

    if (n >= kMfLimit + 1) {
        tab_put(tab, lz4_hash<MODE>(src, u16), 0, u16);
        ip = 1;
        for (;;) {
            // ---- find a match: 64 probes per round
            uint32_t match = 0;
            bool found = false;
            for (uint32_t k0 = 0;; k0 += 64) {
                const uint32_t vi = ip + probe_off(k0 + lane);
                const uint32_t vn = ip + probe_off(k0 + lane + 1);
                const bool act = vn <= search_end;  // the serial loop stops before probing past it
                uint32_t h = 0, cur = 0, cand = 0;
                if (act) {
                    cur = ld32(src + vi);
                    h = u16 ? (cur * 2654435761u) >> 19 : lz4_hash<MODE>(src + vi, false);
                    cand = tab_get(tab, h, u16);
                }
                // probes of this round that share a table entry (or a scratch bucket)
                const uint32_t bkt = h & (kScrBuckets - 1);
                if (act) scr[bkt] = (uint8_t)lane;
                bool cont = act && scr[bkt] != (uint8_t)lane;
                if (cont) scr[bkt] = 0xFF;
                if (act && scr[bkt] == 0xFF) cont = true;
                const uint64_t C = __ballot(cont);
                // serial order: a probe sees the latest earlier probe with its hash
                for (uint64_t m = C; m; m &= m - 1) {
                    const int j = (int)__builtin_ctzll(m);
                    const uint32_t hj = (uint32_t)__builtin_amdgcn_readlane((int)h, j);
                    const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)vi, j);
                    if (cont && (uint32_t)j < lane && hj == h) cand = vj;
                }
                bool eq = false;
                if (act && (u16 || cand + kMaxDistance >= vi)) eq = ld32(src + cand) == cur;
                const uint64_t mact = __ballot(act);
                const uint64_t meq = __ballot(eq);
                const uint32_t fe = ~mact ? (uint32_t)__builtin_ctzll(~mact) : 64u;
                const uint32_t fm = meq ? (uint32_t)__builtin_ctzll(meq) : 64u;
                if (fe < 64 && fe <= fm) break;  // search ended before a match: last literals
                // the table after probes 0..lim: each entry keeps its latest probe
                const uint32_t lim = fm < 64 ? fm : 63;
                bool sup = false;
                for (uint64_t m = C; m; m &= m - 1) {
                    const int j = (int)__builtin_ctzll(m);
                    if ((uint32_t)j > lim) break;
                    const uint32_t hj = (uint32_t)__builtin_amdgcn_readlane((int)h, j);
                    if (cont && (uint32_t)j > lane && hj == h) sup = true;
                }
                if (lane <= lim && act && !sup) tab_put(tab, h, vi, u16);
                asm volatile("" ::: "memory");
                if (fm < 64) {
                    ip = (uint32_t)__builtin_amdgcn_readlane((int)vi, (int)fm);
                    match = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)fm);
                    found = true;
                    break;
                }
            }
            if (!found) break;
            // ---- catch up: extend the match backwards over equal bytes
            {
                const uint32_t B = min(ip - anchor, match);
                uint32_t back = B;
                for (uint32_t base = 0; base < B; base += 64) {
                    const uint32_t l = base + lane;
                    const bool e = l < B && src[ip - 1 - l] == src[match - 1 - l];
                    const uint64_t ne = __ballot(!e);
                    if (ne) {
                        back = base + (uint32_t)__builtin_ctzll(ne);
                        break;
                    }
                }
                ip -= back;
                match -= back;
            }
            // ---- literal run
            uint32_t token = op++;
            uint32_t tokv;
            {
                const uint32_t lit = ip - anchor;
                if (lit >= kRunMask) {
                    tokv = kRunMask << 4;
                    op = put_run(dst, op, lit - kRunMask, lane);
                } else {
                    tokv = lit << 4;
                }
                copy_bytes(dst + op, src + anchor, lit, lane);
                op += lit;
            }
            // ---- a match, possibly followed at once by another one
            for (;;) {
                const uint32_t off = ip - match;
                if (lane == 0) {
                    dst[op] = (uint8_t)off;
                    dst[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                const uint32_t ml = match_count(src, ip + kMinMatch, match + kMinMatch, matchlimit, lane);
                ip += kMinMatch + ml;
                if (ml >= kMlMask) {
                    tokv += kMlMask;
                    op = put_run(dst, op, ml - kMlMask, lane);
                } else {
                    tokv += ml;
                }
                if (lane == 0) dst[token] = (uint8_t)tokv;
                anchor = ip;
                if (ip > mflimit) break;
                // fill the table at ip-2, then test an immediate match at ip
                tab_put(tab, lz4_hash<MODE>(src + ip - 2, u16), ip - 2, u16);
                const uint32_t h = lz4_hash<MODE>(src + ip, u16);
                const uint32_t m = tab_get(tab, h, u16);
                tab_put(tab, h, ip, u16);
                asm volatile("" ::: "memory");
                if ((u16 || m + kMaxDistance >= ip) && ld32(src + m) == ld32(src + ip)) {
                    token = op++;
                    tokv = 0;
                    match = m;
                    continue;
                }
                break;
            }
            if (ip > mflimit) break;
            ip++;
        }
    }
    // ---- last literals
    const uint32_t last = n - anchor;
    if (last >= kRunMask) {
        if (lane == 0) dst[op] = (uint8_t)(kRunMask << 4);
        op = put_run(dst, op + 1, last - kRunMask, lane);
    } else {
        if (lane == 0) dst[op] = (uint8_t)(last << 4);
        op++;
    }
    copy_bytes(dst + op, src + anchor, last, lane);
    return op + last;
}

// One wave per workgroup; chunk c = blockIdx.x + k * gridDim.x (a static stride balances well:
// hundreds of chunks per workgroup, and a shared counter would serialise ~10^6 dequeues).
// GTAB: the hash table lives in global memory (L2 / Infinity Cache) instead of LDS, so LDS no
// longer caps the chunks in flight per CU (1 KiB of LDS per wave instead of 17 KiB).
template <int MODE, bool GTAB = false, int STAGE = 0>
__global__ __launch_bounds__(64) void lz4_compress_kernel(Lz4Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t ltab[GTAB ? 4 : 4096];
    __shared__ uint8_t scr[kScrBuckets];
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE > 0 ? STAGE + 16 : 16];
    uint32_t* tab = GTAB ? a.gtab + (uint64_t)blockIdx.x * 4096 : ltab;
    const uint32_t lane = threadIdx.x;
    const uint64_t n_items = a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
    for (uint64_t i = blockIdx.x; i < n_items; i += gridDim.x) {
        const uint64_t c = a.idx ? a.idx[i] : i;
        const uint32_t n = a.src_len[c];
        const uint8_t* src = a.data + a.src_off[c];
        uint8_t* o = a.out + a.dst_off[c];
        const uint32_t hdr = a.framed ? 4u : 0u;
        uint32_t len;
        if (STAGE > 0 && n <= (uint32_t)STAGE) {
            // STAGE: the chunk's bytes in LDS, so every probe, candidate, catch-up, extension and
            // literal read is an LDS round trip instead of an L2 one
            copy_bytes(stage, src, n, lane);
            __builtin_amdgcn_s_waitcnt(0);  // staged bytes written before any lane reads them
            len = compress_chunk<MODE>((lds_cu8*)stage, n, o + hdr, tab, (lds_vu8*)scr, lane);
        } else {
            len = compress_chunk<MODE>(src, n, o + hdr, tab, (lds_vu8*)scr, lane);
        }
        if (lane == 0) {
            if (hdr) {
                o[0] = (uint8_t)(n >> 24);
                o[1] = (uint8_t)(n >> 16);
                o[2] = (uint8_t)(n >> 8);
                o[3] = (uint8_t)n;
            }
            a.dst_len[c] = len + hdr;
        }
        if (STAGE > 0) __builtin_amdgcn_s_waitcnt(0);  // every lane's stage reads done before the next copy
    }
}

// ---- literal screen (round 5).  Most chunks of a backup stream's file bodies are incompressible,
// and for them LZ4's parse finds no match: every probe of the search (positions 1 + probe_off(i),
// the step growing every 64 misses) compares its 4 bytes with the table's candidate, which is
// either position 0 (the table starts zeroed, and position 0 is put first) or an EARLIER probe
// position.  So when the 4-byte words at position 0 and at every probe position the parse makes
// are pairwise distinct, no compare can succeed, the parse runs to its end, and the block is the
// chunk as one literal run (last_literals with anchor 0) — whatever the mode (R123 / V19 differ in
// the search end, which sets the probe count, and in hashing, which does not matter here).  The
// screen checks exactly that, one wave per chunk: the words go into an LDS hash set (linear
// probing, compare-and-swap); a chunk with all words distinct is written as its literal block, any
// other chunk (a repeated word: compressible, or an accidental repeat) joins the `rest` list that
// the exact kernels then run on.  Output is the same bytes either way (tests/test_lz4.py).
constexpr uint32_t kScreenSlots = 4096;  // LDS set of one one-wave workgroup (16 KiB)
constexpr uint32_t kScreenMaxWords = kScreenSlots / 2;  // load factor <= 1/2 (~32 KiB chunks)
constexpr int kScreenWgPerCu = 9;

// Probes the search makes in a chunk without a match: probe i is made iff the next position,
// 1 + probe_off(i + 1), is <= search_end; returns their count P (probes 0 .. P-1).
__device__ __forceinline__ uint32_t screen_probes(uint32_t search_end) {
    if (search_end < 2) return 0;  // 1 + probe_off(1) = 2
    uint32_t lo = 1, hi = 1u << 16;  // 1 + probe_off(2^16) > 2^27 > any screened chunk
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (1 + probe_off(mid) <= search_end) lo = mid;
        else hi = mid;
    }
    return lo;
}

template <int MODE>
__global__ __launch_bounds__(64) void lz4_literal_screen_kernel(Lz4Args a, uint32_t* rest) {
    __shared__ __attribute__((aligned(16))) uint32_t set[kScreenSlots];
    const uint32_t lane = threadIdx.x;
    const uint64_t n_items = a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
    for (uint64_t i = blockIdx.x; i < n_items; i += gridDim.x) {
        const uint64_t c = a.idx ? a.idx[i] : i;
        const uint32_t n = a.src_len[c];
        const uint8_t* src = a.data + a.src_off[c];
        bool literal = n < kMfLimit + 1;  // too short to search: literals only
        if (!literal && n < (1u << 27)) {
            const uint32_t mflimit = n - kMfLimit;
            const uint32_t search_end = MODE == SDFS_CDC_LZ4_V19 ? mflimit + 1 : mflimit;
            const uint32_t P = screen_probes(search_end);
            // words: position 0, the P probe positions, and (harmless: at worst a false repeat)
            // the first position past the search while it is inside the chunk
            const uint32_t nw = 1 + P + (1 + probe_off(P) + 4 <= n ? 1u : 0u);
            if (nw <= kScreenMaxWords) {
                uint32_t lg = 6;
                while ((1u << lg) < 2 * nw) lg++;
                const uint32_t mask = (1u << lg) - 1;
                for (uint32_t s = lane; 4 * s <= mask; s += 64) reinterpret_cast<uint4*>(set)[s] = make_uint4(0, 0, 0, 0);
                __syncthreads();
                bool dup = false;
                uint32_t zeros = 0;  // the word 0 is the set's empty mark: counted instead
                // a first round of one word per lane (compressible chunks show a repeat there and
                // leave early), then eight per lane
                for (uint32_t k0 = 0, per = 1; k0 < nw && !dup; k0 += 64 * per, per = 8) {
                    uint32_t v[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const uint32_t k = k0 + 64 * j + lane;
                        v[j] = 0xFFFFFFFFu;
                        if ((uint32_t)j < per && k < nw) v[j] = g32(src + (k == 0 ? 0u : 1 + probe_off(k - 1)));
                    }
                    // first probe of every word in straight-line code (eight compare-and-swaps in
                    // flight); only a word whose slot holds another word walks on (rare at load <= 1/2)
                    uint32_t sl[8], old[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const uint32_t k = k0 + 64 * j + lane;
                        const bool ok = (uint32_t)j < per && k < nw && v[j] != 0;
                        zeros += (uint32_t)j < per && k < nw && v[j] == 0;
                        sl[j] = (v[j] * 2654435761u) >> (32 - lg);
                        old[j] = ok ? atomicCAS(&set[sl[j]], 0u, v[j]) : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        dup = dup || (old[j] != 0 && old[j] == v[j]);
                        if (old[j] != 0 && old[j] != v[j]) {
                            uint32_t t = sl[j];
                            for (;;) {
                                t = (t + 1) & mask;
                                const uint32_t o2 = atomicCAS(&set[t], 0u, v[j]);
                                if (o2 == 0) break;
                                if (o2 == v[j]) {
                                    dup = true;
                                    break;
                                }
                            }
                        }
                    }
                    dup = __any(dup) || __any(zeros > 1) || __popcll(__ballot(zeros > 0)) > 1;
                }
                literal = !dup;
                __syncthreads();  // the set is cleared again only after every lane is done with it
            }
        }
        if (!literal) {
            if (lane == 0) rest[1 + atomicAdd(rest, 1u)] = (uint32_t)c;
            continue;
        }
        uint8_t* o = a.out + a.dst_off[c];
        const uint32_t hdr = a.framed ? 4u : 0u;
        uint32_t op = hdr;
        if (lane == 0) {
            if (hdr) {
                o[0] = (uint8_t)(n >> 24);
                o[1] = (uint8_t)(n >> 16);
                o[2] = (uint8_t)(n >> 8);
                o[3] = (uint8_t)n;
            }
            o[hdr] = (uint8_t)((n >= kRunMask ? kRunMask : n) << 4);
        }
        op++;
        if (n >= kRunMask) op = put_run(o, op, n - kRunMask, lane);
        copy_bytes(o + op, src, n, lane);
        if (lane == 0) a.dst_len[c] = op + n;
    }
}

// ---- decompression (the read side: HashBlobArchive.getChunk -> CompressionUtils.decompressLz4,
// HashBlobArchive.java:1927-1933, CompressionUtils.java:122-125; LZ4 block format).  One wave per
// block: the token stream is parsed as wave-uniform scalar work, literal runs are copied 16 bytes
// per lane, and a match is copied lane-parallel — an overlapping match (offset < length) as
// dst[op + k] = dst[op - off + k % off], which only reads bytes written before the match.
struct Lz4DecArgs {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint32_t* d_count;
    uint64_t n_max;
    uint8_t* out;
    const uint64_t* dst_off;
    const uint32_t* dst_cap;
    uint32_t* dst_len;
    uint32_t framed;
    uint32_t route;  // 0: every block; 1: compressible blocks only (lane kernel); 2: the others
};

constexpr uint32_t kLz4Corrupt = 0xFFFFFFFFu;

// Routing of the split decode: a block that saved under 1/16 of its bytes (or a raw record) is
// mostly literal runs, which the wave kernel copies coalesced; the others are short sequences,
// which one lane per block parses without the wave's per-sequence round trips.
__device__ __forceinline__ bool dec_lane_class(const uint8_t* in, uint32_t n, uint32_t cap, uint32_t framed) {
    uint32_t out = cap;
    if (framed) {
        if (n < 4) return false;
        const int32_t nz = (int32_t)((uint32_t)in[0] << 24 | (uint32_t)in[1] << 16 | (uint32_t)in[2] << 8 | in[3]);
        if (nz <= 0) return false;
        out = (uint32_t)nz;
        n -= 4;
    }
    return (uint64_t)n * 16 < (uint64_t)out * 15;
}

// Decode one block of n bytes into dst (cap bytes); returns the decoded length or kLz4Corrupt.

template <typename SrcPtr>
__device__ uint32_t decompress_block(SrcPtr __restrict__ src, uint32_t n, uint8_t* dst, uint32_t cap,
                                     uint32_t lane) {
    uint32_t ip = 0, op = 0;
    for (;;) {
        if (ip >= n) return kLz4Corrupt;
        const uint32_t token = src[ip++];
        uint32_t lit = token >> 4;
        if (lit == kRunMask) {
            uint32_t b;
            do {
                if (ip >= n) return kLz4Corrupt;
                b = src[ip++];
                lit += b;
            } while (b == 255);
        }
        if (ip + lit > n || op + lit > cap) return kLz4Corrupt;
        copy_bytes(dst + op, src + ip, lit, lane);
        ip += lit;
        op += lit;
        if (ip == n) return op;  // the last sequence carries literals only
        if (ip + 2 > n) return kLz4Corrupt;
        const uint32_t off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
        ip += 2;
        if (off == 0 || off > op) return kLz4Corrupt;
        uint32_t ml = token & kMlMask;
        if (ml == kMlMask) {
            uint32_t b;
            do {
                if (ip >= n) return kLz4Corrupt;
                b = src[ip++];
                ml += b;
            } while (b == 255);
        }
        ml += kMinMatch;
        if (op + ml > cap) return kLz4Corrupt;
        if (off >= ml) {
            copy_bytes(dst + op, (const uint8_t*)(dst + op - off), ml, lane);  // disjoint: source ends before op
        } else {
            uint32_t kr = lane % off;  // k % off, stepped by 64 without a division per byte
            const uint32_t sr = 64 % off;
            for (uint32_t k = lane; k < ml; k += 64) {
                dst[op + k] = dst[op - off + kr];
                kr += sr;
                if (kr >= off) kr -= off;
            }
        }
        op += ml;
    }
}

// compressed bytes staged in LDS per wave (larger blocks parse from global) and workgroups per CU:
// 4 KiB x 28 decodes text 12 % faster than 8 KiB x 16 (more blocks in flight outweigh the blocks
// that parse from global; profiles/r01/lz4_dec_sweep.jsonl).  SDFS_LZ4_DEC_STAGE=8192 /
// SDFS_LZ4_DEC_WG_PER_CU select the others for measurements.
constexpr uint32_t kDecStage = 4096;
constexpr int kDecWgPerCu = 28;

// a block: staged through LDS when it fits (the token/length/offset parse and the literal reads
// become LDS round trips), else parsed from global memory
template <uint32_t STAGE>
__device__ __forceinline__ uint32_t decode_any(const uint8_t* in, uint32_t n, uint8_t* o, uint32_t cap, uint8_t* stage,
                                               uint32_t lane) {
    if (n <= STAGE) {
        copy_bytes(stage, in, n, lane);
        __builtin_amdgcn_s_waitcnt(0);  // staged bytes written before any lane parses them
        return decompress_block((lds_cu8*)stage, n, o, cap, lane);
    }
    return decompress_block(in, n, o, cap, lane);
}

template <uint32_t STAGE = kDecStage>
__global__ __launch_bounds__(64) void lz4_decompress_kernel(Lz4DecArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE + 16];  // + the realigning reads' spare dword
    const uint32_t lane = threadIdx.x;
    const uint64_t n_items = a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
    for (uint64_t c = blockIdx.x; c < n_items; c += gridDim.x) {
        const uint8_t* in = a.src + a.src_off[c];
        uint32_t n = a.src_len[c];
        uint8_t* o = a.out + a.dst_off[c];
        uint32_t cap = a.dst_cap[c];
        if (a.route == 2 && dec_lane_class(in, n, cap, a.framed)) continue;  // the lane kernel's
        uint32_t got;
        if (a.framed) {  // [BE32 nz][payload]: nz > 0 = LZ4 block of nz bytes, else raw bytes
            if (n < 4) {
                got = kLz4Corrupt;
            } else {
                const int32_t nz = (int32_t)((uint32_t)in[0] << 24 | (uint32_t)in[1] << 16 | (uint32_t)in[2] << 8 | in[3]);
                in += 4;
                n -= 4;
                if (nz > 0) {
                    got = (uint32_t)nz <= cap ? decode_any<STAGE>(in, n, o, (uint32_t)nz, stage, lane) : kLz4Corrupt;
                    if (got != (uint32_t)nz) got = kLz4Corrupt;
                } else if (n <= cap) {
                    copy_bytes(o, in, n, lane);
                    got = n;
                } else {
                    got = kLz4Corrupt;
                }
            }
        } else {
            got = decode_any<STAGE>(in, n, o, cap, stage, lane);
        }
        if (lane == 0) a.dst_len[c] = got;
    }
}

// One LANE per block (route 1 of the split decode): the serial parse of decompress_block with
// 8-byte literal and match copies (an overlapping match with offset < 8 byte by byte, which
// reads only bytes this lane wrote before).  Same corruption checks, never writes past cap.
__device__ uint32_t decompress_lane(const uint8_t* __restrict__ src, uint32_t n, uint8_t* __restrict__ dst,
                                    uint32_t cap) {
    uint32_t ip = 0, op = 0;
    for (;;) {
        // fast sequence: short literal run (< 15) with its offset inside the next 17 source
        // bytes and room for 16-byte literal / 8-byte-rounded match writes before cap.  The
        // over-written bytes past op are rewritten by the following sequences before anything
        // reads them (a match only reads below its own op).
        if (ip + 17 <= n && op + 16 <= cap) {
            const uint64_t w0 = g64(src + ip), l0 = g64(src + ip + 1), l1 = g64(src + ip + 9);
            const uint32_t token = (uint32_t)w0 & 255u, lit = token >> 4;
            if (lit < kRunMask) {
                __builtin_memcpy(dst + op, &l0, 8);
                __builtin_memcpy(dst + op + 8, &l1, 8);
                // offset bytes at lit, lit + 1 of the 16 loaded after the token
                const uint32_t b0 = lit < 8 ? (uint32_t)(l0 >> (8 * lit)) : (uint32_t)(l1 >> (8 * (lit - 8)));
                const uint32_t b1 = lit + 1 < 8 ? (uint32_t)(l0 >> (8 * (lit + 1))) : (uint32_t)(l1 >> (8 * (lit - 7)));
                const uint32_t off = (b0 & 255u) | ((b1 & 255u) << 8);
                op += lit;
                ip += 3 + lit;
                if (off == 0 || off > op) return kLz4Corrupt;
                uint32_t ml = token & kMlMask;
                if (ml == kMlMask) {
                    uint32_t b;
                    do {
                        if (ip >= n) return kLz4Corrupt;
                        b = src[ip++];
                        ml += b;
                    } while (b == 255);
                }
                ml += kMinMatch;
                if (op + ml > cap) return kLz4Corrupt;
                uint32_t k = 0;
                if (off >= 8) {
                    if (op + ml + 8 <= cap) {  // 8-byte rounded (wild) copy
                        for (; k < ml; k += 8) {
                            const uint64_t v = g64(dst + op - off + k);
                            __builtin_memcpy(dst + op + k, &v, 8);
                        }
                        k = ml;
                    } else {
                        for (; k + 8 <= ml; k += 8) {
                            const uint64_t v = g64(dst + op - off + k);
                            __builtin_memcpy(dst + op + k, &v, 8);
                        }
                    }
                }
                for (; k < ml; k++) dst[op + k] = dst[op - off + k];
                op += ml;
                continue;
            }
        }
        if (ip >= n) return kLz4Corrupt;
        const uint32_t token = src[ip++];
        uint32_t lit = token >> 4;
        if (lit == kRunMask) {
            uint32_t b;
            do {
                if (ip >= n) return kLz4Corrupt;
                b = src[ip++];
                lit += b;
            } while (b == 255);
        }
        if (ip + lit > n || op + lit > cap) return kLz4Corrupt;
        {
            uint32_t k = 0;
            for (; k + 8 <= lit; k += 8) {
                const uint64_t v = g64(src + ip + k);
                __builtin_memcpy(dst + op + k, &v, 8);
            }
            for (; k < lit; k++) dst[op + k] = src[ip + k];
        }
        ip += lit;
        op += lit;
        if (ip == n) return op;
        if (ip + 2 > n) return kLz4Corrupt;
        const uint32_t off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
        ip += 2;
        if (off == 0 || off > op) return kLz4Corrupt;
        uint32_t ml = token & kMlMask;
        if (ml == kMlMask) {
            uint32_t b;
            do {
                if (ip >= n) return kLz4Corrupt;
                b = src[ip++];
                ml += b;
            } while (b == 255);
        }
        ml += kMinMatch;
        if (op + ml > cap) return kLz4Corrupt;
        uint32_t k = 0;
        if (off >= 8) {  // each 8-byte read ends at or before the first byte this step writes
            for (; k + 8 <= ml; k += 8) {
                const uint64_t v = g64(dst + op - off + k);
                __builtin_memcpy(dst + op + k, &v, 8);
            }
        }
        for (; k < ml; k++) dst[op + k] = dst[op - off + k];
        op += ml;
    }
}

__global__ __launch_bounds__(256) void lz4_decompress_lane_kernel(Lz4DecArgs a) {
    const uint64_t n_items = a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < n_items; c += (uint64_t)gridDim.x * 256) {
        const uint8_t* in = a.src + a.src_off[c];
        uint32_t n = a.src_len[c];
        const uint32_t cap = a.dst_cap[c];
        if (!dec_lane_class(in, n, cap, a.framed)) continue;  // the wave kernel's
        uint32_t got;
        if (a.framed) {
            const uint32_t nz = (uint32_t)in[0] << 24 | (uint32_t)in[1] << 16 | (uint32_t)in[2] << 8 | in[3];
            got = nz <= cap ? decompress_lane(in + 4, n - 4, a.out + a.dst_off[c], nz) : kLz4Corrupt;
            if (got != nz) got = kLz4Corrupt;
        } else {
            got = decompress_lane(in, n, a.out + a.dst_off[c], cap);
        }
        a.dst_len[c] = got;
    }
}

// ---- plan: record -> chunk extent and output room (block-local scan, block-sum scan, add)
constexpr int kPlanBlock = 1024;

struct PlanArgs {
    const uint8_t* records;
    const uint32_t* sel;
    const uint32_t* d_count;
    uint64_t n_max;
    uint64_t id_base;
    uint32_t uniform_len;
    uint32_t framed;
    const uint64_t* buf_offs;
    uint64_t* src_off;
    uint32_t* src_len;
    uint64_t* dst_off;
    uint64_t* bsum;
    uint64_t* total;
};

__device__ __forceinline__ uint64_t block_exclusive_scan64(uint64_t v, uint64_t* lds, uint64_t& total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) lds[wv] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint64_t w = threadIdx.x < kPlanBlock / 64 ? lds[threadIdx.x] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(w, o);
            if (lane >= (uint32_t)o) w += y;
        }
        if (threadIdx.x < kPlanBlock / 64) lds[16 + threadIdx.x] = w;
    }
    __syncthreads();
    total = lds[16 + kPlanBlock / 64 - 1];
    const uint64_t before = wv ? lds[16 + wv - 1] : 0;
    const uint64_t res = before + x - v;
    __syncthreads();
    return res;
}

__device__ __forceinline__ uint64_t plan_count(const PlanArgs& a) {
    return a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
}

__global__ __launch_bounds__(kPlanBlock) void lz4_plan_local_kernel(PlanArgs a) {
    __shared__ uint64_t lds[64];
    const uint64_t n = plan_count(a);
    const uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    uint64_t room = 0;
    if (i < n) {
        const uint64_t r = a.sel ? a.sel[i] : i;
        const uint8_t* rec = a.records + r * kRecordBytes;
        uint64_t bid;
        uint32_t st, ln;
        __builtin_memcpy(&bid, rec + 32, 8);
        __builtin_memcpy(&st, rec + 40, 4);
        __builtin_memcpy(&ln, rec + 44, 4);
        const uint64_t b = bid - a.id_base;
        a.src_off[i] = (a.buf_offs ? a.buf_offs[b] : b * a.uniform_len) + st;
        a.src_len[i] = ln;
        room = (uint64_t)ln + ln / 255 + 16 + (a.framed ? 4 : 0);
    }
    uint64_t total;
    const uint64_t ex = block_exclusive_scan64(room, lds, total);
    if (i < n) a.dst_off[i] = ex;
    if (threadIdx.x == 0) a.bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kPlanBlock) void lz4_plan_scan_kernel(uint64_t* bsum, uint32_t nblocks,
                                                                   uint64_t* total_out) {
    __shared__ uint64_t lds[64];
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += kPlanBlock) {
        const uint32_t i = b0 + threadIdx.x;
        const uint64_t v = i < nblocks ? bsum[i] : 0;
        uint64_t total;
        const uint64_t ex = block_exclusive_scan64(v, lds, total);
        if (i < nblocks) bsum[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(kPlanBlock) void lz4_plan_add_kernel(PlanArgs a) {
    const uint64_t n = plan_count(a);
    const uint64_t i = (uint64_t)blockIdx.x * kPlanBlock + threadIdx.x;
    if (i < n) a.dst_off[i] += a.bsum[blockIdx.x];
}

// ---- one LANE per chunk (measurement variant, SDFS_LZ4_LANE=1 in the tuning build): every
// lane runs the byte-serial greedy parse of oracle/lz4_ref.c on its own chunk, so a wave has 64
// chunks in flight instead of one; the lane's table is 2^13 u32 entries in global memory, each
// (generation << 17) | position, so a new chunk starts from an "all zero" table without clearing
// it (an entry of another generation reads as position 0, as LZ4's zeroed table does).
constexpr uint32_t kLaneTabEntries = 1u << 13;
constexpr uint32_t kLanePosBits = 17;  // positions < 128 KiB (the backup profile's maxLen)


template <int MODE>
__device__ __forceinline__ uint32_t lane_hash(const uint8_t* p, bool u16) {
    if (u16) return (g32(p) * 2654435761u) >> 19;
    if constexpr (MODE == SDFS_CDC_LZ4_V19) return (uint32_t)(((g64(p) << 24) * 889523592379ull) >> 52);
    return (g32(p) * 2654435761u) >> 20;
}

__device__ __forceinline__ uint32_t lane_run(uint8_t* dst, uint32_t op, uint32_t len) {
    for (; len >= 255; len -= 255) dst[op++] = 255;
    dst[op++] = (uint8_t)len;
    return op;
}

__device__ __forceinline__ void lane_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
    uint32_t k = 0;
    for (; k + 4 <= n; k += 4) {
        const uint32_t v = g32(src + k);
        __builtin_memcpy(dst + k, &v, 4);
    }
    for (; k < n; k++) dst[k] = src[k];
}

constexpr uint32_t kLaneBailed = 0xffffffffu;
constexpr uint32_t kHybridChunksPerCu = 192;  // auto policy: hybrid from 192 chunks per CU up
constexpr int kLaneDepth = 1;  // probes per search round (SDFS_LZ4_LANE_DEPTH=4|8 in the tuning build:
                               // no gain at 1 GiB batches, where table traffic, not the chain, bounds it)

// The lane's search runs D probes per round: their positions follow from the step rule until a
// match, so the D source words, then the D table entries, then the D candidate words are each
// loaded together (three round trips per D probes instead of two or three per probe).  A probe
// sees the puts of the earlier probes of its round by forwarding (same entry: the latest earlier
// probe's position), exactly as the serial loop's get-after-put would.
template <int MODE, int D>
__device__ uint32_t compress_lane(const uint8_t* __restrict__ src, uint32_t n, uint8_t* __restrict__ dst,
                                  uint32_t* __restrict__ tab, uint32_t tag, uint32_t bail_misses) {
    const bool u16 = n < kLimit64K;
    const uint32_t mflimit = n >= kMfLimit ? n - kMfLimit : 0;
    const uint32_t search_end = MODE == SDFS_CDC_LZ4_V19 ? mflimit + 1 : mflimit;
    const uint32_t matchlimit = n >= kLastLiterals ? n - kLastLiterals : 0;
    const uint32_t tg = tag << kLanePosBits;
    auto get = [&](uint32_t h) -> uint32_t {
        const uint32_t e = tab[h];
        return (e & ~((1u << kLanePosBits) - 1)) == tg ? (e & ((1u << kLanePosBits) - 1)) : 0u;
    };
    auto put = [&](uint32_t h, uint32_t pos) { tab[h] = tg | pos; };
    uint32_t ip = 0, anchor = 0, op = 0;
    if (n >= kMfLimit + 1) {
        put(lane_hash<MODE>(src, u16), 0);
        ip = 1;
        for (;;) {
            uint32_t match = 0;
            bool found = false;
            {
                uint32_t fip = ip, step = 1, nb = 1u << 6;
                for (;;) {
                    if (bail_misses && nb >= bail_misses + 64 && 4 * fip < n) return kLaneBailed;
                    uint32_t pos[D], h[D], m[D], cur[D];
                    int nv = 0;  // probes of this round the serial loop would make
#pragma unroll
                    for (int i = 0; i < D; i++) {
                        pos[i] = fip;
                        if (nv == i && fip + step <= search_end) nv = i + 1;
                        fip += step;
                        step = nb++ >> 6;
                    }
#pragma unroll
                    for (int i = 0; i < D; i++) {
                        cur[i] = i < nv ? g32(src + pos[i]) : 0u;
                        h[i] = i < nv ? lane_hash<MODE>(src + pos[i], u16) : 0u;
                    }
#pragma unroll
                    for (int i = 0; i < D; i++) m[i] = i < nv ? get(h[i]) : 0u;
#pragma unroll
                    for (int i = 1; i < D; i++)
#pragma unroll
                        for (int j = 0; j < i; j++)
                            if (h[j] == h[i]) m[i] = pos[j];
                    int hit = D;
#pragma unroll
                    for (int i = D - 1; i >= 0; i--) {
                        const bool near = u16 || m[i] + kMaxDistance >= pos[i];
                        if (i < nv && near && g32(src + m[i]) == cur[i]) hit = i;
                    }
                    const int last = hit < D ? hit : nv - 1;
#pragma unroll
                    for (int i = 0; i < D; i++)
                        if (i <= last) put(h[i], pos[i]);
                    if (hit < D) {
#pragma unroll
                        for (int i = 0; i < D; i++)
                            if (i == hit) {
                                ip = pos[i];
                                match = m[i];
                            }
                        found = true;
                        break;
                    }
                    if (nv < D) break;
                }
            }
            if (!found) break;
            while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
                ip--;
                match--;
            }
            uint32_t token = op++;
            {
                const uint32_t lit = ip - anchor;
                if (lit >= kRunMask) {
                    dst[token] = (uint8_t)(kRunMask << 4);
                    op = lane_run(dst, op, lit - kRunMask);
                } else {
                    dst[token] = (uint8_t)(lit << 4);
                }
                lane_copy(dst + op, src + anchor, lit);
                op += lit;
            }
            bool done = false;
            for (;;) {
                const uint32_t off = ip - match;
                dst[op++] = (uint8_t)off;
                dst[op++] = (uint8_t)(off >> 8);
                uint32_t a = ip + kMinMatch, b = match + kMinMatch;
                // 32 bytes per round trip (four independent 8-byte pairs), then 8, then bytes
                while (a + 32 <= matchlimit) {
                    uint64_t x[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) x[k] = g64(src + a + 8 * k) ^ g64(src + b + 8 * k);
                    int k = 0;
                    while (k < 4 && x[k] == 0) k++;
                    if (k < 4) {
                        a += 8 * k + ((uint32_t)__builtin_ctzll(x[k]) >> 3);
                        goto counted;
                    }
                    a += 32;
                    b += 32;
                }
                while (a + 8 <= matchlimit) {
                    const uint64_t x = g64(src + a) ^ g64(src + b);
                    if (x) {
                        a += (uint32_t)__builtin_ctzll(x) >> 3;
                        goto counted;
                    }
                    a += 8;
                    b += 8;
                }
                while (a < matchlimit && src[a] == src[b]) {
                    a++;
                    b++;
                }
            counted:
                const uint32_t ml = a - (ip + kMinMatch);
                ip = a;
                if (ml >= kMlMask) {
                    dst[token] += kMlMask;
                    op = lane_run(dst, op, ml - kMlMask);
                } else {
                    dst[token] += (uint8_t)ml;
                }
                anchor = ip;
                if (ip > mflimit) {
                    done = true;
                    break;
                }
                put(lane_hash<MODE>(src + ip - 2, u16), ip - 2);
                const uint32_t h = lane_hash<MODE>(src + ip, u16);
                match = get(h);
                put(h, ip);
                if ((u16 || match + kMaxDistance >= ip) && g32(src + match) == g32(src + ip)) {
                    token = op++;
                    dst[token] = 0;
                    continue;
                }
                break;
            }
            if (done) break;
            ++ip;
        }
    }
    const uint32_t last = n - anchor;
    if (last >= kRunMask) {
        dst[op++] = (uint8_t)(kRunMask << 4);
        op = lane_run(dst, op, last - kRunMask);
    } else {
        dst[op++] = (uint8_t)(last << 4);
    }
    lane_copy(dst + op, src + anchor, last);
    return op + last;
}

// Hybrid pre-test (PT): before parsing, a lane looks at its chunk's first kPretestBytes for
// repeated 4-byte sequences in a 64-entry table of its own in LDS (16-bit tags of the
// multiplicative hash whose top 6 bits pick the entry; entry h of lane t at h * 256 + t).  Incompressible data repeats none (random
// chunks: 0 hits; word-salad text: 21-66, scripts/lz4_bench.py data), so such a chunk goes
// straight to the wave kernel instead of after 128 table-probing misses.  Only the route
// depends on it; the bytes do not.
constexpr uint32_t kPretestBytes = 512, kPretestHits = 4;

template <int MODE, int D, bool PT>
__global__ __launch_bounds__(256) void lz4_lane_kernel(Lz4Args a) {
    __shared__ uint16_t pt[PT ? 64 * 256 : 1];  // 32 KiB: four 256-lane workgroups per CU
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nl = gridDim.x * 256;
    const uint64_t n_items = a.d_count ? min<uint64_t>(*a.d_count, a.n_max) : a.n_max;
    uint32_t* tab = a.gtab + (uint64_t)g * kLaneTabEntries;
    uint32_t tag = a.ltag[g];
    for (uint64_t i = g; i < n_items; i += nl) {
        const uint64_t c = a.idx ? a.idx[i] : i;  // longest-first order: a wave's lanes end together
        const uint32_t n = a.src_len[c];
        const uint8_t* src = a.data + a.src_off[c];
        // A lane's table entries hold (generation << 17) | position: a chunk longer than 128 KiB
        // would spill position bits into the generation field, so it goes to the wave kernel.
        if (n > (1u << kLanePosBits)) {
            a.bail[1 + atomicAdd(a.bail, 1u)] = (uint32_t)c;
            continue;
        }
        if constexpr (PT) {
            if (a.bail_misses) {
                const uint32_t m = n < kPretestBytes ? n : kPretestBytes;
#pragma unroll 8
                for (uint32_t h = 0; h < 64; h++) pt[h * 256 + threadIdx.x] = 0;
                uint32_t hits = 0;
#pragma unroll 4
                for (uint32_t p = 0; p + 4 <= m; p++) {
                    const uint32_t x = g32(src + p) * 2654435761u;  // slot: top 6 bits, tag: low 16
                    const uint32_t h = x >> 26;
                    hits += pt[h * 256 + threadIdx.x] == (uint16_t)x;
                    pt[h * 256 + threadIdx.x] = (uint16_t)x;
                }
                if (hits < kPretestHits && m >= 64) {
                    a.bail[1 + atomicAdd(a.bail, 1u)] = (uint32_t)c;
                    continue;
                }
            }
        }
        if (++tag >= (1u << (32 - kLanePosBits))) {  // generations exhausted: clear once
            for (uint32_t i = 0; i < kLaneTabEntries; i++) tab[i] = 0;
            tag = 1;
        }
        uint8_t* o = a.out + a.dst_off[c];
        const uint32_t hdr = a.framed ? 4u : 0u;
        const uint32_t len = compress_lane<MODE, D>(src, n, o + hdr, tab, tag, a.bail_misses);
        if (len == kLaneBailed) {
            a.bail[1 + atomicAdd(a.bail, 1u)] = (uint32_t)c;
            continue;
        }
        if (hdr) {
            o[0] = (uint8_t)(n >> 24);
            o[1] = (uint8_t)(n >> 16);
            o[2] = (uint8_t)(n >> 8);
            o[3] = (uint8_t)n;
        }
        a.dst_len[c] = len + hdr;
    }
    a.ltag[g] = tag;
}

template <typename T>
struct ZBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(want, 1) * sizeof(T));
        if (e == hipSuccess) n = std::max<size_t>(want, 1);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace
}  // namespace sdfs

using namespace sdfs;

struct sdfs_cdc_lz4 {
    int device = 0;
    int mode = SDFS_CDC_LZ4_R123;
    int num_cus = 256;
    int wg_per_cu = kLz4WgPerCu;  // SDFS_LZ4_WG_PER_CU overrides (measurements)
    int gtab_mode = 0;            // SDFS_LZ4_GTAB=1: hash tables in global memory
    int stage = 0;                // SDFS_LZ4_STAGE=16384|32768: chunks up to that size staged in LDS
    int lane_mode = -1;           // -1 auto (hybrid from kHybridChunksPerCu chunks per CU up), 0 wave
                                  // kernel, 1 lane kernel only, 2 hybrid (SDFS_LZ4_LANE, tuning build)
    int lane_wg_per_cu = 4;       // SDFS_LZ4_LANE_WG_PER_CU: 256-thread workgroups per CU (lane mode)
    int lane_grid = 0;            // SDFS_LZ4_LANE_GRID: at most this many lane workgroups (0 = no cap)
    ZBuf<uint32_t> ltag;
    ZBuf<uint32_t> bail;          // hybrid (lane_mode 2): count + bailed chunk indices
    int screen = 1;               // literal screen before the exact kernels (SDFS_LZ4_SCREEN=0: off, tuning build)
    ZBuf<uint32_t> rest;          // screen: count + the chunks the exact kernels compress
    uint32_t bail_misses = 128;   // SDFS_LZ4_BAIL
    int lane_sort = 0;            // SDFS_LZ4_LANE_SORT=1: lanes take chunks longest first (measured slower)
    int lane_depth = kLaneDepth;  // SDFS_LZ4_LANE_DEPTH
    int pretest = 1;              // SDFS_LZ4_PRETEST=0: no LDS pre-test in the hybrid (tuning build)
    ZBuf<uint32_t> ord;           // launch_extent_order scratch: starts, tasks, total, hist, cursor
    int dec_stage = (int)kDecStage;
    int dec_wg_per_cu = kDecWgPerCu;
    int dec_lane_wg_per_cu = 8;  // SDFS_LZ4_DEC_LANE_WG_PER_CU: 256-lane workgroups per CU (split decode)
    int dec_split = -1;  // -1 auto (split from kHybridChunksPerCu blocks per CU up), 0 wave kernel only,
                         // 1 split: lanes for compressible blocks, waves for the rest (SDFS_LZ4_DEC_LANE)
    ZBuf<uint32_t> gtab;
    hipStream_t stream = nullptr;
    ZBuf<uint64_t> bsum;
    // host-path scratch
    ZBuf<uint8_t> h_in, h_out;
    ZBuf<uint64_t> h_soff, h_doff;
    ZBuf<uint32_t> h_slen, h_dlen;
    StreamOrder order;  // launches that use the shared device scratch, across streams
    std::mutex mu;
};

#define LZ_TRY(expr)                                                                                  \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return fail_status(SDFS_CDC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                               __FILE__, __LINE__);                                                   \
    } while (0)

namespace {

template <int D, bool PT>
hipError_t launch_lane_d(int mode, uint32_t grid, const Lz4Args& g, hipStream_t s) {
    if (mode == SDFS_CDC_LZ4_V19)
        hipLaunchKernelGGL((lz4_lane_kernel<SDFS_CDC_LZ4_V19, D, PT>), dim3(grid), dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL((lz4_lane_kernel<SDFS_CDC_LZ4_R123, D, PT>), dim3(grid), dim3(256), 0, s, g);
    return hipGetLastError();
}

hipError_t launch_lane(int mode, int depth, bool pretest, uint32_t grid, const Lz4Args& g, hipStream_t s) {
#ifdef SDFS_TUNING
    if (depth == 4) return launch_lane_d<4, false>(mode, grid, g, s);
    if (depth == 8) return launch_lane_d<8, false>(mode, grid, g, s);
    if (!pretest) return launch_lane_d<kLaneDepth, false>(mode, grid, g, s);
#endif
    (void)depth;
    (void)pretest;
    return launch_lane_d<kLaneDepth, true>(mode, grid, g, s);
}

// Lane tables for `lanes` lanes (32 KiB each, zeroed once; generations make later chunks start
// from an empty table).  False: not allocatable now (the wave kernel runs instead).
bool lane_tables(sdfs_cdc_lz4* z, uint64_t lanes, hipStream_t s) {
    if (z->ltag.n >= lanes && z->ltag.p) return true;
    if (z->gtab.ensure(lanes * kLaneTabEntries) != hipSuccess || z->ltag.ensure(lanes) != hipSuccess) {
        z->gtab.release();
        z->ltag.release();
        (void)hipGetLastError();
        return false;
    }
    if (hipMemsetAsync(z->gtab.p, 0, lanes * kLaneTabEntries * 4, s) != hipSuccess ||
        hipMemsetAsync(z->ltag.p, 0, lanes * 4, s) != hipSuccess) {
        z->ltag.release();  // tables not known to be zero: allocate and clear again next time
        return false;
    }
    return true;
}

// The compressor's device scratch (lane tables and generations, the bail list, the plan's block
// sums) serves one stream at a time: a launch on another stream than the previous one first
// waits for that one's work (an event recorded after every launch that used the scratch).
int scratch_acquire(sdfs_cdc_lz4* z, hipStream_t s) {
    LZ_TRY(z->order.acquire(s));
    return SDFS_CDC_OK;
}
int scratch_release(sdfs_cdc_lz4* z, hipStream_t s) {
    LZ_TRY(z->order.release(s));
    return SDFS_CDC_OK;
}

int launch_compress_impl(sdfs_cdc_lz4* z, const Lz4Args& a, hipStream_t s);

int launch_compress(sdfs_cdc_lz4* z, const Lz4Args& a, hipStream_t s) {
    if (a.n_max == 0) return SDFS_CDC_OK;
    int rc = scratch_acquire(z, s);
    if (rc) return rc;
    rc = launch_compress_impl(z, a, s);
    const int rr = scratch_release(z, s);
    return rc ? rc : rr;
}

int launch_compress_impl(sdfs_cdc_lz4* z, const Lz4Args& a0, hipStream_t s) {
    // The literal screen first (every batch): chunks whose parse can find no match are written as
    // one literal run here; the exact kernels below run on the `rest` list only.
    Lz4Args a = a0;
    if (z->screen && !a0.idx) {
        LZ_TRY(z->rest.ensure(a0.n_max + 1));
        LZ_TRY(hipMemsetAsync(z->rest.p, 0, 4, s));
        const uint32_t sgrid = (uint32_t)std::min<uint64_t>(a0.n_max, (uint64_t)z->num_cus * kScreenWgPerCu);
        if (z->mode == SDFS_CDC_LZ4_V19)
            hipLaunchKernelGGL(lz4_literal_screen_kernel<SDFS_CDC_LZ4_V19>, dim3(sgrid), dim3(64), 0, s, a0, z->rest.p);
        else
            hipLaunchKernelGGL(lz4_literal_screen_kernel<SDFS_CDC_LZ4_R123>, dim3(sgrid), dim3(64), 0, s, a0, z->rest.p);
        LZ_TRY(hipGetLastError());
        a.d_count = z->rest.p;
        a.idx = z->rest.p + 1;
    }
    // Auto: a batch with enough chunks to fill the chip one lane per chunk runs the hybrid (lanes
    // for compressible chunks, the wave kernel for the ones a lane bails on); smaller batches the
    // wave kernel (scripts/probes/lz4_batch_sweep.sh: the hybrid pays from ~50 000 chunks per 256 CUs).
    // n_max bounds a device-count batch, so the choice follows the capacity the caller gives.
    const int lane_mode = z->lane_mode >= 0 ? z->lane_mode
                                            : (a.n_max >= (uint64_t)z->num_cus * kHybridChunksPerCu ? 2 : 0);
    uint64_t lgrid = std::min<uint64_t>((a.n_max + 255) / 256, (uint64_t)z->num_cus * z->lane_wg_per_cu);
    if (z->lane_grid > 0) lgrid = std::min<uint64_t>(lgrid, (uint64_t)z->lane_grid);  // tuning: fewer chains
    if (lane_mode == 1 && !lane_tables(z, lgrid * 256, s))
        return fail_status(SDFS_CDC_EHIP, "lz4: cannot allocate %llu lane tables", (unsigned long long)(lgrid * 256));
    if (lane_mode == 1 || (lane_mode == 2 && lane_tables(z, lgrid * 256, s))) {
        const uint64_t grid = lgrid;
        Lz4Args g = a;
        g.gtab = z->gtab.p;
        g.ltag = z->ltag.p;
        const bool hybrid = lane_mode == 2;
        if (z->lane_sort) {
            LZ_TRY(z->ord.ensure(2 * a.n_max + kExtentScratchWords));
            ExtentArgs x{a.src_len, a.d_count, a.n_max, z->ord.p, z->ord.p + a.n_max, z->ord.p + 2 * a.n_max,
                         z->ord.p + 2 * a.n_max + 1, z->ord.p + 2 * a.n_max + 1 + 512};
            LZ_TRY(launch_extent_order(x, s));
            g.idx = x.tasks;
        }
        // Both lane modes keep a bail list: chunks over 128 KiB always go to the wave kernel; the
        // hybrid also bails on chunks that look incompressible (pre-test, then bail_misses misses).
        LZ_TRY(z->bail.ensure(a.n_max + 1));
        LZ_TRY(hipMemsetAsync(z->bail.p, 0, 4, s));
        g.bail = z->bail.p;
        g.bail_misses = hybrid ? z->bail_misses : 0u;
        LZ_TRY(launch_lane(z->mode, z->lane_depth, z->pretest != 0, (uint32_t)grid, g, s));
        Lz4Args w = a;  // the bailed chunks, one wave each
        w.d_count = z->bail.p;
        w.idx = z->bail.p + 1;
        const uint32_t wgrid = (uint32_t)std::min<uint64_t>(a.n_max, (uint64_t)z->num_cus * z->wg_per_cu);
        if (z->mode == SDFS_CDC_LZ4_V19)
            hipLaunchKernelGGL(lz4_compress_kernel<SDFS_CDC_LZ4_V19>, dim3(wgrid), dim3(64), 0, s, w);
        else
            hipLaunchKernelGGL(lz4_compress_kernel<SDFS_CDC_LZ4_R123>, dim3(wgrid), dim3(64), 0, s, w);
        LZ_TRY(hipGetLastError());
        return SDFS_CDC_OK;
    }
    const uint64_t grid = std::min<uint64_t>(a.n_max, (uint64_t)z->num_cus * z->wg_per_cu);
    if (z->gtab_mode) {
        LZ_TRY(z->gtab.ensure(grid * 4096));
        Lz4Args g = a;
        g.gtab = z->gtab.p;
        if (z->mode == SDFS_CDC_LZ4_V19)
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_V19, true>), dim3((uint32_t)grid), dim3(64), 0, s, g);
        else
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_R123, true>), dim3((uint32_t)grid), dim3(64), 0, s, g);
    } else if (z->stage == 32768) {
        if (z->mode == SDFS_CDC_LZ4_V19)
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_V19, false, 32768>), dim3((uint32_t)grid), dim3(64), 0, s, a);
        else
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_R123, false, 32768>), dim3((uint32_t)grid), dim3(64), 0, s, a);
    } else if (z->stage == 16384) {
        if (z->mode == SDFS_CDC_LZ4_V19)
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_V19, false, 16384>), dim3((uint32_t)grid), dim3(64), 0, s, a);
        else
            hipLaunchKernelGGL((lz4_compress_kernel<SDFS_CDC_LZ4_R123, false, 16384>), dim3((uint32_t)grid), dim3(64), 0, s, a);
    } else if (z->mode == SDFS_CDC_LZ4_V19) {
        hipLaunchKernelGGL(lz4_compress_kernel<SDFS_CDC_LZ4_V19>, dim3((uint32_t)grid), dim3(64), 0, s, a);
    } else {
        hipLaunchKernelGGL(lz4_compress_kernel<SDFS_CDC_LZ4_R123>, dim3((uint32_t)grid), dim3(64), 0, s, a);
    }
    LZ_TRY(hipGetLastError());
    return SDFS_CDC_OK;
}

}  // namespace

extern "C" {

uint64_t sdfs_cdc_lz4_bound(uint64_t n) { return n + n / 255 + 16; }

int sdfs_cdc_lz4_create(int device, int mode, sdfs_cdc_lz4** out) {
    if (!out) return fail_status(SDFS_CDC_EINVAL, "null output");
    *out = nullptr;
    if (mode != SDFS_CDC_LZ4_R123 && mode != SDFS_CDC_LZ4_V19)
        return fail_status(SDFS_CDC_EINVAL, "bad lz4 mode %d", mode);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail_status(SDFS_CDC_ENODEV, "no HIP device %d", device);
    LZ_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    LZ_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail_status(SDFS_CDC_ENODEV, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    auto* z = new sdfs_cdc_lz4();
    z->device = device;
    z->mode = mode;
    z->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
#ifdef SDFS_TUNING
    // measurement-only layouts (tuning library; DESIGN.md §11 measured them, the product library
    // reads no environment)
    if (const char* v = getenv("SDFS_LZ4_GTAB")) z->gtab_mode = atoi(v);
    if (z->gtab_mode) z->wg_per_cu = 24;
    if (const char* v = getenv("SDFS_LZ4_STAGE")) z->stage = atoi(v);
    if (z->stage != 16384 && z->stage != 32768) z->stage = 0;
    if (z->stage) z->wg_per_cu = z->stage == 32768 ? 3 : 4;  // 16 KiB table + 1 KiB scratch + stage per workgroup
    if (const char* v = getenv("SDFS_LZ4_DEC_STAGE")) z->dec_stage = atoi(v) == 8192 ? 8192 : (int)kDecStage;
    if (const char* v = getenv("SDFS_LZ4_DEC_WG_PER_CU")) z->dec_wg_per_cu = std::max(1, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_DEC_LANE")) z->dec_split = atoi(v);
    if (const char* v = getenv("SDFS_LZ4_DEC_LANE_WG_PER_CU")) z->dec_lane_wg_per_cu = std::max(1, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_WG_PER_CU")) z->wg_per_cu = std::max(1, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_LANE")) z->lane_mode = atoi(v);
    if (const char* v = getenv("SDFS_LZ4_LANE_WG_PER_CU")) z->lane_wg_per_cu = std::max(1, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_LANE_GRID")) z->lane_grid = std::max(0, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_BAIL")) z->bail_misses = (uint32_t)std::max(0, atoi(v));
    if (const char* v = getenv("SDFS_LZ4_LANE_SORT")) z->lane_sort = atoi(v);
    if (const char* v = getenv("SDFS_LZ4_LANE_DEPTH")) z->lane_depth = atoi(v);
    if (const char* v = getenv("SDFS_LZ4_PRETEST")) z->pretest = atoi(v);
    if (const char* v = getenv("SDFS_LZ4_SCREEN")) z->screen = atoi(v);
#endif
    if (hipStreamCreateWithFlags(&z->stream, hipStreamNonBlocking) != hipSuccess) {
        delete z;
        return fail_status(SDFS_CDC_EHIP, "stream creation failed");
    }
    if (z->order.init() != hipSuccess) {
        (void)hipStreamDestroy(z->stream);
        delete z;
        return fail_status(SDFS_CDC_EHIP, "event creation failed");
    }
    *out = z;
    return SDFS_CDC_OK;
}

int sdfs_cdc_lz4_destroy(sdfs_cdc_lz4* z) {
    if (!z) return SDFS_CDC_OK;
    {
        std::lock_guard<std::mutex> lk(z->mu);
        (void)hipSetDevice(z->device);
        if (z->stream) (void)hipStreamSynchronize(z->stream);
        z->bsum.release();
        z->gtab.release();
        z->ltag.release();
        z->bail.release();
        z->rest.release();
        z->ord.release();
        z->h_in.release();
        z->h_out.release();
        z->h_soff.release();
        z->h_doff.release();
        z->h_slen.release();
        z->h_dlen.release();
        if (z->stream) (void)hipStreamDestroy(z->stream);
        z->order.destroy();
    }
    delete z;
    return SDFS_CDC_OK;
}

int sdfs_cdc_lz4_compress_device(sdfs_cdc_lz4* z, const uint8_t* d_data, const uint64_t* d_src_off,
                                 const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max,
                                 uint8_t* d_out, const uint64_t* d_dst_off, uint32_t* d_dst_len, int framed,
                                 void* stream) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null compressor");
    if (n_max && (!d_data || !d_src_off || !d_src_len || !d_out || !d_dst_off || !d_dst_len))
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(z->mu);
    LZ_TRY(hipSetDevice(z->device));
    Lz4Args a{d_data, d_src_off, d_src_len, d_count, n_max, d_out, d_dst_off, d_dst_len, framed ? 1u : 0u};
    return launch_compress(z, a, reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_lz4_plan_records(sdfs_cdc_lz4* z, const uint8_t* d_records, const uint32_t* d_sel,
                              const uint32_t* d_count, uint64_t n_max, uint64_t buffer_id_base,
                              uint32_t uniform_len, const uint64_t* d_buf_offs, int framed, uint64_t* d_src_off,
                              uint32_t* d_src_len, uint64_t* d_dst_off, uint64_t* d_total_bytes, void* stream) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null compressor");
    if (!d_total_bytes) return fail_status(SDFS_CDC_EINVAL, "null total");
    if (n_max && (!d_records || !d_src_off || !d_src_len || !d_dst_off))
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (!d_buf_offs && !uniform_len) return fail_status(SDFS_CDC_EINVAL, "buffer offsets or uniform_len required");
    std::lock_guard<std::mutex> lk(z->mu);
    LZ_TRY(hipSetDevice(z->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (n_max == 0) {
        LZ_TRY(hipMemsetAsync(d_total_bytes, 0, 8, s));
        return SDFS_CDC_OK;
    }
    const uint32_t nblocks = (uint32_t)((n_max + kPlanBlock - 1) / kPlanBlock);
    LZ_TRY(z->bsum.ensure(nblocks));
    if (int rc = scratch_acquire(z, s)) return rc;
    PlanArgs a{d_records, d_sel,     d_count,   n_max,     buffer_id_base, uniform_len,  framed ? 1u : 0u,
               d_buf_offs, d_src_off, d_src_len, d_dst_off, z->bsum.p,      d_total_bytes};
    hipLaunchKernelGGL(lz4_plan_local_kernel, dim3(nblocks), dim3(kPlanBlock), 0, s, a);
    hipLaunchKernelGGL(lz4_plan_scan_kernel, dim3(1), dim3(kPlanBlock), 0, s, z->bsum.p, nblocks, d_total_bytes);
    hipLaunchKernelGGL(lz4_plan_add_kernel, dim3(nblocks), dim3(kPlanBlock), 0, s, a);
    LZ_TRY(hipGetLastError());
    return scratch_release(z, s);
}

int sdfs_cdc_lz4_compress_batch(sdfs_cdc_lz4* z, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                                uint32_t n, uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int framed) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null compressor");
    if (n == 0) return SDFS_CDC_OK;
    if (!base || !offs || !lens || !out || !out_offs || !out_lens)
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(z->mu);
    LZ_TRY(hipSetDevice(z->device));
    // pack the chunks (16-byte aligned) and lay the outputs out back to back
    std::vector<uint64_t> soff(n), doff(n);
    uint64_t in_bytes = 0, out_bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (lens[i] >= (1u << 31)) return fail_status(SDFS_CDC_EINVAL, "chunk %u longer than 2 GiB", i);
        soff[i] = in_bytes;
        in_bytes += (lens[i] + 15ull) & ~15ull;
        doff[i] = out_bytes;
        out_bytes += ((sdfs_cdc_lz4_bound(lens[i]) + (framed ? 4 : 0)) + 15ull) & ~15ull;
    }
    std::vector<uint8_t> packed(in_bytes);
    for (uint32_t i = 0; i < n; i++) memcpy(packed.data() + soff[i], base + offs[i], lens[i]);
    LZ_TRY(z->h_in.ensure(in_bytes + 16));
    LZ_TRY(z->h_out.ensure(out_bytes + 16));
    LZ_TRY(z->h_soff.ensure(n));
    LZ_TRY(z->h_doff.ensure(n));
    LZ_TRY(z->h_slen.ensure(n));
    LZ_TRY(z->h_dlen.ensure(n));
    hipStream_t s = z->stream;
    LZ_TRY(hipMemcpyAsync(z->h_in.p, packed.data(), in_bytes, hipMemcpyHostToDevice, s));
    LZ_TRY(hipMemcpyAsync(z->h_soff.p, soff.data(), n * 8ull, hipMemcpyHostToDevice, s));
    LZ_TRY(hipMemcpyAsync(z->h_doff.p, doff.data(), n * 8ull, hipMemcpyHostToDevice, s));
    LZ_TRY(hipMemcpyAsync(z->h_slen.p, lens, n * 4ull, hipMemcpyHostToDevice, s));
    Lz4Args a{z->h_in.p, z->h_soff.p, z->h_slen.p, nullptr, n, z->h_out.p, z->h_doff.p, z->h_dlen.p,
              framed ? 1u : 0u};
    const int rc = launch_compress(z, a, s);
    if (rc) return rc;
    std::vector<uint8_t> packed_out(out_bytes);
    LZ_TRY(hipMemcpyAsync(packed_out.data(), z->h_out.p, out_bytes, hipMemcpyDeviceToHost, s));
    LZ_TRY(hipMemcpyAsync(out_lens, z->h_dlen.p, n * 4ull, hipMemcpyDeviceToHost, s));
    LZ_TRY(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < n; i++) memcpy(out + out_offs[i], packed_out.data() + doff[i], out_lens[i]);
    return SDFS_CDC_OK;
}

int sdfs_cdc_lz4_compress(sdfs_cdc_lz4* z, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                          uint32_t* out_len) {
    if (!z || !out_len || (n && !src) || !dst) return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (cap < sdfs_cdc_lz4_bound(n))
        return fail_status(SDFS_CDC_ECAP, "cap %u < bound %llu", cap, (unsigned long long)sdfs_cdc_lz4_bound(n));
    const uint64_t off = 0, doff = 0;
    const uint8_t dummy = 0;
    return sdfs_cdc_lz4_compress_batch(z, n ? src : &dummy, &off, &n, 1, dst, &doff, out_len, 0);
}

int sdfs_cdc_lz4_decompress_device(sdfs_cdc_lz4* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                   const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max, uint8_t* d_out,
                                   const uint64_t* d_dst_off, const uint32_t* d_dst_cap, uint32_t* d_dst_len,
                                   int framed, void* stream) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null compressor");
    if (n_max == 0) return SDFS_CDC_OK;
    if (!d_src || !d_src_off || !d_src_len || !d_out || !d_dst_off || !d_dst_cap || !d_dst_len)
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(z->mu);
    LZ_TRY(hipSetDevice(z->device));
    Lz4DecArgs a{d_src, d_src_off, d_src_len, d_count, n_max, d_out, d_dst_off, d_dst_cap, d_dst_len, framed ? 1u : 0u};
    const bool split = z->dec_split >= 0 ? z->dec_split != 0 : n_max >= (uint64_t)z->num_cus * kHybridChunksPerCu;
    if (split) {  // compressible blocks one lane each, then the rest one wave each (same stream)
        a.route = 1;
        const uint64_t lg = std::min<uint64_t>((n_max + 255) / 256, (uint64_t)z->num_cus * z->dec_lane_wg_per_cu);
        hipLaunchKernelGGL(lz4_decompress_lane_kernel, dim3((uint32_t)lg), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        LZ_TRY(hipGetLastError());
        a.route = 2;
    }
    const uint64_t grid = std::min<uint64_t>(n_max, (uint64_t)z->num_cus * z->dec_wg_per_cu);
    if (z->dec_stage == 8192)
        hipLaunchKernelGGL(lz4_decompress_kernel<8192>, dim3((uint32_t)grid), dim3(64), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(lz4_decompress_kernel<kDecStage>, dim3((uint32_t)grid), dim3(64), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
    LZ_TRY(hipGetLastError());
    return SDFS_CDC_OK;
}

int sdfs_cdc_lz4_decompress(sdfs_cdc_lz4* z, const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t dst_len) {
    if (!z || (n && !src) || (dst_len && !dst)) return fail_status(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(z->mu);
    LZ_TRY(hipSetDevice(z->device));
    hipStream_t s = z->stream;
    LZ_TRY(z->h_in.ensure(n + 16));
    LZ_TRY(z->h_out.ensure((uint64_t)dst_len + 16));
    LZ_TRY(z->h_soff.ensure(2));
    LZ_TRY(z->h_slen.ensure(3));
    const uint64_t offs[2] = {0, 0};
    const uint32_t lens[2] = {n, dst_len};
    if (n) LZ_TRY(hipMemcpyAsync(z->h_in.p, src, n, hipMemcpyHostToDevice, s));
    LZ_TRY(hipMemcpyAsync(z->h_soff.p, offs, sizeof(offs), hipMemcpyHostToDevice, s));
    LZ_TRY(hipMemcpyAsync(z->h_slen.p, lens, sizeof(lens), hipMemcpyHostToDevice, s));
    Lz4DecArgs a{z->h_in.p, z->h_soff.p, z->h_slen.p, nullptr, 1, z->h_out.p, z->h_soff.p + 1, z->h_slen.p + 1,
                 z->h_slen.p + 2, 0};
    hipLaunchKernelGGL(lz4_decompress_kernel<kDecStage>, dim3(1), dim3(64), 0, s, a);
    LZ_TRY(hipGetLastError());
    uint32_t got = 0;
    LZ_TRY(hipMemcpyAsync(&got, z->h_slen.p + 2, 4, hipMemcpyDeviceToHost, s));
    LZ_TRY(hipStreamSynchronize(s));
    if (got != dst_len) return fail_status(SDFS_CDC_EINVAL, "malformed LZ4 block (decoded %d of %u bytes)",
                                           got == kLz4Corrupt ? -1 : (int)got, dst_len);
    if (dst_len) {  // on the compressor's own non-blocking stream, not the legacy null stream
        LZ_TRY(hipMemcpyAsync(dst, z->h_out.p, dst_len, hipMemcpyDeviceToHost, s));
        LZ_TRY(hipStreamSynchronize(s));
    }
    return SDFS_CDC_OK;
}

}  // extern "C"
