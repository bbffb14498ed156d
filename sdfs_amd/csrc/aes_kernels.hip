// aes_kernels.hip — AES-CBC of stored chunk records on the MI355X (include/sdfs_aes.h; SURVEY.md
// §8(f) row 4).
//
// Reference: HashBlobArchive.putChunk (HashBlobArchive.java:1280-1294) encrypts each stored record
// [int nz][chunk | LZ4 block] with EncryptUtils.encryptCBC(record, ivspec) (EncryptUtils.java:
// 142-152) = JCE AES/CBC/PKCS5Padding, key = SHA-256(passphrase) (EncryptUtils.java:47-52),
// IV = the archive's (HashBlobArchive.java:91,1028-1032); decryptCBC is the read side
// (HashBlobArchive.java:1923-1925).  oracle/aes_ref.c restates the cipher (FIPS-197, byte form).
//
// MI355X form.  CBC encryption is a serial chain inside a record and independent across
// records, so one LANE encrypts one record (the hash kernel's shape), records scheduled longest
// first so the 64 lanes of a wave finish together.  A round is the 32-bit "T-table" form: 16
// lookups of one 256-word table Te0 (the other three tables are its byte rotations, one
// v_alignbit each), XOR-folded with the round key, which is wave-uniform and lives in the
// kernel arguments (SGPRs).  The table sits in LDS as 32 lane-private copies, word (x, c) at
// byte (x << 7) | (c << 2): lane l reads copy l & 31, so each ds_read_b32 of a 32-lane group
// touches 32 distinct banks whatever the indices (conflict-free; 32 KiB per workgroup, 5
// workgroups per CU).  The last round's S-box bytes are masks of the same Te0 words.
// Decryption of a record is parallel across its 16-byte blocks (P_i = D(C_i) ^ C_{i-1}): one
// wave per record, lanes striding over its blocks, with Td0 and the inverse S-box in LDS the
// same way (64 KiB per workgroup).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/sdfs_aes.h"
#include "cdc_internal.h"
#include "stream_order.h"

namespace sdfs {
namespace {

constexpr int kAesBins = 1024;  // longest-first schedule: bin = min(blocks >> 3, 1023)
constexpr int kAesBinShift = 3;
constexpr int kDecThreads = 256;  // 4 waves = 4 records per workgroup

struct AesEncArgs {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint32_t* count;
    uint64_t n_max;
    const uint32_t* tasks;  // record order, longest first
    uint8_t* out;
    const uint64_t* dst_off;
    uint32_t* dst_len;
    const uint32_t* te0;    // 256 words in global memory (copied into LDS per workgroup)
    const uint8_t* ivs;     // 16 bytes per record, or nullptr
    uint32_t iv[4];         // big-endian words of the shared IV
    uint32_t plen;          // 0 or 4
    uint32_t prefix;        // the big-endian int written before the record (plen == 4)
    uint32_t rk[60];        // encryption round keys, big-endian words
};

struct AesDecArgs {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint32_t* count;
    uint64_t n_max;
    uint8_t* out;
    const uint64_t* dst_off;
    uint32_t* dst_len;
    const uint32_t* td0;    // 256 words
    const uint32_t* isb;    // inverse S-box, 256 words
    const uint8_t* ivs;
    uint32_t iv[4];
    uint32_t dk[60];        // equivalent-inverse-cipher round keys (FIPS-197 §5.3.5), in use order
};

struct AesPlanArgs {
    const uint32_t* src_len;
    const uint32_t* count;
    uint64_t n_max;
    uint32_t plen;
    uint32_t* hist;    // [kAesBins]
    uint32_t* cursor;  // [kAesBins]
    uint32_t* tasks;   // [n_max]
};

__device__ __forceinline__ uint64_t rec_count(const uint32_t* count, uint64_t n_max) {
    return count ? std::min<uint64_t>(*count, n_max) : n_max;
}

__device__ __forceinline__ uint32_t ror(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }

// Table layouts.  COPIES = 32: word (x, c) at byte (x << 7) | (c << 2), lane l reads copy l & 31
// (32 KiB; index = v_bfe + v_lshl_or).  COPIES = 64: word (x, c) at byte (x << 8) | (c << 2), lane l
// reads copy l (64 KiB; the byte address is ONE v_perm_b32 of the state word and the lane's
// offset).  Either way the 32 lanes of a ds_read_b32 group hit 32 distinct banks.
template <int COPIES>
struct Tab {
    static constexpr uint32_t kWords = 256 * COPIES;
    const uint32_t* lds;
    uint32_t l4;  // this lane's copy offset in bytes
    __device__ __forceinline__ uint32_t at(uint32_t addr) const {
        return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + addr);
    }
    // table word indexed by byte K (0 = least significant) of s
    template <int K>
    __device__ __forceinline__ uint32_t get(uint32_t s) const {
        if constexpr (COPIES == 64)
            return at(__builtin_amdgcn_perm(s, l4, 0x0C0C0000u | ((4u + K) << 8)));
        else
            return at((((s >> (8 * K)) & 255u) << 7) | l4);
    }
};

template <int COPIES>
__device__ __forceinline__ void fill_table(uint32_t* lds, const uint32_t* g, uint32_t nthreads) {
    for (uint32_t i = threadIdx.x; i < 256u * COPIES; i += nthreads) lds[i] = g[i / COPIES];
}



template <int COPIES>
__device__ __forceinline__ uint32_t lane_off() {
    return (threadIdx.x & (COPIES - 1)) << 2;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 has no v_xor3_b32
}

__device__ __forceinline__ uint32_t aes_blocks(uint32_t len, uint32_t plen) { return (len + plen) / 16 + 1; }

__device__ __forceinline__ uint32_t enc_bin(uint32_t len, uint32_t plen) {
    const uint32_t b = aes_blocks(len, plen) >> kAesBinShift;
    return b < kAesBins ? b : kAesBins - 1;
}

// Te0[x] = S[x] * {02, 01, 01, 03} (most significant byte first); Te1..3 = ror 8, 16, 24.
template <int NR, int COPIES>
__device__ __forceinline__ void aes_encrypt(uint32_t (&s)[4], const Tab<COPIES>& T, const uint32_t* rk) {
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return xor3(xor3(T.template get<3>(a), ror(T.template get<2>(b), 8), ror(T.template get<1>(c), 16)),
                    ror(T.template get<0>(d), 24), k);
    };
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = col(s0, s1, s2, s3, rk[4 * r]);
        const uint32_t t1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
        const uint32_t t2 = col(s2, s3, s0, s1, rk[4 * r + 2]);
        const uint32_t t3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // last round: S[x] sits in bytes 2 and 1 of Te0[x]
    auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return xor3(xor3((T.template get<3>(a) << 8) & 0xFF000000u, T.template get<2>(b) & 0x00FF0000u,
                         T.template get<1>(c) & 0x0000FF00u),
                    (T.template get<0>(d) >> 8) & 0xFFu, k);
    };
    s[0] = fin(s0, s1, s2, s3, rk[4 * NR]);
    s[1] = fin(s1, s2, s3, s0, rk[4 * NR + 1]);
    s[2] = fin(s2, s3, s0, s1, rk[4 * NR + 2]);
    s[3] = fin(s3, s0, s1, s2, rk[4 * NR + 3]);
}

// Td0[x] = IS[x] * {0e, 09, 0d, 0b}; isb[x] = IS[x].  dk = round keys in use order.
template <int NR, int COPIES>
__device__ __forceinline__ void aes_decrypt(uint32_t (&s)[4], const Tab<COPIES>& D, const Tab<COPIES>& I,
                                            const uint32_t* dk) {
    uint32_t s0 = s[0] ^ dk[0], s1 = s[1] ^ dk[1], s2 = s[2] ^ dk[2], s3 = s[3] ^ dk[3];
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return xor3(xor3(D.template get<3>(a), ror(D.template get<2>(b), 8), ror(D.template get<1>(c), 16)),
                    ror(D.template get<0>(d), 24), k);
    };
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = col(s0, s3, s2, s1, dk[4 * r]);
        const uint32_t t1 = col(s1, s0, s3, s2, dk[4 * r + 1]);
        const uint32_t t2 = col(s2, s1, s0, s3, dk[4 * r + 2]);
        const uint32_t t3 = col(s3, s2, s1, s0, dk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return xor3(xor3(I.template get<3>(a) << 24, I.template get<2>(b) << 16, I.template get<1>(c) << 8),
                    I.template get<0>(d), k);
    };
    s[0] = fin(s0, s3, s2, s1, dk[4 * NR]);
    s[1] = fin(s1, s0, s3, s2, dk[4 * NR + 1]);
    s[2] = fin(s2, s1, s0, s3, dk[4 * NR + 2]);
    s[3] = fin(s3, s2, s1, s0, dk[4 * NR + 3]);
}

__device__ __forceinline__ void load_be(uint32_t (&s)[4], const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // unaligned global_load_dwordx4
    s[0] = __builtin_bswap32(v.x);
    s[1] = __builtin_bswap32(v.y);
    s[2] = __builtin_bswap32(v.z);
    s[3] = __builtin_bswap32(v.w);
}

__device__ __forceinline__ void store_be(uint8_t* p, const uint32_t (&s)[4]) {
    const uint4 v = make_uint4(__builtin_bswap32(s[0]), __builtin_bswap32(s[1]), __builtin_bswap32(s[2]),
                               __builtin_bswap32(s[3]));
    __builtin_memcpy(p, &v, 16);
}

// Block `blk` of the virtual record [prefix: plen bytes][src: len bytes][PKCS#5 padding] assembled
// byte by byte (the first block when plen != 0 and the padded last block: once per record).
__device__ __forceinline__ void gather_block(uint32_t (&s)[4], const uint8_t* p, uint32_t len, uint32_t plen,
                                             uint32_t prefix, uint32_t blk) {
    const uint32_t tot = len + plen;
    const uint32_t pad = 16 - (tot & 15);  // only the last block holds padding
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t k = 16 * blk + 4 * w + j;
            uint32_t b;
            if (k < plen)
                b = (prefix >> (24 - 8 * k)) & 255u;
            else if (k < tot)
                b = p[k - plen];
            else
                b = pad;
            word = (word << 8) | b;
        }
        s[w] = word;
    }
}

template <int NR, int COPIES, int THREADS>
__global__ __launch_bounds__(THREADS) void aes_cbc_encrypt_kernel(AesEncArgs a) {
    __shared__ uint32_t lte[256 * COPIES];
    fill_table<COPIES>(lte, a.te0, THREADS);
    __syncthreads();
    const Tab<COPIES> T{lte, lane_off<COPIES>()};
    const uint64_t n = rec_count(a.count, a.n_max);
    const uint64_t i = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = a.tasks ? a.tasks[i] : (uint32_t)i;
    const uint8_t* p = a.src + a.src_off[r];
    const uint32_t len = a.src_len[r];
    const uint32_t plen = a.plen;
    uint8_t* o = a.out + a.dst_off[r];
    const uint32_t nfull = (len + plen) >> 4;  // whole plaintext blocks before the padded one
    uint32_t c[4];
    if (a.ivs) {
        load_be(c, a.ivs + 16ull * r);
    } else {
        c[0] = a.iv[0]; c[1] = a.iv[1]; c[2] = a.iv[2]; c[3] = a.iv[3];
    }
    uint32_t nx[4];
    if (nfull) {
        if (plen)
            gather_block(nx, p, len, plen, a.prefix, 0);
        else
            load_be(nx, p);
    }
    for (uint32_t b = 0; b < nfull; b++) {
        uint32_t s[4] = {nx[0] ^ c[0], nx[1] ^ c[1], nx[2] ^ c[2], nx[3] ^ c[3]};
        // next whole block (blocks >= 1 are plain loads at p + 16b - plen), clamped in bounds
        const uint32_t bn = b + 1 < nfull ? b + 1 : b;
        if (bn >= 1) load_be(nx, p + 16ull * bn - plen);
        aes_encrypt<NR>(s, T, a.rk);
        store_be(o + 16ull * b, s);
        c[0] = s[0]; c[1] = s[1]; c[2] = s[2]; c[3] = s[3];
    }
    uint32_t s[4];
    gather_block(s, p, len, plen, a.prefix, nfull);
    s[0] ^= c[0]; s[1] ^= c[1]; s[2] ^= c[2]; s[3] ^= c[3];
    aes_encrypt<NR>(s, T, a.rk);
    store_be(o + 16ull * nfull, s);
    a.dst_len[r] = 16 * (nfull + 1);
}

template <int NR>
__global__ __launch_bounds__(kDecThreads) void aes_cbc_decrypt_kernel(AesDecArgs a) {
    __shared__ uint32_t ltd[256 * 32];
    __shared__ uint32_t lis[256 * 32];
    fill_table<32>(ltd, a.td0, kDecThreads);
    fill_table<32>(lis, a.isb, kDecThreads);
    __syncthreads();
    const Tab<32> D{ltd, lane_off<32>()}, I{lis, lane_off<32>()};
    const uint64_t n = rec_count(a.count, a.n_max);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kDecThreads / 64);
    for (uint64_t r = (uint64_t)blockIdx.x * (kDecThreads / 64) + threadIdx.x / 64; r < n; r += waves) {
        const uint32_t len = a.src_len[r];
        const uint8_t* p = a.src + a.src_off[r];
        uint8_t* o = a.out + a.dst_off[r];
        if (len == 0 || (len & 15)) {
            if (lane == 0) a.dst_len[r] = 0xFFFFFFFFu;
            continue;
        }
        const uint32_t nb = len >> 4;
        uint32_t iv[4];
        if (a.ivs) {
            load_be(iv, a.ivs + 16ull * r);
        } else {
            iv[0] = a.iv[0]; iv[1] = a.iv[1]; iv[2] = a.iv[2]; iv[3] = a.iv[3];
        }
        for (uint32_t b = lane; b < nb; b += 64) {
            uint32_t s[4], prev[4];
            load_be(s, p + 16ull * b);
            if (b) {
                load_be(prev, p + 16ull * (b - 1));
            } else {
                prev[0] = iv[0]; prev[1] = iv[1]; prev[2] = iv[2]; prev[3] = iv[3];
            }
            aes_decrypt<NR>(s, D, I, a.dk);
            s[0] ^= prev[0]; s[1] ^= prev[1]; s[2] ^= prev[2]; s[3] ^= prev[3];
            if (b + 1 < nb) {
                store_be(o + 16ull * b, s);
            } else {
                // PKCS#5: the last byte v in 1..16 and the last v bytes all equal v
                const uint32_t v = s[3] & 255u;
                bool ok = v >= 1 && v <= 16;
#pragma unroll
                for (int j = 0; j < 16; j++)
                    if ((uint32_t)j >= 16 - v && ((s[j >> 2] >> (24 - 8 * (j & 3))) & 255u) != v) ok = false;
                if (ok) {
#pragma unroll
                    for (int j = 0; j < 16; j++)
                        if ((uint32_t)j < 16 - v) o[16ull * b + j] = (uint8_t)(s[j >> 2] >> (24 - 8 * (j & 3)));
                }
                a.dst_len[r] = ok ? len - v : 0xFFFFFFFFu;
            }
        }
    }
}

// ---- quad form: one record per 4 lanes (lane q of the quad owns state column q)
// A single lane's CBC chain is a serial ~700-instruction block at 4 cycles per wave64 VALU
// instruction, so the longest record of a batch (2 k blocks at maxLen 32 KiB) sets the kernel's
// floor.  Splitting the block's 4 columns over a lane quad cuts that chain ~3.5x: per round a lane
// fetches its 3 neighbours' columns with DPP quad permutes and does 4 lookups instead of 16.
template <uint32_t CTRL>
__device__ __forceinline__ uint32_t quad_mov(uint32_t v) {
    // mov_dpp (undefined "old"): every lane is written (row/bank masks full), so no zero-init
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr uint32_t kQuadNext1 = 0x39;  // quad_perm [1,2,3,0]: column q+1
constexpr uint32_t kQuadNext2 = 0x4E;  // [2,3,0,1]: column q+2
constexpr uint32_t kQuadNext3 = 0x93;  // [3,0,1,2]: column q+3

template <int NR, int COPIES>
__device__ __forceinline__ uint32_t aes_encrypt_quad(uint32_t s, const Tab<COPIES>& T, const uint32_t (&k)[NR + 1]) {
    s ^= k[0];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t s1 = quad_mov<kQuadNext1>(s), s2 = quad_mov<kQuadNext2>(s), s3 = quad_mov<kQuadNext3>(s);
        s = xor3(xor3(T.template get<3>(s), ror(T.template get<2>(s1), 8), ror(T.template get<1>(s2), 16)),
                 ror(T.template get<0>(s3), 24), k[r]);
    }
    const uint32_t s1 = quad_mov<kQuadNext1>(s), s2 = quad_mov<kQuadNext2>(s), s3 = quad_mov<kQuadNext3>(s);
    return xor3(xor3((T.template get<3>(s) << 8) & 0xFF000000u, T.template get<2>(s1) & 0x00FF0000u,
                     T.template get<1>(s2) & 0x0000FF00u),
                (T.template get<0>(s3) >> 8) & 0xFFu, k[NR]);
}

// big-endian word q of block blk of the virtual record [prefix][src][padding], byte by byte
__device__ __forceinline__ uint32_t gather_word(const uint8_t* p, uint32_t len, uint32_t plen, uint32_t prefix,
                                                uint32_t blk, uint32_t q) {
    const uint32_t tot = len + plen, pad = 16 - (tot & 15);
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t k = 16 * blk + 4 * q + j;
        uint32_t b;
        if (k < plen)
            b = (prefix >> (24 - 8 * k)) & 255u;
        else if (k < tot)
            b = p[k - plen];
        else
            b = pad;
        word = (word << 8) | b;
    }
    return word;
}

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);  // unaligned global_load_dword
    return __builtin_bswap32(v);
}

// PRIO: waves whose records are long raise their issue priority, so the longest serial chains
// (which set the kernel's floor) are not slowed by the short-record waves sharing their SIMD.
template <int NR, int COPIES, int THREADS, bool PRIO = false>
__global__ __launch_bounds__(THREADS) void aes_cbc_encrypt_quad_kernel(AesEncArgs a) {
    __shared__ uint32_t lte[256 * COPIES];
    fill_table<COPIES>(lte, a.te0, THREADS);
    __syncthreads();
    const Tab<COPIES> T{lte, lane_off<COPIES>()};
    const uint64_t n = rec_count(a.count, a.n_max);
    const uint64_t i = ((uint64_t)blockIdx.x * THREADS + threadIdx.x) >> 2;  // whole quads exit together
    if (i >= n) return;
    const uint32_t q = threadIdx.x & 3;
    uint32_t k[NR + 1];
#pragma unroll
    for (int r = 0; r <= NR; r++)
        k[r] = q == 0 ? a.rk[4 * r] : q == 1 ? a.rk[4 * r + 1] : q == 2 ? a.rk[4 * r + 2] : a.rk[4 * r + 3];
    const uint32_t r = a.tasks ? a.tasks[i] : (uint32_t)i;
    const uint8_t* p = a.src + a.src_off[r];
    const uint32_t len = a.src_len[r];
    const uint32_t plen = a.plen;
    uint8_t* o = a.out + a.dst_off[r];
    const uint32_t nfull = (len + plen) >> 4;
    if constexpr (PRIO) {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(nfull);
        if (nb > 1536)
            __builtin_amdgcn_s_setprio(3);
        else if (nb > 1024)
            __builtin_amdgcn_s_setprio(2);
        else if (nb > 512)
            __builtin_amdgcn_s_setprio(1);
    }
    uint32_t c = a.ivs ? load_be32(a.ivs + 16ull * r + 4 * q)
                       : (q == 0 ? a.iv[0] : q == 1 ? a.iv[1] : q == 2 ? a.iv[2] : a.iv[3]);
    uint32_t nx = 0;
    if (nfull) nx = plen ? gather_word(p, len, plen, a.prefix, 0, q) : load_be32(p + 4 * q);
    for (uint32_t b = 0; b < nfull; b++) {
        const uint32_t x = nx ^ c;
        const uint32_t bn = b + 1 < nfull ? b + 1 : b;
        if (bn >= 1) nx = load_be32(p + 16ull * bn + 4 * q - plen);
        c = aes_encrypt_quad<NR>(x, T, k);
        const uint32_t be = __builtin_bswap32(c);
        __builtin_memcpy(o + 16ull * b + 4 * q, &be, 4);
    }
    c = aes_encrypt_quad<NR>(gather_word(p, len, plen, a.prefix, nfull, q) ^ c, T, k);
    const uint32_t be = __builtin_bswap32(c);
    __builtin_memcpy(o + 16ull * nfull + 4 * q, &be, 4);
    if (q == 0) a.dst_len[r] = 16 * (nfull + 1);
}

// ---- longest-first schedule (histogram of block counts, descending prefix, scatter)
__global__ __launch_bounds__(256) void aes_hist_kernel(AesPlanArgs a) {
    __shared__ uint32_t lh[kAesBins];
    for (uint32_t k = threadIdx.x; k < kAesBins; k += 256) lh[k] = 0;
    __syncthreads();
    const uint64_t n = rec_count(a.count, a.n_max);
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) atomicAdd(&lh[enc_bin(a.src_len[i], a.plen)], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kAesBins; k += 256)
        if (lh[k]) atomicAdd(&a.hist[k], lh[k]);
}

__global__ __launch_bounds__(kAesBins) void aes_cursor_kernel(AesPlanArgs a) {
    __shared__ uint32_t part[kAesBins];
    const uint32_t t = threadIdx.x;
    part[t] = a.hist[kAesBins - 1 - t];  // longest bin first
    __syncthreads();
    for (uint32_t d = 1; d < kAesBins; d <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    a.cursor[kAesBins - 1 - t] = part[t] - a.hist[kAesBins - 1 - t];
}

__global__ __launch_bounds__(256) void aes_scatter_kernel(AesPlanArgs a) {
    __shared__ uint32_t lc[kAesBins];
    __shared__ uint32_t lb[kAesBins];
    for (uint32_t k = threadIdx.x; k < kAesBins; k += 256) lc[k] = 0;
    __syncthreads();
    const uint64_t n = rec_count(a.count, a.n_max);
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t bin = 0, rank = 0;
    if (i < n) {
        bin = enc_bin(a.src_len[i], a.plen);
        rank = atomicAdd(&lc[bin], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kAesBins; k += 256)
        if (lc[k]) lb[k] = atomicAdd(&a.cursor[k], lc[k]);
    __syncthreads();
    if (i < n) a.tasks[lb[bin] + rank] = (uint32_t)i;
}

// ---- host-side tables and key schedule (FIPS-197 §5.1.1, §5.2, §5.3.5)
uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (; b; b >>= 1) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0));
    }
    return r;
}

struct AesTables {
    uint8_t sbox[256], isbox[256];
    uint32_t te0[256], td0[256], isb[256];
    AesTables() {
        // multiplicative inverses from a generator walk (3 generates GF(2^8)*): inv(3^k) = 3^(255-k)
        uint8_t pw[255];
        uint8_t x = 1;
        for (int k = 0; k < 255; k++) {
            pw[k] = x;
            x = gf_mul(x, 3);
        }
        uint8_t inv[256] = {0};
        for (int k = 0; k < 255; k++) inv[pw[k]] = pw[(255 - k) % 255];
        for (int v = 0; v < 256; v++) {
            const uint8_t b = inv[v];
            // affine map: b ^ rotl(b,1) ^ rotl(b,2) ^ rotl(b,3) ^ rotl(b,4) ^ 0x63
            uint8_t s = b;
            for (int k = 1; k <= 4; k++) s ^= (uint8_t)((b << k) | (b >> (8 - k)));
            s ^= 0x63;
            sbox[v] = s;
            isbox[s] = (uint8_t)v;
        }
        for (int v = 0; v < 256; v++) {
            const uint8_t s = sbox[v], is = isbox[v];
            te0[v] = (uint32_t)gf_mul(s, 2) << 24 | (uint32_t)s << 16 | (uint32_t)s << 8 | gf_mul(s, 3);
            td0[v] = (uint32_t)gf_mul(is, 14) << 24 | (uint32_t)gf_mul(is, 9) << 16 | (uint32_t)gf_mul(is, 13) << 8 |
                     gf_mul(is, 11);
            isb[v] = is;
        }
    }
};

const AesTables& tables() {
    static const AesTables t;
    return t;
}

uint32_t sub_word(uint32_t w) {
    const uint8_t* s = tables().sbox;
    return (uint32_t)s[w >> 24] << 24 | (uint32_t)s[(w >> 16) & 255] << 16 | (uint32_t)s[(w >> 8) & 255] << 8 |
           s[w & 255];
}

int expand_key(const uint8_t* key, uint32_t key_len, uint32_t rk[60]) {
    const int nk = (int)key_len / 4, nr = nk + 6;
    for (int i = 0; i < nk; i++)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 |
                key[4 * i + 3];
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = sub_word((t << 8) | (t >> 24)) ^ ((uint32_t)rcon << 24);
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = sub_word(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

uint32_t inv_mix_word(uint32_t w) {
    const uint8_t a0 = w >> 24, a1 = w >> 16, a2 = w >> 8, a3 = (uint8_t)w;
    const uint8_t b0 = gf_mul(a0, 14) ^ gf_mul(a1, 11) ^ gf_mul(a2, 13) ^ gf_mul(a3, 9);
    const uint8_t b1 = gf_mul(a0, 9) ^ gf_mul(a1, 14) ^ gf_mul(a2, 11) ^ gf_mul(a3, 13);
    const uint8_t b2 = gf_mul(a0, 13) ^ gf_mul(a1, 9) ^ gf_mul(a2, 14) ^ gf_mul(a3, 11);
    const uint8_t b3 = gf_mul(a0, 11) ^ gf_mul(a1, 13) ^ gf_mul(a2, 9) ^ gf_mul(a3, 14);
    return (uint32_t)b0 << 24 | (uint32_t)b1 << 16 | (uint32_t)b2 << 8 | b3;
}

template <typename T>
struct ABuf {
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

struct sdfs_cdc_aes {
    int device = 0;
    int nr = 14;
    int num_cus = 256;
    int enc_variant = 7;  // quad form, 64 table copies, priority (SDFS_AES_VARIANT for A/B)
    uint32_t rk[60];
    uint32_t dk[60];
    hipStream_t stream = nullptr;
    ABuf<uint32_t> tabs;    // te0 | td0 | isb (3 x 256 words)
    ABuf<uint32_t> plan;    // hist | cursor
    ABuf<uint32_t> tasks;
    ABuf<uint8_t> h_in, h_out;
    ABuf<uint64_t> h_soff, h_doff;
    ABuf<uint32_t> h_slen, h_dlen;
    StreamOrder order;  // encryptions share plan/tasks: ordered across caller streams
    std::mutex mu;
};

#define AES_TRY(expr)                                                                                 \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return fail_status(SDFS_CDC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                               __FILE__, __LINE__);                                                   \
    } while (0)

namespace {

template <int NR, int COPIES, int THREADS>
void launch_enc(uint64_t n_max, const AesEncArgs& a, hipStream_t s) {
    const uint32_t g = (uint32_t)((n_max + THREADS - 1) / THREADS);
    hipLaunchKernelGGL((aes_cbc_encrypt_kernel<NR, COPIES, THREADS>), dim3(g), dim3(THREADS), 0, s, a);
}

template <int NR, int COPIES, int THREADS, bool PRIO = false>
void launch_enc_quad(uint64_t n_max, const AesEncArgs& a, hipStream_t s) {
    const uint32_t g = (uint32_t)((4 * n_max + THREADS - 1) / THREADS);
    hipLaunchKernelGGL((aes_cbc_encrypt_quad_kernel<NR, COPIES, THREADS, PRIO>), dim3(g), dim3(THREADS), 0, s, a);
}

// variant 0: one lane per record, 32 table copies (32 KiB), 256-thread workgroups (5 per CU);
// 3: the quad form (4 lanes per record), 64 copies with the one-v_perm index; 6: quad, 32 copies,
// issue priority; 7 (production): quad, 64 copies, priority.  Measured and dropped (DESIGN.md
// §13): 64 copies per lane (256 / 512 threads), quad with 512 / 1024 threads, four rotated tables.
template <int NR>
void launch_encrypt_nr(int variant, uint64_t n_max, const AesEncArgs& a, hipStream_t s) {
    if (variant == 0)
        launch_enc<NR, 32, 256>(n_max, a, s);
    else if (variant == 3)
        launch_enc_quad<NR, 64, 256>(n_max, a, s);
    else if (variant == 6)
        launch_enc_quad<NR, 32, 256, true>(n_max, a, s);
    else
        launch_enc_quad<NR, 64, 256, true>(n_max, a, s);
}

void launch_encrypt(int nr, int variant, uint64_t n_max, const AesEncArgs& a, hipStream_t s) {
    if (nr == 10)
        launch_encrypt_nr<10>(variant, n_max, a, s);
    else if (nr == 12)
        launch_encrypt_nr<12>(variant, n_max, a, s);
    else
        launch_encrypt_nr<14>(variant, n_max, a, s);
}

void iv_words(const uint8_t* iv, uint32_t (&w)[4]) {
    for (int k = 0; k < 4; k++)
        w[k] = iv ? (uint32_t)iv[4 * k] << 24 | (uint32_t)iv[4 * k + 1] << 16 | (uint32_t)iv[4 * k + 2] << 8 |
                        iv[4 * k + 3]
                  : 0u;
}

int encrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off, const uint32_t* d_src_len,
                   const uint32_t* d_count, uint64_t n_max, int plen, int32_t nz_prefix, const uint8_t* iv,
                   const uint8_t* d_ivs, uint8_t* d_out, const uint64_t* d_dst_off, uint32_t* d_dst_len,
                   hipStream_t s) {
    if (plen != 0 && plen != 4) return fail_status(SDFS_CDC_EINVAL, "plen must be 0 or 4, got %d", plen);
    if (!iv && !d_ivs) return fail_status(SDFS_CDC_EINVAL, "an IV is required");
    if (n_max == 0) return SDFS_CDC_OK;
    if (!d_src || !d_src_off || !d_src_len || !d_out || !d_dst_off || !d_dst_len)
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (n_max >= (1ull << 32)) return fail_status(SDFS_CDC_EINVAL, "more than 2^32 records");
    AES_TRY(z->plan.ensure(2 * kAesBins));
    AES_TRY(z->tasks.ensure(n_max));
    AES_TRY(z->order.acquire(s));
    AesPlanArgs pa{d_src_len, d_count, n_max, (uint32_t)plen, z->plan.p, z->plan.p + kAesBins, z->tasks.p};
    const uint32_t g = (uint32_t)((n_max + 255) / 256);
    AES_TRY(hipMemsetAsync(z->plan.p, 0, kAesBins * sizeof(uint32_t), s));
    hipLaunchKernelGGL(aes_hist_kernel, dim3(g), dim3(256), 0, s, pa);
    hipLaunchKernelGGL(aes_cursor_kernel, dim3(1), dim3(kAesBins), 0, s, pa);
    hipLaunchKernelGGL(aes_scatter_kernel, dim3(g), dim3(256), 0, s, pa);
    AesEncArgs a{};
    a.src = d_src; a.src_off = d_src_off; a.src_len = d_src_len; a.count = d_count; a.n_max = n_max;
    a.tasks = z->tasks.p; a.out = d_out; a.dst_off = d_dst_off; a.dst_len = d_dst_len;
    a.te0 = z->tabs.p; a.ivs = d_ivs; a.plen = (uint32_t)plen; a.prefix = (uint32_t)nz_prefix;
    iv_words(iv, a.iv);
    memcpy(a.rk, z->rk, sizeof(a.rk));
    launch_encrypt(z->nr, z->enc_variant, n_max, a, s);
    AES_TRY(hipGetLastError());
    AES_TRY(z->order.release(s));
    return SDFS_CDC_OK;
}

int decrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off, const uint32_t* d_src_len,
                   const uint32_t* d_count, uint64_t n_max, const uint8_t* iv, const uint8_t* d_ivs, uint8_t* d_out,
                   const uint64_t* d_dst_off, uint32_t* d_dst_len, hipStream_t s) {
    if (!iv && !d_ivs) return fail_status(SDFS_CDC_EINVAL, "an IV is required");
    if (n_max == 0) return SDFS_CDC_OK;
    if (!d_src || !d_src_off || !d_src_len || !d_out || !d_dst_off || !d_dst_len)
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    AesDecArgs a{};
    a.src = d_src; a.src_off = d_src_off; a.src_len = d_src_len; a.count = d_count; a.n_max = n_max;
    a.out = d_out; a.dst_off = d_dst_off; a.dst_len = d_dst_len;
    a.td0 = z->tabs.p + 256; a.isb = z->tabs.p + 512; a.ivs = d_ivs;
    iv_words(iv, a.iv);
    memcpy(a.dk, z->dk, sizeof(a.dk));
    const uint64_t want = (n_max + 3) / 4;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)z->num_cus * 8);
    switch (z->nr) {
    case 10: hipLaunchKernelGGL(aes_cbc_decrypt_kernel<10>, dim3(grid), dim3(kDecThreads), 0, s, a); break;
    case 12: hipLaunchKernelGGL(aes_cbc_decrypt_kernel<12>, dim3(grid), dim3(kDecThreads), 0, s, a); break;
    default: hipLaunchKernelGGL(aes_cbc_decrypt_kernel<14>, dim3(grid), dim3(kDecThreads), 0, s, a); break;
    }
    AES_TRY(hipGetLastError());
    return SDFS_CDC_OK;
}

// Host records packed 16-byte aligned into the device scratch, processed, copied back.
int host_batch(sdfs_cdc_aes* z, bool enc, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
               int plen, int32_t nz_prefix, const uint8_t* iv, uint8_t* out, const uint64_t* out_offs,
               uint32_t* out_lens) {
    std::vector<uint64_t> soff(n), doff(n);
    uint64_t in_bytes = 0, out_bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (lens[i] >= (1u << 31) - 32) return fail_status(SDFS_CDC_EINVAL, "record %u longer than 2 GiB", i);
        soff[i] = in_bytes;
        in_bytes += (lens[i] + 15ull) & ~15ull;
        doff[i] = out_bytes;
        out_bytes += enc ? sdfs_cdc_aes_cbc_bound((uint64_t)lens[i] + (uint64_t)plen) : ((lens[i] + 15ull) & ~15ull);
    }
    std::vector<uint8_t> packed(in_bytes);
    for (uint32_t i = 0; i < n; i++) memcpy(packed.data() + soff[i], base + offs[i], lens[i]);
    AES_TRY(z->h_in.ensure(in_bytes + 16));
    AES_TRY(z->h_out.ensure(out_bytes + 16));
    AES_TRY(z->h_soff.ensure(n));
    AES_TRY(z->h_doff.ensure(n));
    AES_TRY(z->h_slen.ensure(n));
    AES_TRY(z->h_dlen.ensure(n));
    hipStream_t s = z->stream;
    AES_TRY(hipMemcpyAsync(z->h_in.p, packed.data(), in_bytes, hipMemcpyHostToDevice, s));
    AES_TRY(hipMemcpyAsync(z->h_soff.p, soff.data(), n * 8ull, hipMemcpyHostToDevice, s));
    AES_TRY(hipMemcpyAsync(z->h_doff.p, doff.data(), n * 8ull, hipMemcpyHostToDevice, s));
    AES_TRY(hipMemcpyAsync(z->h_slen.p, lens, n * 4ull, hipMemcpyHostToDevice, s));
    const int rc = enc ? encrypt_device(z, z->h_in.p, z->h_soff.p, z->h_slen.p, nullptr, n, plen, nz_prefix, iv,
                                        nullptr, z->h_out.p, z->h_doff.p, z->h_dlen.p, s)
                       : decrypt_device(z, z->h_in.p, z->h_soff.p, z->h_slen.p, nullptr, n, iv, nullptr, z->h_out.p,
                                        z->h_doff.p, z->h_dlen.p, s);
    if (rc) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    std::vector<uint8_t> packed_out(out_bytes);
    AES_TRY(hipMemcpyAsync(packed_out.data(), z->h_out.p, out_bytes, hipMemcpyDeviceToHost, s));
    AES_TRY(hipMemcpyAsync(out_lens, z->h_dlen.p, n * 4ull, hipMemcpyDeviceToHost, s));
    AES_TRY(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < n; i++)
        if (out_lens[i] != 0xFFFFFFFFu) memcpy(out + out_offs[i], packed_out.data() + doff[i], out_lens[i]);
    return SDFS_CDC_OK;
}

}  // namespace

extern "C" {

uint64_t sdfs_cdc_aes_cbc_bound(uint64_t n) { return (n / 16 + 1) * 16; }

int sdfs_cdc_aes_create(int device, const uint8_t* key, uint32_t key_len, sdfs_cdc_aes** out) {
    if (!out) return fail_status(SDFS_CDC_EINVAL, "null output");
    *out = nullptr;
    if (!key || (key_len != 16 && key_len != 24 && key_len != 32))
        return fail_status(SDFS_CDC_EINVAL, "AES key must be 16, 24 or 32 bytes (got %u)", key_len);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail_status(SDFS_CDC_ENODEV, "no HIP device %d", device);
    AES_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    AES_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail_status(SDFS_CDC_ENODEV, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    auto* z = new sdfs_cdc_aes();
    z->device = device;
    z->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
#ifdef SDFS_TUNING
    if (const char* v = getenv("SDFS_AES_VARIANT")) z->enc_variant = atoi(v);  // A/B (tuning library only)
#endif
    z->nr = expand_key(key, key_len, z->rk);
    // equivalent inverse cipher: keys in use order, InvMixColumns on the middle rounds
    for (int r = 0; r <= z->nr; r++)
        for (int c = 0; c < 4; c++) {
            const uint32_t w = z->rk[4 * (z->nr - r) + c];
            z->dk[4 * r + c] = (r == 0 || r == z->nr) ? w : inv_mix_word(w);
        }
    const AesTables& t = tables();
    std::vector<uint32_t> img(768);
    memcpy(img.data(), t.te0, 1024);
    memcpy(img.data() + 256, t.td0, 1024);
    memcpy(img.data() + 512, t.isb, 1024);
    // the upload runs on the component's own non-blocking stream, never the legacy null stream
    // (which would wait for the CDC queue's blocking lane streams)
    if (z->tabs.ensure(768) != hipSuccess ||
        hipStreamCreateWithFlags(&z->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMemcpyAsync(z->tabs.p, img.data(), 768 * 4, hipMemcpyHostToDevice, z->stream) != hipSuccess ||
        hipStreamSynchronize(z->stream) != hipSuccess || z->order.init() != hipSuccess) {
        z->tabs.release();
        if (z->stream) (void)hipStreamDestroy(z->stream);
        delete z;
        return fail_status(SDFS_CDC_EHIP, "AES table upload or stream creation failed");
    }
    *out = z;
    return SDFS_CDC_OK;
}

int sdfs_cdc_aes_destroy(sdfs_cdc_aes* z) {
    if (!z) return SDFS_CDC_OK;
    {
        std::lock_guard<std::mutex> lk(z->mu);
        (void)hipSetDevice(z->device);
        if (z->stream) (void)hipStreamSynchronize(z->stream);
        z->tabs.release();
        z->plan.release();
        z->tasks.release();
        z->h_in.release();
        z->h_out.release();
        z->h_soff.release();
        z->h_doff.release();
        z->h_slen.release();
        z->h_dlen.release();
        if (z->stream) (void)hipStreamDestroy(z->stream);
        z->order.destroy();
        memset(z->rk, 0, sizeof(z->rk));
        memset(z->dk, 0, sizeof(z->dk));
    }
    delete z;
    return SDFS_CDC_OK;
}

int sdfs_cdc_aes_encrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max, int plen,
                                int32_t nz_prefix, const uint8_t* iv, const uint8_t* d_ivs, uint8_t* d_out,
                                const uint64_t* d_dst_off, uint32_t* d_dst_len, void* stream) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null cipher");
    std::lock_guard<std::mutex> lk(z->mu);
    AES_TRY(hipSetDevice(z->device));
    return encrypt_device(z, d_src, d_src_off, d_src_len, d_count, n_max, plen, nz_prefix, iv, d_ivs, d_out,
                          d_dst_off, d_dst_len, reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_aes_decrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max,
                                const uint8_t* iv, const uint8_t* d_ivs, uint8_t* d_out, const uint64_t* d_dst_off,
                                uint32_t* d_dst_len, void* stream) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null cipher");
    std::lock_guard<std::mutex> lk(z->mu);
    AES_TRY(hipSetDevice(z->device));
    return decrypt_device(z, d_src, d_src_off, d_src_len, d_count, n_max, iv, d_ivs, d_out, d_dst_off, d_dst_len,
                          reinterpret_cast<hipStream_t>(stream));
}

int sdfs_cdc_aes_encrypt_batch(sdfs_cdc_aes* z, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                               uint32_t n, int plen, int32_t nz_prefix, const uint8_t* iv, uint8_t* out,
                               const uint64_t* out_offs, uint32_t* out_lens) {
    if (!z) return fail_status(SDFS_CDC_EINVAL, "null cipher");
    if (n == 0) return SDFS_CDC_OK;
    if (!base || !offs || !lens || !out || !out_offs || !out_lens || !iv)
        return fail_status(SDFS_CDC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(z->mu);
    AES_TRY(hipSetDevice(z->device));
    return host_batch(z, true, base, offs, lens, n, plen, nz_prefix, iv, out, out_offs, out_lens);
}

int sdfs_cdc_aes_encrypt(sdfs_cdc_aes* z, const uint8_t* src, uint64_t n, int plen, int32_t nz_prefix,
                         const uint8_t* iv, uint8_t* dst, uint64_t cap, uint64_t* out_len) {
    if (!z || !out_len || (n && !src) || !dst || !iv) return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (n >= (1ull << 31) - 32) return fail_status(SDFS_CDC_EINVAL, "record longer than 2 GiB");
    const uint64_t need = sdfs_cdc_aes_cbc_bound(n + (uint64_t)(plen > 0 ? plen : 0));
    if (cap < need) return fail_status(SDFS_CDC_ECAP, "cap %llu < %llu", (unsigned long long)cap,
                                       (unsigned long long)need);
    const uint64_t off = 0, doff = 0;
    const uint32_t len = (uint32_t)n;
    uint32_t ol = 0;
    const uint8_t dummy = 0;
    std::lock_guard<std::mutex> lk(z->mu);
    AES_TRY(hipSetDevice(z->device));
    const int rc = host_batch(z, true, n ? src : &dummy, &off, &len, 1, plen, nz_prefix, iv, dst, &doff, &ol);
    if (rc == SDFS_CDC_OK) *out_len = ol;
    return rc;
}

int sdfs_cdc_aes_decrypt(sdfs_cdc_aes* z, const uint8_t* src, uint64_t n, const uint8_t* iv, uint8_t* dst,
                         uint64_t cap, uint64_t* out_len) {
    if (!z || !out_len || (n && !src) || !dst || !iv) return fail_status(SDFS_CDC_EINVAL, "null argument");
    if (n == 0 || n % 16) return fail_status(SDFS_CDC_EINVAL, "ciphertext length %llu is not a positive multiple of 16",
                                             (unsigned long long)n);
    if (n >= (1ull << 31) - 32) return fail_status(SDFS_CDC_EINVAL, "record longer than 2 GiB");
    if (cap < n - 1) return fail_status(SDFS_CDC_ECAP, "cap %llu < %llu", (unsigned long long)cap,
                                        (unsigned long long)(n - 1));
    const uint64_t off = 0, doff = 0;
    const uint32_t len = (uint32_t)n;
    uint32_t ol = 0;
    std::vector<uint8_t> tmp(n);
    std::lock_guard<std::mutex> lk(z->mu);
    AES_TRY(hipSetDevice(z->device));
    const int rc = host_batch(z, false, src, &off, &len, 1, 0, 0, iv, tmp.data(), &doff, &ol);
    if (rc) return rc;
    if (ol == 0xFFFFFFFFu) return fail_status(SDFS_CDC_EINVAL, "bad padding");
    if (cap < ol) return fail_status(SDFS_CDC_ECAP, "cap %llu < %u", (unsigned long long)cap, ol);
    memcpy(dst, tmp.data(), ol);
    *out_len = ol;
    return SDFS_CDC_OK;
}

}  // extern "C"
