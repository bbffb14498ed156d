/*
 * aes_ref.c — CPU ORACLE for AES-CBC chunk encryption.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the benches' CPU-baseline
 * legs may load this library, and only as the checker / the timed CPU baseline.  The product
 * path (sdfs_amd/, libsdfs_cdc.so) never links or calls it.
 *
 * Reference call sites: HashBlobArchive.putChunk encrypts the stored record
 * [int nz][chunk or its LZ4 block] with EncryptUtils.encryptCBC(bf.array(), ivspec) when
 * Main.chunkStoreEncryptionEnabled (HashBlobArchive.java:1280-1294); the read side is
 * EncryptUtils.decryptCBC (HashBlobArchive.java:1923-1925).  encryptCBC(chunk, cspec)
 * (EncryptUtils.java:142-152) is Cipher.getInstance("AES/CBC/PKCS5Padding") with
 * key = SHA-256(Main.chunkStoreEncryptionKey.getBytes()) (EncryptUtils.java:47-52: 32 bytes,
 * so AES-256) and the archive's 16-byte IV (HashBlobArchive.java:91,1028-1032,1217-1224).
 * The cipher is the JDK's JCE provider (not in /root/reference).
 *
 * This file restates the published algorithm, byte-oriented and table-free exactly as FIPS-197
 * specifies it (S-box = affine map of the GF(2^8) inverse, SubBytes/ShiftRows/MixColumns/
 * AddRoundKey, the key expansion of §5.2), CBC chaining (NIST SP 800-38A §6.2) and PKCS#5/#7
 * padding (RFC 8018 §6.1.1: 1..16 bytes of value = pad length, a whole block when n % 16 == 0).
 * PARITY STATUS: pinned by the FIPS-197 Appendix C known-answer vectors, the SP 800-38A F.2
 * CBC vectors and records produced by the image's `openssl enc` (tests/golden/aes.json).
 */
#include "aes_ref.h"

#include <pthread.h>
#include <string.h>

static uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

static uint8_t SBOX[256], INV_SBOX[256];
static pthread_once_t sbox_once = PTHREAD_ONCE_INIT;

/* FIPS-197 §5.1.1: b = x^-1 in GF(2^8) (0 -> 0), then b_i ^ b_{i+4} ^ b_{i+5} ^ b_{i+6} ^ b_{i+7} ^ c_i, c = 0x63 */
static void build_sbox(void) {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {  /* x^254 = x^-1 */
            uint8_t p = (uint8_t)x, r = 1;
            for (int e = 254; e; e >>= 1) {
                if (e & 1) r = gmul(r, p);
                p = gmul(p, p);
            }
            inv = r;
        }
        uint8_t s = 0;
        for (int i = 0; i < 8; i++) {
            int bit = ((inv >> i) ^ (inv >> ((i + 4) & 7)) ^ (inv >> ((i + 5) & 7)) ^ (inv >> ((i + 6) & 7)) ^
                       (inv >> ((i + 7) & 7)) ^ (0x63 >> i)) & 1;
            s |= (uint8_t)(bit << i);
        }
        SBOX[x] = s;
        INV_SBOX[s] = (uint8_t)x;
    }
}

uint64_t aes_ref_cbc_bound(uint64_t n) { return (n / 16 + 1) * 16; }

int aes_ref_expand_key(const uint8_t* key, int key_len, uint32_t rk[60]) {
    pthread_once(&sbox_once, build_sbox);
    if (key_len != 16 && key_len != 24 && key_len != 32) return -1;
    const int nk = key_len / 4, nr = nk + 6, total = 4 * (nr + 1);
    for (int i = 0; i < nk; i++)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t << 8) | (t >> 24); /* RotWord */
            t = (uint32_t)SBOX[t >> 24] << 24 | (uint32_t)SBOX[(t >> 16) & 255] << 16 |
                (uint32_t)SBOX[(t >> 8) & 255] << 8 | SBOX[t & 255];
            t ^= (uint32_t)rcon << 24;
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)SBOX[t >> 24] << 24 | (uint32_t)SBOX[(t >> 16) & 255] << 16 |
                (uint32_t)SBOX[(t >> 8) & 255] << 8 | SBOX[t & 255];
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

/* state[r + 4c] = byte r of column c (FIPS-197 §3.4: in[r + 4c]) */
static void add_round_key(uint8_t st[16], const uint32_t* w) {
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) st[r + 4 * c] ^= (uint8_t)(w[c] >> (24 - 8 * r));
}

void aes_ref_encrypt_block(const uint32_t* rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    pthread_once(&sbox_once, build_sbox);
    uint8_t st[16], t[16];
    memcpy(st, in, 16);
    add_round_key(st, rk);
    for (int round = 1; round <= nr; round++) {
        for (int i = 0; i < 16; i++) st[i] = SBOX[st[i]];
        for (int r = 1; r < 4; r++) /* ShiftRows: row r rotates left by r columns */
            for (int c = 0; c < 4; c++) t[r + 4 * c] = st[r + 4 * ((c + r) & 3)];
        for (int r = 1; r < 4; r++)
            for (int c = 0; c < 4; c++) st[r + 4 * c] = t[r + 4 * c];
        if (round != nr) { /* MixColumns */
            for (int c = 0; c < 4; c++) {
                const uint8_t* a = st + 4 * c;  /* {02} = xtime, {03} = xtime ^ identity */
                const uint8_t x0 = xtime(a[0]), x1 = xtime(a[1]), x2 = xtime(a[2]), x3 = xtime(a[3]);
                uint8_t b0 = x0 ^ (x1 ^ a[1]) ^ a[2] ^ a[3];
                uint8_t b1 = a[0] ^ x1 ^ (x2 ^ a[2]) ^ a[3];
                uint8_t b2 = a[0] ^ a[1] ^ x2 ^ (x3 ^ a[3]);
                uint8_t b3 = (x0 ^ a[0]) ^ a[1] ^ a[2] ^ x3;
                st[4 * c] = b0; st[4 * c + 1] = b1; st[4 * c + 2] = b2; st[4 * c + 3] = b3;
            }
        }
        add_round_key(st, rk + 4 * round);
    }
    memcpy(out, st, 16);
}

void aes_ref_decrypt_block(const uint32_t* rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    pthread_once(&sbox_once, build_sbox);
    uint8_t st[16], t[16];
    memcpy(st, in, 16);
    add_round_key(st, rk + 4 * nr);
    for (int round = nr - 1; round >= 0; round--) {
        for (int r = 1; r < 4; r++) /* InvShiftRows */
            for (int c = 0; c < 4; c++) t[r + 4 * ((c + r) & 3)] = st[r + 4 * c];
        for (int r = 1; r < 4; r++)
            for (int c = 0; c < 4; c++) st[r + 4 * c] = t[r + 4 * c];
        for (int i = 0; i < 16; i++) st[i] = INV_SBOX[st[i]];
        add_round_key(st, rk + 4 * round);
        if (round) { /* InvMixColumns */
            for (int c = 0; c < 4; c++) {
                const uint8_t* a = st + 4 * c;
                uint8_t b0 = gmul(a[0], 14) ^ gmul(a[1], 11) ^ gmul(a[2], 13) ^ gmul(a[3], 9);
                uint8_t b1 = gmul(a[0], 9) ^ gmul(a[1], 14) ^ gmul(a[2], 11) ^ gmul(a[3], 13);
                uint8_t b2 = gmul(a[0], 13) ^ gmul(a[1], 9) ^ gmul(a[2], 14) ^ gmul(a[3], 11);
                uint8_t b3 = gmul(a[0], 11) ^ gmul(a[1], 13) ^ gmul(a[2], 9) ^ gmul(a[3], 14);
                st[4 * c] = b0; st[4 * c + 1] = b1; st[4 * c + 2] = b2; st[4 * c + 3] = b3;
            }
        }
    }
    memcpy(out, st, 16);
}

long aes_ref_cbc_encrypt(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* prefix, int plen,
                         const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap) {
    uint32_t rk[60];
    const int nr = aes_ref_expand_key(key, key_len, rk);
    if (nr < 0 || plen < 0 || plen > 16) return -1;
    const uint64_t total = n + (uint64_t)plen, out_len = aes_ref_cbc_bound(total);
    if (cap < out_len) return -1;
    uint8_t chain[16], blk[16];
    memcpy(chain, iv, 16);
    for (uint64_t o = 0; o < out_len; o += 16) {
        for (int j = 0; j < 16; j++) {
            const uint64_t k = o + (uint64_t)j;  /* byte k of [prefix][src][padding] */
            uint8_t b;
            if (k < (uint64_t)plen) b = prefix[k];
            else if (k < total) b = src[k - (uint64_t)plen];
            else b = (uint8_t)(out_len - total);
            blk[j] = b ^ chain[j];
        }
        aes_ref_encrypt_block(rk, nr, blk, chain);
        memcpy(dst + o, chain, 16);
    }
    return (long)out_len;
}

long aes_ref_cbc_decrypt(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* src, uint64_t n,
                         uint8_t* dst, uint64_t cap) {
    uint32_t rk[60];
    const int nr = aes_ref_expand_key(key, key_len, rk);
    if (nr < 0 || n == 0 || n % 16) return -1;
    uint8_t prev[16], p[16];
    memcpy(prev, iv, 16);
    uint8_t last[16];
    for (uint64_t o = 0; o < n; o += 16) {
        aes_ref_decrypt_block(rk, nr, src + o, p);
        for (int j = 0; j < 16; j++) p[j] ^= prev[j];
        memcpy(prev, src + o, 16);
        if (o + 16 < n) {
            if (cap < o + 16) return -1;
            memcpy(dst + o, p, 16);
        } else {
            memcpy(last, p, 16);
        }
    }
    const uint8_t v = last[15];
    if (v < 1 || v > 16) return -1;
    for (int j = 16 - v; j < 16; j++)
        if (last[j] != v) return -1;
    const uint64_t plain = n - v;
    if (cap < plain) return -1;
    memcpy(dst + (n - 16), last, 16 - v);
    return (long)plain;
}

struct aes_job {
    const uint8_t *key, *iv, *prefix, *base;
    int key_len, plen;
    const uint64_t *offs, *out_offs;
    const uint32_t* lens;
    uint8_t* out;
    uint32_t* out_lens;
    uint32_t lo, hi;
    long rc;
};

static void* aes_worker(void* p) {
    struct aes_job* j = (struct aes_job*)p;
    j->rc = 0;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        const uint64_t room = aes_ref_cbc_bound((uint64_t)j->lens[i] + (uint64_t)j->plen);
        long r = aes_ref_cbc_encrypt(j->key, j->key_len, j->iv, j->prefix, j->plen, j->base + j->offs[i], j->lens[i],
                                     j->out + j->out_offs[i], room);
        if (r < 0) { j->rc = -1; return NULL; }
        j->out_lens[i] = (uint32_t)r;
        j->rc += r;
    }
    return NULL;
}

long aes_ref_cbc_encrypt_batch(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* prefix,
                               int plen, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                               uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_once(&sbox_once, build_sbox);
    struct aes_job jobs[256];
    pthread_t th[256];
    const uint32_t per = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        uint32_t lo = (uint32_t)t * per, hi = lo + per < n ? lo + per : n;
        if (lo >= hi) break;
        jobs[t] = (struct aes_job){key, iv, prefix, base, key_len, plen, offs, out_offs, lens, out, out_lens, lo, hi, 0};
        pthread_create(&th[t], NULL, aes_worker, &jobs[t]);
        started++;
    }
    long total = 0;
    for (int t = 0; t < started; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc < 0) total = -1;
        else if (total >= 0) total += jobs[t].rc;
    }
    return total;
}
