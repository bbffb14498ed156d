/*
 * aes_ref.h — CPU ORACLE for AES-CBC chunk encryption (test infrastructure only; see aes_ref.c
 * for what it restates and what pins it).
 */
#ifndef SDFS_AES_REF_H
#define SDFS_AES_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Cipher.doFinal output length of AES/CBC/PKCS5Padding: (n / 16 + 1) * 16 */
uint64_t aes_ref_cbc_bound(uint64_t n);
/* FIPS-197 key expansion for a 16/24/32-byte key: rk[0 .. 4*(Nr+1)) big-endian words; returns Nr
 * (10/12/14) or -1. */
int aes_ref_expand_key(const uint8_t* key, int key_len, uint32_t rk[60]);
void aes_ref_encrypt_block(const uint32_t* rk, int nr, const uint8_t in[16], uint8_t out[16]);
void aes_ref_decrypt_block(const uint32_t* rk, int nr, const uint8_t in[16], uint8_t out[16]);
/* AES/CBC/PKCS5Padding of [prefix (plen bytes)][src (n bytes)] (plen 0 or 4: the big-endian
 * int HashBlobArchive.putChunk writes before an uncompressed chunk); returns bytes written or -1. */
long aes_ref_cbc_encrypt(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* prefix, int plen,
                         const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap);
/* Inverse, with the PKCS5 padding check Cipher.doFinal makes; returns the plain length, -1 on a
 * bad length or padding. */
long aes_ref_cbc_decrypt(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* src, uint64_t n,
                         uint8_t* dst, uint64_t cap);
/* Records base[offs[i] .. + lens[i]) -> out + out_offs[i] (room aes_ref_cbc_bound(len + plen)) on
 * nthreads pthreads; out_lens[i] = bytes written.  Returns the total or -1. */
long aes_ref_cbc_encrypt_batch(const uint8_t* key, int key_len, const uint8_t iv[16], const uint8_t* prefix,
                               int plen, const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                               uint8_t* out, const uint64_t* out_offs, uint32_t* out_lens, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
