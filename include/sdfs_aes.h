/*
 * sdfs_aes.h — C-ABI of the MI355X AES-CBC encryptor for stored chunk records (SURVEY.md §8(f)
 * row 4).
 *
 * When Main.chunkStoreEncryptionEnabled, HashBlobArchive.putChunk (HashBlobArchive.java:1280-1294)
 * encrypts every stored record — [int nz, big-endian][chunk, or its LZ4 block when Main.compress]
 * (nz = -1 for an uncompressed chunk) — with EncryptUtils.encryptCBC(record, ivspec)
 * (EncryptUtils.java:142-152): JCE "AES/CBC/PKCS5Padding", key = SHA-256 of
 * Main.chunkStoreEncryptionKey's bytes (EncryptUtils.java:47-52, a 32-byte key: AES-256), IV = the
 * archive's 16 bytes (HashBlobArchive.java:91,1028-1032).  The read side is
 * EncryptUtils.decryptCBC(record, ivspec) (HashBlobArchive.java:1923-1925, EncryptUtils.java:125-140).
 *
 * These entry points encrypt a whole batch of records on the GPU, byte-identical to that cipher
 * (oracle/aes_ref.c restates FIPS-197 + SP 800-38A CBC + PKCS#5; tests pin it against FIPS/NIST
 * vectors and the image's openssl).  Errors, threading and sdfs_cdc_last_error() as in sdfs_cdc.h.
 * Encryptions enqueued on different streams are ordered (they share the cipher's scheduling scratch).
 */
#ifndef SDFS_AES_H
#define SDFS_AES_H

#include <stdint.h>

#include "sdfs_cdc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sdfs_cdc_aes sdfs_cdc_aes;

/* Cipher.doFinal output length of AES/CBC/PKCS5Padding for n plaintext bytes: (n / 16 + 1) * 16 */
uint64_t sdfs_cdc_aes_cbc_bound(uint64_t n);

/* A cipher for `key` (16, 24 or 32 bytes: AES-128/192/256; SDFS passes SHA-256(passphrase)) on
 * HIP device `device`.  (EncryptUtils' static key, EncryptUtils.java:45-56) */
int sdfs_cdc_aes_create(int device, const uint8_t* key, uint32_t key_len, sdfs_cdc_aes** out);
int sdfs_cdc_aes_destroy(sdfs_cdc_aes* z);

/* Device batch of EncryptUtils.encryptCBC(record, iv).  Record i (i < *d_count when d_count is
 * not NULL, else i < n_max) is [prefix: plen bytes][d_src[d_src_off[i] .. + d_src_len[i])]; plen
 * is 0 (the source already holds the framed record, e.g. sdfs_cdc_lz4_compress_device's framed
 * output) or 4 (the source is a raw chunk and the prefix is the big-endian int nz, -1 for an
 * uncompressed chunk: HashBlobArchive.java:1281-1287).  iv: 16 host bytes used for every record,
 * or d_ivs (16 device bytes per record) when not NULL.  The ciphertext of record i goes to
 * d_out + d_dst_off[i] (room for sdfs_cdc_aes_cbc_bound(len + plen)); d_dst_len[i] = its length.
 * Records are scheduled longest first on the GPU (engine scratch).  Enqueued on `stream`. */
int sdfs_cdc_aes_encrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max, int plen,
                                int32_t nz_prefix, const uint8_t* iv, const uint8_t* d_ivs, uint8_t* d_out,
                                const uint64_t* d_dst_off, uint32_t* d_dst_len, void* stream);

/* Device batch of EncryptUtils.decryptCBC(record, iv): record i = d_src[d_src_off[i] .. +
 * d_src_len[i]) (a positive multiple of 16), its plaintext to d_out + d_dst_off[i] (room
 * d_src_len[i]); d_dst_len[i] = plaintext length, or UINT32_MAX when the length or the PKCS#5
 * padding is invalid (Cipher.doFinal's BadPaddingException). */
int sdfs_cdc_aes_decrypt_device(sdfs_cdc_aes* z, const uint8_t* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, const uint32_t* d_count, uint64_t n_max,
                                const uint8_t* iv, const uint8_t* d_ivs, uint8_t* d_out, const uint64_t* d_dst_off,
                                uint32_t* d_dst_len, void* stream);

/* Host forms (one H2D, the kernels, one D2H): EncryptUtils.encryptCBC(byte[] chunk, ivspec) and
 * decryptCBC.  encrypt: *out_len = bound(n + plen) (cap must hold it); decrypt: returns
 * SDFS_CDC_EINVAL on bad padding. */
int sdfs_cdc_aes_encrypt(sdfs_cdc_aes* z, const uint8_t* src, uint64_t n, int plen, int32_t nz_prefix,
                         const uint8_t* iv, uint8_t* dst, uint64_t cap, uint64_t* out_len);
int sdfs_cdc_aes_decrypt(sdfs_cdc_aes* z, const uint8_t* src, uint64_t n, const uint8_t* iv, uint8_t* dst,
                         uint64_t cap, uint64_t* out_len);
/* Host batch: record i = base[offs[i] .. + lens[i]) -> out + out_offs[i] (room bound(len + plen)). */
int sdfs_cdc_aes_encrypt_batch(sdfs_cdc_aes* z, const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                               uint32_t n, int plen, int32_t nz_prefix, const uint8_t* iv, uint8_t* out,
                               const uint64_t* out_offs, uint32_t* out_lens);

#ifdef __cplusplus
}
#endif
#endif /* SDFS_AES_H */
