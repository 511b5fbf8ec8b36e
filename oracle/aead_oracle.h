/*
 * aead_oracle.h -- CPU restatement of tlslite-ng's pure-Python AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the reported CPU baseline).  The product path (libtlsgpu.so) never
 * links or calls it.
 *
 * Every function restates the reference algorithm it names (file:line under
 * tlslite/utils/ of tlslite-ng 0.8.2).  Parity is pinned by the reference's
 * own known-answer vectors and by golden vectors generated from the reference
 * itself (tests/golden/make_golden.py), see tests/test_oracle_golden.py.
 */
#ifndef TLSGPU_AEAD_ORACLE_H
#define TLSGPU_AEAD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* AES block encrypt (rijndael.py:922-1038).  keylen 16/24/32. */
int oracle_aes_encrypt_block(const uint8_t* key, size_t keylen,
                             const uint8_t in[16], uint8_t out[16]);

/* AESGCM.seal (aesgcm.py:101-124): out = ct || tag (len + 16 bytes).
 * Returns 0, or -1 on bad key/nonce length. */
int oracle_gcm_seal(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* pt, size_t len, uint8_t* out);
/* AESGCM.open (aesgcm.py:126-154): in = ct || tag (inlen bytes).
 * Returns 1 (authentic, pt written: inlen-16 bytes), 0 (reject: None in the
 * reference), -1 (bad nonce: ValueError), -2 (bad key length). */
int oracle_gcm_open(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* in, size_t inlen, uint8_t* pt);

/* AESCCM.seal/open (aesccm.py:85-149), taglen 16 (aes*ccm) or 8 (aes*ccm_8):
 * out = ct || tag (len + taglen).  Conventions as the GCM pair; a rejected
 * open zeroes pt. */
int oracle_ccm_seal(const uint8_t* key, size_t keylen, size_t taglen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* pt, size_t len, uint8_t* out);
int oracle_ccm_open(const uint8_t* key, size_t keylen, size_t taglen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* in, size_t inlen, uint8_t* pt);

/* ChaCha20 keystream XOR (chacha.py:98-153), counter is the initial block. */
int oracle_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12],
                        uint32_t counter, const uint8_t* in, size_t len,
                        uint8_t* out);
/* Poly1305 tag (poly1305.py:32-48) over arbitrary-length data. */
void oracle_poly1305(const uint8_t key[32], const uint8_t* data, size_t len,
                     uint8_t tag[16]);
/* CHACHA20_POLY1305.seal/open (chacha20_poly1305.py:48-94); conventions as
 * the GCM pair. */
int oracle_chacha_seal(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                       size_t noncelen, const uint8_t* aad, size_t aadlen,
                       const uint8_t* pt, size_t len, uint8_t* out);
int oracle_chacha_open(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                       size_t noncelen, const uint8_t* aad, size_t aadlen,
                       const uint8_t* in, size_t inlen, uint8_t* pt);

/* Batch form used for sampled parity checks and the CPU baseline.
 * alg: 0 = AES-GCM, 1 = ChaCha20-Poly1305, 2 = AES-CCM, 3 = AES-CCM_8.
 * op: 0 = seal, 1 = open.
 * keys: nkeys x keylen; key_idx may be NULL (all records use key 0).
 * Record i: input at in + in_off[i], inlen[i] bytes (open: ct||tag);
 * nonce at nonces + 12*i; aad at aad + aad_off[i], aad_len[i] bytes;
 * output at out + out_off[i]; status[i] (open) = 1/0.
 * Work is split over nthreads POSIX threads.  Returns 0 or -1. */
int oracle_batch(int alg, int op, const uint8_t* keys, size_t keylen,
                 const uint32_t* key_idx, const uint8_t* nonces,
                 const uint8_t* aad, const uint64_t* aad_off,
                 const uint32_t* aad_len, const uint8_t* in,
                 const uint64_t* in_off, const uint32_t* inlen, uint8_t* out,
                 const uint64_t* out_off, uint8_t* status, size_t n,
                 int nthreads);

/* GHASH_H(aad, ct) with the length block, i.e. AESGCM._auth before the tag
 * mask (aesgcm.py:60-67), for an arbitrary H (16 bytes, big-endian). */
void oracle_ghash(const uint8_t h[16], const uint8_t* aad, size_t aadlen,
                  const uint8_t* ct, size_t ctlen, uint8_t out[16]);

/* Cross-check of the oracle's fast forms against the reference's own
 * formulations (T-table AES vs byte-wise rounds, byte-wise vs nibble-wise
 * GHASH multiply) on n random cases; returns the number of mismatches. */
int oracle_selfcheck(size_t n, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
