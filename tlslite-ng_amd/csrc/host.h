// host.h -- the host-only half of libtlsgpu: AES key schedules, the GHASH
// tables and the record scanner.  Plain C++ (no HIP), built by g++ into the
// library and, with -fsanitize=address,undefined, into the CPU check
// tests/native/host_check.cpp (tests/test_host_sanitize.py).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace tg {
namespace host {

// Byte image of tg::GcmKeyDev (common.h); api.hip static_asserts that the
// sizes and member offsets agree.
struct GcmKeyImage {
    uint32_t rk[60];
    uint32_t rounds;
    uint32_t pad[3];
    uint32_t ghash[16 * 256][4];
    uint32_t hpow[2048][4];
    uint32_t ghash64[16 * 256][4];
    uint32_t ghash8[16 * 256][4];
    uint32_t bs8mask[15 * 32];
    // the hybrid kernel's key material, built with the key: the bitsliced
    // waves' key rows (keymath.h bs8_row_word) and the T-table waves' rotated
    // round keys (rkrot_word)
    uint32_t bs8rows[15 * 32];
    uint32_t rkrot[64];
};

uint32_t le32(const uint8_t* p);

// FIPS-197 key expansion (rijndael.py:922-993): round-key bytes,
// 16 * (rounds + 1) of them.  Returns the rounds, or -1 for a key length
// other than 16, 24 or 32.
int aes_expand(const uint8_t* key, size_t keylen, uint8_t rk[240]);
void aes_encrypt(const uint8_t* rk, int nr, const uint8_t in[16], uint8_t out[16]);

// The 16 x 256 8-bit GHASH tables of H (block bytes), entry j * 256 + b =
// b * x^(8j) * H as LE words of its GCM bytes.
void ghash_tables(const uint8_t h[16], uint32_t (*table)[4]);

// One AES key's round keys as LE words (the AesKeyDev / GcmTableKey rk):
// returns the rounds or -1.  hn (may be NULL): H = E_K(0^128) in normal
// polynomial order (GcmTableKey::hn).
int aes_round_words(const uint8_t* key, size_t keylen, uint32_t rk[60], uint32_t hn[4]);

// The whole single-key AES-GCM key (AESGCM.__init__, aesgcm.py:27-57, plus
// the kernels' tables): 0, or -1 for a bad key length.
int gcm_key_image(const uint8_t* key, size_t keylen, GcmKeyImage* out);

// Record scanner (RecordSocket.recv, recordlayer.py:169-237).  On success
// returns the number of complete records found (<= max_n) with their offsets
// and lengths (header included) and *consumed = bytes they cover.  On a bad
// header returns -1 with *err filled: code 1 = content type, 2 = body length
// over max_body; index = record number, value = the offending type / length.
struct ScanError {
    int code;
    size_t index;
    uint32_t value;
};
int64_t scan_records(const uint8_t* buf, size_t len, uint32_t max_body, uint64_t* off,
                     uint32_t* rlen, size_t max_n, size_t* consumed, ScanError* err);

// Parallel host copies (hostcopy.cpp): ``rows`` rows of ``row`` bytes from
// src + r * src_stride to dst + r * dst_stride, split over up to ``nthreads``
// threads (the caller and a shared worker pool; <= 0: copy_threads_default()).
// Regions must not overlap.  parallel_copy: one contiguous range.
int copy_threads_default();
void parallel_copy_rows(uint8_t* dst, size_t dst_stride, const uint8_t* src, size_t src_stride, size_t row,
                        size_t rows, int nthreads);
void parallel_copy(void* dst, const void* src, size_t bytes, int nthreads);

}  // namespace host
}  // namespace tg
