// keymath.h -- key-schedule arithmetic shared by the host key setup
// (host.cpp, plain C++) and the device key setup / self-test kernels
// (keysetup.hip, selftest.hip).  No HIP types: it compiles with g++ as well,
// so the sanitizer build of host.cpp (tests/native/host_check.cpp) covers it.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TG_KM_HD __host__ __device__ inline
#else
#define TG_KM_HD inline
#endif

namespace tg {

// a * b in GF(2^128) mod x^128 + x^7 + x^2 + x + 1, normal order (coefficient
// of x^i at bit i, word 0 first), bitwise (key setup only).
TG_KM_HD void gf_mul_norm(const uint32_t a[4], const uint32_t b[4], uint32_t r[4]) {
    uint32_t z[4] = {0, 0, 0, 0}, v[4] = {b[0], b[1], b[2], b[3]};
    for (int i = 0; i < 128; ++i) {
        if ((a[i >> 5] >> (i & 31)) & 1u)
            for (int q = 0; q < 4; ++q) z[q] ^= v[q];
        const uint32_t carry = v[3] >> 31;
        v[3] = (v[3] << 1) | (v[2] >> 31);
        v[2] = (v[2] << 1) | (v[1] >> 31);
        v[1] = (v[1] << 1) | (v[0] >> 31);
        v[0] = (v[0] << 1) ^ (carry ? 0x87u : 0u);
    }
    for (int q = 0; q < 4; ++q) r[q] = z[q];
}

// Normal-order word from a LE word of GCM block bytes: per-byte bit reversal.
TG_KM_HD uint32_t gcm_word_to_norm(uint32_t w) {
    uint32_t r = 0;
    for (int k = 0; k < 32; ++k) r |= ((w >> k) & 1u) << ((k & ~7) + 7 - (k & 7));
    return r;
}

// Entry e = j * 256 + b of the 8-bit GHASH tables of G (hv: G as LE words of
// its GCM bytes): b * x^(8j) * G in the same layout (aesgcm.py:8-14 bit order,
// _mul :86-97 restated bitwise), as 4 LE words.
TG_KM_HD void ghash_table_words(const uint32_t hv[4], int e, uint32_t w[4]) {
    const int j = e >> 8, b = e & 255;
    uint64_t hi = 0, lo = 0;
    for (int k = 0; k < 8; ++k) hi = (hi << 8) | ((hv[k >> 2] >> (8 * (k & 3))) & 0xff);
    for (int k = 8; k < 16; ++k) lo = (lo << 8) | ((hv[k >> 2] >> (8 * (k & 3))) & 0xff);
    uint64_t zh = 0, zl = 0;
    for (int nsh = 0; nsh < 8 * j + 8; ++nsh) {             // V = H * x^nsh
        if (nsh >= 8 * j && (b & (0x80 >> (nsh - 8 * j)))) {
            zh ^= hi;
            zl ^= lo;
        }
        const uint64_t carry = lo & 1;
        lo = (lo >> 1) | (hi << 63);
        hi >>= 1;
        if (carry) hi ^= 0xe1ull << 56;
    }
    for (int q = 0; q < 4; ++q) {
        const uint64_t half = q < 2 ? zh : zl;
        const int sh = q & 1 ? 24 : 56;
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v |= (uint32_t)((half >> (sh - 8 * k)) & 0xff) << (8 * k);
        w[q] = v;
    }
}

// Entry e = (4 r + i) * 8 + b of GcmKeyDev::bs8mask (aes_bs8.h, 8-block
// bitslicing): byte c of the word is 0xff iff bit b of byte i of round-key
// word rk[4 r + c] ^ (r ? 0x63636363 : 0) is set.
TG_KM_HD uint32_t bs8_mask_word(const uint32_t* rk, int e) {
    const int r = e >> 5, i = (e >> 3) & 3, b = e & 7;
    uint32_t m = 0;
    for (int c = 0; c < 4; ++c) {
        const uint32_t w = rk[4 * r + c] ^ (r ? 0x63636363u : 0u);
        if ((w >> (8 * i + b)) & 1u) m |= 0xffu << (8 * c);
    }
    return m;
}

// The MixColumns-folded round-key planes (aes_bs8.h mix_round_folded), entry
// e = (4 r + i) * 8 + b for r >= 1: byte c is 0xff iff bit b of c_i is set,
// where per column c (k_i = byte i of rk[4 r + c] ^ 0x63636363, x = 0x02)
//   c_0 = (k_2 ^ x k_0) / (1 ^ x^2),  c_2 = k_0 ^ x c_0,
//   c_1 = (k_3 ^ x k_1) / (1 ^ x^2),  c_3 = k_1 ^ x c_1,
// so that x c_i ^ c_(i+2) = k_i: MixColumns of T_i = t_i ^ c_i adds the round key
// (1 / (1 ^ x^2) = 0x52 in GF(2^8) mod 0x11b).
TG_KM_HD uint32_t gf8_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k) {
        if ((b >> k) & 1u) r ^= a;
        a = (a << 1) ^ ((a & 0x80u) ? 0x11bu : 0u);
    }
    return r & 0xffu;
}

TG_KM_HD uint32_t bs8_fold_word(const uint32_t* rk, int e) {
    const int r = e >> 5, i = (e >> 3) & 3, b = e & 7;
    uint32_t m = 0;
    for (int c = 0; c < 4; ++c) {
        const uint32_t w = rk[4 * r + c] ^ 0x63636363u;
        const uint32_t lo = i & 1;   // rows lo and lo + 2 form one system
        const uint32_t k0 = (w >> (8 * lo)) & 0xffu, k2 = (w >> (8 * (lo + 2))) & 0xffu;
        const uint32_t cl = gf8_mul(k2 ^ gf8_mul(k0, 2), 0x52);
        const uint32_t ci = i < 2 ? cl : k0 ^ gf8_mul(cl, 2);
        if ((ci >> b) & 1u) m |= 0xffu << (8 * c);
    }
    return m;
}

// Word w = 4 (8 r + bit) + i of the hybrid kernel's bitsliced key rows
// (aes_bs8.h KeyPlanesVmem row layout, GcmKeyDev::bs8rows): the
// MixColumns-folded planes (bs8_fold_word) of rounds 1 .. nr - 1, the plain
// planes (bs8_mask_word) of rounds 0 and nr, zero past them.
TG_KM_HD uint32_t bs8_row_word(const uint32_t* rk, int nr, int w) {
    const int row = w >> 2, i = w & 3, r = row >> 3, bit = row & 7;
    if (r > nr) return 0;
    const int e = 32 * r + 8 * i + bit;
    return r >= 1 && r < nr ? bs8_fold_word(rk, e) : bs8_mask_word(rk, e);
}

// Word w of the T-table waves' round keys (GcmKeyDev::rkrot): round key r
// rotated right by 8 bits for r = 0 .. nr (aes_round.h col_r), then the plain
// last round key; zero past it.
TG_KM_HD uint32_t rkrot_word(const uint32_t* rk, int nr, int w) {
    if (w < 4 * (nr + 1)) return (rk[w] >> 8) | (rk[w] << 24);
    if (w < 4 * (nr + 2)) return rk[w - 4];
    return 0;
}

}  // namespace tg
