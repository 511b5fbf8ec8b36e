// host.cpp -- host key setup and record scanning of libtlsgpu (see host.h).
// Plain C++: the library builds it with g++, and tests/native/host_check.cpp
// builds it again under AddressSanitizer + UBSan.
#include "host.h"

#include <string.h>

#include "keymath.h"

namespace tg {
namespace host {

namespace {

uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// The S-box from GF(2^8) inverses and the affine map (FIPS-197 5.1.1).
struct Sbox {
    uint8_t s[256];
    Sbox() {
        uint8_t exp[256], log[256];
        uint8_t x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = x;
            log[x] = (uint8_t)i;
            x = (uint8_t)(x ^ xt(x));
        }
        for (int v = 0; v < 256; ++v) {
            const uint8_t inv = v ? exp[(255 - log[v]) % 255] : 0;
            uint8_t t = inv, r = inv;
            for (int k = 0; k < 4; ++k) {
                r = (uint8_t)((r << 1) | (r >> 7));
                t = (uint8_t)(t ^ r);
            }
            s[v] = (uint8_t)(t ^ 0x63);
        }
    }
};

const uint8_t* sbox() {
    static const Sbox box;
    return box.s;
}

// H (block bytes) -> normal-order words
void to_norm(const uint8_t h[16], uint32_t hn[4]) {
    for (int w = 0; w < 4; ++w) hn[w] = gcm_word_to_norm(le32(h + 4 * w));
}

// normal-order words -> block bytes
void from_norm(const uint32_t p[4], uint8_t h[16]) {
    for (int w = 0; w < 4; ++w) {
        const uint32_t v = gcm_word_to_norm(p[w]);
        for (int q = 0; q < 4; ++q) h[4 * w + q] = (uint8_t)(v >> (8 * q));
    }
}

}  // namespace

uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

int aes_expand(const uint8_t* key, size_t keylen, uint8_t rk[240]) {
    if (keylen != 16 && keylen != 24 && keylen != 32) return -1;
    const uint8_t* sb = sbox();
    const int nk = (int)keylen / 4, nr = nk + 6, total = 4 * (nr + 1);
    memcpy(rk, key, keylen);
    uint8_t rcon = 1;
    for (int i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            const uint8_t t0 = t[0];
            t[0] = (uint8_t)(sb[t[1]] ^ rcon);
            t[1] = sb[t[2]];
            t[2] = sb[t[3]];
            t[3] = sb[t0];
            rcon = xt(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = sb[t[k]];
        }
        for (int k = 0; k < 4; ++k) rk[4 * i + k] = (uint8_t)(rk[4 * (i - nk) + k] ^ t[k]);
    }
    return nr;
}

void aes_encrypt(const uint8_t* rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    const uint8_t* sb = sbox();
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int r = 1; r <= nr; ++r) {
        for (int c = 0; c < 4; ++c)   // SubBytes + ShiftRows
            for (int row = 0; row < 4; ++row) t[4 * c + row] = sb[s[4 * ((c + row) & 3) + row]];
        if (r != nr) {
            for (int c = 0; c < 4; ++c) {   // MixColumns
                uint8_t* a = t + 4 * c;
                const uint8_t all = (uint8_t)(a[0] ^ a[1] ^ a[2] ^ a[3]), a0 = a[0];
                a[0] = (uint8_t)(a[0] ^ all ^ xt((uint8_t)(a[0] ^ a[1])));
                a[1] = (uint8_t)(a[1] ^ all ^ xt((uint8_t)(a[1] ^ a[2])));
                a[2] = (uint8_t)(a[2] ^ all ^ xt((uint8_t)(a[2] ^ a[3])));
                a[3] = (uint8_t)(a[3] ^ all ^ xt((uint8_t)(a[3] ^ a0)));
            }
        }
        for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(t[i] ^ rk[16 * r + i]);
    }
    memcpy(out, s, 16);
}

// A field element is the 16-byte block read as a big-endian integer whose MSB
// is the x^0 coefficient (aesgcm.py:8-14); multiplying by x is a right shift
// with the 0xe1 << 120 reduction (AESGCM._gcmShift, aesgcm.py:168-178).
// V[n] = H * x^n, and M_j[b] = XOR of V[8j + t] over the bits t (MSB first)
// set in b.  keymath.h ghash_table_words computes one entry from scratch;
// this builds all 4096 from the 128 shifts.
void ghash_tables(const uint8_t h[16], uint32_t (*table)[4]) {
    uint64_t hi = 0, lo = 0;
    for (int i = 0; i < 8; ++i) hi = (hi << 8) | h[i];
    for (int i = 8; i < 16; ++i) lo = (lo << 8) | h[i];
    uint64_t vhi[128], vlo[128];
    for (int n = 0; n < 128; ++n) {
        vhi[n] = hi;
        vlo[n] = lo;
        const uint64_t carry = lo & 1;
        lo = (lo >> 1) | (hi << 63);
        hi >>= 1;
        if (carry) hi ^= 0xe1ull << 56;
    }
    for (int j = 0; j < 16; ++j) {
        for (int b = 0; b < 256; ++b) {
            uint64_t zh = 0, zl = 0;
            for (int t = 0; t < 8; ++t) {
                if (b & (0x80 >> t)) {
                    zh ^= vhi[8 * j + t];
                    zl ^= vlo[8 * j + t];
                }
            }
            uint8_t bytes[16];
            for (int k = 0; k < 8; ++k) {
                bytes[k] = (uint8_t)(zh >> (56 - 8 * k));
                bytes[8 + k] = (uint8_t)(zl >> (56 - 8 * k));
            }
            for (int q = 0; q < 4; ++q) table[j * 256 + b][q] = le32(bytes + 4 * q);
        }
    }
}

int aes_round_words(const uint8_t* key, size_t keylen, uint32_t rk[60], uint32_t hn[4]) {
    uint8_t rkb[240] = {0};
    const int nr = aes_expand(key, keylen, rkb);
    if (nr < 0) return -1;
    memset(rk, 0, 60 * sizeof(uint32_t));
    for (int w = 0; w < 4 * (nr + 1); ++w) rk[w] = le32(rkb + 4 * w);
    if (hn) {
        uint8_t zero[16] = {0}, h[16];
        aes_encrypt(rkb, nr, zero, h);                  // H = E_K(0^128)
        to_norm(h, hn);
        memset(h, 0, sizeof(h));
    }
    memset(rkb, 0, sizeof(rkb));
    return nr;
}

int gcm_key_image(const uint8_t* key, size_t keylen, GcmKeyImage* out) {
    memset(out, 0, sizeof(*out));
    uint8_t rkb[240] = {0};
    const int nr = aes_expand(key, keylen, rkb);
    if (nr < 0) return -1;
    for (int w = 0; w < 4 * (nr + 1); ++w) out->rk[w] = le32(rkb + 4 * w);
    out->rounds = (uint32_t)nr;
    uint8_t zero[16] = {0}, h[16];
    aes_encrypt(rkb, nr, zero, h);                      // H = E_K(0^128)
    ghash_tables(h, out->ghash);
    uint32_t hn[4], p[4];                               // H^1 .. H^2048, normal order
    to_norm(h, hn);
    for (int w = 0; w < 4; ++w) p[w] = hn[w];
    for (int e = 0; e < 2048; ++e) {
        for (int w = 0; w < 4; ++w) out->hpow[e][w] = p[w];
        gf_mul_norm(p, hn, p);
    }
    uint8_t hb[16];
    from_norm(out->hpow[63], hb);                       // tables of H^64 (gcm_wave_kernel)
    ghash_tables(hb, out->ghash64);
    from_norm(out->hpow[7], hb);                        // tables of H^8 (octet kernels)
    ghash_tables(hb, out->ghash8);
    for (int e = 0; e < 32 * (nr + 1); ++e) out->bs8mask[e] = bs8_mask_word(out->rk, e);
    for (int w = 0; w < 15 * 32; ++w) out->bs8rows[w] = bs8_row_word(out->rk, nr, w);
    for (int w = 0; w < 64; ++w) out->rkrot[w] = rkrot_word(out->rk, nr, w);
    memset(rkb, 0, sizeof(rkb));
    memset(h, 0, sizeof(h));
    memset(hb, 0, sizeof(hb));
    return 0;
}

int64_t scan_records(const uint8_t* buf, size_t len, uint32_t max_body, uint64_t* off,
                     uint32_t* rlen, size_t max_n, size_t* consumed, ScanError* err) {
    size_t pos = 0, k = 0;
    *consumed = 0;
    while (k < max_n && len - pos >= 5) {
        const uint8_t type = buf[pos];
        if (type < 20 || type > 24) {
            *err = ScanError{1, k, type};
            return -1;
        }
        const uint32_t body = ((uint32_t)buf[pos + 3] << 8) | buf[pos + 4];
        if (body > max_body) {
            *err = ScanError{2, k, body};
            return -1;
        }
        if (len - pos < 5 + (size_t)body) break;   // incomplete: wait for more bytes
        off[k] = pos;
        rlen[k] = 5 + body;
        pos += 5 + body;
        *consumed = pos;
        ++k;
    }
    return (int64_t)k;
}

}  // namespace host
}  // namespace tg
