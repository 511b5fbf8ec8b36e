/*
 * aead_oracle.c -- CPU restatement of tlslite-ng's pure-Python AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY (see aead_oracle.h).  Parity of this restatement
 * with the reference is pinned in tests/test_oracle_golden.py against
 *   - the reference's own known-answer vectors (unit_tests/
 *     test_tlslite_utils_{aesgcm,aesccm,chacha20_poly1305,chacha,poly1305}.py), and
 *   - golden vectors produced by running the reference itself
 *     (tests/golden/make_golden.py -> tests/golden/ JSON files).
 *
 * Citations are tlslite/utils/<file>:<line> in tlslite-ng 0.8.2.
 */
#include "aead_oracle.h"

#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------ AES --
 * rijndael.py builds its S-box and T-tables from GF(2^8) arithmetic
 * (rijndael.py:51-82 S, :118-377 T1-T4, :898 rcon).  This restatement derives
 * the S-box the same way (multiplicative inverse + affine map) and evaluates
 * the round as SubBytes/ShiftRows/MixColumns on bytes, which is the operation
 * the reference's T-table lookups (rijndael.py:1016-1022) encode.          */

static uint8_t g_sbox[256];
static pthread_once_t g_tables_once = PTHREAD_ONCE_INIT;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void build_sbox(void) {
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; ++y)
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv;
        uint8_t r = inv;
        for (int k = 0; k < 4; ++k) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        g_sbox[x] = (uint8_t)(s ^ 0x63);
    }
}

typedef struct {
    int rounds;
    uint8_t rk[15][16];
    uint32_t rkw[15][4];  /* the same round keys as big-endian column words */
} aes_ctx;

static uint32_t g_te[4][256];
static void build_tables(void);

/* Key expansion, rijndael.py:922-993 (Nk = keylen/4, Nr = 10/12/14). */
static int aes_setup(aes_ctx* c, const uint8_t* key, size_t keylen) {
    pthread_once(&g_tables_once, build_tables);
    if (keylen != 16 && keylen != 24 && keylen != 32) return -1;
    int nk = (int)keylen / 4;
    c->rounds = nk + 6;
    int total = 4 * (c->rounds + 1);
    uint8_t w[60][4];
    for (int i = 0; i < nk; ++i) memcpy(w[i], key + 4 * i, 4);
    uint8_t rcon = 1;
    for (int i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, w[i - 1], 4);
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon);
            t[1] = g_sbox[t[2]];
            t[2] = g_sbox[t[3]];
            t[3] = g_sbox[t0];
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = g_sbox[t[k]];
        }
        for (int k = 0; k < 4; ++k) w[i][k] = (uint8_t)(w[i - nk][k] ^ t[k]);
    }
    for (int r = 0; r <= c->rounds; ++r)
        for (int j = 0; j < 4; ++j) {
            memcpy(&c->rk[r][4 * j], w[4 * r + j], 4);
            c->rkw[r][j] = ((uint32_t)w[4 * r + j][0] << 24) | ((uint32_t)w[4 * r + j][1] << 16) |
                           ((uint32_t)w[4 * r + j][2] << 8) | w[4 * r + j][3];
        }
    return 0;
}

/* Rijndael.encrypt, rijndael.py:995-1038, as the reference evaluates it:
 * big-endian column words, 9 (or 13) rounds of four T-table lookups per
 * column (rijndael.py:1016-1022, tables T1-T4 of :118-377), and a final
 * S-box round (:1024-1038).  The tables are derived here from the S-box
 * (T1[x] = (2s, s, s, 3s) big-endian, T2..T4 its byte rotations), exactly
 * the products rijndael.py's tables hold.  aes_encrypt_bytes() below is the
 * same cipher as SubBytes/ShiftRows/MixColumns on bytes; oracle_selfcheck()
 * compares the two on random blocks. */
static void build_tables(void) {
    build_sbox();
    for (int x = 0; x < 256; ++x) {
        uint32_t s = g_sbox[x], s2 = gf_mul((uint8_t)s, 2), s3 = s2 ^ s;
        uint32_t w = (s2 << 24) | (s << 16) | (s << 8) | s3;
        for (int t = 0; t < 4; ++t) g_te[t][x] = t ? (w >> (8 * t)) | (w << (32 - 8 * t)) : w;
    }
}

static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void aes_encrypt(const aes_ctx* c, const uint8_t in[16], uint8_t out[16]) {
    uint32_t s[4], t[4];
    for (int j = 0; j < 4; ++j) s[j] = be32(in + 4 * j) ^ c->rkw[0][j];
    for (int r = 1; r < c->rounds; ++r) {
        for (int j = 0; j < 4; ++j)
            t[j] = g_te[0][s[j] >> 24] ^ g_te[1][(s[(j + 1) & 3] >> 16) & 0xff] ^
                   g_te[2][(s[(j + 2) & 3] >> 8) & 0xff] ^ g_te[3][s[(j + 3) & 3] & 0xff] ^
                   c->rkw[r][j];
        for (int j = 0; j < 4; ++j) s[j] = t[j];
    }
    for (int j = 0; j < 4; ++j) {
        uint32_t w = ((uint32_t)g_sbox[s[j] >> 24] << 24) |
                     ((uint32_t)g_sbox[(s[(j + 1) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t)g_sbox[(s[(j + 2) & 3] >> 8) & 0xff] << 8) |
                     g_sbox[s[(j + 3) & 3] & 0xff];
        w ^= c->rkw[c->rounds][j];
        out[4 * j] = (uint8_t)(w >> 24); out[4 * j + 1] = (uint8_t)(w >> 16);
        out[4 * j + 2] = (uint8_t)(w >> 8); out[4 * j + 3] = (uint8_t)w;
    }
}

/* The same cipher as SubBytes + ShiftRows + MixColumns on bytes (FIPS-197
 * 5.1); used only by oracle_selfcheck() to cross-check the table form. */
static void aes_encrypt_bytes(const aes_ctx* c, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ c->rk[0][i]);
    for (int r = 1; r <= c->rounds; ++r) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: column j, row i takes column (j+i)%4. */
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 4; ++i) t[4 * j + i] = g_sbox[s[4 * ((j + i) & 3) + i]];
        if (r != c->rounds) {
            for (int j = 0; j < 4; ++j) {
                uint8_t a0 = t[4 * j], a1 = t[4 * j + 1], a2 = t[4 * j + 2], a3 = t[4 * j + 3];
                uint8_t all = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                t[4 * j + 0] = (uint8_t)(a0 ^ all ^ gf_mul((uint8_t)(a0 ^ a1), 2));
                t[4 * j + 1] = (uint8_t)(a1 ^ all ^ gf_mul((uint8_t)(a1 ^ a2), 2));
                t[4 * j + 2] = (uint8_t)(a2 ^ all ^ gf_mul((uint8_t)(a2 ^ a3), 2));
                t[4 * j + 3] = (uint8_t)(a3 ^ all ^ gf_mul((uint8_t)(a3 ^ a0), 2));
            }
        }
        for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(t[i] ^ c->rk[r][i]);
    }
    memcpy(out, s, 16);
}

int oracle_aes_encrypt_block(const uint8_t* key, size_t keylen,
                             const uint8_t in[16], uint8_t out[16]) {
    aes_ctx c;
    if (aes_setup(&c, key, keylen)) return -1;
    aes_encrypt(&c, in, out);
    return 0;
}

/* ----------------------------------------------------------------- GHASH --
 * aesgcm.py:8-14: a field element is the big-endian integer of the 16-byte
 * block, x^0 at the most significant bit.  Held here as (hi, lo) 64-bit
 * halves of that integer.                                                  */
typedef struct { uint64_t hi, lo; } u128;

static const uint16_t k_gcm_reduction[16] = {  /* aesgcm.py:190-193 */
    0x0000, 0x1c20, 0x3840, 0x2460, 0x7080, 0x6ca0, 0x48c0, 0x54e0,
    0xe100, 0xfd20, 0xd940, 0xc560, 0x9180, 0x8da0, 0xa9c0, 0xb5e0,
};

static u128 load_be128(const uint8_t* b) {
    u128 r = {0, 0};
    for (int i = 0; i < 8; ++i) r.hi = (r.hi << 8) | b[i];
    for (int i = 8; i < 16; ++i) r.lo = (r.lo << 8) | b[i];
    return r;
}

static void store_be128(u128 v, uint8_t* b) {
    for (int i = 7; i >= 0; --i) { b[i] = (uint8_t)v.hi; v.hi >>= 8; }
    for (int i = 15; i >= 8; --i) { b[i] = (uint8_t)v.lo; v.lo >>= 8; }
}

static unsigned rev4(unsigned i) {  /* AESGCM._reverseBits, aesgcm.py:157-162 */
    i = ((i << 2) & 0xc) | ((i >> 2) & 0x3);
    return ((i << 1) & 0xa) | ((i >> 1) & 0x5);
}

static u128 gcm_shift(u128 x) {  /* AESGCM._gcmShift, aesgcm.py:168-178 */
    uint64_t high = x.lo & 1;
    x.lo = (x.lo >> 1) | (x.hi << 63);
    x.hi >>= 1;
    if (high) x.hi ^= (uint64_t)0xe1 << 56;
    return x;
}

typedef struct {
    aes_ctx aes;
    u128 table[16];   /* 4-bit multiples of H, aesgcm.py:46-57 */
    u128 table8[256]; /* the same products a byte at a time (see gcm_mul) */
} gcm_ctx;

/* Reduction of the byte shifted out by y*x^8 (the 8-bit widening of the
 * reference's _gcmReductionTable, aesgcm.py:190-193: bit i of the byte is the
 * coefficient of x^(127-i) and folds back as x^(7-i) * (1 + x + x^2 + x^7)). */
static uint16_t g_red8[256];
static pthread_once_t g_red8_once = PTHREAD_ONCE_INIT;

static void build_red8(void) {
    for (unsigned b = 0; b < 256; ++b) {
        uint16_t r = 0;
        for (int i = 0; i < 8; ++i)
            if (b & (1u << i)) r ^= (uint16_t)(0xe100 >> (7 - i));
        g_red8[b] = r;
    }
}

/* AESGCM._mul, aesgcm.py:81-99: y*H, four bits at a time (the reference's
 * own formulation; oracle_selfcheck() compares gcm_mul with it). */
static u128 gcm_mul4(const gcm_ctx* g, u128 y) {
    u128 ret = {0, 0};
    for (int i = 0; i < 32; ++i) {
        unsigned high = (unsigned)(ret.lo & 0xf);
        ret.lo = (ret.lo >> 4) | (ret.hi << 60);
        ret.hi >>= 4;
        ret.hi ^= (uint64_t)k_gcm_reduction[high] << 48;
        u128 p = g->table[y.lo & 0xf];
        ret.hi ^= p.hi; ret.lo ^= p.lo;
        y.lo = (y.lo >> 4) | (y.hi << 60);
        y.hi >>= 4;
    }
    return ret;
}

static void gcm_set_h(gcm_ctx* g, u128 h);

static int gcm_setup(gcm_ctx* g, const uint8_t* key, size_t keylen) {
    if (keylen != 16 && keylen != 32) return -1;  /* aesgcm.py:33-38 */
    if (aes_setup(&g->aes, key, keylen)) return -1;
    uint8_t zero[16] = {0}, hb[16];
    aes_encrypt(&g->aes, zero, hb);                  /* H = E_K(0), :45 */
    gcm_set_h(g, load_be128(hb));
    return 0;
}

/* The product tables of H (aesgcm.py:46-57). */
static void gcm_set_h(gcm_ctx* g, u128 h) {
    pthread_once(&g_red8_once, build_red8);
    memset(g->table, 0, sizeof(g->table));
    g->table[rev4(1)] = h;
    for (unsigned i = 2; i < 16; i += 2) {
        g->table[rev4(i)] = gcm_shift(g->table[rev4(i / 2)]);
        u128 t = g->table[rev4(i)];
        t.hi ^= h.hi; t.lo ^= h.lo;
        g->table[rev4(i + 1)] = t;
    }
    /* table8[b] = H * (b at the top byte): bit 7 of b is x^0, bit 0 is x^7,
     * so table8[0x80 >> k] = H * x^k, and the rest follow by linearity. */
    u128 basis[8];
    basis[0] = h;
    for (int k = 1; k < 8; ++k) basis[k] = gcm_shift(basis[k - 1]);
    for (unsigned b = 0; b < 256; ++b) {
        u128 t = {0, 0};
        for (int k = 0; k < 8; ++k)
            if (b & (0x80u >> k)) { t.hi ^= basis[k].hi; t.lo ^= basis[k].lo; }
        g->table8[b] = t;
    }
}

/* y*H a byte at a time: the Horner loop of AESGCM._mul (aesgcm.py:86-97) with
 * eight-bit digits instead of four. */
static u128 gcm_mul(const gcm_ctx* g, u128 y) {
    u128 ret = {0, 0};
    for (int i = 0; i < 16; ++i) {
        unsigned high = (unsigned)(ret.lo & 0xff);
        ret.lo = (ret.lo >> 8) | (ret.hi << 56);
        ret.hi >>= 8;
        ret.hi ^= (uint64_t)g_red8[high] << 48;
        u128 p = g->table8[y.lo & 0xff];
        ret.hi ^= p.hi; ret.lo ^= p.lo;
        y.lo = (y.lo >> 8) | (y.hi << 56);
        y.hi >>= 8;
    }
    return ret;
}

/* AESGCM._update, aesgcm.py:69-79 (zero-pad the final partial block). */
static u128 gcm_update(const gcm_ctx* g, u128 y, const uint8_t* d, size_t n) {
    size_t full = n / 16;
    for (size_t i = 0; i < full; ++i) {
        u128 b = load_be128(d + 16 * i);
        y.hi ^= b.hi; y.lo ^= b.lo;
        y = gcm_mul(g, y);
    }
    size_t extra = n % 16;
    if (extra) {
        uint8_t blk[16] = {0};
        memcpy(blk, d + 16 * full, extra);
        u128 b = load_be128(blk);
        y.hi ^= b.hi; y.lo ^= b.lo;
        y = gcm_mul(g, y);
    }
    return y;
}

/* AESGCM._auth, aesgcm.py:60-67. */
static void gcm_auth(const gcm_ctx* g, const uint8_t* ct, size_t ctlen,
                     const uint8_t* ad, size_t adlen, const uint8_t mask[16],
                     uint8_t tag[16]) {
    u128 y = {0, 0};
    y = gcm_update(g, y, ad, adlen);
    y = gcm_update(g, y, ct, ctlen);
    y.hi ^= (uint64_t)adlen << 3;
    y.lo ^= (uint64_t)ctlen << 3;
    y = gcm_mul(g, y);
    u128 m = load_be128(mask);
    y.hi ^= m.hi; y.lo ^= m.lo;
    store_be128(y, tag);
}

/* AESGCM._auth without the tag mask, for a given H: the GHASH value the
 * reference's _auth returns before the XOR with E_K(J0) (aesgcm.py:60-67). */
void oracle_ghash(const uint8_t h[16], const uint8_t* aad, size_t aadlen,
                  const uint8_t* ct, size_t ctlen, uint8_t out[16]) {
    static gcm_ctx g;   /* 4.3 KiB of tables: keep them off the caller's stack */
    static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    uint8_t zero[16] = {0};
    pthread_mutex_lock(&mu);
    gcm_set_h(&g, load_be128(h));
    gcm_auth(&g, ct, ctlen, aad, aadlen, zero, out);
    pthread_mutex_unlock(&mu);
}

/* Python_AES_CTR.encrypt with a full 128-bit big-endian counter increment
 * (python_aes.py:101-116). */
static void gcm_ctr(const gcm_ctx* g, uint8_t counter[16], const uint8_t* in,
                    size_t n, uint8_t* out) {
    uint8_t ks[16];
    for (size_t off = 0; off < n; off += 16) {
        aes_encrypt(&g->aes, counter, ks);
        size_t m = n - off < 16 ? n - off : 16;
        for (size_t k = 0; k < m; ++k) out[off + k] = (uint8_t)(in[off + k] ^ ks[k]);
        for (int k = 15; k >= 0; --k)
            if (++counter[k]) break;
    }
}

static int gcm_seal_ctx(const gcm_ctx* g, const uint8_t* nonce,
                        const uint8_t* aad, size_t aadlen, const uint8_t* pt,
                        size_t len, uint8_t* out) {
    uint8_t counter[16] = {0}, mask[16];
    memcpy(counter, nonce, 12);
    counter[15] = 1;                                  /* aesgcm.py:112-115 */
    aes_encrypt(&g->aes, counter, mask);
    counter[15] = 2;                                  /* :118-120 */
    gcm_ctr(g, counter, pt, len, out);
    gcm_auth(g, out, len, aad, aadlen, mask, out + len);
    return 0;
}

static int gcm_open_ctx(const gcm_ctx* g, const uint8_t* nonce,
                        const uint8_t* aad, size_t aadlen, const uint8_t* in,
                        size_t inlen, uint8_t* pt) {
    if (inlen < 16) return 0;                         /* aesgcm.py:135-136 */
    size_t len = inlen - 16;
    uint8_t counter[16] = {0}, mask[16], tag[16];
    memcpy(counter, nonce, 12);
    counter[15] = 1;
    aes_encrypt(&g->aes, counter, mask);
    gcm_auth(g, in, len, aad, aadlen, mask, tag);
    uint8_t diff = 0;                                 /* constanttime.py:209-218 */
    for (int k = 0; k < 16; ++k) diff |= (uint8_t)(tag[k] ^ in[len + k]);
    if (diff) return 0;                               /* aesgcm.py:148-149 */
    counter[15] = 2;
    gcm_ctr(g, counter, in, len, pt);
    return 1;
}

int oracle_gcm_seal(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* pt, size_t len, uint8_t* out) {
    gcm_ctx g;
    if (gcm_setup(&g, key, keylen)) return -2;
    if (noncelen != 12) return -1;                    /* aesgcm.py:107-108 */
    return gcm_seal_ctx(&g, nonce, aad, aadlen, pt, len, out);
}

int oracle_gcm_open(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* in, size_t inlen, uint8_t* pt) {
    gcm_ctx g;
    if (gcm_setup(&g, key, keylen)) return -2;
    if (noncelen != 12) return -1;                    /* aesgcm.py:133-134 */
    return gcm_open_ctx(&g, nonce, aad, aadlen, in, inlen, pt);
}

/* ---------------------------------------------------------------- ChaCha --
 * chacha.py:98-153: state = constants || key words || counter || nonce words
 * (all little-endian), 10 double rounds (column then diagonal order,
 * chacha.py:59-66), feed-forward add, little-endian serialisation.          */
static uint32_t ld32le(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

static void st32le(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                      \
    a += b; d ^= a; d = ROTL32(d, 16);      \
    c += d; b ^= c; b = ROTL32(b, 12);      \
    a += b; d ^= a; d = ROTL32(d, 8);       \
    c += d; b ^= c; b = ROTL32(b, 7);

static void chacha_block(const uint32_t key[8], uint32_t counter,
                         const uint32_t nonce[3], uint8_t out[64]) {
    uint32_t s[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
    for (int i = 0; i < 8; ++i) s[4 + i] = key[i];
    s[12] = counter;
    for (int i = 0; i < 3; ++i) s[13 + i] = nonce[i];
    uint32_t x[16];
    memcpy(x, s, sizeof(x));
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) st32le(out + 4 * i, x[i] + s[i]);
}

int oracle_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12],
                        uint32_t counter, const uint8_t* in, size_t len,
                        uint8_t* out) {
    uint32_t k[8], n[3];
    for (int i = 0; i < 8; ++i) k[i] = ld32le(key + 4 * i);
    for (int i = 0; i < 3; ++i) n[i] = ld32le(nonce + 4 * i);
    uint8_t ks[64];
    for (size_t off = 0, i = 0; off < len; off += 64, ++i) {
        chacha_block(k, counter + (uint32_t)i, n, ks);
        size_t m = len - off < 64 ? len - off : 64;
        for (size_t j = 0; j < m; ++j) out[off + j] = (uint8_t)(in[off + j] ^ ks[j]);
    }
    return 0;
}

/* -------------------------------------------------------------- Poly1305 --
 * poly1305.py:32-48: acc = (acc + LE(chunk || 0x01)) * r mod 2^130-5 per
 * 16-byte chunk (a short final chunk gets its 0x01 right after its bytes),
 * tag = LE16((acc + s) mod 2^128).  Restated with three 44/44/42-bit limbs. */
typedef unsigned __int128 u128n;
#define M44 ((uint64_t)0xfffffffffffULL)
#define M42 ((uint64_t)0x3ffffffffffULL)

typedef struct {
    uint64_t r0, r1, r2, s1, s2;
    uint64_t h0, h1, h2;
    uint64_t pad0, pad1;
} poly_ctx;

static uint64_t ld64le(const uint8_t* p) {
    return (uint64_t)ld32le(p) | ((uint64_t)ld32le(p + 4) << 32);
}

static void poly_init(poly_ctx* p, const uint8_t key[32]) {
    uint64_t t0 = ld64le(key), t1 = ld64le(key + 8);
    t0 &= 0x0ffffffc0fffffffULL;                    /* clamp, poly1305.py:38 */
    t1 &= 0x0ffffffc0ffffffcULL;
    p->r0 = t0 & M44;
    p->r1 = ((t0 >> 44) | (t1 << 20)) & M44;
    p->r2 = (t1 >> 24) & M42;
    p->s1 = p->r1 * 20;  /* 2^132 = 4 * 2^130 == 20 (mod p) */
    p->s2 = p->r2 * 20;
    p->h0 = p->h1 = p->h2 = 0;
    p->pad0 = ld64le(key + 16);
    p->pad1 = ld64le(key + 24);
}

static void poly_block(poly_ctx* p, const uint8_t m[16], uint64_t hibit) {
    uint64_t t0 = ld64le(m), t1 = ld64le(m + 8);
    uint64_t h0 = p->h0 + (t0 & M44);
    uint64_t h1 = p->h1 + (((t0 >> 44) | (t1 << 20)) & M44);
    uint64_t h2 = p->h2 + (((t1 >> 24) & M42) | hibit);
    u128n d0 = (u128n)h0 * p->r0 + (u128n)h1 * p->s2 + (u128n)h2 * p->s1;
    u128n d1 = (u128n)h0 * p->r1 + (u128n)h1 * p->r0 + (u128n)h2 * p->s2;
    u128n d2 = (u128n)h0 * p->r2 + (u128n)h1 * p->r1 + (u128n)h2 * p->r0;
    uint64_t c;
    c = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & M44;
    d1 += c; c = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & M44;
    d2 += c; c = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & M42;
    h0 += c * 5; c = h0 >> 44; h0 &= M44;
    h1 += c;
    p->h0 = h0; p->h1 = h1; p->h2 = h2;
}

static void poly_finish(poly_ctx* p, uint8_t tag[16]) {
    uint64_t h0 = p->h0, h1 = p->h1, h2 = p->h2, c;
    c = h1 >> 44; h1 &= M44; h2 += c;
    c = h2 >> 42; h2 &= M42; h0 += c * 5;
    c = h0 >> 44; h0 &= M44; h1 += c;
    c = h1 >> 44; h1 &= M44; h2 += c;
    c = h2 >> 42; h2 &= M42; h0 += c * 5;
    c = h0 >> 44; h0 &= M44; h1 += c;
    /* g = h + 5 - 2^130; take g when h >= p */
    uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
    uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
    uint64_t g2 = h2 + c - ((uint64_t)1 << 42);
    uint64_t mask = (g2 >> 63) - 1;  /* all ones when g2 did not borrow */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    /* (h + s) mod 2^128 */
    uint64_t lo = h0 | (h1 << 44);
    uint64_t hi = (h1 >> 20) | (h2 << 24);
    u128n acc = ((u128n)hi << 64 | lo) + ((u128n)p->pad1 << 64 | p->pad0);
    for (int i = 0; i < 16; ++i) tag[i] = (uint8_t)(acc >> (8 * i));
}

void oracle_poly1305(const uint8_t key[32], const uint8_t* data, size_t len,
                     uint8_t tag[16]) {
    poly_ctx p;
    poly_init(&p, key);
    size_t off = 0;
    for (; off + 16 <= len; off += 16) poly_block(&p, data + off, (uint64_t)1 << 40);
    if (off < len) {
        uint8_t blk[16] = {0};
        memcpy(blk, data + off, len - off);
        blk[len - off] = 1;
        poly_block(&p, blk, 0);
    }
    poly_finish(&p, tag);
}

/* mac_data = aad || pad16 || ct || pad16 || le64(aadlen) || le64(ctlen),
 * chacha20_poly1305.py:60-63, streamed block by block. */
static void chacha_aead_tag(const uint8_t otk[32], const uint8_t* aad,
                            size_t aadlen, const uint8_t* ct, size_t ctlen,
                            uint8_t tag[16]) {
    poly_ctx p;
    poly_init(&p, otk);
    const uint64_t hb = (uint64_t)1 << 40;
    uint8_t blk[16];
    for (size_t off = 0; off < aadlen; off += 16) {
        size_t m = aadlen - off < 16 ? aadlen - off : 16;
        memset(blk, 0, 16);
        memcpy(blk, aad + off, m);
        poly_block(&p, blk, hb);
    }
    for (size_t off = 0; off < ctlen; off += 16) {
        size_t m = ctlen - off < 16 ? ctlen - off : 16;
        memset(blk, 0, 16);
        memcpy(blk, ct + off, m);
        poly_block(&p, blk, hb);
    }
    for (int i = 0; i < 8; ++i) {
        blk[i] = (uint8_t)((uint64_t)aadlen >> (8 * i));
        blk[8 + i] = (uint8_t)((uint64_t)ctlen >> (8 * i));
    }
    poly_block(&p, blk, hb);
    poly_finish(&p, tag);
}

static void chacha_otk(const uint8_t* key, const uint8_t* nonce, uint8_t otk[32]) {
    uint8_t zero[32] = {0};                  /* chacha20_poly1305.py:35-38 */
    oracle_chacha20_xor(key, nonce, 0, zero, 32, otk);
}

int oracle_chacha_seal(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                       size_t noncelen, const uint8_t* aad, size_t aadlen,
                       const uint8_t* pt, size_t len, uint8_t* out) {
    if (keylen != 32) return -2;                      /* :21-22 */
    if (noncelen != 12) return -1;                    /* :53-54 */
    uint8_t otk[32];
    chacha_otk(key, nonce, otk);
    oracle_chacha20_xor(key, nonce, 1, pt, len, out); /* :58 */
    chacha_aead_tag(otk, aad, aadlen, out, len, out + len);
    return 0;
}

int oracle_chacha_open(const uint8_t* key, size_t keylen, const uint8_t* nonce,
                       size_t noncelen, const uint8_t* aad, size_t aadlen,
                       const uint8_t* in, size_t inlen, uint8_t* pt) {
    if (keylen != 32) return -2;
    if (noncelen != 12) return -1;                    /* :73-74 */
    if (inlen < 16) return 0;                         /* :76-77 */
    size_t len = inlen - 16;
    uint8_t otk[32], tag[16];
    chacha_otk(key, nonce, otk);
    chacha_aead_tag(otk, aad, aadlen, in, len, tag);
    uint8_t diff = 0;
    for (int k = 0; k < 16; ++k) diff |= (uint8_t)(tag[k] ^ in[len + k]);
    if (diff) return 0;                               /* :90-91 */
    oracle_chacha20_xor(key, nonce, 1, in, len, pt);  /* :93 */
    return 1;
}

/* ------------------------------------------------------------------- CCM --
 * AESCCM (aesccm.py:11-155, RFC 3610 with a 12-byte nonce, so L = 3).     */

/* numberToByteArray(v, n) (cryptomath.py:210-225): big-endian, keeping the
 * low n bytes when v does not fit. */
static void put_be(uint8_t* p, uint64_t v, int n) {
    for (int k = n - 1; k >= 0; --k, v >>= 8) p[k] = (uint8_t)v;
}

/* AESCCM._cbcmac_calc, aesccm.py:36-83: CBC-MAC with a zero IV over
 * B_0 || enc(len(aad)) || aad || pad16 || msg || pad16. */
static void ccm_cbcmac(const aes_ctx* c, size_t taglen, const uint8_t* nonce,
                       const uint8_t* aad, size_t aadlen, const uint8_t* msg,
                       size_t len, uint8_t mac[16]) {
    uint8_t x[16], blk[16];
    /* flags (:40-43), B_0 (:46) */
    blk[0] = (uint8_t)(64 * (aadlen > 0) + 8 * ((taglen - 2) / 2) + (3 - 1));
    memcpy(blk + 1, nonce, 12);
    put_be(blk + 13, len, 3);
    aes_encrypt(c, blk, x);
    if (aadlen) {
        /* length encoding (:48-58) then aad, zero-padded to a block (:63-67) */
        uint8_t pre[10];
        size_t np;
        if (aadlen < 0xff00) {
            put_be(pre, aadlen, 2); np = 2;
        } else if ((uint64_t)aadlen < 0x100000000ull) {
            pre[0] = 0xff; pre[1] = 0xfe; put_be(pre + 2, aadlen, 4); np = 6;
        } else {
            pre[0] = 0xff; pre[1] = 0xff; put_be(pre + 2, aadlen, 8); np = 10;
        }
        size_t total = np + aadlen;
        for (size_t off = 0; off < total; off += 16) {
            for (size_t k = 0; k < 16; ++k) {
                size_t s = off + k;
                uint8_t b = s < np ? pre[s] : (s < total ? aad[s - np] : 0);
                blk[k] = (uint8_t)(x[k] ^ b);
            }
            aes_encrypt(c, blk, x);
        }
    }
    for (size_t off = 0; off < len; off += 16) {   /* msg, zero-padded (:68-70) */
        for (size_t k = 0; k < 16; ++k)
            blk[k] = (uint8_t)(x[k] ^ (off + k < len ? msg[off + k] : 0));
        aes_encrypt(c, blk, x);
    }
    memcpy(mac, x, 16);                               /* :78-83 (caller truncates) */
}

/* Python_AES_CTR from counter block s_j = 2 || nonce || be24(j): the
 * reference's 128-bit increment (python_aes.py:101-107) from s_0. */
static void ccm_ctr_block(const aes_ctx* c, const uint8_t* nonce, uint64_t j, uint8_t ks[16]) {
    uint8_t a[16];
    a[0] = 2;                                         /* flags = L - 1 (aesccm.py:99) */
    memcpy(a + 1, nonce, 12);
    a[13] = a[14] = a[15] = 0;
    for (int k = 15; k >= 0 && j; --k) {              /* a += j, big-endian */
        uint64_t v = (uint64_t)a[k] + (j & 0xff);
        a[k] = (uint8_t)v;
        j = (j >> 8) + (v >> 8);
    }
    aes_encrypt(c, a, ks);
}

static void ccm_ctr(const aes_ctx* c, const uint8_t* nonce, const uint8_t* in, size_t n,
                    uint8_t* out) {
    uint8_t ks[16];
    for (size_t off = 0; off < n; off += 16) {
        ccm_ctr_block(c, nonce, 1 + off / 16, ks);   /* S_1.. encrypt the message */
        size_t m = n - off < 16 ? n - off : 16;
        for (size_t k = 0; k < m; ++k) out[off + k] = (uint8_t)(in[off + k] ^ ks[k]);
    }
}

/* AESCCM.seal, aesccm.py:85-113: out = ct || tag (len + taglen bytes). */
static int ccm_seal_ctx(const aes_ctx* c, size_t taglen, const uint8_t* nonce,
                        const uint8_t* aad, size_t aadlen, const uint8_t* pt, size_t len,
                        uint8_t* out) {
    uint8_t mac[16], s0[16];
    ccm_cbcmac(c, taglen, nonce, aad, aadlen, pt, len, mac);
    ccm_ctr_block(c, nonce, 0, s0);                   /* auth value = mac ^ E(S_0) */
    ccm_ctr(c, nonce, pt, len, out);
    for (size_t k = 0; k < taglen; ++k) out[len + k] = (uint8_t)(mac[k] ^ s0[k]);
    return 0;
}

/* AESCCM.open, aesccm.py:115-149: decrypt, recompute the MAC over the
 * plaintext, compare; 0 (None) on mismatch or when inlen < taglen. */
static int ccm_open_ctx(const aes_ctx* c, size_t taglen, const uint8_t* nonce,
                        const uint8_t* aad, size_t aadlen, const uint8_t* in, size_t inlen,
                        uint8_t* pt) {
    if (inlen < taglen) return 0;                     /* :120-123 */
    size_t len = inlen - taglen;
    uint8_t mac[16], s0[16];
    ccm_ctr(c, nonce, in, len, pt);
    ccm_cbcmac(c, taglen, nonce, aad, aadlen, pt, len, mac);
    ccm_ctr_block(c, nonce, 0, s0);
    uint8_t diff = 0;                                 /* received_mac != computed_mac (:145) */
    for (size_t k = 0; k < taglen; ++k) diff |= (uint8_t)(mac[k] ^ s0[k] ^ in[len + k]);
    if (diff) {
        memset(pt, 0, len);
        return 0;
    }
    return 1;
}

int oracle_ccm_seal(const uint8_t* key, size_t keylen, size_t taglen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* pt, size_t len, uint8_t* out) {
    aes_ctx c;
    if ((keylen != 16 && keylen != 32) || (taglen != 8 && taglen != 16)) return -2;  /* :22-30 */
    if (aes_setup(&c, key, keylen)) return -2;
    if (noncelen != 12) return -1;                    /* :87-88 */
    return ccm_seal_ctx(&c, taglen, nonce, aad, aadlen, pt, len, out);
}

int oracle_ccm_open(const uint8_t* key, size_t keylen, size_t taglen, const uint8_t* nonce,
                    size_t noncelen, const uint8_t* aad, size_t aadlen,
                    const uint8_t* in, size_t inlen, uint8_t* pt) {
    aes_ctx c;
    if ((keylen != 16 && keylen != 32) || (taglen != 8 && taglen != 16)) return -2;
    if (aes_setup(&c, key, keylen)) return -2;
    if (noncelen != 12) return -1;                    /* :117-118 */
    return ccm_open_ctx(&c, taglen, nonce, aad, aadlen, in, inlen, pt);
}

/* ----------------------------------------------------------------- batch */
typedef struct {
    int alg, op;
    const uint8_t* keys; size_t keylen; const uint32_t* key_idx;
    const uint8_t* nonces; const uint8_t* aad; const uint64_t* aad_off;
    const uint32_t* aad_len; const uint8_t* in; const uint64_t* in_off;
    const uint32_t* inlen; uint8_t* out; const uint64_t* out_off;
    uint8_t* status; size_t begin, end; int rc;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    gcm_ctx g;
    aes_ctx a;
    uint32_t cur_key = 0xffffffffu;
    for (size_t i = j->begin; i < j->end; ++i) {
        uint32_t ki = j->key_idx ? j->key_idx[i] : 0;
        const uint8_t* key = j->keys + (size_t)ki * j->keylen;
        const uint8_t* nonce = j->nonces + 12 * i;
        const uint8_t* ad = j->aad + j->aad_off[i];
        const uint8_t* src = j->in + j->in_off[i];
        uint8_t* dst = j->out + j->out_off[i];
        int rc;
        if (j->alg == 0) {
            if (ki != cur_key) {
                if (gcm_setup(&g, key, j->keylen)) { j->rc = -1; return NULL; }
                cur_key = ki;
            }
            rc = j->op == 0 ? gcm_seal_ctx(&g, nonce, ad, j->aad_len[i], src, j->inlen[i], dst)
                            : gcm_open_ctx(&g, nonce, ad, j->aad_len[i], src, j->inlen[i], dst);
        } else if (j->alg == 2 || j->alg == 3) {
            size_t tl = j->alg == 2 ? 16 : 8;
            if (ki != cur_key) {
                if (aes_setup(&a, key, j->keylen)) { j->rc = -1; return NULL; }
                cur_key = ki;
            }
            rc = j->op == 0 ? ccm_seal_ctx(&a, tl, nonce, ad, j->aad_len[i], src, j->inlen[i], dst)
                            : ccm_open_ctx(&a, tl, nonce, ad, j->aad_len[i], src, j->inlen[i], dst);
        } else {
            rc = j->op == 0 ? oracle_chacha_seal(key, j->keylen, nonce, 12, ad, j->aad_len[i],
                                                 src, j->inlen[i], dst)
                            : oracle_chacha_open(key, j->keylen, nonce, 12, ad, j->aad_len[i],
                                                 src, j->inlen[i], dst);
        }
        if (rc < 0) { j->rc = -1; return NULL; }
        if (j->op == 1 && j->status) j->status[i] = (uint8_t)rc;
    }
    return NULL;
}

int oracle_batch(int alg, int op, const uint8_t* keys, size_t keylen,
                 const uint32_t* key_idx, const uint8_t* nonces,
                 const uint8_t* aad, const uint64_t* aad_off,
                 const uint32_t* aad_len, const uint8_t* in,
                 const uint64_t* in_off, const uint32_t* inlen, uint8_t* out,
                 const uint64_t* out_off, uint8_t* status, size_t n,
                 int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    batch_job jobs[256];
    pthread_t th[256];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; ++t) {
        batch_job* j = &jobs[t];
        j->alg = alg; j->op = op; j->keys = keys; j->keylen = keylen;
        j->key_idx = key_idx; j->nonces = nonces; j->aad = aad;
        j->aad_off = aad_off; j->aad_len = aad_len; j->in = in;
        j->in_off = in_off; j->inlen = inlen; j->out = out;
        j->out_off = out_off; j->status = status; j->rc = 0;
        j->begin = (size_t)t * per < n ? (size_t)t * per : n;
        j->end = j->begin + per < n ? j->begin + per : n;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    for (int t = 0; t < nthreads; ++t)
        if (jobs[t].rc) return -1;
    return 0;
}

/* ------------------------------------------------------------ self-check --
 * The fast forms above against the reference's own formulations: the T-table
 * cipher against SubBytes/ShiftRows/MixColumns on bytes, and the byte-wise
 * GHASH multiply against the nibble-wise AESGCM._mul.  Returns the number of
 * mismatches over n random (key, block) pairs. */
static uint64_t xs64(uint64_t* s) {
    *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17;
    return *s;
}

int oracle_selfcheck(size_t n, uint64_t seed) {
    int bad = 0;
    uint64_t s = seed | 1;
    for (size_t i = 0; i < n; ++i) {
        uint8_t key[32], blk[16], a[16], b[16];
        for (int k = 0; k < 32; ++k) key[k] = (uint8_t)xs64(&s);
        for (int k = 0; k < 16; ++k) blk[k] = (uint8_t)xs64(&s);
        gcm_ctx g;
        gcm_setup(&g, key, (i & 1) ? 32 : 16);
        aes_encrypt(&g.aes, blk, a);
        aes_encrypt_bytes(&g.aes, blk, b);
        bad += memcmp(a, b, 16) != 0;
        u128 y = load_be128(blk);
        u128 p = gcm_mul(&g, y), q = gcm_mul4(&g, y);
        bad += (p.hi != q.hi) || (p.lo != q.lo);
    }
    return bad;
}
