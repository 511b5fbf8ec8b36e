// bs_check.cpp -- CPU check of the bitsliced AES-CTR core (csrc/aes_bs.h)
// against a byte-wise AES.  g++ -O2 -I tlslite-ng_amd/csrc tools/bs_check.cpp
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <initializer_list>
#include "aes_bs.h"

static uint8_t S[256];
static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
static void make_sbox() {
    uint8_t p = 1, q = 1;
    S[0] = 0x63;
    do {
        p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1b : 0);
        q ^= q << 1; q ^= q << 2; q ^= q << 4;
        if (q & 0x80) q ^= 0x09;
        uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        S[p] = x ^ 0x63;
    } while (p != 1);
}
static void expand(const uint8_t* key, int nk, uint8_t* rk) {  // rk: 16*(nr+1)
    int nr = nk + 6, tot = 4 * (nr + 1);
    memcpy(rk, key, 4 * nk);
    uint8_t rc = 1;
    for (int i = nk; i < tot; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t u = t[0];
            t[0] = S[t[1]] ^ rc; t[1] = S[t[2]]; t[2] = S[t[3]]; t[3] = S[u];
            rc = xt(rc);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = S[t[k]];
        }
        for (int k = 0; k < 4; ++k) rk[4 * i + k] = rk[4 * (i - nk) + k] ^ t[k];
    }
}
static void enc(const uint8_t* rk, int nr, const uint8_t* in, uint8_t* out) {
    uint8_t s[16];
    for (int k = 0; k < 16; ++k) s[k] = in[k] ^ rk[k];
    for (int r = 1; r <= nr; ++r) {
        uint8_t t[16];
        for (int c = 0; c < 4; ++c)
            for (int i = 0; i < 4; ++i) t[i + 4 * c] = S[s[i + 4 * ((c + i) & 3)]];
        if (r < nr) {
            for (int c = 0; c < 4; ++c) {
                uint8_t* a = t + 4 * c;
                uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                a[0] = xt(a0) ^ xt(a1) ^ a1 ^ a2 ^ a3;
                a[1] = a0 ^ xt(a1) ^ xt(a2) ^ a2 ^ a3;
                a[2] = a0 ^ a1 ^ xt(a2) ^ xt(a3) ^ a3;
                a[3] = xt(a0) ^ a0 ^ a1 ^ a2 ^ xt(a3);
            }
        }
        for (int k = 0; k < 16; ++k) s[k] = t[k] ^ rk[16 * r + k];
    }
    memcpy(out, s, 16);
}
static uint32_t le(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

template <int NR>
static int run(int nk, unsigned seed) {
    srand(seed);
    uint8_t key[32], rk[16 * 15], nonce[12];
    for (int i = 0; i < 32; ++i) key[i] = rand();
    for (int i = 0; i < 12; ++i) nonce[i] = rand();
    expand(key, nk, rk);
    uint32_t kw[4 * 15];
    for (int r = 0; r <= NR; ++r)
        for (int q = 0; q < 4; ++q) kw[4 * r + q] = le(rk + 16 * r + 4 * q) ^ (r ? 0x63636363u : 0);
    tg::bs::BsKey bk{kw};
    uint32_t rk0[4];
    for (int q = 0; q < 4; ++q) rk0[q] = le(rk + 4 * q);
    uint8_t sb[12];
    for (int k = 0; k < 12; ++k) sb[k] = S[nonce[k] ^ rk[k]] ^ 0x63;
    uint32_t s1w[3] = {le(sb), le(sb + 4), le(sb + 8)};
    int bad = 0;
    for (uint32_t j : {0u, 1u, 7u, 31u, 0x7ffffu, 0x7fffffeu}) {
        uint32_t base = 2 + 32 * j;
        uint32_t w[4][32];
        tg::bs::ctr32<NR>(bk, rk0[3], s1w, base, w);
        for (int i = 0; i < 32; ++i) {
            uint8_t blk[16], want[16];
            memcpy(blk, nonce, 12);
            uint32_t c = base + i;
            blk[12] = c >> 24; blk[13] = c >> 16; blk[14] = c >> 8; blk[15] = c;
            enc(rk, NR, blk, want);
            for (int q = 0; q < 4; ++q)
                if ((w[q][i] ^ bk.w[4 * NR + q]) != le(want + 4 * q)) { ++bad; break; }
        }
    }
    printf("NR=%d seed=%u mismatching blocks: %d\n", NR, seed, bad);
    return bad;
}

int main() {
    make_sbox();
    int bad = 0;
    for (unsigned s = 1; s < 4; ++s) { bad += run<10>(4, s); bad += run<14>(8, s); }
    return bad != 0;
}
