// bs8_check.cpp -- CPU check of the 8-block bitsliced AES-CTR core
// (tlslite-ng_amd/csrc/aes_bs8.h) against the C oracle's AES block cipher
// (oracle/aead_oracle.c, rijndael.py restated).  TEST INFRASTRUCTURE ONLY.
// Built and run by tests/test_bs8_host.py:
//   g++ -O2 -I tlslite-ng_amd/csrc -I oracle tests/native/bs8_check.cpp oracle/aead_oracle.c
// For AES-128 and AES-256, random keys and nonces, every lane start c0 the GCM
// kernel uses (2..9) and batch indices around every carry boundary, the eight
// keystream blocks nonce || be32(c0 + 64 beta + 8 j) must equal the oracle's.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aead_oracle.h"
#include "aes_bs8.h"

static uint8_t S[256];
static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
static void make_sbox() {   // S from the oracle's own cipher would be circular; build it
    uint8_t p = 1, q = 1;
    S[0] = 0x63;
    do {
        p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1b : 0);
        q ^= q << 1; q ^= q << 2; q ^= q << 4;
        if (q & 0x80) q ^= 0x09;
        const uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                          (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        S[p] = x ^ 0x63;
    } while (p != 1);
}
static void expand(const uint8_t* key, int nk, uint8_t* rk) {   // FIPS-197 key expansion
    const int nr = nk + 6, tot = 4 * (nr + 1);
    memcpy(rk, key, 4 * nk);
    uint8_t rc = 1;
    for (int i = nk; i < tot; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            const uint8_t u = t[0];
            t[0] = S[t[1]] ^ rc; t[1] = S[t[2]]; t[2] = S[t[3]]; t[3] = S[u];
            rc = xt(rc);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = S[t[k]];
        }
        for (int k = 0; k < 4; ++k) rk[4 * i + k] = rk[4 * (i - nk) + k] ^ t[k];
    }
}
static uint32_t le(const uint8_t* p) {
    return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24;
}

// The folded planes (keymath.h bs8_fold_word) in bs8mask order, read as rows:
// encrypt() then runs mix_round_folded (the device's KeyPlanesVmemFolded).
struct FoldedRows {
    static constexpr bool kFolded = true;
    const uint32_t* w;
    tg::bs8::Word4 row4(int r, int b) const {
        return tg::bs8::word4(w[(4 * r) * 8 + b], w[(4 * r + 1) * 8 + b], w[(4 * r + 2) * 8 + b],
                              w[(4 * r + 3) * 8 + b]);
    }
};

// SB: log2 of the lanes per record (3 = the octet kernels; 4..6 = the
// key-grouped kernel with 16 / 32 / 64 lanes per record): block j of a
// lane's batch beta has counter c0 + (j << SB) + (beta << (SB + 3)), c0 =
// 2 + rho, rho < 2^SB.
template <int NR, bool FOLD, int SB = 3>
static int run(int klen, unsigned seed) {
    srand(seed);
    uint8_t key[32], rk[16 * 15], nonce[12];
    for (int i = 0; i < klen; ++i) key[i] = (uint8_t)rand();
    for (int i = 0; i < 12; ++i) nonce[i] = (uint8_t)rand();
    expand(key, klen / 4, rk);
    uint32_t rkw[60];
    for (int q = 0; q < 4 * (NR + 1); ++q) rkw[q] = le(rk + 4 * q);
    uint32_t planes[15 * 32];
    for (int e = 0; e < 32 * (NR + 1); ++e) planes[e] = tg::bs8::mask_word(rkw, e);
    uint32_t folded[15 * 32];
    for (int e = 0; e < 32 * (NR + 1); ++e)
        folded[e] = (e >> 5) >= 1 && (e >> 5) < NR ? tg::bs8_fold_word(rkw, e) : planes[e];
    const tg::bs8::KeyPlanes km{planes};
    const FoldedRows kf{folded};
    const uint32_t u[4] = {le(nonce) ^ rkw[0], le(nonce + 4) ^ rkw[1], le(nonce + 8) ^ rkw[2], rkw[3]};
    int bad = 0, checked = 0;
    const uint32_t betas[] = {0, 1, 2, 3, 7, 15, 16, 255, 256, 1022, 1023, 1024, 1025,
                              65535, 65536, 0x3ffffe, 0x3fffff};
    constexpr uint32_t L = 1u << SB;
    for (uint32_t c0 = 2; c0 <= L + 1; c0 += (SB > 3 ? 3 : 1)) {
        uint32_t lane[SB + 3], kmask;
        tg::bs8::lane_consts<SB>(c0, lane, kmask);
        for (uint32_t beta : betas) {
          if ((uint64_t)beta << (SB + 3) >= (1ull << 31)) continue;   // counters stay 32-bit
          const bool hi = (beta + 1u) >> (16 - (SB + 3));
          // pre01: rows 0-1 enter after round 1's SubBytes, computed once from
          // the record planes (the kernels' path for counters below 2^16)
          for (int pre01 = 0; pre01 <= (hi ? 0 : 1); ++pre01) {
            uint32_t s[4][8], w[4][8];
            for (int i = 0; i < 4; ++i)
                for (int b = 0; b < 8; ++b) s[i][b] = tg::bs8::rec_plane(u, 8 * i + b);
            if (pre01) {
                tg::bs::sbox(s[0]);
                tg::bs::sbox(s[1]);
            }
            for (int b = 0; b < SB + 3; ++b) s[3 - (b >> 3)][b & 7] ^= lane[b];
            tg::bs8::ctr_planes<SB + 3, 16, SB + 3>(s, kmask, beta);
            if (hi) tg::bs8::ctr_planes<16, 32, SB + 3>(s, kmask, beta);
            if (FOLD)
                tg::bs8::encrypt<NR>(s, kf, w, !pre01);
            else
                tg::bs8::encrypt<NR>(s, km, w, !pre01);
            for (int j = 0; j < 8; ++j) {
                const uint32_t ctr = c0 + (beta << (SB + 3)) + ((uint32_t)j << SB);
                uint8_t blk[16], want[16];
                memcpy(blk, nonce, 12);
                blk[12] = (uint8_t)(ctr >> 24); blk[13] = (uint8_t)(ctr >> 16);
                blk[14] = (uint8_t)(ctr >> 8); blk[15] = (uint8_t)ctr;
                oracle_aes_encrypt_block(key, (size_t)klen, blk, want);
                for (int q = 0; q < 4; ++q) {
                    const uint32_t got = w[q][j] ^ rkw[4 * NR + q] ^ 0x63636363u;
                    if (got != le(want + 4 * q)) {
                        if (bad < 5)
                            fprintf(stderr, "NR=%d SB=%d c0=%u beta=%u j=%d q=%d got %08x want %08x\n",
                                    NR, SB, c0, beta, j, q, got, le(want + 4 * q));
                        ++bad;
                    }
                }
                ++checked;
            }
          }
        }
    }
    printf("NR=%d fold=%d lanes=%u seed=%u blocks=%d bad=%d\n", NR, (int)FOLD, L, seed, checked, bad);
    return bad;
}

int main() {
    make_sbox();
    int bad = 0;
    for (unsigned seed = 1; seed <= 4; ++seed) {
        bad += run<10, false>(16, seed);
        bad += run<14, false>(32, 100 + seed);
        bad += run<10, true>(16, seed);
        bad += run<14, true>(32, 100 + seed);
    }
    // the key-grouped kernel's 16 / 32 / 64 lanes per record (key planes unfolded)
    for (unsigned seed = 1; seed <= 2; ++seed) {
        bad += run<14, false, 4>(32, 200 + seed);
        bad += run<14, false, 5>(32, 300 + seed);
        bad += run<14, false, 6>(32, 400 + seed);
        bad += run<10, false, 5>(16, 500 + seed);
    }
    // the per-record plane of a lane equals the plain bit test (GcmKeyDev::bs8mask layout)
    printf(bad ? "FAIL\n" : "OK\n");
    return bad != 0;
}
