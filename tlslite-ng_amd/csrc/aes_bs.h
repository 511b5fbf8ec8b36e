// aes_bs.h -- bitsliced AES counter mode for gfx950: 32 counter blocks per
// lane, one bit of every 32-bit register per block.
//
// Restates Rijndael.encrypt (tlslite/utils/rijndael.py:995-1038) on bit
// planes so that SubBytes runs on the VALU instead of LDS table lookups:
//   * the state is 128 planes st[k][b] = bit b of byte k of 32 blocks (block
//     i in bit i);
//   * SubBytes is the Boyar-Peralta depth-16 circuit (128 gates) fused into
//     84 full-rate v_bitop3_b32 / 2-input gates (tools/gen_bs_sbox.py); its four XNORs
//     are dropped, i.e. every S-box output is S(x) ^ 0x63, and the 0x63 is
//     folded into the next round key (MixColumns maps a column of equal bytes
//     c to itself, so MC(y ^ c) = MC(y) ^ c);
//   * ShiftRows is register renaming (fully unrolled);
//   * AddRoundKey XORs wave-uniform masks 0 / ~0 built on the scalar unit from
//     the round-key words;
//   * counter blocks nonce || be32(base + i): bytes 0..11 are the same for all
//     blocks of a record, so their first S-box is done once per record; bytes 12..15 are the counter, whose planes are
//     wave-uniform when base is (base = 2 + 32 j for chunk j of every lane).
// The planes of the last round are turned back into blocks with a 32 x 32 bit
// transpose per word; the last round key is added by the caller (folded into
// the XOR with the payload).
//
// Usable from host code too (the CPU unit test compiles it with g++).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#if defined(__HIPCC__)
#define TG_BS_HD __host__ __device__ __forceinline__
#define TG_BS_MF __host__ __device__ __forceinline__
#else
#define TG_BS_HD static inline
#define TG_BS_MF inline
#endif

namespace tg {
namespace bs {

// Round-key words in the layout of GcmKeyDev::rk (LE words of the schedule
// bytes): byte k of round key r = rk[4 r + k / 4] >> 8 (k % 4).

// Plane mask of bit p of word w: 0 or ~0.
TG_BS_HD uint32_t bitmask(uint32_t w, int p) { return (uint32_t)((int32_t)(w << (31 - p)) >> 31); }

// Scheduling fence between S-boxes (keeps the scheduler from interleaving
// several S-boxes' temporaries on top of the 128 live state planes).
#if defined(__HIP_DEVICE_COMPILE__)
#define TG_BS_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TG_BS_FENCE() ((void)0)
#endif

// One full-rate v_bitop3_b32: bit i of the result = bit (4 a_i + 2 b_i + c_i) of tt.
#if defined(__HIP_DEVICE_COMPILE__)
#define bop3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#else
TG_BS_HD uint32_t bop3(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k)
        if ((tt >> k) & 1) r |= ((k & 4) ? a : ~a) & ((k & 2) ? b : ~b) & ((k & 1) ? c : ~c);
    return r;
}
#endif
TG_BS_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return bop3(a, b, c, 0x96); }

// v_perm_b32: byte i of the result = byte sel_i of (hi:lo) (0..3 = lo, 4..7 = hi).
TG_BS_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xff) << (8 * i);
    return r;
#endif
}

// In-place S-box (without the affine constant 0x63) on the planes of one byte,
// x[b] = bit b: Boyar & Peralta, "A depth-16 circuit for the AES S-box"
// (2011), 128 gates fused into 84 two- and three-input gates.
#include "aes_bs_sbox.h"

// ShiftRows + MixColumns + AddRoundKey: out column c, row i takes the byte at
// row i, column (c + i) % 4 of the SubBytes output.  k[r][b] = round-key mask
// of byte 4 c + i; out_i = 2 (a_i ^ a_i+1) ^ a_i+1 ^ (a_i+2 ^ a_i+3) ^ k.
template <class KM>
TG_BS_HD void mix_columns(const uint32_t (*st)[8], uint32_t (*out)[8], const KM& km, int r) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t* a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = st[i + 4 * ((c + i) & 3)];
        uint32_t t[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 8; ++b) t[i][b] = a[i][b] ^ a[(i + 1) & 3][b];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t* ti = t[i];
            const uint32_t* a1 = a[(i + 1) & 3];
            const uint32_t* t2 = t[(i + 2) & 3];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t k = km(r, i + 4 * c, b);
                if (b == 1 || b == 3 || b == 4)   // xtime feeds bit 7 back into bits 1, 3, 4
                    out[i + 4 * c][b] = xor3(xor3(ti[b - 1], ti[7], a1[b]), t2[b], k);
                else
                    out[i + 4 * c][b] = xor3(ti[(b + 7) & 7], a1[b], t2[b]) ^ k;
            }
        }
    }
}

// One full middle round, column by column: the four S-boxes a column needs,
// then its MixColumns, so that at most one column's temporaries are live.
template <class KM>
TG_BS_HD void round_by_column(uint32_t (*st)[8], uint32_t (*out)[8], const KM& km, int r) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) sbox(st[i + 4 * ((c + i) & 3)]);
        const uint32_t* a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = st[i + 4 * ((c + i) & 3)];
        uint32_t t[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 8; ++b) t[i][b] = a[i][b] ^ a[(i + 1) & 3][b];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t* ti = t[i];
            const uint32_t* a1 = a[(i + 1) & 3];
            const uint32_t* t2 = t[(i + 2) & 3];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t k = km(r, i + 4 * c, b);
                if (b == 1 || b == 3 || b == 4)
                    out[i + 4 * c][b] = xor3(xor3(ti[b - 1], ti[7], a1[b]), t2[b], k);
                else
                    out[i + 4 * c][b] = xor3(ti[(b + 7) & 7], a1[b], t2[b]) ^ k;
            }
        }
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
}

// Final round: ShiftRows only (out byte i + 4 c <- st byte i + 4 ((c + i) % 4)).
TG_BS_HD void shift_rows(const uint32_t (*st)[8], uint32_t (*out)[8]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 8; ++b) out[i + 4 * c][b] = st[i + 4 * ((c + i) & 3)][b];
}

// 32 x 32 bit transpose in place (a[r] bit c <-> a[c] bit r), in two steps:
// the m = 16 stage over all 32 rows, after which rows 0..15 and 16..31 finish
// independently (stages 8..1 pair rows within a half), so a caller can
// consume half the blocks before the other half is finished.
TG_BS_HD void transpose32_first(uint32_t* a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {   // rows r, r + 16 swap 16-bit halves: two byte permutes
        const uint32_t lo = perm(a[r + 16], a[r], 0x05040100u), hi = perm(a[r + 16], a[r], 0x07060302u);
        a[r] = lo;
        a[r + 16] = hi;
    }
}
TG_BS_HD void transpose32_half(uint32_t* a, int h) {
#pragma unroll
    for (int r = 16 * h; r < 16 * h + 8; ++r) {   // m = 8: byte permutes
        const uint32_t lo = perm(a[r + 8], a[r], 0x06020400u), hi = perm(a[r + 8], a[r], 0x07030501u);
        a[r] = lo;
        a[r + 8] = hi;
    }
#pragma unroll
    for (int l = 2; l >= 0; --l) {   // m = 4, 2, 1: bit-field inserts, no temporaries
        const int m = 1 << l;
        const uint32_t mask = m == 4 ? 0x0f0f0f0fu : m == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int r = 16 * h; r < 16 * h + 16; ++r) {
            if (r & m) continue;
            const uint32_t x = a[r], y = a[r + m];
            a[r] = bop3(mask << m, y << m, x, 0xca);      // (y << m) where mask << m, else x
            a[r + m] = bop3(mask, x >> m, y, 0xca);       // (x >> m) where mask, else y
        }
    }
}

// Round-key masks for one key: rk' = rk ^ 0x63636363 for rounds 1..NR
// (the dropped S-box constant), read from wave-uniform memory (scalar loads)
// and turned into plane masks on the scalar unit.
struct BsKey {
    const uint32_t* w;   // rk' words, 4 (NR + 1)
    TG_BS_MF uint32_t operator()(int r, int k, int b) const { return bitmask(w[4 * r + (k >> 2)], 8 * (k & 3) + b); }
};

// The same keys as precomputed plane masks, mask (r, k, b) at (16 r + k) 8 + b
// (1408 / 1920 words per AES-128 / AES-256 key): scalar loads straight into
// the XORs' SGPR operand, no mask arithmetic per chunk.
struct BsKeyMasks {
    const uint32_t* w;
    TG_BS_MF uint32_t operator()(int r, int k, int b) const {
#if defined(__HIP_DEVICE_COMPILE__)
        // constant address space: a wave-uniform address becomes an s_load
        return ((const __attribute__((address_space(4))) uint32_t*)w)[(16 * r + k) * 8 + b];
#else
        return w[(16 * r + k) * 8 + b];
#endif
    }
};

// Counter planes: bit p (0..31) of base + i for block i, base = 2 mod 32.
// Bits 0..4 are constants; bits >= 5 are those of base for i < 30 and of
// base + 32 for i >= 30.
TG_BS_HD uint32_t ctr_plane(uint32_t base, int p) {
    if (p < 5) {
        constexpr uint32_t lo[5] = {0xaaaaaaaau, 0x33333333u, 0x3c3c3c3cu, 0x3fc03fc0u, 0x3fffc000u};
        return lo[p];
    }
    return (bitmask(base, p) & 0x3fffffffu) | (bitmask(base + 32u, p) & 0xc0000000u);
}

// Keystream of 32 counter blocks nonce || be32(base + i), base = 2 + 32 j.
// s1w: per record, the S-box outputs (without 0x63) of bytes 0..11 of the
// first round (nonce ^ rk0), as 3 LE words; rk0w = word 3 of round key 0.
// Returns the last round's planes in w_out[4][32], transposed (TR = 2):
// w_out[q][i] = word q of block i WITHOUT the last round key; with TR = 1 only
// the first transpose stage is done (finish with transpose32_half).  Rounds 2..NR-1 are a rolled loop (one
// round is ~2 k instructions; the unrolled cipher would not fit the
// instruction cache).
struct NoHook {
    TG_BS_MF void operator()(int, int) {}
};

// hook(r, k) runs after S-box k (0..15) of each middle round r = 2 .. NR-1:
// independent work (the GCM kernel's GHASH of the previous chunk) spread over
// the round in small steps, so each step's LDS / memory latency hides behind
// the next S-box's gates (with FENCE the steps stay where they are put).
template <int NR, int SCHED = 0, class KM = BsKey, int TR = 2, bool FENCE = false, class Hook = NoHook>
TG_BS_HD void ctr32(const KM& key_in, uint32_t rk0w, const uint32_t s1w[3], uint32_t base,
                    uint32_t (*w_out)[32], Hook&& hook = Hook()) {
    KM key = key_in;
#if defined(__HIP_DEVICE_COMPILE__)
    // Nothing of a chunk may be hoisted into the caller's chunk loop: the
    // loop-invariant parts of the first S-boxes (and the scalar loads of the
    // key masks) would stay live (spilled) across the whole cipher.
    asm volatile("" : "+s"(base));
    asm volatile("" : "+s"(key.w));
#endif
    uint32_t st[16][8];
    // round 1 SubBytes: bytes 0..11 per record, bytes 12..15 = be32 counter ^ rk0.
    // The per-record planes are rebuilt per call (96 cheap ops).
    uint32_t s1[3] = {s1w[0], s1w[1], s1w[2]};
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(s1[0]), "+v"(s1[1]), "+v"(s1[2]));
#endif
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
        for (int b = 0; b < 8; ++b) st[k][b] = bitmask(s1[k >> 2], 8 * (k & 3) + b);
#pragma unroll
    for (int k = 12; k < 16; ++k) {
#pragma unroll
        for (int b = 0; b < 8; ++b)
            st[k][b] = ctr_plane(base, 8 * (15 - k) + b) ^ bitmask(rk0w, 8 * (k & 3) + b);
        sbox(st[k]);
        if (FENCE) TG_BS_FENCE();
    }
    uint32_t nx[16][8];
    mix_columns(st, nx, key, 1);
#pragma unroll 1
    for (int r = 2; r < NR; ++r) {
        if (SCHED == 1) {
            round_by_column(nx, st, key, r);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                sbox(nx[k]);
                hook(r, k);
                if (FENCE) TG_BS_FENCE();
            }
            mix_columns(nx, st, key, r);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int b = 0; b < 8; ++b) nx[k][b] = st[k][b];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        sbox(nx[k]);
        if (FENCE) TG_BS_FENCE();
    }
    shift_rows(nx, st);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int p = 0; p < 32; ++p) w_out[q][p] = st[4 * q + (p >> 3)][p & 7];
        transpose32_first(w_out[q]);
        if (TR == 2) {
            transpose32_half(w_out[q], 0);
            transpose32_half(w_out[q], 1);
        }
    }
}

}  // namespace bs
}  // namespace tg
