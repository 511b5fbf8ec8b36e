// ghash.h -- GHASH multiplies and single-block AES helpers shared by the
// AES-GCM kernels (aes_gcm.hip, aes_gcm_bs8.hip) and the self-test entry
// points (selftest.hip).
//
// GHASH (aesgcm.py:60-99, _mul :86-97, bit order :8-14) two ways:
//   * gmul: y * G with the sixteen 8-bit tables of a fixed G staged in LDS
//     at address 0 (entry (j, b) = b * x^(8j) * G at j * 4096 + b * 16);
//   * gf128_mul: a table-free carry-less multiply of two arbitrary elements
//     in normal polynomial order (key tables, the H-power lifts).
// Included by exactly the kernel translation units; everything is internal.
#pragma once
#include "aes_round.h"

namespace tg {
namespace {

// y * H with the sixteen 8-bit tables: X * H = XOR_j M_j[byte j of X]; byte j
// of the block is byte j%4 of word j/4.  Entry (j, b) sits at j * 4096 + b * 16
// (table j is the ds_read offset), so the 16 lanes of a ds_read_b128 group
// land on the 16 bank slots by their own random bytes.
__device__ __forceinline__ uint4 gmul(uint4 y) {
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint4 e[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t v = w[q];
        e[4 * q + 0] = lds_u128(((v << 4) & 0xff0u) + 4096 * (4 * q + 0));
        e[4 * q + 1] = lds_u128(((v >> 4) & 0xff0u) + 4096 * (4 * q + 1));
        e[4 * q + 2] = lds_u128(((v >> 12) & 0xff0u) + 4096 * (4 * q + 2));
        e[4 * q + 3] = lds_u128(((v >> 20) & 0xff0u) + 4096 * (4 * q + 3));
    }
    uint4 z = xor4_3(e[0], e[1], e[2]);
    z = xor4_3(z, e[3], e[4]);
    z = xor4_3(z, e[5], e[6]);
    z = xor4_3(z, e[7], e[8]);
    z = xor4_3(z, e[9], e[10]);
    z = xor4_3(z, e[11], e[12]);
    z = xor4_3(z, e[13], e[14]);
    return xor4(z, e[15]);
}

// gmul with at most eight table rows in flight (32 VGPRs instead of 64), for
// the bitsliced kernel whose keystream chunk already holds 128 VGPRs.
__device__ __forceinline__ uint4 gmul_lowreg(uint4 y) {
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint4 e[8];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t v = w[2 * h + q];
            const int t = 4 * (2 * h + q);
            e[4 * q + 0] = lds_u128(((v << 4) & 0xff0u) + 4096 * (t + 0));
            e[4 * q + 1] = lds_u128(((v >> 4) & 0xff0u) + 4096 * (t + 1));
            e[4 * q + 2] = lds_u128(((v >> 12) & 0xff0u) + 4096 * (t + 2));
            e[4 * q + 3] = lds_u128(((v >> 20) & 0xff0u) + 4096 * (t + 3));
        }
        z = xor4_3(z, e[0], e[1]);
        z = xor4_3(z, e[2], e[3]);
        z = xor4_3(z, e[4], e[5]);
        z = xor4_3(z, e[6], e[7]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return z;
}

// Bank-conflict-free gmul (aes_gcm.hip GhashTablesRotLds): the tables in row
// layout, entry (j, b) at b * 256 + j * 16, so the 16-byte bank slot of a
// lookup is its table j; lane l walks the tables from j = l % 16, so the 16
// lanes of every ds_read_b128 group hit 16 different slots whatever the data.
// y is rotated by l % 16 bytes once per multiply; the four table-offset words
// of lane l come from a 16-row LDS table at ``jt`` (row l % 16: byte k of word
// q = ((l + 4 q + k) % 16) * 16).  lane16 = l % 16.  At most eight table rows
// in flight (32 VGPRs).
// The word rotation by (l % 16) / 4 is two stages of per-lane selects (one
// v_bitop3 each, VGPR operands: full rate); written as conditional swaps the
// compiler emitted exec-masked v_mov chains, 15 moves and 4 exec updates per
// multiply.
__device__ __forceinline__ uint32_t sel32(uint32_t m, uint32_t t, uint32_t f) {   // m ? t : f, bitwise
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(m, t, f, 0xca);
#else
    return (m & t) | (~m & f);
#endif
}
// acc: XORed into the product (y * H ^ acc, Horner's next input) as the first
// level of the XOR tree -- no separate four XORs per block.
__device__ __forceinline__ uint4 gmul_rot_j(uint4 y, uint32_t lane16, uint4 jw,
                                            uint4 acc = make_uint4(0, 0, 0, 0)) {
    const uint32_t m8 = 0u - ((lane16 >> 3) & 1u), m4 = 0u - ((lane16 >> 2) & 1u);
    const uint32_t h0 = sel32(m8, y.z, y.x), h1 = sel32(m8, y.w, y.y);
    const uint32_t h2 = sel32(m8, y.x, y.z), h3 = sel32(m8, y.y, y.w);
    const uint32_t u0 = sel32(m4, h1, h0), u1 = sel32(m4, h2, h1);
    const uint32_t u2 = sel32(m4, h3, h2), u3 = sel32(m4, h0, h3);
    const uint32_t s8 = (lane16 & 3u) << 3;
    const uint32_t v[4] = {__builtin_amdgcn_alignbit(u1, u0, s8), __builtin_amdgcn_alignbit(u2, u1, s8),
                           __builtin_amdgcn_alignbit(u3, u2, s8), __builtin_amdgcn_alignbit(u0, u3, s8)};
    const uint32_t j[4] = {jw.x, jw.y, jw.z, jw.w};
    uint4 z = acc;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint4 e[8];
#pragma unroll
        for (int t = 8 * h; t < 8 * h + 8; ++t) {
            // byte 1 <- v[t/4] byte t%4 (the row b), byte 0 <- j[t/4] byte t%4
            const uint32_t sel = 0x0c0c0000u | ((4u + (t & 3)) << 8) | (uint32_t)(t & 3);
            e[t - 8 * h] = lds_u128(__builtin_amdgcn_perm(v[t >> 2], j[t >> 2], sel));
        }
        z = xor4_3(z, e[0], e[1]);
        z = xor4_3(z, e[2], e[3]);
        z = xor4_3(z, e[4], e[5]);
        z = xor4_3(z, e[6], e[7]);
    }
    return z;
}

// gmul_rot with the lane-offset row read from LDS per multiply.
__device__ __forceinline__ uint4 gmul_rot(uint4 y, uint32_t lane16, uint32_t jt,
                                          uint4 acc = make_uint4(0, 0, 0, 0)) {
    return gmul_rot_j(y, lane16, lds_u128(jt + (lane16 << 4)), acc);
}

// Stage the 8-bit tables of ``src`` (GcmKeyDev layout, entry (j, b) at
// j * 256 + b) in gmul_rot's row layout at LDS 0, and its lane-offset rows at
// ``jt``.  Every thread of the workgroup calls it; a barrier must follow.
__device__ __forceinline__ void stage_ghash_rot(uint4* lds, const uint4* __restrict__ src, uint32_t jt) {
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x) lds[(e & 255) * 16 + (e >> 8)] = src[e];
    if (threadIdx.x < 16) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) w[q] |= (((threadIdx.x + 4 * q + k) & 15u) << 4) << (8 * k);
        }
        lds[jt / 16 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// ---- table-free GHASH for key tables -----------------------------------
// A key table cannot stage 64 KiB of GHASH tables per session, so each lane
// multiplies by its own H with a carry-less multiply built from integer
// multiplies (bits spaced four apart cannot carry into each other: a product
// of two such words, masked to one residue class mod 4, is the carry-less
// product on that class).  Elements are kept in normal polynomial order
// (coefficient of x^i at bit i): a GCM block's bytes keep their positions and
// each byte is bit-reversed (aesgcm.py:8-14).
__device__ __forceinline__ uint32_t to_norm(uint32_t w) {
    return bswap32(__builtin_bitreverse32(w));
}

__device__ __forceinline__ uint64_t mul32(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

__device__ __forceinline__ uint64_t clmul32(uint32_t x, uint32_t y) {
    const uint32_t x0 = x & 0x11111111u, x1 = x & 0x22222222u, x2 = x & 0x44444444u,
                   x3 = x & 0x88888888u;
    const uint32_t y0 = y & 0x11111111u, y1 = y & 0x22222222u, y2 = y & 0x44444444u,
                   y3 = y & 0x88888888u;
    const uint64_t z0 = mul32(x0, y0) ^ mul32(x1, y3) ^ mul32(x2, y2) ^ mul32(x3, y1);
    const uint64_t z1 = mul32(x0, y1) ^ mul32(x1, y0) ^ mul32(x2, y3) ^ mul32(x3, y2);
    const uint64_t z2 = mul32(x0, y2) ^ mul32(x1, y1) ^ mul32(x2, y0) ^ mul32(x3, y3);
    const uint64_t z3 = mul32(x0, y3) ^ mul32(x1, y2) ^ mul32(x2, y1) ^ mul32(x3, y0);
    return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) |
           (z2 & 0x4444444444444444ull) | (z3 & 0x8888888888888888ull);
}

// 64 x 64 -> 128 by one Karatsuba step over 32-bit halves; result words w0..w3.
// sched_barrier between the 32-bit products keeps the scheduler from running
// all nine at once (each holds 16 64-bit partial products).
__device__ __forceinline__ uint4 clmul64(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) {
    const uint64_t lo = clmul32(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t hi = clmul32(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t mid = clmul32(a0 ^ a1, b0 ^ b1) ^ lo ^ hi;
    __builtin_amdgcn_sched_barrier(0);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32) ^ (uint32_t)mid,
                      (uint32_t)(mid >> 32) ^ (uint32_t)hi, (uint32_t)(hi >> 32));
}

// a * b mod x^128 + x^7 + x^2 + x + 1, normal order, 32-bit limbs (x^0 in .x).
__device__ __forceinline__ uint4 gf128_mul(uint4 a, uint4 b) {
    const uint4 L = clmul64(a.x, a.y, b.x, b.y);
    const uint4 Hh = clmul64(a.z, a.w, b.z, b.w);
    const uint4 M = clmul64(a.x ^ a.z, a.y ^ a.w, b.x ^ b.z, b.y ^ b.w);
    const uint32_t m0 = xor3(M.x, L.x, Hh.x), m1 = xor3(M.y, L.y, Hh.y);
    const uint32_t m2 = xor3(M.z, L.z, Hh.z), m3 = xor3(M.w, L.w, Hh.w);
    // 256-bit product p0..p7
    const uint32_t p0 = L.x, p1 = L.y, p2 = L.z ^ m0, p3 = L.w ^ m1;
    const uint32_t t0 = Hh.x ^ m2, t1 = Hh.y ^ m3, t2 = Hh.z, t3 = Hh.w;
    // fold T = p4..p7 (x^128 == x^7 + x^2 + x + 1): r ^= T ^ T<<1 ^ T<<2 ^ T<<7
    const uint32_t v = (t3 >> 31) ^ (t3 >> 30) ^ (t3 >> 25);  // bits pushed past x^127
    uint32_t r0 = xor3(p0, t0, t0 << 1) ^ xor3(t0 << 2, t0 << 7, v);
    r0 ^= xor3(v << 1, v << 2, v << 7);
    const uint32_t r1 = xor3(p1, t1, t1 << 1) ^ xor3(t1 << 2, t1 << 7, (t0 >> 31)) ^
                        ((t0 >> 30) ^ (t0 >> 25));
    const uint32_t r2 = xor3(p2, t2, t2 << 1) ^ xor3(t2 << 2, t2 << 7, (t1 >> 31)) ^
                        ((t1 >> 30) ^ (t1 >> 25));
    const uint32_t r3 = xor3(p3, t3, t3 << 1) ^ xor3(t3 << 2, t3 << 7, (t2 >> 31)) ^
                        ((t2 >> 30) ^ (t2 >> 25));
    return make_uint4(r0, r1, r2, r3);
}

__device__ __forceinline__ uint4 shfl_xor4(uint4 v, int m) {
    return make_uint4((uint32_t)__shfl_xor((int)v.x, m, 64), (uint32_t)__shfl_xor((int)v.y, m, 64),
                      (uint32_t)__shfl_xor((int)v.z, m, 64), (uint32_t)__shfl_xor((int)v.w, m, 64));
}

__device__ __forceinline__ uint4 norm4(uint4 v) {
    return make_uint4(to_norm(v.x), to_norm(v.y), to_norm(v.z), to_norm(v.w));
}

// x^e in GF(2^128), normal order (square and multiply): powers beyond the
// key's table (records over ~18 KiB of AAD + payload).
__device__ __forceinline__ uint4 gf128_pow(uint4 x, uint32_t e) {
    uint4 r = make_uint4(1, 0, 0, 0);
    while (e) {
        if (e & 1) r = gf128_mul(r, x);
        e >>= 1;
        if (e) x = gf128_mul(x, x);
    }
    return r;
}

// ---- 4-bit tables of one key's H^8, one copy per wave (key-table octet
// kernel) ----------------------------------------------------------------
// Entry (j, n) at tab + 256 j + 16 n = n x^(4j) G in the 8-bit tables' byte
// layout: nibble j is the high (j even) or low (j odd) nibble of byte j / 2,
// so M4[2B][n] = M_B[n << 4] and M4[2B + 1][n] = M_B[n].  A 16-entry table is
// 256 B, all 64 banks once: a wave's lookups into one table never conflict.
// 8 KiB per copy; tab must be 256-byte aligned.
//
// In GCM bit order bit 0x80 >> m of byte B is the coefficient of x^(8B + m),
// so M4[j][n] = XOR over k = 0..3 with n & (8 >> k) of x^(4j + k) G.  Lane
// (j, half) of the wave (j = lane % 32) builds the basis x^(4j) G by a
// shift and reduction (gf128_mul_xpow), x^(4j+1..3) G by single shifts, and
// writes the eight entries n = 8 half .. 8 half + 7 of table j when a wave's
// key changes.  gn: G in normal order (a key's H^8 from its
// power table).
__device__ __forceinline__ uint4 gf128_mulx(uint4 v) {   // v * x, normal order
    const uint32_t c = v.w >> 31;
    return make_uint4((v.x << 1) ^ (c * 0x87u), __builtin_amdgcn_alignbit(v.y, v.x, 31),
                      __builtin_amdgcn_alignbit(v.z, v.y, 31), __builtin_amdgcn_alignbit(v.w, v.z, 31));
}

// v * x^s mod x^128 + x^7 + x^2 + x + 1 (normal order), 0 <= s < 128: the
// 256-bit shift v x^s = lo + x^128 hi, then x^128 = 1 + x + x^2 + x^7 twice
// (hi has degree < s, so hi (1 + x + x^2 + x^7) overflows by < 7 bits).
// ~60 VALU instead of a table-free multiply by the monomial (~650).
__device__ __forceinline__ uint32_t funnel_l(uint32_t hi, uint32_t lo, uint32_t b) {   // ({hi, lo} << b) >> 32
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (32u - b));
}
__device__ __forceinline__ uint4 gf128_mul_xpow(uint4 v, uint32_t s) {
    const uint32_t b = s & 31u, q = s >> 5;
    const uint32_t w[5] = {funnel_l(v.x, 0u, b), funnel_l(v.y, v.x, b), funnel_l(v.z, v.y, b),
                           funnel_l(v.w, v.z, b), funnel_l(0u, v.w, b)};
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // t[i] = w[i - q]
        uint32_t x = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            if (i - d >= 0 && i - d < 5) x = q == (uint32_t)d ? w[i - d] : x;
        t[i] = x;
    }
    // + hi (1 + x + x^2 + x^7), hi = t[4..7]
    uint32_t r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t h = t[4 + i], hp = i ? t[3 + i] : 0u;   // hp: the word below (carries in)
        r[i] = t[i] ^ h ^ ((h << 1) | (hp >> 31)) ^ ((h << 2) | (hp >> 30)) ^ ((h << 7) | (hp >> 25));
    }
    // the bits shifted past x^127, once more times 1 + x + x^2 + x^7
    const uint32_t o = (t[7] >> 31) ^ (t[7] >> 30) ^ (t[7] >> 25);
    r[0] ^= o ^ (o << 1) ^ (o << 2) ^ (o << 7);
    return make_uint4(r[0], r[1], r[2], r[3]);
}

__device__ __forceinline__ void build_table4(uint32_t tab, uint4 gn) {
    const uint32_t lane = threadIdx.x & 63u, j = lane & 31u, n0 = (lane >> 5) * 8u;
    uint4 bas[4];
    bas[0] = gf128_mul_xpow(gn, 4u * j);
    bas[1] = gf128_mulx(bas[0]);
    bas[2] = gf128_mulx(bas[1]);
    bas[3] = gf128_mulx(bas[2]);
    // entry n0 + (n + j) % 8 at step n: the 8 lanes of a ds_write_b128 group
    // (8 consecutive lanes, banks (a / 4) mod 32) write 8 different bank
    // slots instead of one -- an 8-way conflict on every store; config 4
    // +0.7 %, two of two rounds on one box (profiles/r05/r5e/)
    uint4 e[8];
#pragma unroll
    for (uint32_t n = 0; n < 8; ++n) {
        const uint32_t nn = n0 + n;
        uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (nn & (8u >> k)) v = xor4(v, bas[k]);
        e[n] = norm4(v);
    }
    // rotate the eight entries by j % 8 (three stages of per-lane selects)
#pragma unroll
    for (int st = 1; st < 8; st <<= 1) {
        const bool sw = (j & (uint32_t)st) != 0;
        uint4 t[8];
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const uint4 a = e[n], b = e[(n + st) & 7];
            t[n] = make_uint4(sw ? b.x : a.x, sw ? b.y : a.y, sw ? b.z : a.z, sw ? b.w : a.w);
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) e[n] = t[n];
    }
#pragma unroll
    for (uint32_t n = 0; n < 8; ++n) lds_st128(tab + 256u * j + 16u * (n0 + ((n + j) & 7u)), e[n]);
}

// y * G through the 4-bit tables at ``tab`` (32 lookups, no reduction).
// tab must be 256-byte aligned (the nibble offsets are ORed in).
__device__ __forceinline__ uint4 gmul4(uint4 y, uint32_t tab, uint4 acc = make_uint4(0, 0, 0, 0)) {
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint4 z = acc;   // y * G ^ acc (see gmul_rot_j)
    // the nibble mask in a VGPR: (x & m) | tab is then one full-rate
    // v_bitop3 (an SGPR or literal operand makes it half rate or two ops)
    uint32_t m = 0xf0u;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_mov_b32 %0, 0xf0" : "=v"(m));
#endif
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 e[8];
        uint32_t w4 = w[q] << 4;   // opaque: or (w4 >> 8k) & m becomes a half-rate v_bfe_u32
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(w4));
#endif
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t B = 4 * q + k;
            const uint32_t hi = ((w[q] >> (8 * k)) & m) | tab;
            const uint32_t lo = ((w4 >> (8 * k)) & m) | tab;
            // nibble | tab, plus a constant that rides in the ds_read offset field
            e[2 * k] = lds_u128(hi + 512u * B);
            e[2 * k + 1] = lds_u128(lo + 512u * B + 256u);
        }
        z = xor4_3(z, e[0], e[1]);
        z = xor4_3(z, e[2], e[3]);
        z = xor4_3(z, e[4], e[5]);
        z = xor4_3(z, e[6], e[7]);
        // eight rows in flight (32 VGPRs): z is made opaque per group, or
        // the XOR tree is reassociated and all 32 rows are held at once
        asm volatile("" : "+v"(z.x), "+v"(z.y), "+v"(z.z), "+v"(z.w));
    }
    return z;
}

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint32_t lds_u8(uint32_t addr) {
    return *(const __attribute__((address_space(3))) uint8_t*)(uintptr_t)addr;
}
#else
__device__ __forceinline__ uint32_t lds_u8(uint32_t) { return 0; }
#endif

// S-box of each byte of w (256-byte LDS table at sbox)
__device__ __forceinline__ uint32_t sub_word(uint32_t w, uint32_t sbox) {
    return lds_u8(sbox + (w & 0xffu)) | (lds_u8(sbox + ((w >> 8) & 0xffu)) << 8) |
           (lds_u8(sbox + ((w >> 16) & 0xffu)) << 16) | (lds_u8(sbox + (w >> 24)) << 24);
}

// MixColumns of one column packed as a LE word (byte i = row i):
// out_i = 2 (a_i ^ a_i+1) ^ a_i+1 ^ a_i+2 ^ a_i+3.
__device__ __forceinline__ uint32_t mix_word(uint32_t w) {
    const uint32_t r1 = __builtin_amdgcn_alignbit(w, w, 8), r2 = __builtin_amdgcn_alignbit(w, w, 16),
                   r3 = __builtin_amdgcn_alignbit(w, w, 24);
    const uint32_t u = w ^ r1;
    const uint32_t xt = ((u & 0x7f7f7f7fu) << 1) ^ (((u >> 7) & 0x01010101u) * 0x1bu);
    return xt ^ xor3(r1, r2, r3);
}

// One block, byte-wise (rijndael.py:995-1038 restated): state words are the
// columns, ShiftRows takes row i of column c from column (c + i) % 4.  For the
// single blocks of the bitsliced kernels (tag masks, partial tails).
template <int NR>
__device__ __forceinline__ uint4 aes_block_sb(const uint32_t* rk, uint4 in, uint32_t sbox) {
    uint32_t s[4] = {in.x ^ rk[0], in.y ^ rk[1], in.z ^ rk[2], in.w ^ rk[3]};
#pragma unroll 1
    for (int r = 1; r <= NR; ++r) {
        uint32_t t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t w = __builtin_amdgcn_perm(s[(c + 1) & 3], s[c], 0x07060500u) & 0xffffu;
            const uint32_t v = (s[(c + 2) & 3] & 0x00ff0000u) | (s[(c + 3) & 3] & 0xff000000u);
            t[c] = sub_word(w | v, sbox);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) s[c] = (r < NR ? mix_word(t[c]) : t[c]) ^ rk[4 * r + c];
    }
    return make_uint4(s[0], s[1], s[2], s[3]);
}

}  // namespace
}  // namespace tg
