// poly1305.h -- the Poly1305 arithmetic of the ChaCha20-Poly1305 kernels
// (chacha_poly.hip) and of the self-test entry point (selftest.hip).
//
// Restates Poly1305 (tlslite/utils/poly1305.py:32-48) in five 26-bit limbs
// with 32 x 32 -> 64 multiply-adds, plus the pieces of the wave-striped
// Horner that the wave-per-record kernel uses: the gap multiply by
// r^(4S - 4), the lift of a thread's partial by r^(blocks after it), and the
// sum of the partials (shuffles, then LDS across a record's waves).
// Included by exactly the kernel translation units; everything is internal.
#pragma once
#include "common.h"

namespace tg {
namespace {

__device__ __forceinline__ uint64_t mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// Poly1305 state in 26-bit limbs (value = sum h_i * 2^(26 i)).
struct Poly {
    uint32_t r0, r1, r2, r3, r4;
    uint32_t s1, s2, s3, s4;  // 5 * r_i: 2^130 == 5 (mod 2^130 - 5)
    uint32_t h0, h1, h2, h3, h4;
    uint32_t p0, p1, p2, p3;  // s half of the one-time key
};

__device__ __forceinline__ void poly_init(Poly& p, const uint32_t (&otk)[16]) {
    // r = LE(key[0:16]) & 0x0ffffffc0ffffffc0ffffffc0fffffff (poly1305.py:37-38)
    p.r0 = otk[0] & 0x3ffffffu;
    p.r1 = __builtin_amdgcn_alignbit(otk[1], otk[0], 26) & 0x3ffff03u;
    p.r2 = __builtin_amdgcn_alignbit(otk[2], otk[1], 20) & 0x3ffc0ffu;
    p.r3 = __builtin_amdgcn_alignbit(otk[3], otk[2], 14) & 0x3f03fffu;
    p.r4 = (otk[3] >> 8) & 0x00fffffu;
    p.s1 = p.r1 * 5; p.s2 = p.r2 * 5; p.s3 = p.r3 * 5; p.s4 = p.r4 * 5;
    p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
    p.p0 = otk[4]; p.p1 = otk[5]; p.p2 = otk[6]; p.p3 = otk[7];
}

// acc = (acc + LE(m || 0x01)) * r mod 2^130-5 for one 16-byte block
// (poly1305.py:43-46).  mac_data is padded to 16 bytes (chacha20_poly1305.py:
// 41-46), so every AEAD block carries the 2^128 bit (hib = 1 << 24 in limb 4);
// a raw message's short last block carries its 0x01 inside m (hib = 0).
__device__ __forceinline__ void poly_block(Poly& p, uint4 m, uint32_t hib = 1u << 24) {
    const uint32_t M26 = 0x3ffffffu;
    uint32_t h0 = p.h0 + (m.x & M26);
    uint32_t h1 = p.h1 + (__builtin_amdgcn_alignbit(m.y, m.x, 26) & M26);
    uint32_t h2 = p.h2 + (__builtin_amdgcn_alignbit(m.z, m.y, 20) & M26);
    uint32_t h3 = p.h3 + (__builtin_amdgcn_alignbit(m.w, m.z, 14) & M26);
    uint32_t h4 = p.h4 + ((m.w >> 8) | hib);
    uint64_t d0 = mul64(h0, p.r0) + mul64(h1, p.s4) + mul64(h2, p.s3) + mul64(h3, p.s2) + mul64(h4, p.s1);
    uint64_t d1 = mul64(h0, p.r1) + mul64(h1, p.r0) + mul64(h2, p.s4) + mul64(h3, p.s3) + mul64(h4, p.s2);
    uint64_t d2 = mul64(h0, p.r2) + mul64(h1, p.r1) + mul64(h2, p.r0) + mul64(h3, p.s4) + mul64(h4, p.s3);
    uint64_t d3 = mul64(h0, p.r3) + mul64(h1, p.r2) + mul64(h2, p.r1) + mul64(h3, p.r0) + mul64(h4, p.s4);
    uint64_t d4 = mul64(h0, p.r4) + mul64(h1, p.r3) + mul64(h2, p.r2) + mul64(h3, p.r1) + mul64(h4, p.r0);
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & M26;
    d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & M26;
    d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & M26;
    d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & M26;
    d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & M26;
    h0 += c * 5; c = h0 >> 26; h0 &= M26;
    h1 += c;
    p.h0 = h0; p.h1 = h1; p.h2 = h2; p.h3 = h3; p.h4 = h4;
}

// tag = LE16((acc + s) mod 2^128) (poly1305.py:47-48)
__device__ __forceinline__ uint4 poly_finish(const Poly& p) {
    const uint32_t M26 = 0x3ffffffu;
    uint32_t h0 = p.h0, h1 = p.h1, h2 = p.h2, h3 = p.h3, h4 = p.h4, c;
    c = h1 >> 26; h1 &= M26; h2 += c;
    c = h2 >> 26; h2 &= M26; h3 += c;
    c = h3 >> 26; h3 &= M26; h4 += c;
    c = h4 >> 26; h4 &= M26; h0 += c * 5;
    c = h0 >> 26; h0 &= M26; h1 += c;
    // g = h + 5 - 2^130; use g when h >= 2^130 - 5
    uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= M26;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= M26;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= M26;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= M26;
    uint32_t g4 = h4 + c - (1u << 26);
    uint32_t sel = (g4 >> 31) - 1u;  // all ones when no borrow
    h0 = (h0 & ~sel) | (g0 & sel);
    h1 = (h1 & ~sel) | (g1 & sel);
    h2 = (h2 & ~sel) | (g2 & sel);
    h3 = (h3 & ~sel) | (g3 & sel);
    h4 = (h4 & ~sel) | (g4 & sel);
    uint32_t w0 = h0 | (h1 << 26);
    uint32_t w1 = (h1 >> 6) | (h2 << 20);
    uint32_t w2 = (h2 >> 12) | (h3 << 14);
    uint32_t w3 = (h3 >> 18) | (h4 << 8);
    uint64_t f = (uint64_t)w0 + p.p0;
    w0 = (uint32_t)f;
    f = (uint64_t)w1 + p.p1 + (f >> 32); w1 = (uint32_t)f;
    f = (uint64_t)w2 + p.p2 + (f >> 32); w2 = (uint32_t)f;
    f = (uint64_t)w3 + p.p3 + (f >> 32); w3 = (uint32_t)f;
    return make_uint4(w0, w1, w2, w3);
}

// ---- radix 2^32 (the lane-per-record kernel) ------------------------------
// h = h0 + h1 2^32 + h2 2^64 + h3 2^96 + h4 2^128 with h0..h3 full words and
// h4 a few bits.  The clamp leaves r0 < 2^28 and r1..r3 < 2^28, multiples of
// 4, so a product term at or above 2^128 folds through 2^130 == 5 as
// h_i * s_j with s_j = r_j + r_j / 4 = 5 r_j / 4 (exact): every column is a
// sum of at most five products < 2^60.4, no 64-bit overflow.  Per 16 bytes:
// 19 v_mad_u64_u32 and one 32-bit multiply, no limb splitting of the message
// (the 26-bit form takes 25 multiply-adds plus the splits and 26-bit
// carries).
struct Poly32 {
    uint32_t r0, r1, r2, r3;
    uint32_t s1, s2, s3;
    uint32_t h0, h1, h2, h3, h4;
    uint32_t p0, p1, p2, p3;  // s half of the one-time key
};

__device__ __forceinline__ void poly_init(Poly32& p, const uint32_t (&otk)[16]) {
    // r = LE(key[0:16]) & 0x0ffffffc0ffffffc0ffffffc0fffffff (poly1305.py:37-38)
    p.r0 = otk[0] & 0x0fffffffu;
    p.r1 = otk[1] & 0x0ffffffcu;
    p.r2 = otk[2] & 0x0ffffffcu;
    p.r3 = otk[3] & 0x0ffffffcu;
    p.s1 = p.r1 + (p.r1 >> 2);
    p.s2 = p.r2 + (p.r2 >> 2);
    p.s3 = p.r3 + (p.r3 >> 2);
    p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
    p.p0 = otk[4]; p.p1 = otk[5]; p.p2 = otk[6]; p.p3 = otk[7];
}

// acc = (acc + LE(m) + hib 2^128) * r mod 2^130 - 5 (poly1305.py:43-46);
// hib = 1 for a full block, 0 for a raw message's short last block (its 0x01
// already inside m).
__device__ __forceinline__ void poly_block(Poly32& p, uint4 m, uint32_t hib = 1u) {
    uint64_t t = (uint64_t)p.h0 + m.x;
    const uint32_t h0 = (uint32_t)t;
    t = (uint64_t)p.h1 + m.y + (t >> 32);
    const uint32_t h1 = (uint32_t)t;
    t = (uint64_t)p.h2 + m.z + (t >> 32);
    const uint32_t h2 = (uint32_t)t;
    t = (uint64_t)p.h3 + m.w + (t >> 32);
    const uint32_t h3 = (uint32_t)t;
    const uint32_t h4 = p.h4 + hib + (uint32_t)(t >> 32);
    const uint64_t d0 = mul64(h0, p.r0) + mul64(h1, p.s3) + mul64(h2, p.s2) + mul64(h3, p.s1);
    uint64_t d1 = mul64(h0, p.r1) + mul64(h1, p.r0) + mul64(h2, p.s3) + mul64(h3, p.s2) + mul64(h4, p.s1);
    uint64_t d2 = mul64(h0, p.r2) + mul64(h1, p.r1) + mul64(h2, p.r0) + mul64(h3, p.s3) + mul64(h4, p.s2);
    uint64_t d3 = mul64(h0, p.r3) + mul64(h1, p.r2) + mul64(h2, p.r1) + mul64(h3, p.r0) + mul64(h4, p.s3);
    d1 += d0 >> 32;
    d2 += d1 >> 32;
    d3 += d2 >> 32;
    // bits 128.. : h4 r0 plus the carry out of d3 (< 2^31 + 2^31)
    const uint32_t d4 = h4 * p.r0 + (uint32_t)(d3 >> 32);
    // fold 2^130 * (d4 >> 2) as 5 (d4 >> 2) = (d4 >> 2) + (d4 & ~3)
    t = (uint64_t)(uint32_t)d0 + (d4 >> 2) + (d4 & ~3u);
    p.h0 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d1 + (t >> 32);
    p.h1 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d2 + (t >> 32);
    p.h2 = (uint32_t)t;
    t = (uint64_t)(uint32_t)d3 + (t >> 32);
    p.h3 = (uint32_t)t;
    p.h4 = (d4 & 3u) + (uint32_t)(t >> 32);
}

// tag = LE16((acc + s) mod 2^128) (poly1305.py:47-48).  h < 5 * 2^128 < 2p,
// so one conditional subtraction of p gives acc mod p.
__device__ __forceinline__ uint4 poly_finish(const Poly32& p) {
    uint64_t t = (uint64_t)p.h0 + 5;
    const uint32_t g0 = (uint32_t)t;
    t = (uint64_t)p.h1 + (t >> 32);
    const uint32_t g1 = (uint32_t)t;
    t = (uint64_t)p.h2 + (t >> 32);
    const uint32_t g2 = (uint32_t)t;
    t = (uint64_t)p.h3 + (t >> 32);
    const uint32_t g3 = (uint32_t)t;
    const uint32_t g4 = p.h4 + (uint32_t)(t >> 32);
    const uint32_t sel = 0u - (g4 >> 2);   // all ones when h + 5 >= 2^130, i.e. h >= p
    const uint32_t w0 = (p.h0 & ~sel) | (g0 & sel), w1 = (p.h1 & ~sel) | (g1 & sel);
    const uint32_t w2 = (p.h2 & ~sel) | (g2 & sel), w3 = (p.h3 & ~sel) | (g3 & sel);
    t = (uint64_t)w0 + p.p0;
    const uint32_t o0 = (uint32_t)t;
    t = (uint64_t)w1 + p.p1 + (t >> 32);
    const uint32_t o1 = (uint32_t)t;
    t = (uint64_t)w2 + p.p2 + (t >> 32);
    const uint32_t o2 = (uint32_t)t;
    t = (uint64_t)w3 + p.p3 + (t >> 32);
    return make_uint4(o0, o1, o2, (uint32_t)t);
}

struct F5 {
    uint32_t h0, h1, h2, h3, h4;
};

// a * b mod 2^130 - 5, limbs of both < 2^26 (a little above for a's h1)
__device__ __forceinline__ F5 fmul(const F5& a, const F5& b) {
    const uint32_t M26 = 0x3ffffffu;
    const uint32_t s1 = b.h1 * 5, s2 = b.h2 * 5, s3 = b.h3 * 5, s4 = b.h4 * 5;
    uint64_t d0 = mul64(a.h0, b.h0) + mul64(a.h1, s4) + mul64(a.h2, s3) + mul64(a.h3, s2) + mul64(a.h4, s1);
    uint64_t d1 = mul64(a.h0, b.h1) + mul64(a.h1, b.h0) + mul64(a.h2, s4) + mul64(a.h3, s3) + mul64(a.h4, s2);
    uint64_t d2 = mul64(a.h0, b.h2) + mul64(a.h1, b.h1) + mul64(a.h2, b.h0) + mul64(a.h3, s4) + mul64(a.h4, s3);
    uint64_t d3 = mul64(a.h0, b.h3) + mul64(a.h1, b.h2) + mul64(a.h2, b.h1) + mul64(a.h3, b.h0) + mul64(a.h4, s4);
    uint64_t d4 = mul64(a.h0, b.h4) + mul64(a.h1, b.h3) + mul64(a.h2, b.h2) + mul64(a.h3, b.h1) + mul64(a.h4, b.h0);
    F5 r;
    uint32_t c;
    c = (uint32_t)(d0 >> 26); r.h0 = (uint32_t)d0 & M26;
    d1 += c; c = (uint32_t)(d1 >> 26); r.h1 = (uint32_t)d1 & M26;
    d2 += c; c = (uint32_t)(d2 >> 26); r.h2 = (uint32_t)d2 & M26;
    d3 += c; c = (uint32_t)(d3 >> 26); r.h3 = (uint32_t)d3 & M26;
    d4 += c; c = (uint32_t)(d4 >> 26); r.h4 = (uint32_t)d4 & M26;
    r.h0 += c * 5; c = r.h0 >> 26; r.h0 &= M26;
    r.h1 += c;
    return r;
}

__device__ __forceinline__ F5 fnorm_add(const F5& a, const F5& b) {
    const uint32_t M26 = 0x3ffffffu;
    F5 r = {a.h0 + b.h0, a.h1 + b.h1, a.h2 + b.h2, a.h3 + b.h3, a.h4 + b.h4};
    uint32_t c;
    c = r.h0 >> 26; r.h0 &= M26; r.h1 += c;
    c = r.h1 >> 26; r.h1 &= M26; r.h2 += c;
    c = r.h2 >> 26; r.h2 &= M26; r.h3 += c;
    c = r.h3 >> 26; r.h3 &= M26; r.h4 += c;
    c = r.h4 >> 26; r.h4 &= M26; r.h0 += c * 5;
    c = r.h0 >> 26; r.h0 &= M26; r.h1 += c;
    return r;
}

__device__ __forceinline__ F5 fpow(F5 x, uint32_t e) {
    F5 r = {1, 0, 0, 0, 0};
    while (e) {
        if (e & 1) r = fmul(r, x);
        e >>= 1;
        if (e) x = fmul(x, x);
    }
    return r;
}

__device__ __forceinline__ F5 fshfl_xor(const F5& v, int m) {
    return F5{(uint32_t)__shfl_xor((int)v.h0, m, 64), (uint32_t)__shfl_xor((int)v.h1, m, 64),
              (uint32_t)__shfl_xor((int)v.h2, m, 64), (uint32_t)__shfl_xor((int)v.h3, m, 64),
              (uint32_t)__shfl_xor((int)v.h4, m, 64)};
}


// ---- wave-striped Horner (chacha_wave_kernel) --------------------------
// S threads share one message; thread seg takes the 64-byte chunks
// q = seg, seg + S, ... (four Poly1305 blocks each).  Between two of its
// chunks its Horner value skips the other threads' 4 (S - 1) blocks.
// Before chunk q: h <- h * r^(4S - 4) unless q is the thread's first chunk
// (rgap computed on the first gap only).
template <uint32_t S>
__device__ __forceinline__ void stripe_gap(Poly& p, const F5& r, uint32_t q, uint32_t seg, F5& rgap) {
    if (q == seg) return;
    if (q == seg + S) rgap = fpow(r, 4 * S - 4);   // only threads with a gap
    const F5 h = fmul(F5{p.h0, p.h1, p.h2, p.h3, p.h4}, rgap);
    p.h0 = h.h0; p.h1 = h.h1; p.h2 = h.h2; p.h3 = h.h3; p.h4 = h.h4;
}

// The thread's partial lifted by r^after (after = Poly1305 blocks of the
// message behind the thread's last one); cb = 0 means the thread had none.
__device__ __forceinline__ F5 stripe_lift(const Poly& p, const F5& r, uint32_t cb, uint32_t after) {
    F5 z = F5{p.h0, p.h1, p.h2, p.h3, p.h4};
    if (cb) z = fmul(z, fpow(r, after));
    return z;
}

// Sum of the partials of the W waves (64 W threads) of one message: a
// shuffle tree per wave, then through s_part (W entries per message slot)
// across waves.  All threads of the workgroup must call it when W > 1.
template <int W>
__device__ __forceinline__ F5 stripe_sum(F5 z, F5* s_part, uint32_t seg, uint32_t slot) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) z = fnorm_add(z, fshfl_xor(z, m));
    if (W > 1) {
        if ((seg & 63u) == 0) s_part[slot * W + (seg >> 6)] = z;
        __syncthreads();
        z = s_part[slot * W];
#pragma unroll
        for (int w = 1; w < W; ++w) z = fnorm_add(z, s_part[slot * W + w]);
    }
    return z;
}

// ---- octet striping (chacha_octet_kernel, selftest mode 4) ----------------
// Eight lanes per message; lane l owns the 64-byte chunks b = l, l + 8, ...
// (ChaCha blocks b of the record), i.e. the Poly1305 blocks 4 b .. 4 b + 3.
// Its Horner multiplies by r within a chunk and by r^29 after a chunk's last
// block (the other seven lanes' 28 blocks lie between), and by r after its
// own last block; its value is then lifted by r^f (octet_lift_exp) and the
// eight partials are summed over the octet.  All in 26-bit limbs: r^29 and
// the lift powers are general 130-bit values, which the radix-2^32 clamp
// trick (Poly32) cannot multiply by.

// A multiplier in 26-bit limbs with 5 x limbs 1..4 (2^130 == 5).
struct Mul26 {
    uint32_t r0, r1, r2, r3, r4, s1, s2, s3, s4;
};

__device__ __forceinline__ Mul26 mul26(const F5& r) {
    return Mul26{r.h0, r.h1, r.h2, r.h3, r.h4, r.h1 * 5, r.h2 * 5, r.h3 * 5, r.h4 * 5};
}

// h = (h + LE(m) + hib 2^128) * R mod 2^130 - 5 (poly1305.py:43-46 with any
// multiplier): poly_block with R instead of the key's r.
__device__ __forceinline__ void fblock(F5& h, uint4 m, const Mul26& R, uint32_t hib = 1u << 24) {
    const uint32_t M26 = 0x3ffffffu;
    uint32_t h0 = h.h0 + (m.x & M26);
    uint32_t h1 = h.h1 + (__builtin_amdgcn_alignbit(m.y, m.x, 26) & M26);
    uint32_t h2 = h.h2 + (__builtin_amdgcn_alignbit(m.z, m.y, 20) & M26);
    uint32_t h3 = h.h3 + (__builtin_amdgcn_alignbit(m.w, m.z, 14) & M26);
    uint32_t h4 = h.h4 + ((m.w >> 8) | hib);
    uint64_t d0 = mul64(h0, R.r0) + mul64(h1, R.s4) + mul64(h2, R.s3) + mul64(h3, R.s2) + mul64(h4, R.s1);
    uint64_t d1 = mul64(h0, R.r1) + mul64(h1, R.r0) + mul64(h2, R.s4) + mul64(h3, R.s3) + mul64(h4, R.s2);
    uint64_t d2 = mul64(h0, R.r2) + mul64(h1, R.r1) + mul64(h2, R.r0) + mul64(h3, R.s4) + mul64(h4, R.s3);
    uint64_t d3 = mul64(h0, R.r3) + mul64(h1, R.r2) + mul64(h2, R.r1) + mul64(h3, R.r0) + mul64(h4, R.s4);
    uint64_t d4 = mul64(h0, R.r4) + mul64(h1, R.r3) + mul64(h2, R.r2) + mul64(h3, R.r1) + mul64(h4, R.r0);
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & M26;
    d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & M26;
    d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & M26;
    d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & M26;
    d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & M26;
    h0 += c * 5; c = h0 >> 26; h0 &= M26;
    h1 += c;
    h.h0 = h0; h.h1 = h1; h.h2 = h2; h.h3 = h3; h.h4 = h4;
}

// The per-message powers of r the octet lanes use: r (F5), r^2, r^4, r^8,
// r^16 (the lift), r^29 (the jump), and s.  36 words (144 bytes) per
// message, written by chacha_otk_kernel (the one-time key, block 0).
struct OctetPoly {
    uint32_t r[5], r2[5], r4[5], r8[5], r16[5], r29[5];
    uint32_t s[4];
    uint32_t pad[2];
};
static_assert(sizeof(OctetPoly) == 144, "OctetPoly layout");

__device__ __forceinline__ F5 f5_at(const uint32_t* w) { return F5{w[0], w[1], w[2], w[3], w[4]}; }

// The powers from the clamped r (poly1305.py:37-38) in 26-bit limbs.
__device__ __forceinline__ void octet_powers(const F5& r, OctetPoly& o) {
    const F5 r2 = fmul(r, r), r4 = fmul(r2, r2), r8 = fmul(r4, r4), r16 = fmul(r8, r8);
    const F5 r29 = fmul(fmul(fmul(r16, r8), r4), r);
    const F5* src[6] = {&r, &r2, &r4, &r8, &r16, &r29};
    uint32_t* dst[6] = {o.r, o.r2, o.r4, o.r8, o.r16, o.r29};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        dst[k][0] = src[k]->h0; dst[k][1] = src[k]->h1; dst[k][2] = src[k]->h2;
        dst[k][3] = src[k]->h3; dst[k][4] = src[k]->h4;
    }
}

// The lift exponent of an octet lane: lanes own 64-byte chunks b = l mod 8;
// nch chunks in all (the last holding mlast Poly1305 blocks, 1..4).  The lane
// whose chunk is the last (b_last = nch - 1) needs nothing more (0); the
// lane d chunks before it (d = 1..7) had its Horner end d chunks early and
// needs r^(4 (d - 1) + mlast).  Lanes without a chunk return 0 (their value
// is zero, whatever the lift).
__device__ __forceinline__ uint32_t octet_lift_exp(uint32_t l, uint32_t nch, uint32_t mlast) {
    if (nch == 0 || l >= nch) return 0;
    const uint32_t d = (nch - 1u - l) & 7u;
    return d ? 4u * (d - 1u) + mlast : 0u;
}

// v * r^f for f < 32 from the stored powers (one multiply per set bit).
__device__ __forceinline__ F5 octet_lift(F5 v, uint32_t f, const uint32_t* r, const uint32_t* r2,
                                         const uint32_t* r4, const uint32_t* r8, const uint32_t* r16) {
    if (f & 1u) v = fmul(v, f5_at(r));
    if (f & 2u) v = fmul(v, f5_at(r2));
    if (f & 4u) v = fmul(v, f5_at(r4));
    if (f & 8u) v = fmul(v, f5_at(r8));
    if (f & 16u) v = fmul(v, f5_at(r16));
    return v;
}

// Sum of the eight partials of an octet (lanes 8 q .. 8 q + 7).
__device__ __forceinline__ F5 octet_sum(F5 z) {
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) z = fnorm_add(z, fshfl_xor(z, m));
    return z;
}

// tag = LE16((acc + s) mod 2^128) for an F5 accumulator (poly1305.py:47-48).
__device__ __forceinline__ uint4 octet_finish(const F5& h, const uint32_t* s) {
    Poly p;
    p.h0 = h.h0; p.h1 = h.h1; p.h2 = h.h2; p.h3 = h.h3; p.h4 = h.h4;
    p.p0 = s[0]; p.p1 = s[1]; p.p2 = s[2]; p.p3 = s[3];
    return poly_finish(p);
}

}  // namespace
}  // namespace tg
