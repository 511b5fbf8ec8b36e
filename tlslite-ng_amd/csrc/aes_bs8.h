// aes_bs8.h -- bitsliced AES counter mode for gfx950, 8 counter blocks per
// lane in 32 registers ("row planes").
//
// Restates Rijndael.encrypt (tlslite/utils/rijndael.py:995-1038) on bit
// planes, like aes_bs.h, but with a state small enough for four or more
// waves per SIMD:
//   * s[i][b] = bit plane b of state row i: byte c of the register is column
//     c, bit j of that byte is block j of the lane's eight blocks;
//   * SubBytes is the 72-gate Boyar-Peralta cover of aes_bs.h (one
//     call covers the four bytes of a row for all eight blocks), its 0x63
//     folded into the next round key;
//   * ShiftRows rotates row i right by i bytes (one v_alignbit per plane);
//   * MixColumns + AddRoundKey are plane XORs with the round-key planes
//     (scalar operands, or broadcast LDS reads: KeyPlanesLds);
//   * the last round's ShiftRows is folded into the conversion back to block
//     words (a byte gather by v_perm plus an 8 x 8 bit transpose per byte).
// Counter blocks are nonce || be32(c), c = c0 + 64 beta + 8 j for block j of
// batch beta (the GCM kernel gives a lane every eighth block of its record),
// so bytes 0..11 are per-record constants, counter bits 0..5 per-lane
// constants and only bits >= 6 change per batch (wave-uniformly).
//
// Usable from host code too (the CPU unit test compiles it with g++).
#pragma once
#include "aes_bs.h"
#include "keymath.h"

namespace tg {
namespace bs8 {

#if !defined(__HIP_DEVICE_COMPILE__)
using bs::bop3;   // a macro (one v_bitop3_b32) in device code
#endif
using bs::perm;
using bs::xor3;

// Rotate right by 8 i bits: byte c of the result = byte (c + i) % 4 of x.
TG_BS_HD uint32_t rotr_bytes(uint32_t x, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(x, x, 8 * i);
#else
    return i ? (x >> (8 * i)) | (x << (32 - 8 * i)) : x;
#endif
}

// Round-key plane (r, i, b) at index (4 r + i) 8 + b: byte c = 0xff iff bit b
// of byte i of round-key word rk[4 r + c] ^ (r ? 0x63636363 : 0) is set
// (the S-box constant dropped by the circuit, see aes_bs.h; keymath.h).  rk: LE words of
// the schedule bytes (GcmKeyDev::rk).  (NR + 1) * 32 words per key.
TG_BS_HD uint32_t mask_word(const uint32_t* rk, int e) { return bs8_mask_word(rk, e); }

#if defined(__HIPCC__)
using Word4 = uint4;
#else
struct Word4 {   // the host build (g++, tests/native/bs8_check.cpp) has no HIP vector types
    uint32_t x, y, z, w;
};
#endif
TG_BS_HD Word4 word4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return Word4{a, b, c, d}; }

// Key-plane providers: row4(r, b) = the planes (r, i, b) of rows i = 0..3.
struct KeyPlanes {   // key planes in memory (host: plain reads; device: scalar loads)
    static constexpr bool kFolded = false;
    const uint32_t* w;
    TG_BS_MF uint32_t operator()(int r, int i, int b) const {
#if defined(__HIP_DEVICE_COMPILE__)
        return ((const __attribute__((address_space(4))) uint32_t*)w)[(4 * r + i) * 8 + b];
#else
        return w[(4 * r + i) * 8 + b];
#endif
    }
    TG_BS_MF Word4 row4(int r, int b) const {
        return word4((*this)(r, 0, b), (*this)(r, 1, b), (*this)(r, 2, b), (*this)(r, 3, b));
    }
};

// The same planes re-laid out in LDS as (8 r + b) * 16 + 4 i: one broadcast
// ds_read_b128 per (round, bit), so the key XORs take VGPR operands (a
// v_bitop3 with an SGPR operand issues at half rate on gfx950,
// profiles/r02/v5_issue_probe2.txt).  stage_lds_planes writes the layout.
#if defined(__HIPCC__)
struct KeyPlanesLds {
    static constexpr bool kFolded = false;
    uint32_t base;
    __device__ __forceinline__ uint4 row4(int r, int b) const {
#if defined(__HIP_DEVICE_COMPILE__)
        return *(const __attribute__((address_space(3))) uint4*)(uintptr_t)(base + 16u * (8 * r + b));
#else
        return uint4();
#endif
    }
};

// The KeyPlanesLds layout in global memory (L1/L2-resident, 1 920 B per
// key): one vector load per (round, bit) through the vector-memory path,
// which the octet kernels barely use, so neither the VALU (SGPR operands) nor
// the LDS (the T-table waves' pipe) pays for the key planes.
struct KeyPlanesVmem {
    static constexpr bool kFolded = false;
    const uint4* rows;
    __device__ __forceinline__ uint4 row4(int r, int b) const {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u v = *(const __attribute__((address_space(1))) v4u*)(rows + 8 * r + b);
        return make_uint4(v.x, v.y, v.z, v.w);
#else
        return rows[8 * r + b];
#endif
    }
};

// The same row layout holding the folded planes (keymath.h bs8_fold_word) of
// rounds 1 .. NR - 1: encrypt() runs mix_round_folded.  The rows' addresses
// are wave-uniform, so the compiler reads them with s_load_dwordx16 (both
// providers): the folded gates take SGPR operands and still win, 20 gates
// per round fewer (profiles/r02/v58_fold_keys/; from LDS, VGPR operands,
// they measured no better).
struct KeyPlanesVmemFolded : KeyPlanesVmem {
    static constexpr bool kFolded = true;
    static constexpr bool kRound = false;
};

// The folded rows by VECTOR loads: the address carries the lane's opaque zero
// ``zv``, so the compiler cannot scalarise it and the words arrive in VGPRs.
// As SGPR operands the 32 T gates of every round issue at half rate (any VALU
// instruction that reads an SGPR does on gfx950, profiles/r04/probe4.txt).
// encrypt() fetches a whole round's eight rows (32 VGPRs) at the start of the
// round, so the S-box gates hide the load latency; the vector-memory path is
// otherwise idle in the octet kernels.
struct KeyPlanesVec {
    static constexpr bool kFolded = true;
    static constexpr bool kRound = true;
    const uint4* rows;
    uint32_t zv;
    TG_BS_MF void round(int r, Word4 (&c)[8]) const {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const uint8_t* base = reinterpret_cast<const uint8_t*>(rows + 8 * r) + zv;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const v4u v = *(const __attribute__((address_space(1))) v4u*)(base + 16 * b);
            c[b] = make_uint4(v.x, v.y, v.z, v.w);
        }
#else
        for (int b = 0; b < 8; ++b) c[b] = rows[8 * r + b];
#endif
    }
    TG_BS_MF Word4 row4(int r, int b) const { return rows[8 * r + b]; }
};

// Plane (r, i, b) of the (NR + 1) * 32 in ``src`` (GcmKeyDev::bs8mask order)
// to LDS ``base`` in KeyPlanesLds order; all threads of the workgroup call it.
__device__ __forceinline__ void stage_lds_planes(uint32_t base, const uint32_t* src, int nr) {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int e = threadIdx.x; e < 32 * (nr + 1); e += blockDim.x) {
        const int r = e >> 5, i = (e >> 3) & 3, b = e & 7;
        *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(base + 16u * (8 * r + b) + 4u * i) = src[e];
    }
#endif
}
#endif

// The per-record part of the first state (after AddRoundKey 0): plane e =
// 8 i + b, byte c < 3 = bit e of u[c] (nonce word c ^ rk word c) spread to
// 0x00 / 0xff, byte 3 = the same of rk word 3 (the counter column's key
// byte; the counter itself is added per lane and batch).
TG_BS_HD uint32_t rec_plane(const uint32_t u[4], int e) {
    return (bs::bitmask(u[0], e) & 0x000000ffu) | (bs::bitmask(u[1], e) & 0x0000ff00u) |
           (bs::bitmask(u[2], e) & 0x00ff0000u) | (bs::bitmask(u[3], e) & 0xff000000u);
}

// Per-lane counter constants: block j of a lane's batch has counter
// c0 + (j << SB) (SB = 3 for eight lanes per record: blocks 8 apart; 4 / 5 /
// 6 for 16 / 32 / 64 lanes), c0 = the lane's first counter.  Counter bits
// 0 .. SB + 2 differ per block j but not per batch: lane[b] is their
// byte-3 plane for bit b (bits 0..7 belong to row 3, bit 8 to row 2); no
// carry leaves them except out of block 7 into the batch bits when
// c0 mod 2^(SB+3) >= 2^SB, which kmask = ~0 marks (see ctr_planes).
template <int SB = 3>
TG_BS_HD void lane_consts(uint32_t c0, uint32_t (&lane)[SB + 3], uint32_t& kmask) {
#pragma unroll
    for (int b = 0; b < SB + 3; ++b) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) m |= (((c0 + ((uint32_t)j << SB)) >> b) & 1u) << j;
        lane[b] = m << 24;
    }
    kmask = (c0 >> SB) & 1u ? 0xffffffffu : 0u;
}

// XOR the batch part of the counters (bits p >= Q0 = SB + 3: beta, or
// beta + 1 for block 7 of lanes with kmask) into the state, for counter bits
// [P0, P1).  The kernel does bits Q0..15 (rows 3 and 2) every batch and bits
// 16..31 only once beta + 1 >= 2^(16 - Q0) (records over 1 MiB for eight
// lanes per record; a wave-uniform test).
template <int P0, int P1, int Q0 = 6>
TG_BS_HD void ctr_planes(uint32_t (*s)[8], uint32_t kmask, uint32_t beta) {
    const uint32_t flip = beta ^ (beta + 1u);
#pragma unroll
    for (int p = P0; p < P1; ++p) {
        const uint32_t q = (uint32_t)(p - Q0);
        const uint32_t A = ((beta >> q) & 1u) ? 0xff000000u : 0u;
        const uint32_t D = ((flip >> q) & 1u) ? 0x80000000u : 0u;
        uint32_t& r = s[3 - (p >> 3)][p & 7];
        r = bop3(r, kmask, D, 0x78) ^ A;   // r ^ (kmask & D) ^ A
    }
}

// MixColumns(ShiftRows(x)) ^ K_r on the SubBytes output x, in place.
// out_i = 2 (a_i ^ a_i+1) ^ a_i+1 ^ (a_i+2 ^ a_i+3) ^ k with a_i = row i of
// the shifted state; 2x on planes: bit b <- bit b-1, bit 7 fed back into
// bits 0, 1, 3, 4 (0x11b).  Plane by plane (t_i of plane 7 first, it feeds
// the xtime of planes 0, 1, 3, 4), with scheduling fences between planes, so
// that only about 48 state-sized values are live instead of a, t and the
// output all at once (occupancy).
#if defined(__HIP_DEVICE_COMPILE__)
#define TG_BS8_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TG_BS8_FENCE() ((void)0)
#endif
template <class KM>
TG_BS_HD void mix_round(uint32_t (*s)[8], const KM& km, int r) {
    uint32_t a7[4], t7[4], tp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a7[i] = rotr_bytes(s[i][7], i);
#pragma unroll
    for (int i = 0; i < 4; ++i) t7[i] = a7[i] ^ a7[(i + 1) & 3];
    TG_BS8_FENCE();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t a[4], t[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = b == 7 ? a7[i] : rotr_bytes(s[i][b], i);
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i] = b == 7 ? t7[i] : a[i] ^ a[(i + 1) & 3];
        const Word4 k4 = km.row4(r, b);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = i == 0 ? k4.x : (i == 1 ? k4.y : (i == 2 ? k4.z : k4.w));
            const uint32_t tprev = b == 0 ? t7[i] : tp[i];
            if (b == 1 || b == 3 || b == 4)
                s[i][b] = xor3(xor3(tprev, t7[i], a[(i + 1) & 3]), t[(i + 2) & 3], k);
            else
                s[i][b] = xor3(tprev, a[(i + 1) & 3], t[(i + 2) & 3]) ^ k;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) tp[i] = t[i];
        TG_BS8_FENCE();
    }
}

// mix_round with the round key folded into the column XORs: with the planes
// c of bs8_fold_word (x c_i ^ c_(i+2) = k_i), T_i = a_i ^ a_(i+1) ^ c_i is one
// 3-input gate and out_i = x T_i ^ a_(i+1) ^ T_(i+2) already carries k_i, so
// the five planes without xtime feedback take one gate per row instead of
// two (20 gates per round fewer).  Provider: KeyPlanesVmemFolded (the
// hybrid kernel's default).
template <class KM>
TG_BS_HD void mix_round_folded(uint32_t (*s)[8], const KM& km, int r) {
    uint32_t a7[4], T7[4], Tp[4];
    const Word4 c7 = km.row4(r, 7);
    const uint32_t c7w[4] = {c7.x, c7.y, c7.z, c7.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) a7[i] = rotr_bytes(s[i][7], i);
#pragma unroll
    for (int i = 0; i < 4; ++i) T7[i] = xor3(a7[i], a7[(i + 1) & 3], c7w[i]);
    TG_BS8_FENCE();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t a[4], T[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = b == 7 ? a7[i] : rotr_bytes(s[i][b], i);
        if (b == 7) {
#pragma unroll
            for (int i = 0; i < 4; ++i) T[i] = T7[i];
        } else {
            const Word4 c4 = km.row4(r, b);
            const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) T[i] = xor3(a[i], a[(i + 1) & 3], cw[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t Tprev = b == 0 ? T7[i] : Tp[i];
            if (b == 1 || b == 3 || b == 4)
                s[i][b] = xor3(Tprev, T7[i], a[(i + 1) & 3]) ^ T[(i + 2) & 3];
            else
                s[i][b] = xor3(Tprev, a[(i + 1) & 3], T[(i + 2) & 3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Tp[i] = T[i];
        TG_BS8_FENCE();
    }
}

// mix_round_folded from a round's rows already in registers (KeyPlanesVec).
TG_BS_HD void mix_round_rows(uint32_t (*s)[8], const Word4 (&c)[8]) {
    uint32_t a7[4], T7[4], Tp[4];
    const uint32_t c7w[4] = {c[7].x, c[7].y, c[7].z, c[7].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) a7[i] = rotr_bytes(s[i][7], i);
#pragma unroll
    for (int i = 0; i < 4; ++i) T7[i] = xor3(a7[i], a7[(i + 1) & 3], c7w[i]);
    TG_BS8_FENCE();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t a[4], T[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = b == 7 ? a7[i] : rotr_bytes(s[i][b], i);
        if (b == 7) {
#pragma unroll
            for (int i = 0; i < 4; ++i) T[i] = T7[i];
        } else {
            const uint32_t cw[4] = {c[b].x, c[b].y, c[b].z, c[b].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) T[i] = xor3(a[i], a[(i + 1) & 3], cw[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t Tprev = b == 0 ? T7[i] : Tp[i];
            if (b == 1 || b == 3 || b == 4)
                s[i][b] = xor3(Tprev, T7[i], a[(i + 1) & 3]) ^ T[(i + 2) & 3];
            else
                s[i][b] = xor3(Tprev, a[(i + 1) & 3], T[(i + 2) & 3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Tp[i] = T[i];
        TG_BS8_FENCE();
    }
}

// 8 x 8 bit transpose inside every byte of a[0..7]: bit j of byte c of a[b]
// <-> bit b of byte c of a[j] (three swap stages, two shifts + two bitop3
// per pair).
// The stage masks in VGPRs: as SGPR or literal operands they make every
// v_bitop3 of the transposes half rate (VOP3 with a scalar operand), 96 of
// them per batch of eight blocks.  mask << m is ~mask, so one mask per stage
// serves both selects (operands swapped).
struct TransposeMasks {
    uint32_t m4, m2, m1;   // 0x0f0f0f0f, 0x33333333, 0x55555555
};
TG_BS_HD TransposeMasks transpose_masks() {
    TransposeMasks t{0x0f0f0f0fu, 0x33333333u, 0x55555555u};
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_mov_b32 %0, 0x0f0f0f0f" : "=v"(t.m4));
    asm volatile("v_mov_b32 %0, 0x33333333" : "=v"(t.m2));
    asm volatile("v_mov_b32 %0, 0x55555555" : "=v"(t.m1));
#endif
    return t;
}

TG_BS_HD void transpose8(uint32_t* a, const TransposeMasks& tm) {
#pragma unroll
    for (int l = 2; l >= 0; --l) {
        const int m = 1 << l;
        const uint32_t mask = m == 4 ? tm.m4 : m == 2 ? tm.m2 : tm.m1;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (r & m) continue;
            const uint32_t x = a[r], y = a[r + m];
            // y << 1 as y + y: v_lshlrev_b32 issues at half rate, v_add_u32 at
            // full (in asm: the compiler turns y + y back into a shift)
            uint32_t ys = y << m;
#if defined(__HIP_DEVICE_COMPILE__)
            if (m == 1) asm("v_add_u32 %0, %1, %1" : "=v"(ys) : "v"(y));
#endif
            a[r] = bop3(mask, x, ys, 0xca);           // (y << m) where ~mask, else x
            a[r + m] = bop3(mask, x >> m, y, 0xca);   // (x >> m) where mask, else y
        }
    }
}

// The last SubBytes output x (rows, pre-ShiftRows) -> block words:
// w[q][j] = word q (column q, LE) of block j's keystream WITHOUT the last
// round key.  Column q of the shifted state takes row i from column
// (q + i) % 4, gathered by v_perm, then each column's eight planes are
// transposed into the eight blocks.
TG_BS_HD void to_blocks(uint32_t (*x)[8], uint32_t (*w)[8]) {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t s0 = x[0][b], s1 = x[1][b], s2 = x[2][b], s3 = x[3][b];
        const uint32_t A = perm(s1, s0, 0x07020500u);    // s0.0 s1.1 s0.2 s1.3
        const uint32_t B = perm(s3, s2, 0x05000702u);    // s2.2 s3.3 s2.0 s3.1
        const uint32_t A2 = perm(s1, s0, 0x04030601u);   // s0.1 s1.2 s0.3 s1.0
        const uint32_t B2 = perm(s3, s2, 0x06010403u);   // s2.3 s3.0 s2.1 s3.2
        w[0][b] = perm(B, A, 0x05040100u);
        w[2][b] = perm(B, A, 0x07060302u);
        w[1][b] = perm(B2, A2, 0x05040100u);
        w[3][b] = perm(B2, A2, 0x07060302u);
        TG_BS8_FENCE();
    }
    const TransposeMasks tm = transpose_masks();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        transpose8(w[q], tm);
        TG_BS8_FENCE();
    }
}

// Rounds 1..NR on the state after AddRoundKey 0 (in place); w receives the
// blocks (to_blocks).  Middle rounds are a rolled loop on the device (a
// round is ~500 instructions).
//
// sub01 = false: rows 0 and 1 of s already hold round 1's SubBytes output.
// In counter mode with counters below 2^16 those rows are the nonce bytes and
// counter bytes 12-13 (zero), the same for every block of a record, so the
// caller computes their S-box once per record (rows 2 and 3 carry counter
// bytes 14 and 15): two of the four S-box calls of round 1 (144 of ~4 500
// instructions per batch of eight blocks).
template <class KM, class = void>
struct RoundRows {
    static constexpr bool value = false;
};
template <class KM>
struct RoundRows<KM, decltype((void)KM::kRound)> {
    static constexpr bool value = KM::kRound;
};
template <class KM>
TG_BS_HD constexpr bool round_rows() { return RoundRows<KM>::value; }

template <int NR, class KM>
TG_BS_HD void encrypt(uint32_t (*s)[8], const KM& km, uint32_t (*w)[8], bool sub01 = true) {
    // KeyPlanesVec: the round's key rows are fetched before its S-box gates
    Word4 c[8];
    if constexpr (round_rows<KM>()) km.round(1, c);
    // round 1 peeled off the rolled loop: its S-box of rows 0-1 is optional
    if (sub01) {
        bs::sbox(s[0]);
        TG_BS8_FENCE();
        bs::sbox(s[1]);
        TG_BS8_FENCE();
    }
    bs::sbox(s[2]);
    TG_BS8_FENCE();
    bs::sbox(s[3]);
    TG_BS8_FENCE();
    if constexpr (round_rows<KM>())
        mix_round_rows(s, c);
    else if constexpr (KM::kFolded)
        mix_round_folded(s, km, 1);
    else
        mix_round(s, km, 1);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
    for (int r = 2; r < NR; ++r) {
        if constexpr (round_rows<KM>()) km.round(r, c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bs::sbox(s[i]);
            TG_BS8_FENCE();
        }
        if constexpr (round_rows<KM>())
            mix_round_rows(s, c);
        else if constexpr (KM::kFolded)
            mix_round_folded(s, km, r);
        else
            mix_round(s, km, r);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bs::sbox(s[i]);
        TG_BS8_FENCE();
    }
    to_blocks(s, w);
}

}  // namespace bs8
}  // namespace tg
