// aes_round.h -- the AES T-table round shared by the GCM and CCM kernels.
//
// Restates Rijndael.encrypt (tlslite/utils/rijndael.py:995-1038) for one
// block per lane with Te0 and Te2 = rotl16(Te0) in LDS:
//   * each table row x (256 B) = {Te0[x] x 32 copies, Te2[x] x 32 copies};
//     lane l reads copy l % 32, i.e. bank l % 32, so ds_read_b32 lookups are
//     conflict-free whatever the data;
//   * a column needs one rotation instead of three:
//       Te0[a] ^ rotl8(Te0[b]) ^ rotl16(Te0[c]) ^ rotl24(Te0[d])
//         = Te0[a] ^ Te2[c] ^ rotl8(Te0[b] ^ Te2[d]);
//   * each lookup address is one v_perm_b32 (or one full-rate v_bitop3 for
//     byte 1) of the state word and the lane's copy offset ``lane4``, which
//     also carries the table's LDS base (absolute LDS addressing: no static
//     LDS in these kernels, so offsets ride in the DS instruction);
//   * the final round's S-box byte is byte 1 of Te0[x].
// Included by exactly the kernel translation units; everything is internal.
#pragma once
#include "common.h"

namespace tg {
namespace {

// ---- Te0 generated at compile time from GF(2^8) exp/log tables ----------
struct TeTable {
    uint32_t te0[256];
};

constexpr uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

constexpr TeTable make_te() {
    uint8_t exp[256] = {};
    uint8_t log[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {
        exp[i] = x;
        log[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime(x));  // times generator 3
    }
    TeTable t = {};
    for (int v = 0; v < 256; ++v) {
        uint8_t inv = v ? exp[(255 - log[v]) % 255] : 0;
        uint8_t s = inv, r = inv;
        for (int k = 0; k < 4; ++k) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s = (uint8_t)(s ^ r);
        }
        s = (uint8_t)(s ^ 0x63);
        uint8_t s2 = xtime(s);
        uint8_t s3 = (uint8_t)(s2 ^ s);
        // column contribution of a row-0 byte: rows (2s, s, s, 3s), LE word
        t.te0[v] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
    return t;
}

__constant__ TeTable c_te = make_te();

#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(3))) uint32_t* lds_u32_ptr;
typedef const __attribute__((address_space(3))) uint4* lds_u128_ptr;
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) { return *(lds_u32_ptr)(uintptr_t)addr; }
__device__ __forceinline__ uint4 lds_u128(uint32_t addr) { return *(lds_u128_ptr)(uintptr_t)addr; }
__device__ __forceinline__ void lds_st128(uint32_t addr, uint4 v) {
    *(__attribute__((address_space(3))) uint4*)(uintptr_t)addr = v;
}
__device__ __forceinline__ void lds_st32(uint32_t addr, uint32_t v) {
    *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)addr = v;
}
__device__ __forceinline__ uint4 lds_u128_v(uint32_t addr) {
    const volatile __attribute__((address_space(3))) uint4* p =
        (const volatile __attribute__((address_space(3))) uint4*)(uintptr_t)addr;
    uint4 v;
    v.x = p->x; v.y = p->y; v.z = p->z; v.w = p->w;
    return v;
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t b, uint32_t c) {  // (a & b) | c
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xEA);
}
#else
__device__ __forceinline__ uint32_t lds_u32(uint32_t) { return 0; }
__device__ __forceinline__ uint4 lds_u128(uint32_t) { return uint4(); }
__device__ __forceinline__ uint4 lds_u128_v(uint32_t) { return uint4(); }
__device__ __forceinline__ void lds_st128(uint32_t, uint4) {}
__device__ __forceinline__ void lds_st32(uint32_t, uint32_t) {}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t b, uint32_t c) { return (a & b) | c; }
#endif

__device__ __forceinline__ uint4 xor4_3(uint4 a, uint4 b, uint4 c) {
    return make_uint4(xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y), xor3(a.z, b.z, c.z),
                      xor3(a.w, b.w, c.w));
}

// Byte address of row (byte K of x) for this lane; lane4 = 0x10000 | (lane%32)*4.
template <int K>
__device__ __forceinline__ uint32_t te_addr(uint32_t x, uint32_t lane4) {
    if (K == 1) return and_or(x, 0xff00u, lane4);   // one full-rate bitop3
    return __builtin_amdgcn_perm(x, lane4, 0x0c020000u | ((4u + K) << 8));
}
template <int K>
__device__ __forceinline__ uint32_t T0(uint32_t x, uint32_t lane4) { return lds_u32(te_addr<K>(x, lane4)); }
template <int K>
__device__ __forceinline__ uint32_t T2(uint32_t x, uint32_t lane4) { return lds_u32(te_addr<K>(x, lane4) + 128); }

// One T-table round column: rows from s_a byte 0, s_b byte 1, s_c byte 2, s_d byte 3.
__device__ __forceinline__ uint32_t col(uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd,
                                        uint32_t rk, uint32_t lane4) {
    return xor3(T0<0>(sa, lane4), T2<2>(sc, lane4), rk) ^
           rotl32(T0<1>(sb, lane4) ^ T2<3>(sd, lane4), 8);
}

// col with the round key pre-rotated (rkr = rotr8(rk)) and XORed inside the
// rotation: rotl8(x ^ rotr8(k)) = rotl8(x) ^ k, so a column is two 3-input
// XORs and one rotation (4 issue slots) instead of a 3-input XOR, two XORs
// and the rotation (5).
__device__ __forceinline__ uint32_t col_r(uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd,
                                          uint32_t rkr, uint32_t lane4) {
    return xor3(T0<0>(sa, lane4), T2<2>(sc, lane4), rotl32(xor3(T0<1>(sb, lane4), T2<3>(sd, lane4), rkr), 8));
}

// Final round column: S(x) is byte 1 of Te0[x].
__device__ __forceinline__ uint32_t col_last(uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd,
                                             uint32_t rk, uint32_t lane4) {
    const uint32_t lo = __builtin_amdgcn_perm(T0<1>(sb, lane4), T0<0>(sa, lane4), 0x0c0c0501u);
    const uint32_t hi = __builtin_amdgcn_perm(T0<3>(sd, lane4), T0<2>(sc, lane4), 0x05010c0cu);
    return xor3(lo, hi, rk);
}

// Round-key providers: get(r) = the four words of round key r.
template <int NR>
struct RkRegs {  // single key per launch: wave-uniform, lives in SGPRs
    uint32_t w[4 * (NR + 1)];
    __device__ __forceinline__ uint4 get(int r) const {
        return make_uint4(w[4 * r], w[4 * r + 1], w[4 * r + 2], w[4 * r + 3]);
    }
};
struct RkLds {  // key table: this lane's schedule staged in an LDS row
    uint32_t base;
    const uint4* rot = nullptr;   // hybrid AES-GCM: round keys rotated right by 8 (global, wave-uniform)
    // volatile: re-read per round instead of being hoisted into 60 VGPRs
    __device__ __forceinline__ uint4 get(int r) const { return lds_u128_v(base + 16 * r); }
};
// A wave-uniform key of a key table in global memory (scalar loads): the
// schedule words ``rk`` (GcmTableKey::rk) and the rotated copy ``rot`` (the
// key-table hybrid kernel's T-table waves, aes_gcm_bs8.hip).
struct RkTab {
    const uint32_t* rk;
    const uint4* rot;
    __device__ __forceinline__ uint4 get(int r) const {
        return make_uint4(rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3]);
    }
};

// Per-record round-1 constants for counter mode: after AddRoundKey the state
// words s0..s2 (nonce ^ rk0) are the same for every block of the record, so
// each round-1 column is a constant K_c XOR the one term that reads s3.
struct CtrCache {
    uint32_t k0, k1, k2, k3;
};

template <int NR, class RK>
__device__ __forceinline__ CtrCache ctr_cache(uint32_t lane4, const RK& rkp, uint4 nv) {
    const uint4 k0 = rkp.get(0), k1 = rkp.get(1);
    const uint32_t s0 = nv.x ^ k0.x, s1 = nv.y ^ k0.y, s2 = nv.z ^ k0.z;
    const uint32_t rk[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
    CtrCache c;
    // column 0: a=s0.b0 b=s1.b1 c=s2.b2 d=s3.b3(varies)
    c.k0 = T0<0>(s0, lane4) ^ T2<2>(s2, lane4) ^ rotl32(T0<1>(s1, lane4), 8) ^ rk[4];
    // column 1: a=s1.b0 b=s2.b1 c=s3.b2(varies) d=s0.b3
    c.k1 = T0<0>(s1, lane4) ^ rotl32(T0<1>(s2, lane4) ^ T2<3>(s0, lane4), 8) ^ rk[5];
    // column 2: a=s2.b0 b=s3.b1(varies) c=s0.b2 d=s1.b3
    c.k2 = T0<0>(s2, lane4) ^ T2<2>(s0, lane4) ^ rotl32(T2<3>(s1, lane4), 8) ^ rk[6];
    // column 3: a=s3.b0(varies) b=s0.b1 c=s1.b2 d=s2.b3
    c.k3 = T2<2>(s1, lane4) ^ rotl32(T0<1>(s0, lane4) ^ T2<3>(s2, lane4), 8) ^ rk[7];
    return c;
}

// E_K(w0 w1 w2 w3) for the counter block whose first three words the cache
// was built from; w3 is the last word as it sits in memory (LE of bytes 12..15).
template <int NR, class RK>
__device__ __forceinline__ uint4 aes_ctr_w(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                           uint32_t w3) {
    uint32_t s3 = w3 ^ rkp.get(0).w;
    uint32_t s0 = cc.k0 ^ rotl32(T2<3>(s3, lane4), 8);
    uint32_t s1 = cc.k1 ^ T2<2>(s3, lane4);
    uint32_t s2 = cc.k2 ^ rotl32(T0<1>(s3, lane4), 8);
    uint32_t t3 = cc.k3 ^ T0<0>(s3, lane4);
    uint32_t t0, t1, t2;
    s3 = t3;
#pragma unroll
    for (int r = 2; r < NR; ++r) {
        const uint4 k = rkp.get(r);
        t0 = col(s0, s1, s2, s3, k.x, lane4);
        t1 = col(s1, s2, s3, s0, k.y, lane4);
        t2 = col(s2, s3, s0, s1, k.z, lane4);
        t3 = col(s3, s0, s1, s2, k.w, lane4);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = rkp.get(NR);
    return make_uint4(col_last(s0, s1, s2, s3, k.x, lane4), col_last(s1, s2, s3, s0, k.y, lane4),
                      col_last(s2, s3, s0, s1, k.z, lane4), col_last(s3, s0, s1, s2, k.w, lane4));
}

// E_K(nonce || be32(ctr)) (the GCM counter block).
template <int NR, class RK>
__device__ __forceinline__ uint4 aes_ctr(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                         uint32_t ctr) {
    return aes_ctr_w<NR>(lane4, rkp, cc, bswap32(ctr));
}

// ---- 256-block counter windows (round-2 cache) ---------------------------
// Within a window of 256 counters (ctr >> 8 fixed) only byte 15 of the
// counter block changes.  After round 1 just state word 0 (A) depends on it
// (the s3 byte-3 term of column 0); words 1..3 (B, C, D) are fixed, so each
// round-2 column is a per-window constant W_c XOR the one lookup that reads
// A.  A block then costs 1 + 4 lookups for rounds 1-2 instead of 4 + 16.
// win_refresh computes W for the window holding ctr and stores it at the
// lane's LDS slot ``win`` (16 B); aes_ctr_win runs one block from it.
// Same function as aes_ctr (the windows are an algebraic regrouping of the
// T-table rounds of rijndael.py:995-1038, not a different cipher).
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void lds_st_u128(uint32_t addr, uint4 v) {
    *(__attribute__((address_space(3))) uint4*)(uintptr_t)addr = v;
}
#else
__device__ __forceinline__ void lds_st_u128(uint32_t, uint4) {}
#endif

// w3: the counter block's last word as it sits in memory (its byte 3, the
// counter's low byte, is ignored); win_consts(ctr) for the GCM layout.
template <int NR, class RK>
__device__ __forceinline__ uint4 win_consts_w(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                              uint32_t w3) {
    const uint32_t s3 = w3 ^ rkp.get(0).w;
    const uint32_t B = cc.k1 ^ T2<2>(s3, lane4);
    const uint32_t C = cc.k2 ^ rotl32(T0<1>(s3, lane4), 8);
    const uint32_t D = cc.k3 ^ T0<0>(s3, lane4);
    const uint4 k = rkp.get(2);
    uint4 w;
    w.x = xor3(T2<2>(C, lane4), k.x, rotl32(T0<1>(B, lane4) ^ T2<3>(D, lane4), 8));
    w.y = xor3(T0<0>(B, lane4), T2<2>(D, lane4), k.y) ^ rotl32(T0<1>(C, lane4), 8);
    w.z = xor3(T0<0>(C, lane4), k.z, rotl32(T0<1>(D, lane4) ^ T2<3>(B, lane4), 8));
    w.w = xor3(T0<0>(D, lane4), T2<2>(B, lane4), k.w) ^ rotl32(T2<3>(C, lane4), 8);
    return w;
}

template <int NR, class RK>
__device__ __forceinline__ uint4 win_consts(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                            uint32_t ctr) {
    return win_consts_w<NR>(lane4, rkp, cc, bswap32(ctr));
}

template <int NR, class RK>
__device__ __forceinline__ void win_refresh(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                            uint32_t win, uint32_t ctr) {
    lds_st_u128(win, win_consts<NR>(lane4, rkp, cc, ctr));
}

template <int NR, class RK>
__device__ __forceinline__ uint4 aes_ctr_win(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                             const uint4 w, uint32_t ctr) {
    const uint32_t A = cc.k0 ^ rotl32(T2<3>((ctr << 24) ^ rkp.get(0).w, lane4), 8);
    uint32_t s0 = w.x ^ T0<0>(A, lane4);
    uint32_t s1 = w.y ^ rotl32(T2<3>(A, lane4), 8);
    uint32_t s2 = w.z ^ T2<2>(A, lane4);
    uint32_t s3 = w.w ^ rotl32(T0<1>(A, lane4), 8);
    uint32_t t0, t1, t2, t3;
#pragma unroll
    for (int r = 3; r < NR; ++r) {
        const uint4 k = rkp.get(r);
        t0 = col(s0, s1, s2, s3, k.x, lane4);
        t1 = col(s1, s2, s3, s0, k.y, lane4);
        t2 = col(s2, s3, s0, s1, k.z, lane4);
        t3 = col(s3, s0, s1, s2, k.w, lane4);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = rkp.get(NR);
    return make_uint4(col_last(s0, s1, s2, s3, k.x, lane4), col_last(s1, s2, s3, s0, k.y, lane4),
                      col_last(s2, s3, s0, s1, k.z, lane4), col_last(s3, s0, s1, s2, k.w, lane4));
}

// Keystream of counters ctr0 .. ctr0 + G - 1.  WIN = 0: full rounds.  WIN:
// through the window cache at LDS ``win``, refreshed when the group is the
// first of a window (or ``first``); a group that straddles two windows runs
// full rounds.  ctr0 is the same for every lane of a lane-per-record wave, so
// both branches are wave-uniform.
template <int NR, int G, bool WIN, class RK>
__device__ __forceinline__ void ctr_keystream(uint32_t lane4, const RK& rkp, const CtrCache& cc,
                                              uint32_t win, uint32_t ctr0, bool first,
                                              uint4 (&ks)[G]) {
    if (!WIN || ((ctr0 ^ (ctr0 + G - 1)) >> 8) != 0) {
#pragma unroll
        for (int q = 0; q < G; ++q) ks[q] = aes_ctr<NR>(lane4, rkp, cc, ctr0 + q);
        return;
    }
    if (first || (ctr0 & 255u) < (uint32_t)G) win_refresh<NR>(lane4, rkp, cc, win, ctr0);
    const uint4 w = lds_u128(win);
#pragma unroll
    for (int q = 0; q < G; ++q) ks[q] = aes_ctr_win<NR>(lane4, rkp, cc, w, ctr0 + q);
}

// Full AES encryption of one block (all rounds from the table).
template <int NR, class RK>
__device__ __forceinline__ uint4 aes_block(uint32_t lane4, const RK& rkp, uint4 in) {
    const uint4 k0 = rkp.get(0);
    uint32_t s0 = in.x ^ k0.x, s1 = in.y ^ k0.y, s2 = in.z ^ k0.z, s3 = in.w ^ k0.w;
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint4 k = rkp.get(r);
        const uint32_t t0 = col(s0, s1, s2, s3, k.x, lane4);
        const uint32_t t1 = col(s1, s2, s3, s0, k.y, lane4);
        const uint32_t t2 = col(s2, s3, s0, s1, k.z, lane4);
        const uint32_t t3 = col(s3, s0, s1, s2, k.w, lane4);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = rkp.get(NR);
    return make_uint4(col_last(s0, s1, s2, s3, k.x, lane4), col_last(s1, s2, s3, s0, k.y, lane4),
                      col_last(s2, s3, s0, s1, k.z, lane4), col_last(s3, s0, s1, s2, k.w, lane4));
}

// Fill the 64 KiB Te0/Te2 copy block (``te`` points at its first word):
// row x = 8 x uint4{Te0[x]} then 8 x uint4{rotl16(Te0[x])}; consecutive
// threads write consecutive 16-byte slots (conflict-free ds_write_b128) and
// the 16 threads of a row read the same Te0 entry (one broadcast load).
__device__ __forceinline__ void stage_te(uint32_t* te) {
    uint4* t4 = reinterpret_cast<uint4*>(te);
#pragma unroll 4
    for (int e = threadIdx.x; e < 256 * 16; e += blockDim.x) {
        const uint32_t v = c_te.te0[e >> 4];
        const uint32_t w = (e & 8) ? rotl32(v, 16) : v;
        t4[e] = make_uint4(w, w, w, w);
    }
}

}  // namespace
}  // namespace tg
