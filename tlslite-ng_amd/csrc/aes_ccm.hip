// aes_ccm.hip -- batched AES-CCM / CCM_8 seal/open for gfx950 (SURVEY.md
// section 8(f) row 2).
//
// Restates AESCCM (tlslite/utils/aesccm.py:11-155, RFC 3610 with a 12-byte
// nonce, so the length field is L = 3 bytes), one record per lane:
//   _cbcmac_calc :36-83   CBC-MAC with a zero IV over
//                         B_0 || enc(len(aad)) || aad || pad16 || msg || pad16,
//                         B_0 = flags || nonce || be24(len(msg)),
//                         flags = 64*(aad != "") + 8*((tag_len - 2)/2) + (L - 1)
//   seal         :85-113  T = MAC[:tag_len] ^ E(S_0), C = P ^ E(S_1..)
//   open         :115-149 P = C ^ E(S_1..), MAC recomputed over P, compared
// with counter blocks S_j = (L - 1) || nonce || be24(j).  The AES round is the
// shared T-table round (aes_round.h); both block streams of a record run in
// one pass over its payload: the keystream block of j+1 is computed while
// block j's CBC-MAC step runs, so the lane always has two independent AES
// encryptions in flight (the CBC-MAC chain itself is serial per record,
// parallel across records -- as SURVEY.md section 8(f) notes).
//
// Only the 64 KiB Te block lives in LDS (no GHASH tables), so two workgroups
// share a CU: 1024 threads each with a single key (round keys wave-uniform in
// SGPRs, < 64 VGPRs -> 8 waves/SIMD), 512 with a key table (this lane's
// schedule in VGPRs, < 128 VGPRs -> 4 waves/SIMD).
//
// Counter words: bytes 12..15 of S_j are nonce[11] || be24(j), i.e. the LE
// word nonce[11] | (bswap32(j) & 0xffffff00) for j < 2^24.  A record is
// therefore limited to 2^24 - 2 blocks (256 MiB); past that the reference's
// 128-bit increment would carry into the nonce (tlsgpu.h documents the limit).
#include <stdlib.h>

#include "aes_bs8.h"
#include "aes_round.h"
#include "options.h"

namespace tg {
namespace {

constexpr size_t kCcmLds = 65536;
template <bool TABLE>
constexpr int ccm_threads() { return TABLE ? 512 : 1024; }

extern __shared__ __attribute__((aligned(16))) uint4 g_lds_ccm[];

// v shifted towards higher byte positions by n in {2, 6} bytes (n % 4 == 2).
__device__ __forceinline__ uint4 shl_bytes(uint4 v, uint32_t n) {
    if (n >= 4) v = make_uint4(0u, v.x, v.y, v.z);
    return make_uint4(v.x << 16, (v.y << 16) | (v.x >> 16), (v.z << 16) | (v.y >> 16),
                      (v.w << 16) | (v.z >> 16));
}

__device__ __forceinline__ uint4 xor_blk(uint4 a, uint4 b) { return xor4(a, b); }

// CBC-MAC over B_0 and the encoded AAD blocks (aesccm.py:40-67): step(blk)
// performs x = E(x ^ blk) on the caller's state (x = 0 before B_0).
// B_0 = flags || nonce || be24(len), then enc(len(aad)) || aad, zero-padded.
// nv: the nonce as LE words; a1, a2, a3 its words shifted by one byte.
template <int TAG, class Step>
__device__ __forceinline__ void ccm_mac_head(Step&& step, uint4 nv, uint32_t a1, uint32_t a2,
                                             uint32_t a3, uint32_t len, const uint8_t* ad,
                                             uint32_t alen) {
    // B_0 (aesccm.py:40-46); the length is numberToByteArray(len, 3)
    const uint32_t flags = (alen ? 64u : 0u) + 8u * ((TAG - 2) / 2) + 2u;
    step(make_uint4(flags | (nv.x << 8), a1, a2, a3 | (bswap32(len) & 0xffffff00u)));
    // enc(len(aad)) || aad, zero-padded (aesccm.py:48-67)
    if (alen) {
        const uint32_t np = alen < 0xff00u ? 2u : 6u;
        const uint4 pre = np == 2 ? make_uint4(((alen >> 8) & 0xffu) | ((alen & 0xffu) << 8), 0, 0, 0)
                                  : make_uint4(0xfeffu | (((alen >> 24) & 0xffu) << 16) |
                                                   (((alen >> 16) & 0xffu) << 24),
                                               ((alen >> 8) & 0xffu) | ((alen & 0xffu) << 8), 0, 0);
        const uint32_t first = alen < 16 - np ? alen : 16 - np;
        uint4 blk = shl_bytes(load_partial(ad, first), np);
        step(make_uint4(blk.x | pre.x, blk.y | pre.y, blk.z, blk.w));
        for (uint32_t off = first; off < alen; off += 16) {
            const uint32_t m = alen - off < 16 ? alen - off : 16;
            step(load_partial(ad + off, m));
        }
    }
}

template <int NR, bool OPEN, int TAG, bool WIN, class RK, int G = 0>
__device__ __forceinline__ void ccm_record(const tg_batch& b, uint64_t i, uint32_t lane4,
                                           const RK& rk) {
    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;

    // nonce bytes n0..n11 as LE words; S_j = 2 || n || be24(j)
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const uint32_t a0 = 2u | (nv.x << 8);
    const uint32_t a1 = (nv.x >> 24) | (nv.y << 8);
    const uint32_t a2 = (nv.y >> 24) | (nv.z << 8);
    const uint32_t a3 = nv.z >> 24;                       // n11, counter bytes zero
    const CtrCache cc = ctr_cache<NR>(lane4, rk, make_uint4(a0, a1, a2, 0u));
    const uint4 s0 = aes_ctr_w<NR>(lane4, rk, cc, a3);   // E(S_0) masks the tag

    uint4 x = make_uint4(0, 0, 0, 0);
    ccm_mac_head<TAG>([&](uint4 blk) { x = aes_block<NR>(lane4, rk, xor_blk(x, blk)); }, nv, a1, a2,
                      a3, len, ad, alen);

    // payload: keystream S_1.., CBC-MAC over the plaintext (aesccm.py:68-70)
    const uint32_t nfull = len >> 4;
    const uint32_t tail = len & 15;
    // keystream through the 256-counter window cache (aes_round.h): the
    // counter is be24 in bytes 13..15, byte 15 its low byte as in GCM
    uint4 wc = win_consts_w<NR>(lane4, rk, cc, a3);
    uint32_t whi = 0;
    uint4 ks = aes_ctr_win<NR>(lane4, rk, cc, wc, 1u);
    // one block of the loop: XOR, store, MAC step, the next block's keystream
    auto step = [&](uint32_t j, const uint4& d) {
        const uint4 c = xor4(d, ks);
        store16(out + 16 * j, c, aligned);
        // next block's keystream is independent of this block's CBC step
        if (!WIN) {
            ks = aes_ctr_w<NR>(lane4, rk, cc, a3 | (bswap32(j + 2u) & 0xffffff00u));
        } else {
            if (((j + 2u) >> 8) != whi) {      // all lanes at the same j: uniform
                whi = (j + 2u) >> 8;
                wc = win_consts_w<NR>(lane4, rk, cc, a3 | (bswap32(j + 2u) & 0xffffff00u));
            }
            ks = aes_ctr_win<NR>(lane4, rk, cc, wc, j + 2u);
        }
        x = aes_block<NR>(lane4, rk, xor_blk(x, OPEN ? c : d));
    };
    // the payload G blocks at a time, the next group's loads issued before
    // this group's blocks run (G = 0: a dependent load per block)
    uint32_t j = 0;
    if (G > 0 && nfull >= (uint32_t)G) {
        uint4 d[G > 0 ? G : 1];
#pragma unroll
        for (int q = 0; q < G; ++q) d[q] = load16(in + 16 * q, aligned);
        for (; j + 2 * G <= nfull; j += G) {
            uint4 nx[G > 0 ? G : 1];
#pragma unroll
            for (int q = 0; q < G; ++q) nx[q] = load16(in + 16 * (j + G + q), aligned);
#pragma unroll
            for (int q = 0; q < G; ++q) step(j + q, d[q]);
#pragma unroll
            for (int q = 0; q < G; ++q) d[q] = nx[q];
        }
#pragma unroll
        for (int q = 0; q < G; ++q) step(j + q, d[q]);
        j += G;
    }
    for (; j < nfull; ++j) step(j, load16(in + 16 * j, aligned));
    if (tail) {
        const uint4 d = load_partial(in + 16 * nfull, tail);
        const uint4 c = mask_tail(xor4(d, ks), tail);
        store_partial(out + 16 * nfull, c, tail);
        x = aes_block<NR>(lane4, rk, xor_blk(x, OPEN ? c : d));
    }

    const uint4 t = xor4(x, s0);   // the auth value; CCM_8 keeps its first 8 bytes
    if (!OPEN) {
        if (TAG == 16) {
            store16(out + len, t, aligned && tail == 0);
        } else {
            store_partial(out + len, t, 8);
        }
        return;
    }
    // open: received_mac != computed_mac -> None (aesccm.py:144-146)
    const uint4 exp = TAG == 16 ? load16(in + len, aligned && tail == 0) : load_partial(in + len, 8);
    uint32_t diff = (exp.x ^ t.x) | (exp.y ^ t.y);
    if (TAG == 16) diff |= (exp.z ^ t.z) | (exp.w ^ t.w);
    if (b.status) b.status[i] = diff == 0;
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t k = 0; k < nfull; ++k) store16(out + 16 * k, z, aligned);
        if (tail) store_partial(out + 16 * nfull, z, tail);
    }
}

// WIN: the keystream through the 256-counter window cache (default);
// option ccm_variant 1 runs full rounds (measurement).  A key-table record
// whose key_idx is not below nkeys is skipped (open: status 0).
// Single key: two 1024-thread workgroups per CU (64 KiB of Te each) need <= 64
// VGPRs (8 waves per SIMD, HIP's second launch bound), so the one-block
// prefetch (G = 1) is held to that; deeper prefetch takes one workgroup per CU.
template <int NR, bool OPEN, int TAG, bool TABLE, bool WIN, int G = 0>
__global__ __launch_bounds__(ccm_threads<TABLE>(), (!TABLE && G <= 1) ? 8 : 1) void ccm_kernel(const AesKeyDev* __restrict__ keys,
                                                          uint64_t nkeys, tg_batch b) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_ccm));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    if (TABLE && b.key_idx[i] >= nkeys) {
        if (OPEN && b.status) b.status[i] = 0;
        return;
    }
    const AesKeyDev* kp = TABLE ? keys + b.key_idx[i] : keys;
    RkRegs<NR> rk;
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    ccm_record<NR, OPEN, TAG, WIN, RkRegs<NR>, G>(b, i, lane4, rk);
}

// ---- one block on the four lanes of a quad (the serial CBC-MAC chain) ----
// Quad table (wave kernel LDS at 0): row x (256 B apart, 128 B used) holds 4
// copies each of T0[x], T1[x] = rotl8 T0[x], T2[x] = rotl16 T0[x],
// T3[x] = rotl24 T0[x] and S[x] << 8k (k = 0..3); lane c reads copy c % 4, so
// the four lanes of a quad never share a bank.  Table t of row x sits at
// (x << 8) + 16 t + 4 c: te_addr() builds (x.byteK << 8) | lc with one v_perm
// and the 16 t rides in the DS offset.
constexpr uint32_t kQuadRows = 256 * 256;
template <int T, int K>
__device__ __forceinline__ uint32_t Q(uint32_t x, uint32_t lc) { return lds_u32(te_addr<K>(x, lc) + 16 * T); }

__device__ __forceinline__ void stage_quad(uint4* q) {
    for (int e = threadIdx.x; e < 256 * 8; e += blockDim.x) {
        const uint32_t x = e >> 3, t = e & 7, v = c_te.te0[x];
        const uint32_t w = t < 4 ? rotl32(v, 8 * t) : ((v >> 8) & 0xffu) << (8 * (t - 4));
        q[16 * x + t] = make_uint4(w, w, w, w);
    }
}

// Lane c holds state column c and the column-c words of the round keys.  It
// looks up its own column's four bytes -- T0(b0) for column c, T1(b1) for
// c - 1, T2(b2) for c - 2, T3(b3) for c - 3 (the terms of col()) -- and
// gathers column c's other three terms from lanes c + 1 .. c + 3 with DPP
// quad permutes fused into the XORs: 4 lookups per round and lane instead of
// 16 on one lane.
// acc ^ (v of lane (c + K) % 4), one v_xor_b32 with a DPP quad permute on its
// first operand (the compiler would build v_mov_b32_dpp + v_bitop3 and put
// two dependent instructions on the chain).  v comes from an LDS read, not a
// VALU write, so the DPP read needs no wait states.
template <int K>
__device__ __forceinline__ uint32_t xor_from(uint32_t v, uint32_t acc) {
    uint32_t d;
#if defined(__HIP_DEVICE_COMPILE__)
    if (K == 1)
        asm volatile("v_xor_b32_dpp %0, %1, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
                     : "=v"(d) : "v"(v), "v"(acc));
    else if (K == 2)
        asm volatile("v_xor_b32_dpp %0, %1, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
                     : "=v"(d) : "v"(v), "v"(acc));
    else
        asm volatile("v_xor_b32_dpp %0, %1, %2 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf"
                     : "=v"(d) : "v"(v), "v"(acc));
#else
    d = v ^ acc;
#endif
    return d;
}

template <int NR>
__device__ __forceinline__ uint32_t aes_quad(uint32_t lc, const uint32_t (&rkc)[NR + 1], uint32_t x) {
    uint32_t s = x ^ rkc[0];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint32_t p0 = Q<0, 0>(s, lc), p1 = Q<1, 1>(s, lc), p2 = Q<2, 2>(s, lc), p3 = Q<3, 3>(s, lc);
        s = xor_from<3>(p3, xor_from<2>(p2, xor_from<1>(p1, p0 ^ rkc[r])));
    }
    const uint32_t p0 = Q<4, 0>(s, lc), p1 = Q<5, 1>(s, lc), p2 = Q<6, 2>(s, lc), p3 = Q<7, 3>(s, lc);
    return xor_from<3>(p3, xor_from<2>(p2, xor_from<1>(p1, p0 ^ rkc[NR])));
}

// One full block on one lane from the quad table (the stream wave's counter
// blocks; up to 16-way bank conflicts, off the critical path).
template <int NR, class RK>
__device__ __forceinline__ uint4 aes_block_q(uint32_t lc, const RK& rkp, uint4 in) {
    const uint4 k0 = rkp.get(0);
    uint32_t s0 = in.x ^ k0.x, s1 = in.y ^ k0.y, s2 = in.z ^ k0.z, s3 = in.w ^ k0.w;
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint4 k = rkp.get(r);
        const uint32_t t0 = xor3(Q<0, 0>(s0, lc), Q<1, 1>(s1, lc), k.x) ^ (Q<2, 2>(s2, lc) ^ Q<3, 3>(s3, lc));
        const uint32_t t1 = xor3(Q<0, 0>(s1, lc), Q<1, 1>(s2, lc), k.y) ^ (Q<2, 2>(s3, lc) ^ Q<3, 3>(s0, lc));
        const uint32_t t2 = xor3(Q<0, 0>(s2, lc), Q<1, 1>(s3, lc), k.z) ^ (Q<2, 2>(s0, lc) ^ Q<3, 3>(s1, lc));
        const uint32_t t3 = xor3(Q<0, 0>(s3, lc), Q<1, 1>(s0, lc), k.w) ^ (Q<2, 2>(s1, lc) ^ Q<3, 3>(s2, lc));
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = rkp.get(NR);
    return make_uint4(xor3(Q<4, 0>(s0, lc), Q<5, 1>(s1, lc), k.x) ^ (Q<6, 2>(s2, lc) ^ Q<7, 3>(s3, lc)),
                      xor3(Q<4, 0>(s1, lc), Q<5, 1>(s2, lc), k.y) ^ (Q<6, 2>(s3, lc) ^ Q<7, 3>(s0, lc)),
                      xor3(Q<4, 0>(s2, lc), Q<5, 1>(s3, lc), k.z) ^ (Q<6, 2>(s0, lc) ^ Q<7, 3>(s1, lc)),
                      xor3(Q<4, 0>(s3, lc), Q<5, 1>(s0, lc), k.w) ^ (Q<6, 2>(s1, lc) ^ Q<7, 3>(s2, lc)));
}

__device__ __forceinline__ uint32_t word_of(uint4 v, uint32_t c) {
    return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

// ---- wave-per-record kernel (per-record calls and small batches) --------
// The CBC-MAC chain is serial, the CTR keystream is not.  One record per
// 128-thread workgroup, two wave roles:
//   wave 1 (stream wave): for 64-block chunk k, lane t loads payload block
//     64k + t (one coalesced 1 KiB row per instruction, the next chunk's row
//     already in flight), XORs it with E(S_{64k+t+1}), stores the output and
//     stages the MAC input block (plaintext: seal's input, open's output) in
//     LDS buffer k % 2;
//   wave 0 (MAC wave): lanes 0-3 run B_0, the AAD blocks and then
//     x = E(x ^ m) (aes_quad) over the staged blocks of chunk k - 1 while the
//     stream wave fills chunk k.
// One workgroup barrier per chunk hands the buffers over, so the record takes
// about (blocks + 2) serial quad encryptions with the payload's HBM latency
// and the keystream hidden behind them (the lane kernel pays a dependent HBM
// load per block).  Both waves read the quad table.
constexpr int kCcmWaveThreads = 128;
constexpr uint32_t kCcmStage = kQuadRows;       // 2 x 64 x 16 B staged MAC input
constexpr uint32_t kCcmMisc = 65536 + 2048;     // E(S_0), open verdict
constexpr uint32_t kCcmRk = 65536 + 2048 + 32;  // the record's round keys
constexpr size_t kCcmWaveLds = 65536 + 2048 + 32 + 240;

template <int NR, bool OPEN, int TAG, bool TABLE>
__global__ __launch_bounds__(kCcmWaveThreads) void ccm_wave_kernel(const AesKeyDev* __restrict__ keys,
                                                                   uint64_t nkeys, tg_batch b) {
    const uint64_t i = blockIdx.x;                 // the record (workgroup-uniform)
    if (TABLE && b.key_idx[i] >= nkeys) {          // out-of-range key index: skipped
        if (OPEN && b.status && threadIdx.x == 0) b.status[i] = 0;
        return;
    }
    stage_quad(g_lds_ccm);
    const AesKeyDev* kp = TABLE ? keys + b.key_idx[i] : keys;
    uint32_t* rkw = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(g_lds_ccm) + kCcmRk);
    if (threadIdx.x < 4 * (NR + 1)) rkw[threadIdx.x] = kp->rk[threadIdx.x];
    const RkLds rk{kCcmRk};                        // round keys read per round from LDS
    const uint32_t lane = threadIdx.x & 63u, lc = (threadIdx.x & 3u) << 2;
    const bool mac_wave = threadIdx.x < 64;
    uint4* stage = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(g_lds_ccm) + kCcmStage);
    uint4* misc = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(g_lds_ccm) + kCcmMisc);

    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const uint32_t a0 = 2u | (nv.x << 8);
    const uint32_t a1 = (nv.x >> 24) | (nv.y << 8);
    const uint32_t a2 = (nv.y >> 24) | (nv.z << 8);
    const uint32_t a3 = nv.z >> 24;
    const uint32_t nfull = len >> 4, tail = len & 15, nblk = (len + 15) >> 4;
    const uint32_t nch = (nblk + 63) >> 6;
    __syncthreads();                               // Te staged

    uint32_t xc = 0;                               // MAC lanes 0-3: column lane of x
    uint32_t rkc[NR + 1];
    if (mac_wave && lane < 4) {
#pragma unroll
        for (int r = 0; r <= NR; ++r) rkc[r] = rkw[4 * r + lane];
    }
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (!mac_wave) {
        if (lane == 0) misc[0] = aes_block_q<NR>(lc, rk, make_uint4(a0, a1, a2, a3));   // E(S_0) masks the tag
        if (lane < nfull) nxt = load16(in + 16 * lane, aligned);
    }
    for (uint32_t k = 0; k <= nch; ++k) {
        if (!mac_wave && k < nch) {
            const uint32_t j = 64 * k + lane;
            const uint4 d = nxt;
            if (j + 64 < nfull) nxt = load16(in + 16 * (j + 64), aligned);
            uint4 m = make_uint4(0, 0, 0, 0);
            if (j < nblk) {
                const uint4 ks = aes_block_q<NR>(lc, rk, make_uint4(a0, a1, a2, a3 | (bswap32(j + 1u) & 0xffffff00u)));
                if (j < nfull) {
                    const uint4 c = xor4(d, ks);
                    store16(out + 16 * j, c, aligned);
                    m = OPEN ? c : d;
                } else {                           // the partial last block
                    const uint4 dt = load_partial(in + 16 * j, tail);
                    const uint4 c = mask_tail(xor4(dt, ks), tail);
                    store_partial(out + 16 * j, c, tail);
                    m = OPEN ? c : dt;
                }
            }
            stage[64 * (k & 1) + lane] = m;
        }
        if (mac_wave && lane < 4) {
            if (k == 0) {
                ccm_mac_head<TAG>([&](uint4 blk) { xc = aes_quad<NR>(lc, rkc, xc ^ word_of(blk, lane)); },
                                  nv, a1, a2, a3, len, ad, alen);
            } else {
                const uint32_t q0 = 64 * (k - 1), cnt = nblk - q0 < 64 ? nblk - q0 : 64;
                const uint32_t* sb = reinterpret_cast<const uint32_t*>(stage + 64 * ((k - 1) & 1)) + lane;
                for (uint32_t q = 0; q < cnt; ++q) xc = aes_quad<NR>(lc, rkc, xc ^ sb[4 * q]);
            }
        }
        __syncthreads();
    }
    if (mac_wave && lane < 4) {
        const uint32_t tc = xc ^ reinterpret_cast<const uint32_t*>(misc)[lane];
        // the auth value (CCM_8 keeps its first 8 bytes), assembled on lane 0
        const uint4 t = make_uint4(__builtin_amdgcn_readlane(tc, 0), __builtin_amdgcn_readlane(tc, 1),
                                   __builtin_amdgcn_readlane(tc, 2), __builtin_amdgcn_readlane(tc, 3));
        if (lane == 0 && !OPEN) {
            if (TAG == 16) {
                store16(out + len, t, aligned && tail == 0);
            } else {
                store_partial(out + len, t, 8);
            }
        } else if (lane == 0) {   // received_mac != computed_mac -> None (aesccm.py:144-146)
            const uint4 exp = TAG == 16 ? load16(in + len, aligned && tail == 0) : load_partial(in + len, 8);
            uint32_t diff = (exp.x ^ t.x) | (exp.y ^ t.y);
            if (TAG == 16) diff |= (exp.z ^ t.z) | (exp.w ^ t.w);
            if (b.status) b.status[i] = diff == 0;
            misc[1] = make_uint4(diff, 0, 0, 0);
        }
    }
    if (!OPEN) return;
    __syncthreads();
    if (misc[1].x != 0) {                          // zero the released plaintext
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t q = threadIdx.x; q < nfull; q += kCcmWaveThreads) store16(out + 16 * q, z, aligned);
        if (tail && threadIdx.x == 0) store_partial(out + 16 * nfull, z, tail);
    }
}

// ---- hybrid lane-per-record kernel (large single-key batches) ----------
// The lane kernel above runs both AES streams of a block as T-table rounds
// (~293 LDS lookups per block) and is bound by the LDS.  Here the keystream
// of most records comes from the 8-block bitsliced cipher (aes_bs8.h) on the
// VALU, and only the serial CBC-MAC chain stays on the T-table rounds:
//   * a lane owns a record (as in ccm_kernel); batch beta of the lane is its
//     blocks 8 beta .. 8 beta + 7, i.e. counters S_(8 beta + 1 .. 8 beta + 8)
//     -- eight consecutive counters, the bs8 counter layout with SB = 0
//     (blocks one apart): counter bits 0..2 per block, bits >= 3 from beta,
//     the same for every lane of the wave (aesccm.py:36-38, :72-83);
//   * the counter block flags || nonce || be24(j) has bytes 0..12 constant
//     per record (nonce[11] is row 0 of column 3, where GCM has a zero
//     counter byte) and bytes 14..15 in rows 2-3 of column 3 exactly where
//     the GCM counter's low bytes sit, so round 1's S-box of rows 0-1 is a
//     per-record constant (kept in a lane-private LDS area) while the
//     counter stays below 2^16;
//   * the eight keystream blocks of a batch go to the payload (CTR) and the
//     eight plaintext blocks through the MAC chain x = E(x ^ m) by T-table
//     rounds (aes_block), the batch's payload loaded ahead of the chain.
// Waves 0 .. nt - 1 run the whole record on T-table rounds (ccm_record,
// the lane kernel's code), the rest as above; all take 64-record jobs from
// one queue, so the LDS pipe (MAC chains, T-table keystreams) and the VALU
// (bitsliced keystreams) are busy at the same time -- the AES-GCM hybrid's
// split (aes_gcm_bs8.hip gcm_hy_kernel).
constexpr int kCcmHyThreads = 768;                        // 12 waves (3 per SIMD, <= 168 VGPRs)
constexpr uint32_t kCcmHyRows = 65536;                    // after the Te block
constexpr uint32_t kCcmHyRowArea = 16 * 64 * 4;           // rows 0-1 planes, lane-major
constexpr uint32_t kCcmHyRk = kCcmHyRows + (kCcmHyThreads / 64) * kCcmHyRowArea;   // round keys
constexpr size_t kCcmHyLds = kCcmHyRk + 240;
constexpr int kCcmHyTDefault = 4;

// aes_block with the middle rounds as a loop: the MAC steps of a bitsliced
// batch are eight dependent blocks, and unrolled they spilled the cipher's
// registers.
template <int NR, class RK>
__device__ __forceinline__ uint4 aes_block_rolled(uint32_t lane4, const RK& rkp, uint4 in) {
    const uint4 k0 = rkp.get(0);
    uint32_t s0 = in.x ^ k0.x, s1 = in.y ^ k0.y, s2 = in.z ^ k0.z, s3 = in.w ^ k0.w;
#pragma unroll 1
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

template <int NR, bool OPEN, int TAG>
__device__ __forceinline__ void ccm_bs_record(const tg_batch& b, uint64_t i, bool valid, uint32_t lane4,
                                              const RkLds& rk, const bs8::KeyPlanesVmemFolded& km,
                                              uint32_t rows) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint8_t* in = valid ? rec_in(b, i) : nullptr;
    uint8_t* out = valid ? rec_out(b, i) : nullptr;
    const uint32_t len = valid ? rec_len(b, i) : 0u;
    const uint8_t* ad = valid ? rec_aad(b, i) : nullptr;
    const uint32_t alen = valid ? rec_aad_len(b, i) : 0u;
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = valid ? load_partial(b.nonce + 12 * i, 12) : make_uint4(0, 0, 0, 0);
    const uint32_t a0 = 2u | (nv.x << 8);
    const uint32_t a1 = (nv.x >> 24) | (nv.y << 8);
    const uint32_t a2 = (nv.y >> 24) | (nv.z << 8);
    const uint32_t a3 = nv.z >> 24;                       // n11, counter bytes zero
    // the first state's per-record words (S_j ^ rk0 without the counter)
    const uint4 k0 = rk.get(0);
    const uint32_t u[4] = {a0 ^ k0.x, a1 ^ k0.y, a2 ^ k0.z, a3 ^ k0.w};
    // rows 0 and 1 after round 1's SubBytes: no counter byte below 2^16
    {
        uint32_t r0[8], r1[8];
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            r0[bb] = bs8::rec_plane(u, bb);
            r1[bb] = bs8::rec_plane(u, 8 + bb);
        }
        bs::sbox(r0);
        bs::sbox(r1);
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            lds_st32(rows + 4u * (64u * bb + lane), r0[bb]);
            lds_st32(rows + 4u * (64u * (8 + bb) + lane), r1[bb]);
        }
    }
    // the last round key (the bitsliced rounds leave it out; its planes
    // carry the S-box constant, see aes_bs8.h)
    const uint4 kl = rk.get(NR);
    const uint4 rkl = make_uint4(kl.x ^ 0x63636363u, kl.y ^ 0x63636363u, kl.z ^ 0x63636363u, kl.w ^ 0x63636363u);
    uint32_t lanec[3], kmask;
    bs8::lane_consts<0>(1u, lanec, kmask);                // block j of a batch: counter 8 beta + 1 + j

    // E(S_0) masks the tag; B_0 and the AAD blocks start the MAC (aesccm.py:40-67)
    const uint4 s0 = aes_block<NR>(lane4, rk, make_uint4(a0, a1, a2, a3));
    uint4 x = make_uint4(0, 0, 0, 0);
    if (valid)
        ccm_mac_head<TAG>([&](uint4 blk) { x = aes_block<NR>(lane4, rk, xor_blk(x, blk)); }, nv, a1, a2, a3,
                          len, ad, alen);
    const uint32_t nfull = len >> 4, tail = len & 15, nblk = (len + 15) >> 4;
    uint32_t nb = (nblk + 7) >> 3;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)nb, off, 64);
        nb = o > nb ? o : nb;
    }
    nb = (uint32_t)__builtin_amdgcn_readfirstlane((int)nb);
    uint32_t u0 = u[0], u1 = u[1], u2 = u[2], u3 = u[3];
    for (uint32_t beta = 0; beta < nb; ++beta) {
        const uint32_t blk0 = 8u * beta;
        // the planes are rebuilt (rows 2-3) and re-read (rows 0-1) per batch:
        // hoisted out of the loop they held 32 more registers across the
        // cipher and spilled
        asm volatile("" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) :: "memory");
        const uint32_t uu[4] = {u0, u1, u2, u3};
        const bool hi = (beta + 1u) >> 13;                // counters >= 2^16 (records over 1 MiB)
        uint32_t s[4][8];
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            s[0][bb] = hi ? bs8::rec_plane(uu, bb) : lds_u32(rows + 4u * (64u * bb + lane));
            s[1][bb] = hi ? bs8::rec_plane(uu, 8 + bb) : lds_u32(rows + 4u * (64u * (8 + bb) + lane));
            s[2][bb] = bs8::rec_plane(uu, 16 + bb);
            s[3][bb] = bs8::rec_plane(uu, 24 + bb);
        }
#pragma unroll
        for (int bb = 0; bb < 3; ++bb) s[3][bb] ^= lanec[bb];
        bs8::ctr_planes<3, 16, 3>(s, kmask, beta);
        if (hi) bs8::ctr_planes<16, 32, 3>(s, kmask, beta);
        uint32_t w[4][8];
        bs8::encrypt<NR>(s, km, w, hi);
        __builtin_amdgcn_sched_barrier(0);   // the payload loads stay behind the cipher
        if (!valid) continue;
        // the batch's payload (held across the cipher it would spill): the
        // eight loads go out together, the MAC chain waits for the first
        uint4 d[8];
        const bool full = blk0 + 8u <= nfull;
        if (full) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = load16(in + 16u * (blk0 + j), aligned);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint4 ks = make_uint4(w[0][j] ^ rkl.x, w[1][j] ^ rkl.y, w[2][j] ^ rkl.z, w[3][j] ^ rkl.w);
            const uint32_t blk = blk0 + j;
            uint4 m = make_uint4(0, 0, 0, 0);
            if (full || blk < nfull) {
                const uint4 dd = full ? d[j] : load16(in + 16u * blk, aligned);
                const uint4 c = xor4(dd, ks);
                store16(out + 16u * blk, c, aligned);
                m = OPEN ? c : dd;
            } else if (blk < nblk) {                      // the partial last block
                const uint4 dd = load_partial(in + 16u * blk, tail);
                const uint4 c = mask_tail(xor4(dd, ks), tail);
                store_partial(out + 16u * blk, c, tail);
                m = OPEN ? c : dd;
            }
            if (blk < nblk) x = aes_block_rolled<NR>(lane4, rk, xor_blk(x, m));
        }
    }
    if (!valid) return;
    const uint4 t = xor4(x, s0);   // the auth value; CCM_8 keeps its first 8 bytes
    if (!OPEN) {
        if (TAG == 16) {
            store16(out + len, t, aligned && tail == 0);
        } else {
            store_partial(out + len, t, 8);
        }
        return;
    }
    // open: received_mac != computed_mac -> None (aesccm.py:144-146)
    const uint4 exp = TAG == 16 ? load16(in + len, aligned && tail == 0) : load_partial(in + len, 8);
    uint32_t diff = (exp.x ^ t.x) | (exp.y ^ t.y);
    if (TAG == 16) diff |= (exp.z ^ t.z) | (exp.w ^ t.w);
    if (b.status) b.status[i] = diff == 0;
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t k = 0; k < nfull; ++k) store16(out + 16 * k, z, aligned);
        if (tail) store_partial(out + 16 * nfull, z, tail);
    }
}

template <int NR, bool OPEN, int TAG>
__global__ __launch_bounds__(kCcmHyThreads) void ccm_hy_kernel(const AesKeyDev* __restrict__ key,
                                                               const tg_batch* bp,
                                                               const uint4* __restrict__ krows,
                                                               uint32_t* __restrict__ queue, uint32_t nt) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_ccm));   // Te0/Te2 copies at LDS 0
    // the round keys from LDS (broadcast reads): the bitsliced role's key rows
    // arrive by scalar loads, and both in SGPRs spilled
    if (threadIdx.x < 4 * (NR + 1))
        reinterpret_cast<uint32_t*>(g_lds_ccm)[kCcmHyRk / 4 + threadIdx.x] = key->rk[threadIdx.x];
    const RkLds rk{kCcmHyRk};
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    const uint64_t njobs = (bp->n + 63) / 64;
    const uint32_t rows = kCcmHyRows + wave * kCcmHyRowArea;
    for (;;) {
        uint32_t job = 0;
        if ((threadIdx.x & 63u) == 0) job = atomicAdd(queue, 1u);
        job = (uint32_t)__builtin_amdgcn_readfirstlane((int)job);
        if (job >= njobs) break;
        // the batch descriptor re-read per job (device copy): held in SGPRs
        // across the persistent loop it crowds out the ciphers' own scalars
        asm volatile("" ::: "memory");
        const tg_batch b = *bp;
        const uint64_t i = 64ull * job + (threadIdx.x & 63u);
        const bool valid = i < b.n;
        if (wave < nt) {
            if (valid) ccm_record<NR, OPEN, TAG, true, RkLds, 4>(b, i, lane4, rk);
        } else {
            ccm_bs_record<NR, OPEN, TAG>(b, i, valid, lane4, rk, bs8::KeyPlanesVmemFolded{{krows}}, rows);
        }
    }
}

// The hybrid kernel's scratch: the job counter, a device copy of the batch
// descriptor at word 16, then the key's bitsliced rows at word 128
// (aes_bs8.h KeyPlanesVmem layout, keymath.h bs8_row_word: the
// MixColumns-folded planes of the middle rounds), 480 words.
constexpr size_t kCcmHyScratch = 512 + 15 * 32 * 4;
static_assert(sizeof(tg_batch) <= 512 - 64, "batch copy");
__global__ void ccm_hy_setup_kernel(const AesKeyDev* __restrict__ key, int nr, tg_batch b, uint32_t* scratch) {
    const int t = (int)threadIdx.x;
    if (t == 0) {
        scratch[0] = 0;
        *reinterpret_cast<tg_batch*>(scratch + 16) = b;
    }
    for (int w = t; w < 15 * 32; w += (int)blockDim.x) scratch[128 + w] = bs8_row_word(key->rk, nr, w);
}

template <int NR, bool OPEN, int TAG>
int launch_hy(const AesKeyDev* key, const tg_batch& b, hipStream_t s) {
    const int o = opt(kOptCcmHyT);
    if (o > kCcmHyThreads / 64) return TG_EINVAL;
    const uint32_t nt = o < 0 ? 0u : o == 0 ? (uint32_t)kCcmHyTDefault : (uint32_t)o;
    if (lds_attr((const void*)ccm_hy_kernel<NR, OPEN, TAG>, (int)kCcmHyLds)) return TG_EHIP;
    if ((b.n + 63) / 64 > 0xffffffffull) return TG_EINVAL;
    uint32_t* scratch = nullptr;
    if (stream_alloc((void**)&scratch, kCcmHyScratch, s)) return TG_EHIP;
    hipLaunchKernelGGL(ccm_hy_setup_kernel, dim3(1), dim3(256), 0, s, key, NR, b, scratch);
    int rc = hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    if (!rc) {
        hipLaunchKernelGGL((ccm_hy_kernel<NR, OPEN, TAG>), dim3((unsigned)device_cus()), dim3(kCcmHyThreads),
                           kCcmHyLds, s, key, reinterpret_cast<const tg_batch*>(scratch + 16),
                           reinterpret_cast<const uint4*>(scratch + 128), scratch, nt);
        rc = hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    }
    if (stream_free(scratch, s) && !rc) rc = TG_EHIP;
    return rc;
}

template <int NR, bool OPEN, int TAG, bool TABLE>
int launch_wave(const AesKeyDev* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s) {
    if (lds_attr((const void*)ccm_wave_kernel<NR, OPEN, TAG, TABLE>, (int)kCcmWaveLds)) return TG_EHIP;
    if (b.n > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((ccm_wave_kernel<NR, OPEN, TAG, TABLE>), dim3((unsigned)b.n),
                       dim3(kCcmWaveThreads), kCcmWaveLds, s, keys, nkeys, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Up to this many records a batch runs the wave-per-record kernel (two
// workgroups of 66 KiB LDS per CU: 512 records in flight; at 16 KiB the two
// kernels meet near 4096 records: profiles/r02/v22_ccm_wave.txt).
constexpr uint64_t kCcmWaveMaxRecords = 4096;

template <int NR, bool OPEN, int TAG, bool TABLE, bool WIN, int G = 0>
int launch_w(const AesKeyDev* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s) {
    if (lds_attr((const void*)ccm_kernel<NR, OPEN, TAG, TABLE, WIN, G>, (int)kCcmLds)) return TG_EHIP;
    constexpr int threads = ccm_threads<TABLE>();
    const uint64_t blocks = (b.n + threads - 1) / threads;
    if (blocks > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((ccm_kernel<NR, OPEN, TAG, TABLE, WIN, G>), dim3((unsigned)blocks),
                       dim3(threads), kCcmLds, s, keys, nkeys, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Option ccm_variant (tests and measurement): 0 = auto (wave per record up
// to kCcmWaveMaxRecords, else lane per record with the window cache), 1 =
// lane per record, full rounds, 2 = wave per record, 3 = lane per record
// with the window cache, 4 = the hybrid lane-per-record kernel (single key),
// 5 / 6 / 7 / 8 = 3 with the payload loaded 1 / 2 / 4 / 8 blocks ahead.
template <int NR, bool OPEN, int TAG, bool TABLE>
int launch(const AesKeyDev* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s) {
    switch (opt(kOptCcmVariant)) {
        case 0:
            if (b.n <= kCcmWaveMaxRecords) return launch_wave<NR, OPEN, TAG, TABLE>(keys, nkeys, b, s);
            // single key: the payload four blocks ahead (one 1024-thread
            // workgroup per CU at 95 VGPRs): 612 against 502 GiB/s for the
            // dependent load per block at two workgroups per CU
            // (profiles/r05/r5d, r5e; 2 / 8 blocks: 604 / 589)
            if (!TABLE) return launch_w<NR, OPEN, TAG, TABLE, true, 4>(keys, nkeys, b, s);
            return launch_w<NR, OPEN, TAG, TABLE, true>(keys, nkeys, b, s);
        case 1: return launch_w<NR, OPEN, TAG, TABLE, false>(keys, nkeys, b, s);
        case 2: return launch_wave<NR, OPEN, TAG, TABLE>(keys, nkeys, b, s);
        case 3: return launch_w<NR, OPEN, TAG, TABLE, true>(keys, nkeys, b, s);
        case 4:
            if (TABLE) return launch_w<NR, OPEN, TAG, TABLE, true>(keys, nkeys, b, s);
            return launch_hy<NR, OPEN, TAG>(keys, b, s);
        case 5: return launch_w<NR, OPEN, TAG, TABLE, true, 1>(keys, nkeys, b, s);
        case 6: return launch_w<NR, OPEN, TAG, TABLE, true, 2>(keys, nkeys, b, s);
        case 7: return launch_w<NR, OPEN, TAG, TABLE, true, 4>(keys, nkeys, b, s);
        case 8: return launch_w<NR, OPEN, TAG, TABLE, true, 8>(keys, nkeys, b, s);

        default: return TG_EINVAL;
    }
}

template <int NR, int TAG, bool TABLE>
int launch_op(const AesKeyDev* keys, uint64_t nkeys, const tg_batch& b, bool open, hipStream_t s) {
    return open ? launch<NR, true, TAG, TABLE>(keys, nkeys, b, s) : launch<NR, false, TAG, TABLE>(keys, nkeys, b, s);
}

template <int NR, bool TABLE>
int launch_tag(const AesKeyDev* keys, uint64_t nkeys, int taglen, const tg_batch& b, bool open, hipStream_t s) {
    return taglen == 16 ? launch_op<NR, 16, TABLE>(keys, nkeys, b, open, s)
                        : launch_op<NR, 8, TABLE>(keys, nkeys, b, open, s);
}

}  // namespace
}  // namespace tg

int tg_launch_ccm(const tg::AesKeyDev* keys, uint64_t nkeys, int rounds, int taglen,
                  const tg_batch& b, bool open, hipStream_t s) {
    if (taglen != 16 && taglen != 8) return TG_EINVAL;
    const bool table = nkeys > 1;
    if (rounds == 10)
        return table ? tg::launch_tag<10, true>(keys, nkeys, taglen, b, open, s)
                     : tg::launch_tag<10, false>(keys, nkeys, taglen, b, open, s);
    if (rounds == 14)
        return table ? tg::launch_tag<14, true>(keys, nkeys, taglen, b, open, s)
                     : tg::launch_tag<14, false>(keys, nkeys, taglen, b, open, s);
    return TG_EINVAL;
}
