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

#include "aes_round.h"

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

template <int NR, bool OPEN, int TAG, bool WIN, class RK>
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

    // B_0 (aesccm.py:40-46); the length is numberToByteArray(len, 3)
    const uint32_t flags = (alen ? 64u : 0u) + 8u * ((TAG - 2) / 2) + 2u;
    uint4 x = aes_block<NR>(lane4, rk,
                            make_uint4(flags | (nv.x << 8), a1, a2, a3 | (bswap32(len) & 0xffffff00u)));

    // enc(len(aad)) || aad, zero-padded (aesccm.py:48-67)
    if (alen) {
        const uint32_t np = alen < 0xff00u ? 2u : 6u;
        const uint4 pre = np == 2 ? make_uint4(((alen >> 8) & 0xffu) | ((alen & 0xffu) << 8), 0, 0, 0)
                                  : make_uint4(0xfeffu | (((alen >> 24) & 0xffu) << 16) |
                                                   (((alen >> 16) & 0xffu) << 24),
                                               ((alen >> 8) & 0xffu) | ((alen & 0xffu) << 8), 0, 0);
        const uint32_t first = alen < 16 - np ? alen : 16 - np;
        uint4 blk = shl_bytes(load_partial(ad, first), np);
        blk = make_uint4(blk.x | pre.x, blk.y | pre.y, blk.z, blk.w);
        x = aes_block<NR>(lane4, rk, xor_blk(x, blk));
        for (uint32_t off = first; off < alen; off += 16) {
            const uint32_t m = alen - off < 16 ? alen - off : 16;
            x = aes_block<NR>(lane4, rk, xor_blk(x, load_partial(ad + off, m)));
        }
    }

    // payload: keystream S_1.., CBC-MAC over the plaintext (aesccm.py:68-70)
    const uint32_t nfull = len >> 4;
    const uint32_t tail = len & 15;
    // keystream through the 256-counter window cache (aes_round.h): the
    // counter is be24 in bytes 13..15, byte 15 its low byte as in GCM
    uint4 wc = win_consts_w<NR>(lane4, rk, cc, a3);
    uint32_t whi = 0;
    uint4 ks = aes_ctr_win<NR>(lane4, rk, cc, wc, 1u);
    for (uint32_t j = 0; j < nfull; ++j) {
        const uint4 d = load16(in + 16 * j, aligned);
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
    }
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
// TLSGPU_CCM_VARIANT=1 runs full rounds (measurement).
template <int NR, bool OPEN, int TAG, bool TABLE, bool WIN>
__global__ __launch_bounds__(ccm_threads<TABLE>()) void ccm_kernel(const AesKeyDev* __restrict__ keys,
                                                          tg_batch b) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_ccm));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const AesKeyDev* kp = TABLE ? keys + b.key_idx[i] : keys;
    RkRegs<NR> rk;
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    ccm_record<NR, OPEN, TAG, WIN>(b, i, lane4, rk);
}

template <int NR, bool OPEN, int TAG, bool TABLE, bool WIN>
int launch_w(const AesKeyDev* keys, const tg_batch& b, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)ccm_kernel<NR, OPEN, TAG, TABLE, WIN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCcmLds) !=
            hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    constexpr int threads = ccm_threads<TABLE>();
    const uint64_t blocks = (b.n + threads - 1) / threads;
    hipLaunchKernelGGL((ccm_kernel<NR, OPEN, TAG, TABLE, WIN>), dim3((unsigned)blocks),
                       dim3(threads), kCcmLds, s, keys, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

template <int NR, bool OPEN, int TAG, bool TABLE>
int launch(const AesKeyDev* keys, const tg_batch& b, hipStream_t s) {
    const char* e = getenv("TLSGPU_CCM_VARIANT");   // read per launch (tests, measurement)
    if (e && atoi(e) == 1) return launch_w<NR, OPEN, TAG, TABLE, false>(keys, b, s);
    return launch_w<NR, OPEN, TAG, TABLE, true>(keys, b, s);
}

template <int NR, int TAG, bool TABLE>
int launch_op(const AesKeyDev* keys, const tg_batch& b, bool open, hipStream_t s) {
    return open ? launch<NR, true, TAG, TABLE>(keys, b, s) : launch<NR, false, TAG, TABLE>(keys, b, s);
}

template <int NR, bool TABLE>
int launch_tag(const AesKeyDev* keys, int taglen, const tg_batch& b, bool open, hipStream_t s) {
    return taglen == 16 ? launch_op<NR, 16, TABLE>(keys, b, open, s)
                        : launch_op<NR, 8, TABLE>(keys, b, open, s);
}

}  // namespace
}  // namespace tg

int tg_launch_ccm(const tg::AesKeyDev* keys, bool table, int rounds, int taglen,
                  const tg_batch& b, bool open, hipStream_t s) {
    if (taglen != 16 && taglen != 8) return TG_EINVAL;
    if (rounds == 10)
        return table ? tg::launch_tag<10, true>(keys, taglen, b, open, s)
                     : tg::launch_tag<10, false>(keys, taglen, b, open, s);
    if (rounds == 14)
        return table ? tg::launch_tag<14, true>(keys, taglen, b, open, s)
                     : tg::launch_tag<14, false>(keys, taglen, b, open, s);
    return TG_EINVAL;
}
