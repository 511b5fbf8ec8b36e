// gcm_lane.h -- one AES-GCM record per lane: the T-table CTR keystream and
// the record's GHASH, seal or open (aesgcm.py:101-154).  Shared by the lane
// kernels of aes_gcm.hip and by the key-table hybrid of aes_gcm_bs8.hip, whose
// waves take the short records once the long ones are done (round 6).
#pragma once
#include "aes_round.h"
#include "common.h"
#include "ghash.h"

namespace tg {

struct GhashClmul {  // y kept in normal order; hn = H in normal order
    uint4 hn;
    __device__ __forceinline__ uint4 update(uint4 y, uint4 blk) const {
        const uint4 x = make_uint4(y.x ^ to_norm(blk.x), y.y ^ to_norm(blk.y),
                                   y.z ^ to_norm(blk.z), y.w ^ to_norm(blk.w));
        return gf128_mul(x, hn);
    }
    __device__ __forceinline__ uint4 finish(uint4 y) const {
        return make_uint4(to_norm(y.x), to_norm(y.y), to_norm(y.z), to_norm(y.w));
    }
};

// Full 16-byte blocks [0, G*ngroups) in groups of G.  The keystream of group
// g+1 and the payload of group g+1 are produced while group g is XORed and
// hashed, so the GHASH chain of seal (which needs the ciphertext) overlaps the
// next group's AES rounds.
// WIN: keystream through the lane's 256-counter window cache at LDS ``win``
// (aes_round.h, ctr_keystream).
template <int NR, bool OPEN, bool ALIGNED, int G, bool WIN, class RK, class GH>
__device__ __forceinline__ uint4 ctr_groups(uint32_t lane4, const RK& rk, const GH& gh,
                                            const CtrCache& cc, uint32_t win, const uint8_t* in,
                                            uint8_t* out, uint32_t ngroups, uint4 y) {
    if (ngroups == 0) return y;
    uint4 d[G], ks[G];
#pragma unroll
    for (int q = 0; q < G; ++q) d[q] = load16(in + 16 * q, ALIGNED);
    ctr_keystream<NR, G, WIN>(lane4, rk, cc, win, 2u, true, ks);
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint32_t gn = g + 1 < ngroups ? g + 1 : g;
        uint4 nx[G], c[G];
#pragma unroll
        for (int q = 0; q < G; ++q) nx[q] = load16(in + 16 * (G * gn + q), ALIGNED);
#pragma unroll
        for (int q = 0; q < G; ++q) {
            c[q] = xor4(d[q], ks[q]);
            store16(out + 16 * (G * g + q), c[q], ALIGNED);
        }
        ctr_keystream<NR, G, WIN>(lane4, rk, cc, win, 2u + G * (g + 1), false, ks);
#pragma unroll
        for (int q = 0; q < G; ++q) y = gh.update(y, OPEN ? d[q] : c[q]);
#pragma unroll
        for (int q = 0; q < G; ++q) d[q] = nx[q];
    }
    return y;
}

// One record: AESGCM.seal / AESGCM.open (aesgcm.py:101-154) for lane i.
template <int NR, bool OPEN, int G, class RK, class GH, bool WIN = false>
__device__ __forceinline__ void gcm_record(const tg_batch& b, uint64_t i, uint32_t lane4,
                                           const RK& rk, const GH& gh, uint32_t win = 0) {
    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;

    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const CtrCache cc = ctr_cache<NR>(lane4, rk, nv);
    // J0 = nonce || be32(1): the tag mask (aesgcm.py:112-115)
    const uint4 mask = aes_ctr<NR>(lane4, rk, cc, 1u);

    // GHASH over the AAD, zero-padded (aesgcm.py:69-79)
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < alen; off += 16) {
        uint32_t m = alen - off < 16 ? alen - off : 16;
        y = gh.update(y, load_partial(ad + off, m));
    }

    // CTR from nonce || be32(2) (aesgcm.py:118-120), GHASH over the ciphertext
    const uint32_t nfull = len >> 4;
    const uint32_t tail = len & 15;
    const uint32_t ngroups = nfull / G;
    y = aligned
            ? ctr_groups<NR, OPEN, true, G, WIN>(lane4, rk, gh, cc, win, in, out, ngroups, y)
            : ctr_groups<NR, OPEN, false, G, WIN>(lane4, rk, gh, cc, win, in, out, ngroups, y);
    for (uint32_t j = G * ngroups; j < nfull; ++j) {
        const uint4 ks = aes_ctr<NR>(lane4, rk, cc, 2u + j);
        const uint4 d = load16(in + 16 * j, aligned);
        const uint4 c = xor4(d, ks);
        store16(out + 16 * j, c, aligned);
        y = gh.update(y, OPEN ? d : c);
    }
    if (tail) {
        const uint4 ks = aes_ctr<NR>(lane4, rk, cc, 2u + nfull);
        const uint4 d = load_partial(in + 16 * nfull, tail);
        const uint4 c = mask_tail(xor4(d, ks), tail);
        store_partial(out + 16 * nfull, c, tail);
        y = gh.update(y, OPEN ? d : c);
    }

    // length block: be64(8*alen) || be64(8*len) (aesgcm.py:64)
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
    y = gh.update(y, make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                                bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits)));
    const uint4 tag = xor4(gh.finish(y), mask);
    if (!OPEN) {
        store16(out + len, tag, aligned && tail == 0);
        return;
    }
    // open: compare before releasing (aesgcm.py:148-149, constanttime.py:209-218)
    const uint4 exp = load16(in + len, aligned && tail == 0);
    const uint32_t diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
    if (b.status) b.status[i] = diff == 0;
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t k = 0; k < nfull; ++k) store16(out + 16 * k, z, aligned);
        if (tail) store_partial(out + 16 * nfull, z, tail);
    }
}

}  // namespace tg
