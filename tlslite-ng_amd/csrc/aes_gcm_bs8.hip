// aes_gcm_bs8.hip -- batched single-key AES-GCM seal/open with the AES on the
// VALU (8-block bitslicing, aes_bs8.h) for gfx950 (CDNA4).
//
// Restates AESGCM.seal/open (tlslite/utils/aesgcm.py:101-154) with the CTR
// keystream of Python_AES_CTR (python_aes.py:101-116) and GHASH
// (aesgcm.py:60-99), eight lanes per TLS record ("octet"), eight records per
// wavefront:
//
//   * the GHASH input AAD || C || length block is front-padded with zero
//     blocks (neutral) to P = 8 ceil(M / 8) blocks; lane l of the octet owns
//     the padded positions l, l + 8, l + 16, ... and folds them by Horner with
//     stride H^8 (y <- y H^8 ^ X, the 8-bit tables of H^8 staged in LDS);
//     since GHASH = sum_t X_t H^(P - t) its value is lifted once by H^(8 - l)
//     (a table-free multiply by a power from the key's table) and the eight
//     partials are XOR-reduced by shuffles;
//   * ciphertext block k sits at position pad + na + k, so lane l owns the
//     blocks k = rho + 8 v, rho = (l + nc + 1) mod 8; batch beta of the lane
//     is its blocks v = 8 beta .. 8 beta + 7, i.e. counters
//     2 + rho + 64 beta + 8 j, encrypted together by the bitsliced cipher;
//     for a fixed j the octet's eight lanes cover 128 consecutive record
//     bytes, so every load and store instruction moves whole 128-byte lines;
//   * the nonce part of the first state is built once per record into LDS
//     (32 planes, shared by the octet), the counter part per lane and batch
//     from a few wave-uniform masks;
//   * the tag mask E_K(J0) is one byte-wise AES block (S-box in LDS).
// LDS: the H^8 tables (64 KiB) + S-box + 4 KiB of record planes per 512-thread
// workgroup, two workgroups per CU.
#include <cstdlib>

#include "aes_bs8.h"
#include "aes_round.h"
#include "ghash.h"

namespace tg {
namespace {

constexpr int kBs8Threads = 512;
constexpr int kBs8Recs = kBs8Threads / 8;               // record slots per workgroup
constexpr uint32_t kBs8Sbox = 65536;                      // 256-byte S-box
constexpr uint32_t kBs8RecBase = 65536 + 256;             // 128 B of planes per record slot
constexpr size_t kBs8Lds = kBs8RecBase + kBs8Recs * 128;

// No static __shared__ in this file: the GHASH tables sit at LDS address 0
// (gmul's absolute addresses).
extern __shared__ __attribute__((aligned(16))) uint4 g_lds_bs8[];

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o < v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

template <int NR, bool OPEN>
__global__ __launch_bounds__(kBs8Threads, 4) void gcm_bs8_kernel(const GcmKeyDev* __restrict__ key,
                                                                tg_batch b,
                                                                const uint32_t* __restrict__ order) {
    for (int e = threadIdx.x; e < kGhashEntries; e += kBs8Threads) g_lds_bs8[e] = key->ghash8[e];
    if (threadIdx.x < 64) {   // S(x) = byte 1 of Te0[x]
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v |= ((c_te.te0[4 * threadIdx.x + q] >> 8) & 0xffu) << (8 * q);
        reinterpret_cast<uint32_t*>(g_lds_bs8)[kBs8Sbox / 4 + threadIdx.x] = v;
    }
    const uint32_t* rk = key->rk;
    const uint32_t l = threadIdx.x & 7u;
    const uint32_t slot = threadIdx.x >> 3;
    const uint64_t t = (uint64_t)blockIdx.x * kBs8Recs + slot;
    const bool valid = t < b.n;
    const uint64_t i = valid ? (order ? order[t] : t) : 0;
    uint32_t len = 0, alen = 0;
    const uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    const uint8_t* ad = nullptr;
    uint4 nv = make_uint4(0, 0, 0, 0);
    if (valid) {
        len = rec_len(b, i);
        alen = rec_aad_len(b, i);
        in = rec_in(b, i);
        out = rec_out(b, i);
        ad = rec_aad(b, i);
        nv = load_partial(b.nonce + 12 * i, 12);
    }
    asm volatile("" ::: "memory");
    const uint32_t nfull = len >> 4, tail = len & 15, nc = (len + 15) >> 4, na = (alen + 15) >> 4;
    const uint32_t rho = (l + nc + 1u) & 7u;   // this lane's ciphertext blocks: rho + 8 v
    const uint32_t recb = kBs8RecBase + slot * 128u;
    {   // the record's first-state planes 4 l .. 4 l + 3 (nonce ^ rk0 spread to bytes)
        const uint32_t u[4] = {nv.x ^ rk[0], nv.y ^ rk[1], nv.z ^ rk[2], rk[3]};
        const uint4 rp = make_uint4(bs8::rec_plane(u, 4 * l), bs8::rec_plane(u, 4 * l + 1),
                                    bs8::rec_plane(u, 4 * l + 2), bs8::rec_plane(u, 4 * l + 3));
        lds_st128(recb + 16u * l, rp);
    }
    __syncthreads();

    uint32_t lanec[6], kmask;
    bs8::lane_consts(2u + rho, lanec, kmask);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint32_t nvl = nc > rho ? (nc - rho + 7u) >> 3 : 0u;          // blocks of this lane
    const uint32_t nfl = nfull > rho ? (nfull - rho + 7u) >> 3 : 0u;    // full ones
    const uint32_t nbatch = wave_max_u32((nvl + 7u) >> 3);
    // batches in which every valid lane of the wave has all eight blocks full
    const uint32_t nfast = __all(!valid || aligned) ? wave_min_u32(valid ? nfl >> 3 : 0xffffffffu) : 0u;

    // GHASH over this lane's AAD positions (aesgcm.py:69-79), zero-padded blocks
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t a = (l + na + nc + 1u) & 7u; a < na; a += 8) {
        const uint32_t m = alen - 16 * a < 16 ? alen - 16 * a : 16;
        y = xor4(gmul(y), load_partial(ad + 16 * a, m));
    }

    const bs8::KeyPlanes km{key->bs8mask};
    const uint4 rkl = make_uint4(rk[4 * NR] ^ 0x63636363u, rk[4 * NR + 1] ^ 0x63636363u,
                                 rk[4 * NR + 2] ^ 0x63636363u, rk[4 * NR + 3] ^ 0x63636363u);
    for (uint32_t beta = 0; beta < nbatch; ++beta) {
        uint32_t s[4][8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = lds_u128(recb + 16u * q);
            s[q >> 1][4 * (q & 1) + 0] = v.x;
            s[q >> 1][4 * (q & 1) + 1] = v.y;
            s[q >> 1][4 * (q & 1) + 2] = v.z;
            s[q >> 1][4 * (q & 1) + 3] = v.w;
        }
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) s[3][bb] ^= lanec[bb];
        bs8::ctr_planes<6, 16>(s, kmask, beta);
        if ((beta + 1u) >> 10) bs8::ctr_planes<16, 32>(s, kmask, beta);
        uint32_t w[4][8];
        bs8::encrypt<NR>(s, km, w);
        const uint32_t blk0 = rho + 64u * beta;   // block of slot j: blk0 + 8 j
        auto ks = [&](int j) { return make_uint4(w[0][j], w[1][j], w[2][j], w[3][j]); };
        if (beta < nfast) {
            if (valid) {
                // XOR + store first (the keystream dies block by block), then the
                // GHASH chain over the eight inputs held in d
                uint4 d[8];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    d[j] = *reinterpret_cast<const uint4*>(in + 16u * (blk0 + 8u * j));
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint4 k = ks(j);
                    const uint4 c = make_uint4(xor3(d[j].x, k.x, rkl.x), xor3(d[j].y, k.y, rkl.y),
                                               xor3(d[j].z, k.z, rkl.z), xor3(d[j].w, k.w, rkl.w));
                    *reinterpret_cast<uint4*>(out + 16u * (blk0 + 8u * j)) = c;
                    if (!OPEN) d[j] = c;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) y = xor4(gmul_lowreg(y), d[j]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t blk = blk0 + 8u * j;
                if (!valid || blk >= nc) continue;
                const uint4 k = ks(j);
                const uint4 kk = make_uint4(k.x ^ rkl.x, k.y ^ rkl.y, k.z ^ rkl.z, k.w ^ rkl.w);
                uint4 d, c;
                if (blk < nfull) {
                    d = load16(in + 16u * blk, aligned);
                    c = xor4(d, kk);
                    store16(out + 16u * blk, c, aligned);
                } else {                                  // the partial last block
                    d = load_partial(in + 16u * blk, tail);
                    c = mask_tail(xor4(d, kk), tail);
                    store_partial(out + 16u * blk, c, tail);
                }
                y = xor4(gmul_lowreg(y), OPEN ? d : c);
            }
        }
    }
    if (!__any(valid)) return;
    // length block be64(8 alen) || be64(8 len) (aesgcm.py:64): the last position
    if (l == 7) {
        const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
        y = xor4(gmul(y), make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                                     bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits)));
    }
    // lift by H^(8 - l) and XOR-reduce over the octet
    uint4 yn = norm4(y);
    if (yn.x | yn.y | yn.z | yn.w) yn = gf128_mul(yn, key->hpow[7 - l]);
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) yn = xor4(yn, shfl_xor4(yn, m));
    // tag = GHASH ^ E_K(J0), J0 = nonce || be32(1) (aesgcm.py:112-122)
    if (valid) nv = load_partial(b.nonce + 12 * i, 12);   // reloaded: not held across the loop
    const uint4 mask = aes_block_sb<NR>(rk, make_uint4(nv.x, nv.y, nv.z, bswap32(1u)), kBs8Sbox);
    const uint4 tag = xor4(norm4(yn), mask);
    const bool tag_aligned = aligned && tail == 0;
    if (!OPEN) {
        if (valid && l == 0) store16(out + len, tag, tag_aligned);
        return;
    }
    // open: compare before releasing (aesgcm.py:148-149, constanttime.py:209-218)
    uint32_t diff = 0;
    if (valid && l == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status) b.status[i] = diff == 0;
    }
    diff = (uint32_t)__shfl((int)diff, (int)(threadIdx.x & 56u), 64);
    if (valid && diff) {   // a rejected record's plaintext is zeroed: each lane its own blocks
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t blk = rho; blk < nfull; blk += 8) store16(out + 16u * blk, z, aligned);
        if (tail && (nfull & 7u) == rho) store_partial(out + 16u * nfull, z, tail);
    }
}

template <int NR, bool OPEN>
int launch_bs8(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_bs8_kernel<NR, OPEN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBs8Lds) != hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t groups = (b.n + kBs8Recs - 1) / kBs8Recs;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_bs8_kernel<NR, OPEN>), dim3((unsigned)groups), dim3(kBs8Threads), kBs8Lds, s,
                       key, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

}  // namespace
}  // namespace tg

int tg_launch_gcm_bs8(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                      hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch_bs8<10, true>(key, b, s, order) : tg::launch_bs8<10, false>(key, b, s, order);
    if (rounds == 14)
        return open ? tg::launch_bs8<14, true>(key, b, s, order) : tg::launch_bs8<14, false>(key, b, s, order);
    return TG_EINVAL;
}
