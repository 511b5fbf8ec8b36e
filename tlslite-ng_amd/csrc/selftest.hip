// selftest.hip -- test-only entry points that run the engine's device
// Poly1305 and GHASH arithmetic on raw messages, so the reference's own
// known answers (RFC 7539 A.3 #1-11, unit_tests/test_tlslite_utils_poly1305.py
// :52-210; GHASH values of the reference's AESGCM._auth, aesgcm.py:60-99) can
// be checked against the exact device code the AEAD kernels use.  Not on the
// record path.
//
// Poly1305 modes (poly1305.h):
//   0  lane Horner in radix 2^32 (Poly32), as chacha_kernel (one message per lane);
//   1  wave-striped Horner with the r^(4S-4) gaps, the lift and the shuffle
//      sum of chacha_wave_kernel, W = 1 (S = 64 threads per message);
//   2  the same with W = 4;  3  W = 16;
//   4  the octet striping of chacha_octet_kernel: eight lanes per message,
//      lane l the 64-byte chunks l, l + 8, ..., r within a chunk and r^29
//      across the other lanes' chunks, the lift and the octet sum.
// GHASH modes (ghash.h):
//   0  Horner with gmul (8-bit tables, j * 4096 + b * 16: the T-table lane
//      kernel and the wave kernel);  1  gmul_lowreg;
//   2  gmul_rot (row layout + lane rotation: the octet kernels and seal);
//   3  gf128_mul, table-free (the key-table kernels);
//   4  the octet structure of aes_gcm_bs8.hip: eight lanes, front padding to
//      a multiple of 8 blocks, stride H^8 (gmul_rot tables of H^8), lift by
//      H^(8 - l) (gf128_mul), XOR over the octet;
//   5  the wave structure of gcm_wave_kernel (W = 1): front padding to a
//      multiple of 64, stride H^64 (gmul tables of H^64), lift by H^(64 - l);
//   6  the octet structure of the key-table octet kernel (gcm_kt_kernel):
//      stride H^8 through the wave's 4-bit tables (build_table4 / gmul4).
#include <hip/hip_runtime.h>

#include <cstring>

#include "aes_round.h"
#include "ghash.h"
#include "poly1305.h"

namespace tg {
namespace {

extern __shared__ __attribute__((aligned(16))) uint4 g_lds_st[];

// 16-byte block k of a message of n bytes; RFC padding for Poly1305 (the
// short last block gets 0x01 after its bytes, hib = 0), zero padding for GHASH.
__device__ __forceinline__ uint4 msg_block(const uint8_t* m, uint32_t n, uint32_t k, bool poly,
                                           uint32_t& hib) {
    const uint32_t rem = n - 16 * k;
    if (rem >= 16) {
        hib = 1u << 24;
        return load_partial(m + 16 * k, 16);
    }
    uint4 v = load_partial(m + 16 * k, rem);
    hib = 0;
    if (poly) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            if (rem >> 2 == q) w[q] |= 1u << (8 * (rem & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return v;
}

// ---- Poly1305 -------------------------------------------------------------
__global__ void poly_lane_kernel(const uint8_t* keys, const uint8_t* msgs, const uint64_t* off,
                                 const uint32_t* len, uint64_t n, uint8_t* tags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t otk[16] = {0};
    const uint4 k0 = load_partial(keys + 32 * i, 16), k1 = load_partial(keys + 32 * i + 16, 16);
    otk[0] = k0.x; otk[1] = k0.y; otk[2] = k0.z; otk[3] = k0.w;
    otk[4] = k1.x; otk[5] = k1.y; otk[6] = k1.z; otk[7] = k1.w;
    Poly32 p;   // as chacha_kernel
    poly_init(p, otk);
    const uint8_t* m = msgs + off[i];
    const uint32_t nb = (len[i] + 15) >> 4;
    for (uint32_t k = 0; k < nb; ++k) {
        uint32_t hib;
        const uint4 blk = msg_block(m, len[i], k, true, hib);
        poly_block(p, blk, hib ? 1u : 0u);   // radix 2^32: the 2^128 bit is 1 in h4
    }
    store_partial(tags + 16 * i, poly_finish(p), 16);
}

// One message per workgroup of S = 64 W threads.
template <int W>
__global__ __launch_bounds__(64 * W) void poly_wave_kernel(const uint8_t* keys, const uint8_t* msgs,
                                                           const uint64_t* off, const uint32_t* len,
                                                           uint8_t* tags) {
    constexpr uint32_t S = 64u * W;
    __shared__ F5 s_part[W];
    const uint64_t i = blockIdx.x;
    const uint32_t seg = threadIdx.x;
    uint32_t otk[16] = {0};
    const uint4 k0 = load_partial(keys + 32 * i, 16), k1 = load_partial(keys + 32 * i + 16, 16);
    otk[0] = k0.x; otk[1] = k0.y; otk[2] = k0.z; otk[3] = k0.w;
    otk[4] = k1.x; otk[5] = k1.y; otk[6] = k1.z; otk[7] = k1.w;
    Poly p;
    poly_init(p, otk);
    const F5 r = {p.r0, p.r1, p.r2, p.r3, p.r4};
    const uint8_t* m = msgs + off[i];
    const uint32_t n = len[i], nb = (n + 15) >> 4, nq = (nb + 3) >> 2;
    F5 rgap = {0, 0, 0, 0, 0};
    uint32_t cb = 0;
    for (uint32_t q = seg; q < nq; q += S) {   // as chacha_wave_kernel, chunks of 4 blocks
        stripe_gap<S>(p, r, q, seg, rgap);
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            const uint32_t c = 4 * q + sb;
            if (c < nb) {
                uint32_t hib;
                const uint4 blk = msg_block(m, n, c, true, hib);
                poly_block(p, blk, hib);
            }
        }
        cb = 4 * q + 4 < nb ? 4 * q + 4 : nb;
    }
    F5 z = stripe_lift(p, r, cb, nb - cb);      // no length block behind a raw message
    z = stripe_sum<W>(z, s_part, seg, 0);
    p.h0 = z.h0; p.h1 = z.h1; p.h2 = z.h2; p.h3 = z.h3; p.h4 = z.h4;
    const uint4 tag = poly_finish(p);
    if (seg == 0) store_partial(tags + 16 * i, tag, 16);
}

// Eight messages per 64-thread workgroup, one octet each (mode 4).
__global__ __launch_bounds__(64) void poly_octet_kernel(const uint8_t* keys, const uint8_t* msgs,
                                                        const uint64_t* off, const uint32_t* len, uint64_t n,
                                                        uint8_t* tags) {
    const uint32_t l = threadIdx.x & 7u;
    const uint64_t i = (uint64_t)blockIdx.x * 8 + (threadIdx.x >> 3);
    const bool valid = i < n;
    uint32_t otk[16] = {0};
    const uint64_t ik = valid ? i : 0;
    const uint4 k0 = load_partial(keys + 32 * ik, 16), k1 = load_partial(keys + 32 * ik + 16, 16);
    otk[0] = k0.x; otk[1] = k0.y; otk[2] = k0.z; otk[3] = k0.w;
    otk[4] = k1.x; otk[5] = k1.y; otk[6] = k1.z; otk[7] = k1.w;
    Poly p;
    poly_init(p, otk);
    OctetPoly o;   // as chacha_otk_kernel
    octet_powers(F5{p.r0, p.r1, p.r2, p.r3, p.r4}, o);
    const Mul26 R = mul26(f5_at(o.r)), R29 = mul26(f5_at(o.r29));
    const uint8_t* m = msgs + (valid ? off[i] : 0);
    const uint32_t nbytes = valid ? len[i] : 0, nb = (nbytes + 15) >> 4, nch = (nb + 3) >> 2;
    F5 h = {0, 0, 0, 0, 0};
    for (uint32_t c = l; c < nch; c += 8) {   // the lane's chunks, as chacha_octet_kernel's blocks
        const bool last = c + 8 >= nch;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t k = 4 * c + q;
            if (k >= nb) break;
            uint32_t hib;
            const uint4 blk = msg_block(m, nbytes, k, true, hib);
            fblock(h, blk, (q == 3 && !last) ? R29 : R, hib);
        }
    }
    const uint32_t mlast = nch ? nb - 4u * (nch - 1u) : 0u;
    h = octet_lift(h, octet_lift_exp(l, nch, mlast), o.r, o.r2, o.r4, o.r8, o.r16);
    h = octet_sum(h);
    const uint4 tag = octet_finish(h, (const uint32_t[4]){p.p0, p.p1, p.p2, p.p3});
    if (valid && l == 0) store_partial(tags + 16 * i, tag, 16);
}

// ---- GHASH ----------------------------------------------------------------
constexpr uint32_t kStJt = 65536;   // gmul_rot lane-offset rows after the tables

__device__ __forceinline__ uint4 len_block(uint32_t alen, uint32_t clen) {
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)clen << 3;
    return make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                      bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits));
}

// GHASH input block t of aad || pad || ct || pad || len (M blocks in all).
__device__ __forceinline__ uint4 gh_block(const uint8_t* ad, uint32_t alen, const uint8_t* ct,
                                          uint32_t clen, uint32_t t) {
    const uint32_t na = (alen + 15) >> 4, nc = (clen + 15) >> 4;
    uint32_t hib;
    if (t < na) return msg_block(ad, alen, t, false, hib);
    if (t < na + nc) return msg_block(ct, clen, t - na, false, hib);
    return len_block(alen, clen);
}

// One item per 256-thread workgroup: stage the tables of G = H^e (e = 1, 8 or
// 64 by mode) in LDS, then wave 0 (lane 0, or the octet, or the whole wave)
// computes the GHASH the way its kernel does.
template <int MODE>
__global__ __launch_bounds__(256) void ghash_kernel(const uint8_t* hs, const uint8_t* aad,
                                                    const uint64_t* aad_off, const uint32_t* aad_len,
                                                    const uint8_t* cts, const uint64_t* ct_off,
                                                    const uint32_t* ct_len, uint8_t* out) {
    const uint64_t i = blockIdx.x;
    const uint4 hw = load_partial(hs + 16 * i, 16);
    const uint4 hn = make_uint4(gcm_word_to_norm(hw.x), gcm_word_to_norm(hw.y), gcm_word_to_norm(hw.z),
                                gcm_word_to_norm(hw.w));
    constexpr uint32_t E = (MODE == 4 || MODE == 6) ? 8 : MODE == 5 ? 64 : 1;
    const uint4 gn = E == 1 ? hn : gf128_pow(hn, E);           // G = H^E, normal order
    if (MODE == 6) {
        if (threadIdx.x < 64) build_table4(0, gn);
    } else if (MODE != 3) {
        const uint32_t gv[4] = {gcm_word_to_norm(gn.x), gcm_word_to_norm(gn.y), gcm_word_to_norm(gn.z),
                                gcm_word_to_norm(gn.w)};
        const bool rot = MODE == 2 || MODE == 4;
        for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x)
            g_lds_st[rot ? (e & 255) * 16 + (e >> 8) : e] = ghash_table_entry(gv, e);
        if (rot && threadIdx.x < 16) {
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[q] = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) w[q] |= (((threadIdx.x + 4 * q + k) & 15u) << 4) << (8 * k);
            }
            g_lds_st[kStJt / 16 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    const uint8_t* ad = aad + aad_off[i];
    const uint8_t* ct = cts + ct_off[i];
    const uint32_t alen = aad_len[i], clen = ct_len[i];
    const uint32_t M = ((alen + 15) >> 4) + ((clen + 15) >> 4) + 1;
    if (MODE <= 3) {   // one lane, plain Horner y <- (y ^ X) G (aesgcm.py:60-79)
        if (lane) return;
        uint4 y = make_uint4(0, 0, 0, 0);
        for (uint32_t t = 0; t < M; ++t) {
            const uint4 x = gh_block(ad, alen, ct, clen, t);
            if (MODE == 0) y = gmul(xor4(y, x));
            else if (MODE == 1) y = gmul_lowreg(xor4(y, x));
            else if (MODE == 2) y = gmul_rot(xor4(y, x), lane & 15u, kStJt);
            else y = gf128_mul(xor4(y, norm4(x)), hn);
        }
        if (MODE == 3) y = norm4(y);
        store_partial(out + 16 * i, y, 16);
        return;
    }
    // striped: S lanes, front padding to P = S ceil(M / S); lane l owns the
    // positions l, l + S, ... ; y <- y G ^ X (G = H^S), lifted by H^(S - l)
    constexpr uint32_t S = (MODE == 4 || MODE == 6) ? 8 : 64;
    if (lane >= S) return;
    const uint32_t P = S * ((M + S - 1) / S), pad = P - M;
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t t = lane; t < P; t += S) {
        if (t < pad) continue;   // leading zero blocks: y stays 0
        const uint4 x = gh_block(ad, alen, ct, clen, t - pad);
        y = xor4(MODE == 4 ? gmul_rot(y, lane & 15u, kStJt) : MODE == 6 ? gmul4(y, 0) : gmul(y), x);
    }
    uint4 yn = norm4(y);
    if (yn.x | yn.y | yn.z | yn.w) yn = gf128_mul(yn, gf128_pow(hn, S - lane));
#pragma unroll
    for (uint32_t m = 1; m < S; m <<= 1) yn = xor4(yn, shfl_xor4(yn, (int)m));
    if (lane == 0) store_partial(out + 16 * i, norm4(yn), 16);
}

}  // namespace
}  // namespace tg

namespace {

// Device copies of the host arrays, freed on scope exit.
struct DevBufs {
    void* p[8] = {nullptr};
    int k = 0;
    ~DevBufs() {
        for (int i = 0; i < k; ++i)
            if (p[i]) (void)hipFree(p[i]);
    }
    template <class T>
    T* up(const T* h, size_t bytes) {
        void* d = nullptr;
        if (hipMalloc(&d, bytes ? bytes : 16) != hipSuccess) return nullptr;
        p[k++] = d;
        if (bytes && hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return static_cast<T*>(d);
    }
};

size_t span(const uint64_t* off, const uint32_t* len, uint64_t n) {
    size_t m = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (off[i] + len[i] > m) m = off[i] + len[i];
    return m;
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int tg_selftest_poly1305(
    int mode, const uint8_t* keys, const uint8_t* msgs, const uint64_t* off, const uint32_t* len,
    uint64_t n, uint8_t* tags) {
    if (!keys || !off || !len || !tags || mode < 0 || mode > 4 || n == 0 || n > (1u << 20))
        return TG_EINVAL;
    DevBufs d;
    const size_t ms = span(off, len, n);
    uint8_t* dk = d.up(keys, 32 * n);
    uint8_t* dm = d.up(msgs, ms);
    uint64_t* doff = d.up(off, 8 * n);
    uint32_t* dlen = d.up(len, 4 * n);
    uint8_t* dt = d.up(tags, 16 * n);
    if (!dk || !dm || !doff || !dlen || !dt) return TG_EHIP;
    if (mode == 0)
        hipLaunchKernelGGL(tg::poly_lane_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, dk, dm, doff,
                           dlen, n, dt);
    else if (mode == 1)
        hipLaunchKernelGGL(tg::poly_wave_kernel<1>, dim3((unsigned)n), dim3(64), 0, 0, dk, dm, doff, dlen, dt);
    else if (mode == 2)
        hipLaunchKernelGGL(tg::poly_wave_kernel<4>, dim3((unsigned)n), dim3(256), 0, 0, dk, dm, doff, dlen, dt);
    else if (mode == 3)
        hipLaunchKernelGGL(tg::poly_wave_kernel<16>, dim3((unsigned)n), dim3(1024), 0, 0, dk, dm, doff, dlen, dt);
    else
        hipLaunchKernelGGL(tg::poly_octet_kernel, dim3((unsigned)((n + 7) / 8)), dim3(64), 0, 0, dk, dm, doff, dlen,
                           n, dt);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TG_EHIP;
    return hipMemcpy(tags, dt, 16 * n, hipMemcpyDeviceToHost) == hipSuccess ? TG_OK : TG_EHIP;
}

extern "C" __attribute__((visibility("default"))) int tg_selftest_ghash(
    int mode, const uint8_t* h, const uint8_t* aad, const uint64_t* aad_off, const uint32_t* aad_len,
    const uint8_t* ct, const uint64_t* ct_off, const uint32_t* ct_len, uint64_t n, uint8_t* out) {
    if (!h || !aad_off || !aad_len || !ct_off || !ct_len || !out || mode < 0 || mode > 6 || n == 0 ||
        n > (1u << 16))
        return TG_EINVAL;
    DevBufs d;
    uint8_t* dh = d.up(h, 16 * n);
    uint8_t* da = d.up(aad, span(aad_off, aad_len, n));
    uint64_t* dao = d.up(aad_off, 8 * n);
    uint32_t* dal = d.up(aad_len, 4 * n);
    uint8_t* dc = d.up(ct, span(ct_off, ct_len, n));
    uint64_t* dco = d.up(ct_off, 8 * n);
    uint32_t* dcl = d.up(ct_len, 4 * n);
    uint8_t* dout = d.up(out, 16 * n);
    if (!dh || !da || !dao || !dal || !dc || !dco || !dcl || !dout) return TG_EHIP;
    const size_t lds = 65536 + 256;
#define TG_ST_GHASH(M)                                                                                    \
    do {                                                                                                  \
        if (hipFuncSetAttribute((const void*)tg::ghash_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)lds) != hipSuccess)                                                  \
            return TG_EHIP;                                                                               \
        hipLaunchKernelGGL(tg::ghash_kernel<M>, dim3((unsigned)n), dim3(256), lds, 0, dh, da, dao, dal, dc, \
                           dco, dcl, dout);                                                               \
    } while (0)
    switch (mode) {
        case 0: TG_ST_GHASH(0); break;
        case 1: TG_ST_GHASH(1); break;
        case 2: TG_ST_GHASH(2); break;
        case 3: TG_ST_GHASH(3); break;
        case 4: TG_ST_GHASH(4); break;
        case 5: TG_ST_GHASH(5); break;
        default: TG_ST_GHASH(6); break;
    }
#undef TG_ST_GHASH
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TG_EHIP;
    return hipMemcpy(out, dout, 16 * n, hipMemcpyDeviceToHost) == hipSuccess ? TG_OK : TG_EHIP;
}
