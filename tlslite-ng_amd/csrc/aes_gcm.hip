// aes_gcm.hip -- batched AES-GCM seal/open for gfx950 (CDNA4).
//
// Restates AESGCM.seal/open (tlslite/utils/aesgcm.py:101-154) with the CTR
// keystream of Python_AES_CTR (python_aes.py:101-116) and the Rijndael round
// (rijndael.py:995-1038), one TLS record per lane:
//
//   * the AES round is a T-table round; Te0 (1 KiB) is replicated 32x in LDS
//     so lane l always reads bank l%32 (ds_read_b32 is conflict-free);
//     Te1..Te3 are byte rotations of Te0 (v_alignbit), the final round's
//     S-box byte is Te0[x] >> 8.
//   * GHASH multiplies by H with sixteen 8-bit tables M_j[b] = b*x^(8j)*H
//     (64 KiB, staged into LDS once per workgroup): X*H = XOR_j M_j[X_j],
//     i.e. 16 ds_read_b128 per block, no shifts and no reduction steps.
//   * round keys are wave-uniform (single key per launch) and live in SGPRs.
//
// Counter blocks are nonce || be32(2 + j); the reference's 128-bit
// increment equals this 32-bit one because a record has < 2^28 blocks.
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

constexpr int kGcmThreads = 1024;
constexpr int kTeWords = 256 * 32;                       // replicated Te0
constexpr size_t kGcmLds = kTeWords * 4 + kGhashEntries * 16;  // 96 KiB

__device__ __forceinline__ uint32_t TE(const uint32_t* tl, uint32_t x) { return tl[x << 5]; }

template <int NR>
__device__ __forceinline__ uint4 aes_enc(const uint32_t* tl, const uint32_t (&rk)[4 * (NR + 1)],
                                         uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3) {
    uint32_t s0 = i0 ^ rk[0], s1 = i1 ^ rk[1], s2 = i2 ^ rk[2], s3 = i3 ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        uint32_t t0 = TE(tl, s0 & 0xff) ^ rotl32(TE(tl, (s1 >> 8) & 0xff), 8) ^
                      rotl32(TE(tl, (s2 >> 16) & 0xff), 16) ^ rotl32(TE(tl, s3 >> 24), 24) ^ rk[4 * r];
        uint32_t t1 = TE(tl, s1 & 0xff) ^ rotl32(TE(tl, (s2 >> 8) & 0xff), 8) ^
                      rotl32(TE(tl, (s3 >> 16) & 0xff), 16) ^ rotl32(TE(tl, s0 >> 24), 24) ^
                      rk[4 * r + 1];
        uint32_t t2 = TE(tl, s2 & 0xff) ^ rotl32(TE(tl, (s3 >> 8) & 0xff), 8) ^
                      rotl32(TE(tl, (s0 >> 16) & 0xff), 16) ^ rotl32(TE(tl, s1 >> 24), 24) ^
                      rk[4 * r + 2];
        uint32_t t3 = TE(tl, s3 & 0xff) ^ rotl32(TE(tl, (s0 >> 8) & 0xff), 8) ^
                      rotl32(TE(tl, (s1 >> 16) & 0xff), 16) ^ rotl32(TE(tl, s2 >> 24), 24) ^
                      rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // final round: SubBytes + ShiftRows + AddRoundKey; S(x) = byte 1 of Te0[x]
#define SB(x) ((TE(tl, (x)) >> 8) & 0xff)
    uint32_t o0 = SB(s0 & 0xff) | (SB((s1 >> 8) & 0xff) << 8) | (SB((s2 >> 16) & 0xff) << 16) |
                  (SB(s3 >> 24) << 24);
    uint32_t o1 = SB(s1 & 0xff) | (SB((s2 >> 8) & 0xff) << 8) | (SB((s3 >> 16) & 0xff) << 16) |
                  (SB(s0 >> 24) << 24);
    uint32_t o2 = SB(s2 & 0xff) | (SB((s3 >> 8) & 0xff) << 8) | (SB((s0 >> 16) & 0xff) << 16) |
                  (SB(s1 >> 24) << 24);
    uint32_t o3 = SB(s3 & 0xff) | (SB((s0 >> 8) & 0xff) << 8) | (SB((s1 >> 16) & 0xff) << 16) |
                  (SB(s2 >> 24) << 24);
#undef SB
    return make_uint4(o0 ^ rk[4 * NR], o1 ^ rk[4 * NR + 1], o2 ^ rk[4 * NR + 2], o3 ^ rk[4 * NR + 3]);
}

// y * H with the sixteen 8-bit tables (byte j of the block = byte j%4 of word j/4).
__device__ __forceinline__ uint4 gmul(const uint4* gt, uint4 y) {
    uint4 z = gt[y.x & 0xff];
    z = xor4(z, gt[256 + ((y.x >> 8) & 0xff)]);
    z = xor4(z, gt[512 + ((y.x >> 16) & 0xff)]);
    z = xor4(z, gt[768 + (y.x >> 24)]);
    z = xor4(z, gt[1024 + (y.y & 0xff)]);
    z = xor4(z, gt[1280 + ((y.y >> 8) & 0xff)]);
    z = xor4(z, gt[1536 + ((y.y >> 16) & 0xff)]);
    z = xor4(z, gt[1792 + (y.y >> 24)]);
    z = xor4(z, gt[2048 + (y.z & 0xff)]);
    z = xor4(z, gt[2304 + ((y.z >> 8) & 0xff)]);
    z = xor4(z, gt[2560 + ((y.z >> 16) & 0xff)]);
    z = xor4(z, gt[2816 + (y.z >> 24)]);
    z = xor4(z, gt[3072 + (y.w & 0xff)]);
    z = xor4(z, gt[3328 + ((y.w >> 8) & 0xff)]);
    z = xor4(z, gt[3584 + ((y.w >> 16) & 0xff)]);
    z = xor4(z, gt[3840 + (y.w >> 24)]);
    return z;
}

template <int NR, bool OPEN>
__global__ __launch_bounds__(kGcmThreads) void gcm_kernel(const GcmKeyDev* __restrict__ key,
                                                          tg_batch b) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* te = lds;
    uint4* gt = reinterpret_cast<uint4*>(lds + kTeWords);
    for (int e = threadIdx.x; e < kTeWords; e += blockDim.x) te[e] = c_te.te0[e >> 5];
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x) gt[e] = key->ghash[e];
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk[k] = key->rk[k];
    __syncthreads();

    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const uint32_t* tl = te + (threadIdx.x & 31);

    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;

    // J0 = nonce || be32(1): the tag mask (aesgcm.py:112-115)
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const uint32_t n0 = nv.x, n1 = nv.y, n2 = nv.z;
    const uint4 mask = aes_enc<NR>(tl, rk, n0, n1, n2, bswap32(1u));

    // GHASH over the AAD, zero-padded (aesgcm.py:69-79)
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < alen; off += 16) {
        uint32_t m = alen - off < 16 ? alen - off : 16;
        y = gmul(gt, xor4(y, load_partial(ad + off, m)));
    }

    // CTR from nonce || be32(2) (aesgcm.py:118-120) with GHASH over the ciphertext
    const uint32_t nfull = len >> 4;
    const uint32_t tail = len & 15;
    uint32_t j = 0;
    for (; j + 4 <= nfull; j += 4) {
        uint4 ks[4], d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ks[q] = aes_enc<NR>(tl, rk, n0, n1, n2, bswap32(2u + j + q));
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = load16(in + 16 * (j + q), aligned);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint4 c = xor4(d[q], ks[q]);
            store16(out + 16 * (j + q), c, aligned);
            y = gmul(gt, xor4(y, OPEN ? d[q] : c));
        }
    }
    for (; j < nfull; ++j) {
        uint4 ks = aes_enc<NR>(tl, rk, n0, n1, n2, bswap32(2u + j));
        uint4 d = load16(in + 16 * j, aligned);
        uint4 c = xor4(d, ks);
        store16(out + 16 * j, c, aligned);
        y = gmul(gt, xor4(y, OPEN ? d : c));
    }
    if (tail) {
        uint4 ks = aes_enc<NR>(tl, rk, n0, n1, n2, bswap32(2u + nfull));
        uint4 d = load_partial(in + 16 * nfull, tail);
        uint4 c = mask_tail(xor4(d, ks), tail);
        store_partial(out + 16 * nfull, c, tail);
        y = gmul(gt, xor4(y, OPEN ? d : c));
    }

    // length block: be64(8*alen) || be64(8*len) (aesgcm.py:64)
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
    y = gmul(gt, xor4(y, make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                                    bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits))));
    const uint4 tag = xor4(y, mask);
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

template <int NR, bool OPEN>
int launch(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_kernel<NR, OPEN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGcmLds) !=
            hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + kGcmThreads - 1) / kGcmThreads;
    hipLaunchKernelGGL((gcm_kernel<NR, OPEN>), dim3((unsigned)blocks), dim3(kGcmThreads), kGcmLds,
                       s, key, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

}  // namespace
}  // namespace tg

int tg_launch_gcm(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                  hipStream_t s) {
    if (rounds == 10) return open ? tg::launch<10, true>(key, b, s) : tg::launch<10, false>(key, b, s);
    if (rounds == 14) return open ? tg::launch<14, true>(key, b, s) : tg::launch<14, false>(key, b, s);
    return TG_EINVAL;
}
