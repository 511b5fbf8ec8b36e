// aes_gcm.hip -- batched AES-GCM seal/open for gfx950 (CDNA4).
//
// Restates AESGCM.seal/open (tlslite/utils/aesgcm.py:101-154) with the CTR
// keystream of Python_AES_CTR (python_aes.py:101-116) and the Rijndael round
// (rijndael.py:995-1038), one TLS record per lane:
//
//   * the AES round is a T-table round; Te0 (1 KiB) is replicated 64x in LDS
//     so lane l always reads its own bank (ds_read_b32 is conflict-free) and
//     each lookup address is one v_perm_b32; Te1..Te3 are byte rotations of
//     Te0 (v_alignbit), the final round's S-box byte is byte 1 of Te0[x].
//   * GHASH multiplies by H with sixteen 8-bit tables M_j[b] = b*x^(8j)*H
//     (64 KiB, staged into LDS once per workgroup): X*H = XOR_j M_j[X_j],
//     i.e. 16 ds_read_b128 per block, no shifts and no reduction steps.
//   * round keys are wave-uniform (single key per launch) and live in SGPRs.
//
// Counter blocks are nonce || be32(2 + j); the reference's 128-bit
// increment equals this 32-bit one because a record has < 2^28 blocks.
#include <cstdlib>

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
// LDS map (one workgroup per CU):
//   [0, 64 KiB)        GHASH tables M_j[b] (16 x 256 x 16 B)
//   [64 KiB, 128 KiB)  Te0, one copy per lane: entry x for lane l at
//                      64 KiB + x * 256 + l * 4, so every lane reads its own
//                      bank (ds_read_b32 conflict-free) and the byte address
//                      is assembled by ONE v_perm_b32 from the state word.
constexpr uint32_t kTeBase = 65536;
constexpr size_t kGcmLds = 2 * 65536;

extern __shared__ __attribute__((aligned(16))) uint4 g_lds[];

// The kernel declares no static LDS, so the dynamic block starts at LDS
// address 0 and table addresses are absolute: the perm/shift result is the
// ds_read address itself (constant parts go in the instruction's offset).
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(3))) uint32_t* lds_u32_ptr;
typedef const __attribute__((address_space(3))) uint4* lds_u128_ptr;
__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) { return *(lds_u32_ptr)(uintptr_t)addr; }
__device__ __forceinline__ uint4 lds_u128(uint32_t addr) { return *(lds_u128_ptr)(uintptr_t)addr; }
#else
__device__ __forceinline__ uint32_t lds_u32(uint32_t) { return 0; }
__device__ __forceinline__ uint4 lds_u128(uint32_t) { return uint4(); }
#endif

// Te0[byte K of x] for this lane; lane4 = {lane * 4, 0, 1, 0} (bytes 0..3).
template <int K>
__device__ __forceinline__ uint32_t TE(uint32_t x, uint32_t lane4) {
    return lds_u32(__builtin_amdgcn_perm(x, lane4, 0x0c020000u | ((4u + K) << 8)));
}

template <int NR>
__device__ __forceinline__ uint4 aes_enc(uint32_t lane4, const uint32_t (&rk)[4 * (NR + 1)],
                                         uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3) {
    uint32_t s0 = i0 ^ rk[0], s1 = i1 ^ rk[1], s2 = i2 ^ rk[2], s3 = i3 ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        uint32_t t0 = TE<0>(s0, lane4) ^ rotl32(TE<1>(s1, lane4), 8) ^
                      rotl32(TE<2>(s2, lane4), 16) ^ rotl32(TE<3>(s3, lane4), 24) ^ rk[4 * r];
        uint32_t t1 = TE<0>(s1, lane4) ^ rotl32(TE<1>(s2, lane4), 8) ^
                      rotl32(TE<2>(s3, lane4), 16) ^ rotl32(TE<3>(s0, lane4), 24) ^ rk[4 * r + 1];
        uint32_t t2 = TE<0>(s2, lane4) ^ rotl32(TE<1>(s3, lane4), 8) ^
                      rotl32(TE<2>(s0, lane4), 16) ^ rotl32(TE<3>(s1, lane4), 24) ^ rk[4 * r + 2];
        uint32_t t3 = TE<0>(s3, lane4) ^ rotl32(TE<1>(s0, lane4), 8) ^
                      rotl32(TE<2>(s1, lane4), 16) ^ rotl32(TE<3>(s2, lane4), 24) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // final round: SubBytes + ShiftRows + AddRoundKey; S(x) is byte 1 of Te0[x],
    // gathered from four lookups with two v_perm_b32 and an OR.
#define SBW(a, b, c, d)                                                                  \
    (__builtin_amdgcn_perm(TE<1>(b, lane4), TE<0>(a, lane4), 0x0c0c0501u) |                \
     __builtin_amdgcn_perm(TE<3>(d, lane4), TE<2>(c, lane4), 0x05010c0cu))
    const uint32_t o0 = SBW(s0, s1, s2, s3), o1 = SBW(s1, s2, s3, s0);
    const uint32_t o2 = SBW(s2, s3, s0, s1), o3 = SBW(s3, s0, s1, s2);
#undef SBW
    return make_uint4(o0 ^ rk[4 * NR], o1 ^ rk[4 * NR + 1], o2 ^ rk[4 * NR + 2], o3 ^ rk[4 * NR + 3]);
}

// y * H with the sixteen 8-bit tables (byte j of the block = byte j%4 of word
// j/4): entry (j, b) at LDS byte j * 4096 + b * 16.
__device__ __forceinline__ uint4 gmul(uint4 y) {
    const uint32_t w[4] = {y.x, y.y, y.z, y.w};
    uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t v = w[j >> 2];
        const int sh = 8 * (j & 3) - 4;
        const uint32_t off = (sh < 0 ? (v << 4) : (v >> sh)) & 0xff0u;
        z = xor4(z, lds_u128(off + 4096u * j));
    }
    return z;
}

// Blocks [0, G*ngroups) of a record in groups of G (16*G bytes), the next
// group's payload loaded one iteration ahead.
template <int NR, bool OPEN, bool ALIGNED, int G>
__device__ __forceinline__ uint4 ctr_groups(uint32_t lane4, const uint32_t (&rk)[4 * (NR + 1)],
                                            uint4 nv, const uint8_t* in, uint8_t* out,
                                            uint32_t ngroups, uint4 y) {
    if (ngroups == 0) return y;
    uint4 d[G];
#pragma unroll
    for (int q = 0; q < G; ++q) d[q] = load16(in + 16 * q, ALIGNED);
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint32_t gn = g + 1 < ngroups ? g + 1 : g;
        uint4 nx[G];
#pragma unroll
        for (int q = 0; q < G; ++q) nx[q] = load16(in + 16 * (G * gn + q), ALIGNED);
        uint4 ks[G];
#pragma unroll
        for (int q = 0; q < G; ++q)
            ks[q] = aes_enc<NR>(lane4, rk, nv.x, nv.y, nv.z, bswap32(2u + G * g + q));
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const uint4 c = xor4(d[q], ks[q]);
            store16(out + 16 * (G * g + q), c, ALIGNED);
            y = gmul(xor4(y, OPEN ? d[q] : c));
        }
#pragma unroll
        for (int q = 0; q < G; ++q) d[q] = nx[q];
    }
    return y;
}

template <int NR, bool OPEN, int G, int THREADS>
__global__ __launch_bounds__(THREADS) void gcm_kernel(const GcmKeyDev* __restrict__ key,
                                                      tg_batch b) {
    uint4* lds = g_lds;
    // stage the GHASH tables and the per-lane Te0 copies
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x) lds[e] = key->ghash[e];
    {
        uint32_t* te = reinterpret_cast<uint32_t*>(lds) + kTeBase / 4;
        for (int e = threadIdx.x; e < 256 * 64; e += blockDim.x) te[e] = c_te.te0[e >> 6];
    }
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk[k] = key->rk[k];
    __syncthreads();

    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const uint32_t lane4 = ((threadIdx.x & 63u) << 2) | 0x00010000u;

    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;

    // J0 = nonce || be32(1): the tag mask (aesgcm.py:112-115)
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const uint4 mask = aes_enc<NR>(lane4, rk, nv.x, nv.y, nv.z, bswap32(1u));

    // GHASH over the AAD, zero-padded (aesgcm.py:69-79)
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < alen; off += 16) {
        uint32_t m = alen - off < 16 ? alen - off : 16;
        y = gmul(xor4(y, load_partial(ad + off, m)));
    }

    // CTR from nonce || be32(2) (aesgcm.py:118-120), GHASH over the ciphertext
    const uint32_t nfull = len >> 4;
    const uint32_t tail = len & 15;
    const uint32_t ngroups = nfull / G;
    y = aligned ? ctr_groups<NR, OPEN, true, G>(lane4, rk, nv, in, out, ngroups, y)
                : ctr_groups<NR, OPEN, false, G>(lane4, rk, nv, in, out, ngroups, y);
    for (uint32_t j = G * ngroups; j < nfull; ++j) {
        const uint4 ks = aes_enc<NR>(lane4, rk, nv.x, nv.y, nv.z, bswap32(2u + j));
        const uint4 d = load16(in + 16 * j, aligned);
        const uint4 c = xor4(d, ks);
        store16(out + 16 * j, c, aligned);
        y = gmul(xor4(y, OPEN ? d : c));
    }
    if (tail) {
        const uint4 ks = aes_enc<NR>(lane4, rk, nv.x, nv.y, nv.z, bswap32(2u + nfull));
        const uint4 d = load_partial(in + 16 * nfull, tail);
        const uint4 c = mask_tail(xor4(d, ks), tail);
        store_partial(out + 16 * nfull, c, tail);
        y = gmul(xor4(y, OPEN ? d : c));
    }

    // length block: be64(8*alen) || be64(8*len) (aesgcm.py:64)
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
    y = gmul(xor4(y, make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
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

template <int NR, bool OPEN, int G, int THREADS>
int launch_v(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_kernel<NR, OPEN, G, THREADS>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGcmLds) !=
            hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + THREADS - 1) / THREADS;
    hipLaunchKernelGGL((gcm_kernel<NR, OPEN, G, THREADS>), dim3((unsigned)blocks), dim3(THREADS),
                       kGcmLds, s, key, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Tuning variants (TLSGPU_GCM_VARIANT, for measurement only): blocks per
// iteration x threads per workgroup.
int variant() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("TLSGPU_GCM_VARIANT");
        v = e ? atoi(e) : 0;
    }
    return v;
}

template <int NR, bool OPEN>
int launch(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    switch (variant()) {
        case 1: return launch_v<NR, OPEN, 4, 1024>(key, b, s);
        case 2: return launch_v<NR, OPEN, 4, 512>(key, b, s);
        case 3: return launch_v<NR, OPEN, 2, 512>(key, b, s);
        default: return launch_v<NR, OPEN, 2, 1024>(key, b, s);
    }
}

}  // namespace
}  // namespace tg

int tg_launch_gcm(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                  hipStream_t s) {
    if (rounds == 10) return open ? tg::launch<10, true>(key, b, s) : tg::launch<10, false>(key, b, s);
    if (rounds == 14) return open ? tg::launch<14, true>(key, b, s) : tg::launch<14, false>(key, b, s);
    return TG_EINVAL;
}
