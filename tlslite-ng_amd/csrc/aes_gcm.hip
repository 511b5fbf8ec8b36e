// aes_gcm.hip -- batched AES-GCM seal/open for gfx950 (CDNA4).
//
// Restates AESGCM.seal/open (tlslite/utils/aesgcm.py:101-154) with the CTR
// keystream of Python_AES_CTR (python_aes.py:101-116) and the Rijndael round
// (rijndael.py:995-1038), one TLS record per lane:
//
//   * the AES round is a T-table round over Te0 and Te2 = rotl16(Te0), each
//     replicated 32x in LDS so lane l always reads bank l%32 (ds_read_b32 is
//     conflict-free); a column needs one rotation (v_alignbit) instead of
//     three; each lookup address is one v_perm_b32 or one full-rate bitop3;
//     the final round's S-box byte is byte 1 of Te0[x].
//   * counter mode: round 1 is cached per record (only the counter word
//     changes between blocks), so it costs 4 lookups instead of 16.
//   * GHASH multiplies by H with sixteen 8-bit tables M_j[b] = b*x^(8j)*H
//     (64 KiB, staged into LDS once per workgroup): X*H = XOR_j M_j[X_j],
//     i.e. 16 ds_read_b128 per block, no shifts and no reduction steps;
//     3-input XORs are single full-rate v_bitop3_b32.
//   * round keys are wave-uniform (single key per launch) and live in SGPRs.
//
// Counter blocks are nonce || be32(2 + j); the reference's 128-bit
// increment equals this 32-bit one because a record has < 2^28 blocks.
#include <cstdlib>
#include <type_traits>

#include "aes_bs.h"
#include "aes_round.h"
#include "ghash.h"

namespace tg {
namespace {

// LDS map (one workgroup per CU, no static LDS so the dynamic block is at 0):
//   [0, 64 KiB)        GHASH tables, entry (j, b) = M_j[b] at j * 4096 + b * 16
//   [64 KiB, 128 KiB)  Te0 and Te2 = rotl16(Te0), row x (256 B) =
//                      {Te0[x] x 32 copies, Te2[x] x 32 copies}; lane l reads
//                      copy l % 32, i.e. bank l % 32 (conflict-free ds_read_b32)
//   A round column then needs one rotation instead of three:
//     Te0[a] ^ rotl8(Te0[b]) ^ rotl16(Te0[c]) ^ rotl24(Te0[d])
//       = Te0[a] ^ Te2[c] ^ rotl8(Te0[b] ^ Te2[d]).
constexpr uint32_t kTeBase = 65536;
constexpr size_t kGcmLds = 2 * 65536 + 256;   // + the GhashTablesRotLds offsets

extern __shared__ __attribute__((aligned(16))) uint4 g_lds[];

struct GhashTables {  // single key: the 8-bit tables staged in LDS; y in block byte layout
    __device__ __forceinline__ uint4 update(uint4 y, uint4 blk) const { return gmul(xor4(y, blk)); }
    __device__ __forceinline__ uint4 finish(uint4 y) const { return y; }
};

// Bank-conflict-free variant.  Tables in row layout, entry (j, b) at
// b * 256 + j * 16, so the 16-byte bank slot of a lookup is its table j.  Lane
// l walks the tables starting at j = l % 16: at step t it looks up table
// (t + l) % 16 with byte (t + l) % 16 of y, so the 16 lanes of every
// ds_read_b128 group hit 16 different slots whatever the data.  y is rotated
// by l % 16 bytes once per multiply (word rotation by two selects, byte
// rotation by v_alignbit), after which byte t of the rotated value is static;
// each address is one v_perm_b32 of (rotated word, lane's table-offset bytes).
struct GhashTablesRot {
    uint32_t r2, r1;   // lane & 8, lane & 4: word-rotation steps
    uint32_t s8;       // 8 * (lane & 3): byte rotation in bits
    uint32_t jt[4];    // byte t%4 of jt[t/4] = ((t + lane) % 16) * 16
    __device__ __forceinline__ void init(uint32_t lane) {
        const uint32_t l16 = lane & 15;
        r2 = l16 & 8;
        r1 = l16 & 4;
        s8 = 8 * (l16 & 3);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) v |= (((l16 + 4 * q + k) & 15u) << 4) << (8 * k);
            jt[q] = v;
        }
    }
    __device__ __forceinline__ uint4 mul(uint4 y) const {
        uint32_t u0 = y.x, u1 = y.y, u2 = y.z, u3 = y.w;
        if (r2) { uint32_t t = u0; u0 = u2; u2 = t; t = u1; u1 = u3; u3 = t; }
        if (r1) { uint32_t t = u0; u0 = u1; u1 = u2; u2 = u3; u3 = t; }
        const uint32_t v[4] = {__builtin_amdgcn_alignbit(u1, u0, s8),
                               __builtin_amdgcn_alignbit(u2, u1, s8),
                               __builtin_amdgcn_alignbit(u3, u2, s8),
                               __builtin_amdgcn_alignbit(u0, u3, s8)};
        uint4 e[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            // byte 1 <- v[t/4] byte t%4 (the row b), byte 0 <- jt[t/4] byte t%4
            const uint32_t sel = 0x0c0c0000u | ((4u + (t & 3)) << 8) | (uint32_t)(t & 3);
            e[t] = lds_u128(__builtin_amdgcn_perm(v[t >> 2], jt[t >> 2], sel));
        }
        uint4 z = xor4_3(e[0], e[1], e[2]);
        z = xor4_3(z, e[3], e[4]);
        z = xor4_3(z, e[5], e[6]);
        z = xor4_3(z, e[7], e[8]);
        z = xor4_3(z, e[9], e[10]);
        z = xor4_3(z, e[11], e[12]);
        z = xor4_3(z, e[13], e[14]);
        return xor4(z, e[15]);
    }
    __device__ __forceinline__ uint4 update(uint4 y, uint4 blk) const { return mul(xor4(y, blk)); }
    __device__ __forceinline__ uint4 finish(uint4 y) const { return y; }
};

// GhashTablesRot without persistent per-lane state: the rotation amounts are
// bits of lane4 (the AES lookup register, bits 2..5 = lane % 16) and the four
// table-offset words come from a 16-row LDS table (one conflict-free
// ds_read_b128 per multiply), which frees the 7 VGPRs GhashTablesRot holds.
constexpr uint32_t kJtBase = 2 * 65536;
struct GhashTablesRotLds {
    uint32_t lane4;
    __device__ __forceinline__ uint4 mul(uint4 y) const {
        const uint4 jt = lds_u128(kJtBase + ((lane4 & 0x3cu) << 2));
        uint32_t u0 = y.x, u1 = y.y, u2 = y.z, u3 = y.w;
        if (lane4 & 0x20u) { uint32_t t = u0; u0 = u2; u2 = t; t = u1; u1 = u3; u3 = t; }
        if (lane4 & 0x10u) { uint32_t t = u0; u0 = u1; u1 = u2; u2 = u3; u3 = t; }
        const uint32_t s8 = (lane4 & 0xcu) << 1;
        const uint32_t v[4] = {__builtin_amdgcn_alignbit(u1, u0, s8),
                               __builtin_amdgcn_alignbit(u2, u1, s8),
                               __builtin_amdgcn_alignbit(u3, u2, s8),
                               __builtin_amdgcn_alignbit(u0, u3, s8)};
        const uint32_t j[4] = {jt.x, jt.y, jt.z, jt.w};
        uint4 e[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t sel = 0x0c0c0000u | ((4u + (t & 3)) << 8) | (uint32_t)(t & 3);
            e[t] = lds_u128(__builtin_amdgcn_perm(v[t >> 2], j[t >> 2], sel));
        }
        uint4 z = xor4_3(e[0], e[1], e[2]);
        z = xor4_3(z, e[3], e[4]);
        z = xor4_3(z, e[5], e[6]);
        z = xor4_3(z, e[7], e[8]);
        z = xor4_3(z, e[9], e[10]);
        z = xor4_3(z, e[11], e[12]);
        z = xor4_3(z, e[13], e[14]);
        return xor4(z, e[15]);
    }
    __device__ __forceinline__ uint4 update(uint4 y, uint4 blk) const { return mul(xor4(y, blk)); }
    __device__ __forceinline__ uint4 finish(uint4 y) const { return y; }
};

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
// SPLIT: a scheduling fence between the AES of group g+1 and the GHASH of
// group g, so their register peaks do not add up (the waves' own
// interleaving still overlaps the two).
// WIN: keystream through the lane's 256-counter window cache at LDS ``win``
// (aes_round.h, ctr_keystream).
template <int NR, bool OPEN, bool ALIGNED, int G, int SPLIT, bool WIN, class RK, class GH>
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
        if (SPLIT) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < G; ++q) y = gh.update(y, OPEN ? d[q] : c[q]);
#pragma unroll
        for (int q = 0; q < G; ++q) d[q] = nx[q];
    }
    return y;
}

// One record: AESGCM.seal / AESGCM.open (aesgcm.py:101-154) for lane i.
template <int NR, bool OPEN, int G, class RK, class GH, int SPLIT = 0, bool WIN = false>
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
            ? ctr_groups<NR, OPEN, true, G, SPLIT, WIN>(lane4, rk, gh, cc, win, in, out, ngroups, y)
            : ctr_groups<NR, OPEN, false, G, SPLIT, WIN>(lane4, rk, gh, cc, win, in, out, ngroups, y);
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


// GHASH flavours of the single-key kernel (GH % 10): 0 = GhashTables,
// 1 = GhashTablesRot, 2 = GhashTablesRotLds; GH / 10 = 1 adds the SPLIT fence.
template <int NR, bool OPEN, int G, int THREADS, int GH>
__global__ __launch_bounds__(THREADS) void gcm_kernel(const GcmKeyDev* __restrict__ key,
                                                      tg_batch b, const uint32_t* __restrict__ order) {
    constexpr int GHK = GH % 10, SPLIT = (GH / 10) % 10;   // GHASH flavour, split schedule
    constexpr bool WIN = GH >= 100;                         // 256-counter window cache
    constexpr bool ROT = GHK != 0;
    uint4* lds = g_lds;
    // stage the GHASH tables (ROT: row layout b * 16 + j) and the Te0/Te2 copies
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x)
        lds[ROT ? (e & 255) * 16 + (e >> 8) : e] = key->ghash[e];
    if (GHK == 2 && threadIdx.x < 16) {   // row l: byte k of word q = ((l + 4q + k) % 16) * 16
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) w[q] |= (((threadIdx.x + 4 * q + k) & 15u) << 4) << (8 * k);
        }
        lds[kJtBase / 16 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    stage_te(reinterpret_cast<uint32_t*>(lds) + kTeBase / 4);
    RkRegs<NR> rk;
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = key->rk[k];
    __syncthreads();

    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n) return;
    const uint64_t i = order ? order[t] : t;
    const uint32_t lane4 = ((threadIdx.x & 31u) << 2) | kTeBase;
    const uint32_t win = (uint32_t)kGcmLds + 16u * threadIdx.x;   // this lane's window slot
    if constexpr (GHK == 0) {
        gcm_record<NR, OPEN, G, RkRegs<NR>, GhashTables, SPLIT, WIN>(b, i, lane4, rk,
                                                                    GhashTables{}, win);
    } else if constexpr (GHK == 1) {
        GhashTablesRot gh;
        gh.init(threadIdx.x & 63);
        gcm_record<NR, OPEN, G, RkRegs<NR>, GhashTablesRot, SPLIT, WIN>(b, i, lane4, rk, gh, win);
    } else {
        gcm_record<NR, OPEN, G, RkRegs<NR>, GhashTablesRotLds, SPLIT, WIN>(
            b, i, lane4, rk, GhashTablesRotLds{lane4}, win);
    }
}

// ---- bitsliced single-key kernel ---------------------------------------
// AES on the VALU (aes_bs.h): each lane runs its record in chunks of 32
// counter blocks, 2 + 32 j ... 33 + 32 j, bitsliced across the 32 bits of
// every register; the wave walks the chunks in lock step (j is wave-uniform,
// so the counter planes are scalar), up to the longest record of the wave.
// LDS holds only the GHASH tables (64 KiB) and a 256-byte S-box for the
// per-record work: the first-round S-box of the nonce bytes, the tag mask
// E_K(J0) and the keystream of a trailing partial block, which are single
// blocks done with a byte-wise AES (aes_block_sb).  512 threads = two waves
// per SIMD (the cipher keeps 128 state planes + S-box temporaries live).
constexpr int kBsThreads = 512;
constexpr uint32_t kSboxBase = 65536;
// GHASH staging (hooked path): per wave two buffers of 4 blocks x 64 lanes x 16 B
constexpr uint32_t kStageBase = 65536 + 256;
constexpr uint32_t kStageWave = 2 * 4 * 1024;
constexpr size_t kBsLds = kStageBase + (kBsThreads / 64) * kStageWave;

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

// The chunk loop.  HOOKED (every record of the wave 16-byte aligned): the
// GHASH of chunk j-1 runs inside chunk j's middle AES rounds, GH blocks per
// round, so that its serial chain of table lookups hides behind the S-box
// gates of both waves of the SIMD.  Its input (the ciphertext just stored for
// seal, the input for open) is re-read from memory one round ahead straight
// into a per-wave LDS staging buffer (global_load_lds_dwordx4: no VGPRs held
// across the round); out-of-range blocks read a harmless address and leave y
// unchanged, so the round stays one basic block.  The last chunk's blocks are
// hashed after the loop.  Not HOOKED: GHASH block by block after the XOR.
template <int NR, bool OPEN, bool HOOKED>
__device__ __forceinline__ uint4 gcm_bs_chunks(const bs::BsKeyMasks& km, const uint32_t* rk,
                                               const uint32_t* s1w, uint4 rkl, const uint8_t* in,
                                               uint8_t* out, uint32_t nfull, uint32_t nch,
                                               uint32_t stage, const uint8_t* safe, uint4 y,
                                               bool valid) {
    // fewest full blocks over the wave's valid lanes (wave-uniform)
    uint32_t nmin = valid ? nfull : 0xffffffffu;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)nmin, off, 64);
        nmin = o < nmin ? o : nmin;
    }
    nmin = __builtin_amdgcn_readfirstlane(nmin);
    constexpr int GH = (32 + NR - 3) / (NR - 2);   // 4 for AES-128, 3 for AES-256
    const uint8_t* ghsrc = OPEN ? in : out;
    const uint32_t lane16 = (threadIdx.x & 63u) << 4;
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    for (uint32_t j = 0; j < nch; ++j) {
        const uint32_t g0 = 32u * (j - 1), glim = nfull < 32u * j ? nfull : 32u * j;
        // stage round r's GH blocks (of chunk j-1) into buffer r & 1 (for
        // r = NR, a harmless reload of block 0's slot address)
        auto prefetch = [&](int r) {
#pragma unroll
            for (int u = 0; u < GH; ++u) {
                const uint32_t gb = g0 + GH * (r - 2) + u;
                const uint8_t* p = (j != 0 && gb < glim) ? ghsrc + 16 * gb : safe;
                __builtin_amdgcn_global_load_lds((gvoid*)p,
                                                 (lvoid*)(uintptr_t)(stage + ((r & 1) * 4 + u) * 1024),
                                                 16, 0, 0);
            }
        };
        // one GHASH block per four S-box steps, four table rows in flight at
        // a time (16 VGPRs): step 4u: read block u from the staging buffer,
        // x = y ^ c, issue rows 0-3; steps 4u+1..4u+3: fold the rows in
        // flight, issue the next four; the fold of rows 12-15 (at the next
        // block's first step, or after the last S-box) yields y.  A select
        // keeps y for blocks outside the previous chunk / the record.
        uint4 x = make_uint4(0, 0, 0, 0), z = make_uint4(0, 0, 0, 0);
        uint4 e[4], c[GH];
        auto rows = [&](int g) {   // table rows 4g .. 4g+3: byte positions of word g
            const uint32_t v = g == 0 ? x.x : g == 1 ? x.y : g == 2 ? x.z : x.w;
            e[0] = lds_u128(((v << 4) & 0xff0u) + 4096 * (4 * g + 0));
            e[1] = lds_u128(((v >> 4) & 0xff0u) + 4096 * (4 * g + 1));
            e[2] = lds_u128(((v >> 12) & 0xff0u) + 4096 * (4 * g + 2));
            e[3] = lds_u128(((v >> 20) & 0xff0u) + 4096 * (4 * g + 3));
        };
        auto fold = [&]() {
            z = xor4_3(z, e[0], e[1]);
            z = xor4_3(z, e[2], e[3]);
        };
        auto finish = [&](int r, int u) {   // rows 12-15 of block u are in flight
            fold();
            const bool ok = j != 0 && g0 + GH * (r - 2) + u < glim;
            y.x = ok ? z.x : y.x;
            y.y = ok ? z.y : y.y;
            y.z = ok ? z.z : y.z;
            y.w = ok ? z.w : y.w;
        };
        auto hook = [&](int r, int k) {
            if (!HOOKED) return;
            if (k == 0) {
                // this round's blocks out of staging buffer r & 1 (the DMA of the
                // previous round), then the next round's DMA into the other one
#pragma unroll
                for (int u = 0; u < GH; ++u) c[u] = lds_u128(stage + ((r & 1) * 4 + u) * 1024 + lane16);
                prefetch(r + 1);
            }
#pragma unroll
            for (int u = 0; u < GH; ++u) {
                if (k == 4 * u) {
                    if (u) finish(r, u - 1);
                    x = xor4(y, c[u]);
                    z = make_uint4(0, 0, 0, 0);
                    rows(0);
                } else if (k == 4 * u + 1 || k == 4 * u + 2 || k == 4 * u + 3) {
                    fold();
                    rows(k - 4 * u);
                }
            }
            if (k == 15) finish(r, GH - 1);
        };
        if (HOOKED) {
            __builtin_amdgcn_s_waitcnt(0);   // chunk j-1's stores are done before they are re-read
            prefetch(2);
        }
        uint32_t w[4][32];
        bs::ctr32<NR, 0, bs::BsKeyMasks, 1, HOOKED>(km, rk[3], s1w, 2u + 32u * j, w, hook);
        auto xor_ks = [&](uint4 d, int q) {
            return make_uint4(xor3(d.x, w[0][q], rkl.x), xor3(d.y, w[1][q], rkl.y),
                              xor3(d.z, w[2][q], rkl.z), xor3(d.w, w[3][q], rkl.w));
        };
        if (HOOKED && 32u * j + 32u <= nmin) {
            // Every valid lane of the wave has all 32 blocks.  Loads run one
            // batch of 8 ahead of the XOR/stores and are issued before the
            // transposes they wait behind: the vector memory counter is in
            // order over loads AND stores, so a load issued after a store
            // would also wait for that store.
            if (valid) {
                const uint8_t* ip = in + 512u * j;
                uint8_t* op = out + 512u * j;
                constexpr int B = 4;   // blocks per batch; two batches in flight
                uint4 dv[2][B];
                auto ld = [&](int bt) {
#pragma unroll
                    for (int t = 0; t < B; ++t)
                        dv[bt & 1][t] = *reinterpret_cast<const uint4*>(ip + 16 * (B * bt + t));
                };
                auto st = [&](int bt) {
#pragma unroll
                    for (int t = 0; t < B; ++t)
                        *reinterpret_cast<uint4*>(op + 16 * (B * bt + t)) = xor_ks(dv[bt & 1][t], B * bt + t);
                };
                auto tr = [&](int h) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) bs::transpose32_half(w[q], h);
                };
#define TG_SB __builtin_amdgcn_sched_barrier(0)
                ld(0); TG_SB; ld(1); TG_SB; tr(0); TG_SB;
#pragma unroll
                for (int bt = 0; bt < 32 / B; ++bt) {
                    st(bt); TG_SB;
                    if (bt + 2 < 32 / B) { ld(bt + 2); TG_SB; }
                    if (B * (bt + 2) == 16) { tr(1); TG_SB; }
                }
#undef TG_SB
            }
            continue;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) bs::transpose32_half(w[q], h);
            __builtin_amdgcn_sched_barrier(0);
            auto block = [&](int q) {
                const uint32_t blk = 32u * j + q;
                const uint4 d = load16(in + 16 * blk, HOOKED);
                const uint4 c = xor_ks(d, q);
                store16(out + 16 * blk, c, HOOKED);
                if (!HOOKED) y = gmul_lowreg(xor4(y, OPEN ? d : c));
            };
            if (32u * j + 16u * h + 16u <= nmin) {
                // every valid lane of the wave has these 16 blocks: one basic
                // block, so the loads are issued together, not one latency each
                if (valid) {
#pragma unroll
                    for (int q = 16 * h; q < 16 * h + 16; ++q) block(q);
                }
            } else {
#pragma unroll
                for (int q = 16 * h; q < 16 * h + 16; ++q)
                    if (32u * j + q < nfull) block(q);
            }
        }
    }
    // HOOKED: GHASH of the last chunk's blocks (stored above; reread in order)
    if (HOOKED && nch) {
        // the cipher state is dead here: load the (up to 32) blocks first,
        // eight at a time, so only the multiply chain is serial
        for (uint32_t b0 = 32u * (nch - 1); b0 < nfull; b0 += 8) {
            uint4 cb[8];
#pragma unroll
            for (int t = 0; t < 8; ++t)
                cb[t] = b0 + t < nfull ? *reinterpret_cast<const uint4*>(ghsrc + 16 * (b0 + t))
                                       : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (b0 + t < nfull) y = gmul(xor4(y, cb[t]));
        }
    }
    return y;
}

template <int NR, bool OPEN>
__global__ __launch_bounds__(kBsThreads, 1) void gcm_bs_kernel(const GcmKeyDev* __restrict__ key,
                                                              tg_batch b) {
    uint4* lds = g_lds;
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x) lds[e] = key->ghash[e];
    if (threadIdx.x < 64) {   // S(x) = byte 1 of Te0[x]
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v |= ((c_te.te0[4 * threadIdx.x + q] >> 8) & 0xffu) << (8 * q);
        reinterpret_cast<uint32_t*>(lds)[kSboxBase / 4 + threadIdx.x] = v;
    }
    __syncthreads();

    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < b.n;
    const uint32_t* rk = key->rk;
    const uint32_t len = valid ? rec_len(b, i) : 0u;
    const uint32_t nfull = len >> 4, tail = len & 15;
    const uint32_t nch = wave_max((nfull + 31) >> 5);
    const uint8_t* in = valid ? rec_in(b, i) : nullptr;
    uint8_t* out = valid ? rec_out(b, i) : nullptr;
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;

    uint4 nv = make_uint4(0, 0, 0, 0);
    if (valid) nv = load_partial(b.nonce + 12 * i, 12);
    // first-round S-box of the nonce bytes, without the 0x63 (see aes_bs.h)
    const uint32_t s1w[3] = {sub_word(nv.x ^ rk[0], kSboxBase) ^ 0x63636363u, sub_word(nv.y ^ rk[1], kSboxBase) ^ 0x63636363u,
                             sub_word(nv.z ^ rk[2], kSboxBase) ^ 0x63636363u};
    const uint4 rkl = make_uint4(rk[4 * NR] ^ 0x63636363u, rk[4 * NR + 1] ^ 0x63636363u,
                                 rk[4 * NR + 2] ^ 0x63636363u, rk[4 * NR + 3] ^ 0x63636363u);

    // GHASH over the AAD, zero-padded (aesgcm.py:69-79)
    uint4 y = make_uint4(0, 0, 0, 0);
    if (valid) {
        const uint8_t* ad = rec_aad(b, i);
        const uint32_t alen = rec_aad_len(b, i);
        for (uint32_t off = 0; off < alen; off += 16) {
            const uint32_t m = alen - off < 16 ? alen - off : 16;
            y = gmul_lowreg(xor4(y, load_partial(ad + off, m)));
        }
    }

    // CTR from nonce || be32(2) (aesgcm.py:118-120), GHASH over the ciphertext
    // (aesgcm.py:69-79).
    const bs::BsKeyMasks km{key->bsmask};
    const uint32_t stage = kStageBase + (threadIdx.x >> 6) * kStageWave;
    if (__all(aligned))
        y = gcm_bs_chunks<NR, OPEN, true>(km, rk, s1w, rkl, in, out, nfull, nch, stage,
                                          reinterpret_cast<const uint8_t*>(key->ghash), y, valid);
    else
        y = gcm_bs_chunks<NR, OPEN, false>(km, rk, s1w, rkl, in, out, nfull, nch, stage,
                                           reinterpret_cast<const uint8_t*>(key->ghash), y, valid);
    if (!valid) return;
    if (tail) {
        const uint4 ks = aes_block_sb<NR>(rk, make_uint4(nv.x, nv.y, nv.z, bswap32(2u + nfull)), kSboxBase);
        const uint4 d = load_partial(in + 16 * nfull, tail);
        const uint4 c = mask_tail(xor4(d, ks), tail);
        store_partial(out + 16 * nfull, c, tail);
        y = gmul_lowreg(xor4(y, OPEN ? d : c));
    }
    // length block: be64(8*alen) || be64(8*len) (aesgcm.py:64)
    const uint64_t abits = (uint64_t)rec_aad_len(b, i) << 3, cbits = (uint64_t)len << 3;
    y = gmul_lowreg(xor4(y, make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                                bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits))));
    // J0 = nonce || be32(1): the tag mask (aesgcm.py:112-115)
    const uint4 tag = xor4(y, aes_block_sb<NR>(rk, make_uint4(nv.x, nv.y, nv.z, bswap32(1u)), kSboxBase));
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
int launch_bs(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_bs_kernel<NR, OPEN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBsLds) != hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + kBsThreads - 1) / kBsThreads;
    hipLaunchKernelGGL((gcm_bs_kernel<NR, OPEN>), dim3((unsigned)blocks), dim3(kBsThreads), kBsLds, s,
                       key, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// ---- wave-per-record kernel (small batches and the per-record calls) ----
// One record per wavefront (the layout of the north star), or W waves per
// record.  The GHASH input AAD || C || length block is front-padded with zero
// blocks (neutral for GHASH: y stays 0) to P = 64 W Bw blocks; wave w of the
// record takes the padded blocks [64 Bw w, 64 Bw (w + 1)) and lane l of it the
// blocks 64 Bw w + 64 j + l (j < Bw), so every load and store instruction of
// the wave covers 1 KiB of consecutive record bytes.  Lane l encrypts its
// blocks (T-table CTR, counters 2 + c) and folds them by Horner with stride
// H^64 (y <- y H^64 ^ X, the 8-bit tables of H^64 staged in LDS); since
// GHASH = sum_t X_t H^(P - t), its value is then lifted by
// H^(64 Bw (W - 1 - w) + 64 - l) -- one table-free multiply by a power from
// the key's H^e table (GcmKeyDev::hpow) -- and the lifted values are
// XOR-reduced by shuffles (and across the record's waves through LDS).
constexpr int kWaveThreads = 1024;   // 16 waves share one LDS copy of the tables
// GHASH tables at 0, Te0/Te2 copies at 64 KiB, then the per-wave partials
// (16 x 16 B) and the per-record open verdicts (16 x 4 B).  The table lookups
// use absolute LDS addresses, so this kernel must not declare static
// __shared__ variables (they would move the dynamic region).
constexpr size_t kWavePartBase = 2 * 65536;
constexpr size_t kWaveLds = kWavePartBase + 16 * 16 + 16 * 4;

// W waves per record (1, 4 or 16; 16 / W records per workgroup): more waves
// per record for batches too small to fill the chip (the per-record calls).
// (A persistent grid that stages the tables once per CU and loops over the
// record groups measured slower: profiles/r01/v20_smallbatch.txt.)
// All waves of a workgroup reach the barriers: a record slot past the end of
// the batch recomputes the last record with its stores switched off.
template <int NR, bool OPEN, int W>
__device__ __forceinline__ void gcm_wave_record(const GcmKeyDev* __restrict__ key, const tg_batch& b,
                                                const RkRegs<NR>& rk, uint64_t i, bool live,
                                                uint32_t slot) {
    constexpr uint32_t S = 64u * W;            // segments (threads) per record
    uint4* s_part = g_lds + kWavePartBase / 16;
    uint32_t* s_diff = reinterpret_cast<uint32_t*>(g_lds + kWavePartBase / 16 + 16);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t seg = threadIdx.x & (S - 1u);
    const uint32_t lane4 = ((lane & 31u) << 2) | kTeBase;
    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const CtrCache cc = ctr_cache<NR>(lane4, rk, nv);
    const uint32_t na = (alen + 15) >> 4, nc = (len + 15) >> 4, nfull = len >> 4, tail = len & 15;
    const uint32_t M = na + nc + 1;            // GHASH blocks (aesgcm.py:60-79)
    const uint32_t Bw = (M + S - 1) / S, pad = S * Bw - M;
    const uint32_t wv = seg >> 6;              // the record's wave
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
    uint4 y = make_uint4(0, 0, 0, 0);
    // 256-counter window cache in registers (aes_round.h): the lane's counter
    // steps by 64, so it enters a new window every fourth block
    uint4 wc = make_uint4(0, 0, 0, 0);
    uint32_t whi = 0xffffffffu;
    for (uint32_t j = 0; j < Bw; ++j) {
        if (j) y = gmul(y);                     // y H^64 (wave-uniform)
        const uint32_t t = 64 * (Bw * wv + j) + lane;
        if (t < pad) continue;                  // leading zero blocks
        const uint32_t k = t - pad;
        uint4 x;
        if (k < na) {
            const uint32_t m = alen - 16 * k < 16 ? alen - 16 * k : 16;
            x = load_partial(ad + 16 * k, m);
        } else if (k < na + nc) {               // CTR block c (python_aes.py:101-116)
            const uint32_t c = k - na;
            if (((2u + c) >> 8) != whi) {
                whi = (2u + c) >> 8;
                wc = win_consts<NR>(lane4, rk, cc, 2u + c);
            }
            const uint4 ks = aes_ctr_win<NR>(lane4, rk, cc, wc, 2u + c);
            if (c < nfull) {
                const uint4 d = load16(in + 16 * c, aligned);
                const uint4 ct = xor4(d, ks);
                if (live) store16(out + 16 * c, ct, aligned);
                x = OPEN ? d : ct;
            } else {
                const uint4 d = load_partial(in + 16 * c, tail);
                const uint4 ct = mask_tail(xor4(d, ks), tail);
                if (live) store_partial(out + 16 * c, ct, tail);
                x = OPEN ? d : ct;
            }
        } else {                                // be64(8 alen) || be64(8 len) (aesgcm.py:64)
            x = make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                           bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits));
        }
        y = xor4(y, x);
    }
    // lift by H^(64 Bw (W - 1 - w) + 64 - l) and XOR-reduce
    uint4 yn = norm4(y);
    if (y.x | y.y | y.z | y.w) {
        const uint32_t e = 64 * Bw * (W - 1 - wv) + 64 - lane;
        const uint4 hp = e <= (uint32_t)kHPow ? key->hpow[e - 1] : gf128_pow(key->hpow[0], e);
        yn = gf128_mul(yn, hp);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) yn = xor4(yn, shfl_xor4(yn, m));
    if (W > 1) {
        if (lane == 0) s_part[threadIdx.x >> 6] = yn;
        __syncthreads();
        yn = s_part[slot * W];
#pragma unroll
        for (int w = 1; w < W; ++w) yn = xor4(yn, s_part[slot * W + w]);
    }
    // tag = GHASH ^ E_K(J0) (aesgcm.py:112-122)
    const uint4 mask = aes_ctr<NR>(lane4, rk, cc, 1u);
    const uint4 tag = xor4(norm4(yn), mask);
    const bool tag_aligned = aligned && tail == 0;
    if (!OPEN) {
        if (seg == 0 && live) store16(out + len, tag, tag_aligned);
        return;
    }
    // open: compare (aesgcm.py:148-149); a rejected record's plaintext is zeroed
    uint32_t diff = 0;
    if (seg == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status && live) b.status[i] = diff == 0;
        if (W > 1) s_diff[slot] = diff;
    }
    if (W > 1) {
        __syncthreads();
        diff = live ? s_diff[slot] : 0;
    } else {
        diff = (uint32_t)__shfl((int)diff, 0, 64);
    }
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t c = seg; c < nfull; c += S) store16(out + 16 * c, z, aligned);
        if (tail && seg == 0) store_partial(out + 16 * nfull, z, tail);
    }
}

template <int NR, bool OPEN, int W>
__global__ __launch_bounds__(kWaveThreads) void gcm_wave_kernel(const GcmKeyDev* __restrict__ key,
                                                                tg_batch b) {
    constexpr uint32_t R = kWaveThreads / (64u * W);   // records per group
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x) g_lds[e] = key->ghash64[e];
    stage_te(reinterpret_cast<uint32_t*>(g_lds) + kTeBase / 4);
    RkRegs<NR> rk;
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = key->rk[k];
    __syncthreads();
    // wave-uniform (readfirstlane): the record's fields become scalar loads
    const uint32_t slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / (64u * W)));
    const uint64_t i0 = (uint64_t)blockIdx.x * R + slot;
    const bool live = i0 < b.n;
    if (W == 1 && !live) return;             // whole wave; no barriers for W = 1
    gcm_wave_record<NR, OPEN, W>(key, b, rk, live ? i0 : b.n - 1, live, slot);
}

// Waves per record: enough for n * W waves to give each CU a 16-wave
// workgroup (profiles/r01/v21_smallbatch.txt).
int waves_per_record(uint64_t n) {
    const char* env = getenv("TLSGPU_WAVES_PER_RECORD");
    if (env) return atoi(env);
    return n <= 256 ? 16 : n <= 2048 ? 4 : 1;
}

template <int NR, bool OPEN, int W>
int launch_wave_w(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_wave_kernel<NR, OPEN, W>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWaveLds) != hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    constexpr uint64_t per_group = kWaveThreads / (64 * W);
    const uint64_t groups = (b.n + per_group - 1) / per_group;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_wave_kernel<NR, OPEN, W>), dim3((unsigned)groups), dim3(kWaveThreads),
                       kWaveLds, s, key, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

template <int NR, bool OPEN>
int launch_wave(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    switch (waves_per_record(b.n)) {
        case 16: return launch_wave_w<NR, OPEN, 16>(key, b, s);
        case 4: return launch_wave_w<NR, OPEN, 4>(key, b, s);
        default: return launch_wave_w<NR, OPEN, 1>(key, b, s);
    }
}

// Key-table kernel (many sessions per batch, BASELINE config 4): lane i uses
// key key_idx[i] and GHASH is the table-free multiply.  This first layout
// stages each lane's round keys into a private LDS row (272-byte stride:
// conflict-free ds_read_b128); gcm_table_vkernel below keeps them in VGPRs
// and is the default.
constexpr int kMkThreads = 256;
constexpr uint32_t kMkRowBytes = 272;
constexpr size_t kMkLds = 65536 + kMkThreads * kMkRowBytes;

template <int NR, bool OPEN, int G>
__global__ __launch_bounds__(kMkThreads, 4) void gcm_table_kernel(const GcmTableKey* __restrict__ keys,
                                                              tg_batch b,
                                                              const uint32_t* __restrict__ order) {
    uint4* lds = g_lds;
    stage_te(reinterpret_cast<uint32_t*>(lds));  // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n) return;
    const uint64_t i = order ? order[t] : t;
    const GcmTableKey* kp = keys + b.key_idx[i];
    const RkLds rk{65536u + threadIdx.x * kMkRowBytes};
    uint4* row = lds + rk.base / 16;
#pragma unroll
    for (int r = 0; r <= NR; ++r) row[r] = reinterpret_cast<const uint4*>(kp->rk)[r];
    const GhashClmul gh{*reinterpret_cast<const uint4*>(kp->hn)};
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    gcm_record<NR, OPEN, G>(b, i, lane4, rk, gh);
}

// Key-table kernel with the lane's round keys in VGPRs (60 words for
// AES-256) instead of an LDS row: LDS holds only the 64 KiB Te block, so a
// 768-thread workgroup (three waves per SIMD) fits where the LDS-row layout
// (64 KiB + 68 KiB of rows) allowed one wave per SIMD.
// WIN: 256-counter window cache in a 16-byte LDS slot per lane after the Te
// block (aes_round.h, ctr_keystream).
template <int NR, bool OPEN, int THREADS, bool WIN = true>
__global__ __launch_bounds__(THREADS) void gcm_table_vkernel(const GcmTableKey* __restrict__ keys,
                                                             tg_batch b,
                                                             const uint32_t* __restrict__ order) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n) return;
    const uint64_t i = order ? order[t] : t;
    const GcmTableKey* kp = keys + b.key_idx[i];
    RkRegs<NR> rk;   // per-lane values: VGPRs
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const GhashClmul gh{*reinterpret_cast<const uint4*>(kp->hn)};
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    gcm_record<NR, OPEN, 1, RkRegs<NR>, GhashClmul, 0, WIN>(b, i, lane4, rk, gh,
                                                           65536u + 16u * threadIdx.x);
}

template <int NR, bool OPEN, int THREADS, bool WIN = true>
int launch_table_v(const GcmTableKey* keys, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    constexpr int lds = 65536 + (WIN ? 16 * THREADS : 0);
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_table_vkernel<NR, OPEN, THREADS, WIN>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + THREADS - 1) / THREADS;
    hipLaunchKernelGGL((gcm_table_vkernel<NR, OPEN, THREADS, WIN>), dim3((unsigned)blocks),
                       dim3(THREADS), lds, s, keys, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Key-table wave-per-record kernel (many sessions, mixed lengths; BASELINE
// config 4).  Wave w of the workgroup seals / opens record i with key
// key_idx[i]: the index is wave-uniform, so the round keys are scalar loads
// into SGPRs (no VGPRs, no LDS rows).  The layout is the single-key wave
// kernel's with W = 1 (lane l takes blocks l, l + 64, ...: coalesced), but
// GHASH is the table-free multiply: Horner with stride H^64 and one lift by
// H^(64 - l), both read from the key's 64 precomputed powers
// (hpow[64 k + e - 1] = H^e, built at key setup by table_hpow_kernel).
// No length planning: a wave takes as long as its own record.
template <int NR, bool OPEN>
__device__ __forceinline__ void gcm_table_wave_record(const GcmTableKey* __restrict__ keys,
                                                      const uint4* __restrict__ hpow,
                                                      const tg_batch& b, uint64_t i, uint32_t lane) {
    const uint32_t ki = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b.key_idx ? b.key_idx[i] : 0u));
    const GcmTableKey* kp = keys + ki;
    RkRegs<NR> rk;   // wave-uniform: SGPRs
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const uint4* hp = hpow + 64ull * ki;
    const uint4 h64 = hp[63];
    const uint32_t lane4 = (lane & 31u) << 2;
    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    const CtrCache cc = ctr_cache<NR>(lane4, rk, nv);
    const uint32_t na = (alen + 15) >> 4, nc = (len + 15) >> 4, nfull = len >> 4, tail = len & 15;
    const uint32_t M = na + nc + 1;            // GHASH blocks (aesgcm.py:60-79)
    const uint32_t Bw = (M + 63) >> 6, pad = 64 * Bw - M;
    const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
    uint4 y = make_uint4(0, 0, 0, 0);          // normal order
    uint4 wc = make_uint4(0, 0, 0, 0);         // 256-counter window cache (aes_round.h)
    uint32_t whi = 0xffffffffu;
    for (uint32_t j = 0; j < Bw; ++j) {
        if (j) y = gf128_mul(y, h64);           // y H^64 (wave-uniform)
        const uint32_t t = 64 * j + lane;
        if (t < pad) continue;                  // leading zero blocks
        const uint32_t k = t - pad;
        uint4 x;
        if (k < na) {
            const uint32_t m = alen - 16 * k < 16 ? alen - 16 * k : 16;
            x = load_partial(ad + 16 * k, m);
        } else if (k < na + nc) {               // CTR block c (python_aes.py:101-116)
            const uint32_t c = k - na;
            if (((2u + c) >> 8) != whi) {
                whi = (2u + c) >> 8;
                wc = win_consts<NR>(lane4, rk, cc, 2u + c);
            }
            const uint4 ks = aes_ctr_win<NR>(lane4, rk, cc, wc, 2u + c);
            if (c < nfull) {
                const uint4 d = load16(in + 16 * c, aligned);
                const uint4 ct = xor4(d, ks);
                store16(out + 16 * c, ct, aligned);
                x = OPEN ? d : ct;
            } else {
                const uint4 d = load_partial(in + 16 * c, tail);
                const uint4 ct = mask_tail(xor4(d, ks), tail);
                store_partial(out + 16 * c, ct, tail);
                x = OPEN ? d : ct;
            }
        } else {                                // be64(8 alen) || be64(8 len) (aesgcm.py:64)
            x = make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                           bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits));
        }
        y = xor4(y, norm4(x));
    }
    if (y.x | y.y | y.z | y.w) y = gf128_mul(y, hp[63 - lane]);   // lift by H^(64 - l)
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) y = xor4(y, shfl_xor4(y, m));
    // tag = GHASH ^ E_K(J0) (aesgcm.py:112-122)
    const uint4 tag = xor4(norm4(y), aes_ctr<NR>(lane4, rk, cc, 1u));
    const bool tag_aligned = aligned && tail == 0;
    if (!OPEN) {
        if (lane == 0) store16(out + len, tag, tag_aligned);
        return;
    }
    uint32_t diff = 0;                          // aesgcm.py:148-149
    if (lane == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status) b.status[i] = diff == 0;
    }
    diff = (uint32_t)__shfl((int)diff, 0, 64);
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t c = lane; c < nfull; c += 64) store16(out + 16 * c, z, aligned);
        if (tail && lane == 0) store_partial(out + 16 * nfull, z, tail);
    }
}

// A persistent grid (two workgroups per CU): wave g takes records g, g + G,
// g + 2G, ... so a workgroup's waves finish together however the lengths mix
// (one workgroup per record group would hold its LDS until its longest
// record is done).
template <int NR, bool OPEN, int kTwThreads>
__global__ __launch_bounds__(kTwThreads) void gcm_table_wave_kernel(
    const GcmTableKey* __restrict__ keys, const uint4* __restrict__ hpow, tg_batch b) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t G = (uint64_t)gridDim.x * (kTwThreads / 64);
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (uint64_t i = (uint64_t)blockIdx.x * (kTwThreads / 64) + wave; i < b.n; i += G)
        gcm_table_wave_record<NR, OPEN>(keys, hpow, b, i, threadIdx.x & 63u);
}

// Threads per workgroup: two workgroups (2 x 64 KiB of T-tables) per CU.
template <int NR, bool OPEN, int kTwThreads>
int launch_table_wave_t(const GcmTableKey* keys, const uint4* hpow, const tg_batch& b,
                        hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_table_wave_kernel<NR, OPEN, kTwThreads>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 65536) != hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t groups = (b.n + kTwThreads / 64 - 1) / (kTwThreads / 64);
    const uint64_t cap = 2ull * (uint64_t)device_cus();
    hipLaunchKernelGGL((gcm_table_wave_kernel<NR, OPEN, kTwThreads>), dim3((unsigned)(groups < cap ? groups : cap)),
                       dim3(kTwThreads), 65536, s, keys, hpow, b);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

template <int NR, bool OPEN>
int launch_table_wave(const GcmTableKey* keys, const uint4* hpow, const tg_batch& b, hipStream_t s) {
    const char* e = getenv("TLSGPU_GCM_TABLE_WAVE_THREADS");   // measurement
    switch (e ? atoi(e) : 768) {
        case 512: return launch_table_wave_t<NR, OPEN, 512>(keys, hpow, b, s);
        case 1024: return launch_table_wave_t<NR, OPEN, 1024>(keys, hpow, b, s);
        default: return launch_table_wave_t<NR, OPEN, 768>(keys, hpow, b, s);
    }
}

// The key table's GHASH powers for gcm_table_wave_kernel: one wave per key,
// lane l ends with H^(l + 1) (normal order); after the step with distance d
// lanes [0, 2d) hold their powers (H^(l + 1) = H^(l + 1 - d) * H^d).
__global__ __launch_bounds__(256) void table_hpow_kernel(const GcmTableKey* __restrict__ keys,
                                                         uint64_t n, uint4* __restrict__ hpow) {
    const uint64_t key = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (key >= n) return;
    const int lane = threadIdx.x & 63;
    const uint4 h = *reinterpret_cast<const uint4*>(keys[key].hn);
    uint4 p = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint4 hd = make_uint4((uint32_t)__shfl((int)p.x, d - 1, 64), (uint32_t)__shfl((int)p.y, d - 1, 64),
                                    (uint32_t)__shfl((int)p.z, d - 1, 64), (uint32_t)__shfl((int)p.w, d - 1, 64));
        const int src = lane >= d ? lane - d : lane;
        const uint4 q = make_uint4((uint32_t)__shfl((int)p.x, src, 64), (uint32_t)__shfl((int)p.y, src, 64),
                                   (uint32_t)__shfl((int)p.z, src, 64), (uint32_t)__shfl((int)p.w, src, 64));
        if (lane >= d && lane < 2 * d) p = gf128_mul(q, hd);
    }
    hpow[64 * key + lane] = p;
}

int table_variant() {
    const char* e = getenv("TLSGPU_GCM_TABLE_VARIANT");
    return e ? atoi(e) : 0;
}

template <int NR, bool OPEN, int G, int THREADS, int GH>
int launch_v(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    // GH >= 100: + one 16-byte window slot per thread after the fixed tables
    constexpr size_t lds = kGcmLds + (GH >= 100 ? 16 * THREADS : 0);
    static_assert(lds <= 160 * 1024, "LDS per workgroup");
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_kernel<NR, OPEN, G, THREADS, GH>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + THREADS - 1) / THREADS;
    hipLaunchKernelGGL((gcm_kernel<NR, OPEN, G, THREADS, GH>), dim3((unsigned)blocks), dim3(THREADS),
                       lds, s, key, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Kernel choice (TLSGPU_GCM_VARIANT, read per launch, for tests and measurement):
//   0 / unset  the wave-per-record kernel up to kWaveMaxRecords records, the
//              hybrid octet kernel (15) above;
//   1..3       T-table tuning variants;
//   4          the bitsliced kernel (gcm_bs_kernel);
//   5          G = 4, 1024 threads, full rounds (no counter-window cache);
//   7..13      counter-window tuning variants (G, threads, GHASH flavour);
//   6          the wave-per-record kernel (gcm_wave_kernel), which is also what
//              batches of at most kWaveMaxRecords records use;
//   14         the 8-block bitsliced octet kernel (aes_gcm_bs8.hip);
//   15         the hybrid octet kernel (T-table + bitsliced waves), the default
//              above kWaveMaxRecords (TLSGPU_HY_T / TLSGPU_HY_PRIO tune it);
//   16         the T-table lane-per-record kernel that was the default before.
// Up to this many records a batch runs one record per wavefront; above it the
// hybrid octet kernel, whose floor is one octet job (8 records on one wave,
// ~0.42 ms at 16 KiB): at 16 KiB the two meet between 16 384 and 32 768
// records (profiles/r02/v28_wave_vs_hybrid.txt; against the T-table lane
// kernel it was 196 608, profiles/r01/v31_smallbatch.txt), and the wave
// kernel needs no length planning for mixed batches.
constexpr uint64_t kWaveMaxRecords = 24576;

int variant() {
    const char* e = getenv("TLSGPU_GCM_VARIANT");
    return e ? atoi(e) : 0;
}

template <int NR, bool OPEN>
int launch(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    switch (variant()) {   // profiles/r01/gcm_variant_sweep.txt
        case 1: return launch_v<NR, OPEN, 2, 1024, 0>(key, b, s, order);
        case 2: return launch_v<NR, OPEN, 2, 1024, 2>(key, b, s, order);
        case 3: return launch_v<NR, OPEN, 2, 512, 1>(key, b, s, order);
        case 4: return launch_bs<NR, OPEN>(key, b, s);
        case 5: return launch_v<NR, OPEN, 4, 1024, 0>(key, b, s, order);   // no window cache
        case 6: return launch_wave<NR, OPEN>(key, b, s);
        case 7: return launch_v<NR, OPEN, 4, 1024, 100>(key, b, s, order);
        case 8: return launch_v<NR, OPEN, 2, 1024, 100>(key, b, s, order);
        case 9: return launch_v<NR, OPEN, 4, 1024, 102>(key, b, s, order);
        case 10: return launch_v<NR, OPEN, 2, 1024, 102>(key, b, s, order);
        case 11: return launch_v<NR, OPEN, 2, 512, 101>(key, b, s, order);
        case 12: return launch_v<NR, OPEN, 4, 768, 100>(key, b, s, order);
        case 13: return launch_v<NR, OPEN, 3, 1024, 100>(key, b, s, order);
        case 14: return tg_launch_gcm_bs8(key, NR, b, OPEN, s, order);
        case 15: return tg_launch_gcm_hy(key, NR, b, OPEN, s, order);
        case 16:
            return OPEN ? launch_v<NR, OPEN, 4, 1024, 100>(key, b, s, order)
                        : launch_v<NR, OPEN, 4, 1024, 102>(key, b, s, order);
        default:
            if (b.n <= kWaveMaxRecords) return launch_wave<NR, OPEN>(key, b, s);
            // larger batches: the hybrid octet kernel (T-table waves beside
            // bitsliced waves, aes_gcm_bs8.hip): 15.1 / 15.2 ms against the
            // T-table lane kernel's 16.5 / 17.1 at 2^20 x 16 KiB
            // (profiles/r02/v10_gcm_kernel_probe.txt)
            return tg_launch_gcm_hy(key, NR, b, OPEN, s, order);
    }
}

bool wave_path(uint64_t n) {
    const int v = variant();
    return v == 6 || (v == 0 && n <= kWaveMaxRecords);
}

bool table_wave_path(uint64_t n) {
    (void)n;
    return table_variant() == 5;
}

template <int NR, bool OPEN>
int launch_table(const GcmTableKey* keys, const uint4* hpow, const tg_batch& b, hipStream_t s,
                 const uint32_t* order) {
    // TLSGPU_GCM_TABLE_VARIANT (measurement): 0 = lane per record, round keys
    // in VGPRs, 768 threads (config 4: 368 GiB/s); 2 = the same at 512 threads
    // (346); 3 = at 1024 threads (217, spills); 9 = round keys in LDS rows
    // (230); 5 = wave per record (gcm_table_wave_kernel: 358, both bound by the
    // table-free GHASH multiply; profiles/r01/v24_c4_*.json).
    if (table_wave_path(b.n) && hpow) return launch_table_wave<NR, OPEN>(keys, hpow, b, s);
    switch (table_variant()) {
        case 2: return launch_table_v<NR, OPEN, 512>(keys, b, s, order);
        case 6: return launch_table_v<NR, OPEN, 768, false>(keys, b, s, order);   // full rounds
        case 3: return launch_table_v<NR, OPEN, 1024>(keys, b, s, order);
        case 9: break;
        default: return launch_table_v<NR, OPEN, 768>(keys, b, s, order);
    }
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)gcm_table_kernel<NR, OPEN, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMkLds) !=
            hipSuccess)
            return TG_EHIP;
        attr_set = true;
    }
    const uint64_t blocks = (b.n + kMkThreads - 1) / kMkThreads;
    hipLaunchKernelGGL((gcm_table_kernel<NR, OPEN, 1>), dim3((unsigned)blocks), dim3(kMkThreads),
                       kMkLds, s, keys, b, order);  // G = 1: one block in flight per lane
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

}  // namespace
}  // namespace tg

bool tg_gcm_table_wave_path(uint64_t n) { return tg::table_wave_path(n); }

int tg_launch_table_hpow(const tg::GcmTableKey* keys, uint64_t n, uint4* hpow, hipStream_t s) {
    const uint64_t groups = (n + 3) / 4;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL(tg::table_hpow_kernel, dim3((unsigned)groups), dim3(256), 0, s, keys, n, hpow);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

int tg_launch_gcm_table(const tg::GcmTableKey* keys, const uint4* hpow, int rounds,
                        const tg_batch& b, bool open, hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch_table<10, true>(keys, hpow, b, s, order)
                    : tg::launch_table<10, false>(keys, hpow, b, s, order);
    if (rounds == 14)
        return open ? tg::launch_table<14, true>(keys, hpow, b, s, order)
                    : tg::launch_table<14, false>(keys, hpow, b, s, order);
    return TG_EINVAL;
}

bool tg_gcm_wave_path(uint64_t n) { return tg::wave_path(n); }

int tg_launch_gcm(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                  hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch<10, true>(key, b, s, order) : tg::launch<10, false>(key, b, s, order);
    if (rounds == 14)
        return open ? tg::launch<14, true>(key, b, s, order) : tg::launch<14, false>(key, b, s, order);
    return TG_EINVAL;
}
