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

#include "aes_round.h"
#include "ghash.h"
#include "gcm_lane.h"
#include "options.h"

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

// Bank-conflict-free GHASH (ghash.h gmul_rot): tables in row layout, entry
// (j, b) at b * 256 + j * 16; the rotation amounts are bits of lane4 (the AES
// lookup register, bits 2..5 = lane % 16) and the four table-offset words
// come from a 16-row LDS table (one conflict-free ds_read_b128 per multiply).
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

// The T-table lane-per-record kernel (round 1's default, now the forced
// fallback gcm_variant 16): four blocks per group, 1024 threads, keystream
// through the lane's 256-counter window slot after the fixed LDS tables.
// ROT: the conflict-free GHASH tables (seal); plain 8-bit tables otherwise
// (open: the payload is already in flight, the plain tables measured equal).
constexpr int kLaneThreads = 1024;
constexpr int kLaneG = 4;
constexpr size_t kLaneLds = kGcmLds + 16 * kLaneThreads;
static_assert(kLaneLds <= 160 * 1024, "LDS per workgroup");

template <int NR, bool OPEN, bool ROT>
__global__ __launch_bounds__(kLaneThreads) void gcm_kernel(const GcmKeyDev* __restrict__ key,
                                                           tg_batch b, const uint32_t* __restrict__ order) {
    uint4* lds = g_lds;
    // stage the GHASH tables (ROT: row layout b * 16 + j) and the Te0/Te2 copies
    for (int e = threadIdx.x; e < kGhashEntries; e += blockDim.x)
        lds[ROT ? (e & 255) * 16 + (e >> 8) : e] = key->ghash[e];
    if (ROT && threadIdx.x < 16) {   // row l: byte k of word q = ((l + 4q + k) % 16) * 16
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
    if constexpr (!ROT) {
        gcm_record<NR, OPEN, kLaneG, RkRegs<NR>, GhashTables, true>(b, i, lane4, rk, GhashTables{}, win);
    } else {
        gcm_record<NR, OPEN, kLaneG, RkRegs<NR>, GhashTablesRotLds, true>(b, i, lane4, rk,
                                                                         GhashTablesRotLds{lane4}, win);
    }
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
// workgroup (profiles/r01/v21_smallbatch.txt); option waves_per_record forces.
int waves_per_record(uint64_t n) {
    const int w = opt(kOptWavesPerRecord);
    if (w) return w;
    return n <= 256 ? 16 : n <= 2048 ? 4 : 1;
}

template <int NR, bool OPEN, int W>
int launch_wave_w(const GcmKeyDev* key, const tg_batch& b, hipStream_t s) {
    if (lds_attr((const void*)gcm_wave_kernel<NR, OPEN, W>, (int)kWaveLds)) return TG_EHIP;
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
        case 1: return launch_wave_w<NR, OPEN, 1>(key, b, s);
        default: return TG_EINVAL;
    }
}

// Key-table kernel (BASELINE config 4's short records): one record per
// lane, the lane's round keys in VGPRs (60 words for AES-256), LDS holding
// only the 64 KiB Te block plus a 16-byte 256-counter window slot per lane
// (aes_round.h ctr_keystream), 768 threads = three waves per SIMD; GHASH is
// the table-free multiply by the record's H.  Thread t takes slot *first + t
// of ``order`` (first: NULL = 0, else a device count -- the key-table plan
// puts the long records, which the octet kernel takes, in front); a record
// whose key_idx is not below nkeys is skipped (open: status 0).
#ifndef TG_TV_G
#define TG_TV_G 1   // blocks per step (A/B builds, tools/build_variant.sh -DTG_TV_G=n)
#endif
#ifndef TG_TV_THREADS
#define TG_TV_THREADS 512
#endif
constexpr int kTvThreads = TG_TV_THREADS;
constexpr int kTvLds = 65536 + 16 * kTvThreads;

template <int NR, bool OPEN>
__global__ __launch_bounds__(kTvThreads) void gcm_table_vkernel(const GcmTableKey* __restrict__ keys,
                                                               uint64_t nkeys, tg_batch b,
                                                               const uint32_t* __restrict__ order,
                                                               const uint32_t* __restrict__ first) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + (first ? *first : 0u);
    if (t >= b.n) return;
    const uint64_t i = order ? order[t] : t;
    const uint32_t ki = b.key_idx[i];
    if (ki >= nkeys) {
        if (OPEN && b.status) b.status[i] = 0;
        return;
    }
    const GcmTableKey* kp = keys + ki;
    RkRegs<NR> rk;   // per-lane values: VGPRs
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const GhashClmul gh{*reinterpret_cast<const uint4*>(kp->hn)};
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;
    gcm_record<NR, OPEN, TG_TV_G, RkRegs<NR>, GhashClmul, true>(b, i, lane4, rk, gh, 65536u + 16u * threadIdx.x);
}

template <int NR, bool OPEN>
int launch_table_v(const GcmTableKey* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s,
                   const uint32_t* order, const uint32_t* first) {
    if (lds_attr((const void*)gcm_table_vkernel<NR, OPEN>, kTvLds)) return TG_EHIP;
    const uint64_t blocks = (b.n + kTvThreads - 1) / kTvThreads;
    if (blocks > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_table_vkernel<NR, OPEN>), dim3((unsigned)blocks), dim3(kTvThreads), kTvLds, s,
                       keys, nkeys, b, order, first);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Key-table wave-per-record kernel (many sessions, mixed lengths; BASELINE
// config 4).  Wave w of the workgroup seals / opens record i with key
// key_idx[i]: the index is wave-uniform, so the round keys are scalar loads
// into SGPRs (no VGPRs, no LDS rows).  The layout is the single-key wave
// kernel's with W = 1 (lane l takes blocks l, l + 64, ...: coalesced);
// GHASH is Horner with stride H^64 and one lift by H^(64 - l), from the
// key's 64 precomputed powers (hpow[64 k + e - 1] = H^e, built at key setup
// by table_hpow_kernel).  T4: the stride multiply goes through 4-bit tables
// of the record's H^64 that the wave builds in its own 8 KiB of LDS at
// ``tab`` (ghash.h build_table4 / gmul4: 32 conflict-free lookups instead
// of the table-free multiply's ~650 VALU slots; ~700 VALU per lane to build,
// i.e. ~45 per block of a 16 KiB record); otherwise the table-free multiply.
template <int NR, bool OPEN, bool T4>
__device__ __forceinline__ void gcm_table_wave_record(const GcmTableKey* __restrict__ keys,
                                                      uint64_t nkeys, const uint4* __restrict__ hpow,
                                                      const tg_batch& b, uint64_t i, uint32_t lane,
                                                      uint32_t tab, uint32_t& tab_key) {
    const uint32_t ki = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b.key_idx ? b.key_idx[i] : 0u));
    if (ki >= nkeys) {   // out-of-range key index: skipped (open: rejected)
        if (OPEN && b.status && lane == 0) b.status[i] = 0;
        return;
    }
    const GcmTableKey* kp = keys + ki;
    RkRegs<NR> rk;   // wave-uniform: SGPRs
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = kp->rk[k];
    const uint4* hp = hpow + 64ull * ki;
    const uint4 h64 = hp[63];
    if (T4 && ki != tab_key) {   // this wave's tables of H^64 (kept while the key repeats)
        build_table4(tab, h64);
        __builtin_amdgcn_wave_barrier();
        tab_key = ki;
    }
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
        // y H^64 (T4: y in block byte layout, else normal order)
        if (j) y = T4 ? gmul4(y, tab) : gf128_mul(y, h64);
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
        y = xor4(y, T4 ? x : norm4(x));
    }
    if (T4) y = norm4(y);
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

// A persistent grid: wave g takes plan slots g, g + G, g + 2G, ... of
// [0, count) (count: NULL = all n records; order: NULL = identity), so a
// workgroup's waves finish together however the lengths mix (one workgroup
// per record group would hold its LDS until its longest record is done).
// Table-free GHASH: 768 threads, two workgroups (2 x 64 KiB of T-tables) per
// CU (512 / 1024 measured no better, profiles/r01/v24_c4_*.json).  T4: 512
// threads, one workgroup per CU: 64 KiB of T-tables + 8 KiB of GHASH tables
// per wave.
template <bool T4>
constexpr int tw_threads() { return T4 ? 512 : 768; }
template <bool T4>
constexpr int tw_lds() { return 65536 + (T4 ? 8192 * (tw_threads<T4>() / 64) : 0); }

template <int NR, bool OPEN, bool T4>
__global__ __launch_bounds__(tw_threads<T4>()) void gcm_table_wave_kernel(
    const GcmTableKey* __restrict__ keys, uint64_t nkeys, const uint4* __restrict__ hpow, tg_batch b,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ count) {
    constexpr int kW = tw_threads<T4>() / 64;
    stage_te(reinterpret_cast<uint32_t*>(g_lds));   // Te0/Te2 copies at LDS 0
    __syncthreads();
    const uint64_t G = (uint64_t)gridDim.x * kW;
    const uint64_t nslots = count ? *count : b.n;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t tab = 65536u + 8192u * wave;
    uint32_t tab_key = 0xffffffffu;
    for (uint64_t t = (uint64_t)blockIdx.x * kW + wave; t < nslots; t += G)
        gcm_table_wave_record<NR, OPEN, T4>(keys, nkeys, hpow, b, order ? gld(order, t) : t, threadIdx.x & 63u,
                                            tab, tab_key);
}

template <int NR, bool OPEN, bool T4>
int launch_table_wave(const GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, const tg_batch& b,
                      hipStream_t s, const uint32_t* order, const uint32_t* count) {
    constexpr int thr = tw_threads<T4>(), lds = tw_lds<T4>();
    if (lds_attr((const void*)gcm_table_wave_kernel<NR, OPEN, T4>, lds)) return TG_EHIP;
    const uint64_t groups = (b.n + thr / 64 - 1) / (thr / 64);
    const uint64_t cap = (T4 ? 1ull : 2ull) * (uint64_t)device_cus();
    hipLaunchKernelGGL((gcm_table_wave_kernel<NR, OPEN, T4>), dim3((unsigned)(groups < cap ? groups : cap)),
                       dim3(thr), lds, s, keys, nkeys, hpow, b, order, count);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
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

template <int NR, bool OPEN, bool ROT>
int launch_lane(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    if (lds_attr((const void*)gcm_kernel<NR, OPEN, ROT>, (int)kLaneLds)) return TG_EHIP;
    const uint64_t blocks = (b.n + kLaneThreads - 1) / kLaneThreads;
    if (blocks > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_kernel<NR, OPEN, ROT>), dim3((unsigned)blocks), dim3(kLaneThreads), kLaneLds, s,
                       key, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Single-key kernel choice (option gcm_variant; tests and measurement):
//   0   auto: the wave-per-record kernel up to kWaveMaxRecords records, the
//       hybrid octet kernel above;
//   6   the wave-per-record kernel (gcm_wave_kernel);
//   14  the 8-block bitsliced octet kernel alone (aes_gcm_bs8.hip);
//   15  the hybrid octet kernel (T-table + bitsliced waves);
//   16  the T-table lane-per-record kernel (round 1's default).
// Up to this many records a batch runs one record per wavefront; above it the
// hybrid octet kernel, whose floor is one octet job (8 records on one wave,
// ~0.42 ms at 16 KiB): at 16 KiB the two meet between 16 384 and 32 768
// records (profiles/r02/v28_wave_vs_hybrid.txt; against the T-table lane
// kernel it was 196 608, profiles/r01/v31_smallbatch.txt), and the wave
// kernel needs no length planning for mixed batches.
constexpr uint64_t kWaveMaxRecords = 24576;

template <int NR, bool OPEN>
int launch(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    switch (opt(kOptGcmVariant)) {
        case 0:
            if (b.n <= kWaveMaxRecords) return launch_wave<NR, OPEN>(key, b, s);
            // larger batches: the hybrid octet kernel (T-table waves beside
            // bitsliced waves, aes_gcm_bs8.hip): 15.1 / 15.2 ms against the
            // T-table lane kernel's 16.5 / 17.1 at 2^20 x 16 KiB
            // (profiles/r02/v10_gcm_kernel_probe.txt)
            return tg_launch_gcm_hy(key, NR, b, OPEN, s, order);
        case 6: return launch_wave<NR, OPEN>(key, b, s);
        case 14: return tg_launch_gcm_bs8(key, NR, b, OPEN, s, order);
        case 15: return tg_launch_gcm_hy(key, NR, b, OPEN, s, order);
        case 16: return launch_lane<NR, OPEN, !OPEN>(key, b, s, order);
        default: return TG_EINVAL;
    }
}

bool wave_path(uint64_t n) {
    const int v = opt(kOptGcmVariant);
    return v == 6 || (v == 0 && n <= kWaveMaxRecords);
}

}  // namespace
}  // namespace tg

bool tg_gcm_wave_path(uint64_t n) { return tg::wave_path(n); }

int tg_launch_table_hpow(const tg::GcmTableKey* keys, uint64_t n, uint4* hpow, hipStream_t s) {
    const uint64_t groups = (n + 3) / 4;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL(tg::table_hpow_kernel, dim3((unsigned)groups), dim3(256), 0, s, keys, n, hpow);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

int tg_launch_gcm_table_lane(const tg::GcmTableKey* keys, uint64_t nkeys, int rounds, const tg_batch& b,
                             bool open, hipStream_t s, const uint32_t* order, const uint32_t* first) {
    if (rounds == 10)
        return open ? tg::launch_table_v<10, true>(keys, nkeys, b, s, order, first)
                    : tg::launch_table_v<10, false>(keys, nkeys, b, s, order, first);
    if (rounds == 14)
        return open ? tg::launch_table_v<14, true>(keys, nkeys, b, s, order, first)
                    : tg::launch_table_v<14, false>(keys, nkeys, b, s, order, first);
    return TG_EINVAL;
}

int tg_launch_gcm_table_wave(const tg::GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, int rounds,
                             const tg_batch& b, bool open, hipStream_t s, bool t4, const uint32_t* order,
                             const uint32_t* count) {
#define TG_TW(NR, OP, T)                                                                           \
    return tg::launch_table_wave<NR, OP, T>(keys, nkeys, hpow, b, s, order, count)
    if (rounds == 10) {
        if (open) { if (t4) TG_TW(10, true, true); TG_TW(10, true, false); }
        if (t4) TG_TW(10, false, true);
        TG_TW(10, false, false);
    }
    if (rounds == 14) {
        if (open) { if (t4) TG_TW(14, true, true); TG_TW(14, true, false); }
        if (t4) TG_TW(14, false, true);
        TG_TW(14, false, false);
    }
#undef TG_TW
    return TG_EINVAL;
}

int tg_launch_gcm(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                  hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch<10, true>(key, b, s, order) : tg::launch<10, false>(key, b, s, order);
    if (rounds == 14)
        return open ? tg::launch<14, true>(key, b, s, order) : tg::launch<14, false>(key, b, s, order);
    return TG_EINVAL;
}
