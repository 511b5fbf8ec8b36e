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
//   * the tag mask E_K(J0) is one byte-wise AES block (S-box in LDS at ``sbox``).
// LDS: the H^8 tables (64 KiB) + S-box + 4 KiB of record planes per 512-thread
// workgroup, two workgroups per CU.
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "aes_bs8.h"
#include "aes_round.h"
#include "gcm_lane.h"
#include "ghash.h"
#include "options.h"

namespace tg {
namespace {

// Per-wave LDS of octet_job: the first-state planes of each record (128 B per
// record slot, up to 8) at recw, and round 1's S-box output of their rows 0
// and 1 (64 B per slot) at recw + 1024.
constexpr uint32_t kRecArea = 1536;

constexpr int kBs8Threads = 512;
constexpr int kBs8Recs = kBs8Threads / 8;               // record slots per workgroup
constexpr uint32_t kTeBase = 65536;                       // hybrid kernel: Te0/Te2 copies
constexpr uint32_t kBs8Sbox = 65536;                      // 256-byte S-box
constexpr uint32_t kBs8Jt = 65536 + 256;                  // gmul_rot lane-offset rows (256 B)
constexpr uint32_t kBs8Keys = kBs8Jt + 256;               // round-key planes (bs8::KeyPlanesLds)
constexpr uint32_t kBs8RecBase = kBs8Keys + 2048;          // kRecArea per wave (octet_job)
constexpr size_t kBs8Lds = kBs8RecBase + (kBs8Threads / 64) * kRecArea;

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

// Measurement build TG_ROLE_PROBE (tools/role_probe.py): wave-cycles of the
// single-key hybrid's octet jobs by role and phase, from s_memtime stamps at
// the phase boundaries -- 0 record setup (counter cache / first-state planes,
// AAD GHASH), 1 keystream (T-table halves / bitsliced cipher), 2 consume
// (payload loads, XOR, stores, GHASH chain), 3 tail (length block, lift,
// reduction, tag), 4 queue grab (the atomicAdd, gcm_hy_kernel) -- plus jobs,
// blocks, and each wave's span from its first grab to its exit.  Summed over
// the dispatch with atomics; printed by role_probe_print.
#if defined(TG_ROLE_PROBE)
__device__ unsigned long long g_rp[2][10];   // [T-table role][phase 0-4, jobs, blocks, span, waves, spare]
struct RoleProbe {
    uint64_t last = 0;
    uint64_t acc[4] = {0, 0, 0, 0};
    __device__ __forceinline__ void start() { last = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        acc[k] += t - last;
        last = t;
    }
    __device__ __forceinline__ void flush(bool trole, uint32_t blocks) {
        if ((threadIdx.x & 63u) == 0) {
            for (int k = 0; k < 4; ++k) atomicAdd(&g_rp[trole][k], (unsigned long long)acc[k]);
            atomicAdd(&g_rp[trole][5], 1ull);
            atomicAdd(&g_rp[trole][6], (unsigned long long)blocks);
        }
    }
};
__global__ void role_probe_print() {
    for (int r = 0; r < 2; ++r) {
        printf("ROLE_PROBE role %s setup %llu cipher %llu consume %llu tail %llu grab %llu jobs %llu blocks %llu span %llu waves %llu\n",
               r ? "ttable" : "bitsliced", g_rp[r][0], g_rp[r][1], g_rp[r][2], g_rp[r][3], g_rp[r][4], g_rp[r][5],
               g_rp[r][6], g_rp[r][7], g_rp[r][8]);
        for (int k = 0; k < 10; ++k) g_rp[r][k] = 0;
    }
}
#else
struct RoleProbe {
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(bool, uint32_t) {}
};
#endif

// The T-table keystream of half h of a lane's batch: counters c0 + 8 j,
// j = 4 h .. 4 h + 3, in lock step (one round-key read per round for the four), through
// the 256-counter window cache (aes_round.h) when no lane of the wave crosses
// a window in this batch (a wave-uniform test), else full rounds.  Round keys
// are read from LDS (wave-uniform address: one broadcast ds_read_b128 per
// round), which keeps the 44 / 60 key words out of the SGPR file.
// The hybrid kernel's T-table columns of rounds 2 .. NR - 1 take the round keys
// rotated right by 8 bits (aes_round.h col_r, one XOR per column fewer), from
// a wave-uniform global copy the setup kernel writes (RkLds::rot: scalar
// loads, so the LDS pipe the T-table waves are bound by carries no key reads).

// LPR: the lanes per record of the job -- a lane's blocks are LPR apart (8:
// the single-key hybrid's octets; 32: the key-table hybrid's pairs).
template <int NR, int LPR = 8, class RK = RkLds>
__device__ __forceinline__ void t_half(uint32_t lane4, const RK& rk, const CtrCache& cc,
                                       uint32_t c0, bool win, const uint4& wc, uint32_t k0w, int h,
                                       uint4 (&ks)[4]) {
    uint32_t s[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t ctr = c0 + (uint32_t)LPR * (4 * h + q);
        if (win) {   // rounds 1-2 from the window constants (aes_ctr_win)
            const uint32_t A = cc.k0 ^ rotl32(T2<3>((ctr << 24) ^ k0w, lane4), 8);
            s[q][0] = wc.x ^ T0<0>(A, lane4);
            s[q][1] = wc.y ^ rotl32(T2<3>(A, lane4), 8);
            s[q][2] = wc.z ^ T2<2>(A, lane4);
            s[q][3] = wc.w ^ rotl32(T0<1>(A, lane4), 8);
        } else {     // round 1 from the record cache, then round 2 (aes_ctr_w)
            const uint32_t s3 = bswap32(ctr) ^ k0w;
            const uint32_t a0 = cc.k0 ^ rotl32(T2<3>(s3, lane4), 8);
            const uint32_t a1 = cc.k1 ^ T2<2>(s3, lane4);
            const uint32_t a2 = cc.k2 ^ rotl32(T0<1>(s3, lane4), 8);
            const uint32_t a3 = cc.k3 ^ T0<0>(s3, lane4);
            const uint4 k = rk.rot[2];
            s[q][0] = col_r(a0, a1, a2, a3, k.x, lane4);
            s[q][1] = col_r(a1, a2, a3, a0, k.y, lane4);
            s[q][2] = col_r(a2, a3, a0, a1, k.z, lane4);
            s[q][3] = col_r(a3, a0, a1, a2, k.w, lane4);
        }
    }
    // two rounds per iteration: fully unrolled, the T-table code did not fit
    // the instruction cache beside the bitsliced role's; one
    // round per iteration measured 1.3 % slower than two (measurement builds:
    // TG_T_UNROLL, TG_T_UNROLL1)
#if defined(TG_T_UNROLL)
#pragma unroll
#elif defined(TG_T_UNROLL1)
#pragma unroll 1
#else
#pragma unroll 2
#endif
    for (int r = 3; r < NR; ++r) {
        const uint4 k = rk.rot[r];   // rotr8 of round key r (col_r), scalar loads
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t t0 = col_r(s[q][0], s[q][1], s[q][2], s[q][3], k.x, lane4);
            const uint32_t t1 = col_r(s[q][1], s[q][2], s[q][3], s[q][0], k.y, lane4);
            const uint32_t t2 = col_r(s[q][2], s[q][3], s[q][0], s[q][1], k.z, lane4);
            const uint32_t t3 = col_r(s[q][3], s[q][0], s[q][1], s[q][2], k.w, lane4);
            s[q][0] = t0; s[q][1] = t1; s[q][2] = t2; s[q][3] = t3;
        }
    }
    const uint4 k = rk.rot[NR + 1];   // the plain last round key, after the rotated ones
#pragma unroll
    for (int q = 0; q < 4; ++q)
        ks[q] = make_uint4(col_last(s[q][0], s[q][1], s[q][2], s[q][3], k.x, lane4),
                           col_last(s[q][1], s[q][2], s[q][3], s[q][0], k.y, lane4),
                           col_last(s[q][2], s[q][3], s[q][0], s[q][1], k.z, lane4),
                           col_last(s[q][3], s[q][0], s[q][1], s[q][2], k.w, lane4));
}

// Key contexts of octet_job: the round-key words (GcmKeyDev / GcmTableKey
// ``rk`` layout), H^e in normal order for the lift, and y * H^8 for the
// stride-8 Horner.
struct SingleKeyCtx {   // one key for the batch: 8-bit H^8 tables in LDS (gmul_rot)
    const GcmKeyDev* key;
    uint32_t jt;
    __device__ __forceinline__ const uint32_t* rk() const { return key->rk; }
    __device__ __forceinline__ uint4 hpow(int e) const { return key->hpow[e - 1]; }
    __device__ __forceinline__ uint4 gmul(uint4 y) const { return gmul_rot(y, threadIdx.x & 15u, jt); }
    // y * H^8 ^ x: Horner's step with the input folded into the XOR tree
    __device__ __forceinline__ uint4 gmulx(uint4 y, uint4 x) const { return gmul_rot(y, threadIdx.x & 15u, jt, x); }
    __device__ __forceinline__ const uint4* masks() const { return nullptr; }
};
// SingleKeyCtx with the lane's offset row held in registers (the hybrid
// kernel's waves of both roles: one ds_read_b128 fewer per block; T-table
// waves ~0.3 %, profiles/r02/v52_ghash_row/; bitsliced ~0.5 %, v76_bs_row/)
struct SingleKeyRowCtx {
    const GcmKeyDev* key;
    uint4 jw;
    const uint4* mt = nullptr;   // per slot E_K(J0) (hy_mask_kernel), or computed per record
    uint32_t tid = threadIdx.x;  // (gcm_hy_kernel passes it through an empty asm per job)
    __device__ __forceinline__ const uint32_t* rk() const { return key->rk; }
    __device__ __forceinline__ uint4 hpow(int e) const { return key->hpow[e - 1]; }
    __device__ __forceinline__ uint4 gmul(uint4 y) const { return gmul_rot_j(y, tid & 15u, jw); }
    __device__ __forceinline__ uint4 gmulx(uint4 y, uint4 x) const { return gmul_rot_j(y, tid & 15u, jw, x); }
    __device__ __forceinline__ const uint4* masks() const { return mt; }
};
struct TableKeyCtx {    // a key of a key table: the wave's 4-bit H^8 tables in LDS (gmul4)
    const uint32_t* rkw;
    const uint4* hp;    // H^1 .. H^64 of this key (tg_launch_table_hpow)
    uint32_t tab;
    const uint4* mt = nullptr;   // per plan slot E_K(J0) (kt_mask_kernel), or computed per record
    __device__ __forceinline__ const uint32_t* rk() const { return rkw; }
    __device__ __forceinline__ const uint4* masks() const { return mt; }
    __device__ __forceinline__ uint4 hpow(int e) const { return hp[e - 1]; }
#if defined(TG_KT_NO_GHASH)   // measurement build: no GHASH multiply (wrong tags)
    __device__ __forceinline__ uint4 gmul(uint4 y) const { return y; }
#else
    __device__ __forceinline__ uint4 gmul(uint4 y) const { return gmul4(y, tab); }
#endif
#if defined(TG_KT_NO_GHASH)
    __device__ __forceinline__ uint4 gmulx(uint4 y, uint4 x) const { return xor4(y, x); }
#else
    __device__ __forceinline__ uint4 gmulx(uint4 y, uint4 x) const { return gmul4(y, tab, x); }
#endif
};

// One octet job: the eight records of record slots t0 .. t0 + 7 on this wave
// (lane 8 q + l = lane l of slot t0 + q).  TROLE: the keystream comes from the
// T-table cipher (aes_round.h, Te tables at kTeBase, round keys in SGPRs)
// instead of the bitsliced one; everything else is shared.  ``recb``: this
// wave's 1 KiB of LDS for the records' first-state planes.
// LPR (lanes per record, 8 / 16 / 32 / 64; bitsliced only above 8): the same
// job with a group of LPR lanes per record and 64 / LPR records per wave --
// lane l of a group owns the GHASH positions l, l + LPR, ... (stride H^LPR:
// kc.gmul multiplies by H^LPR), batch beta of the lane holds its blocks
// rho + LPR (8 beta + j), j = 0..7, so each load / store instruction still
// moves LPR x 16 consecutive bytes per record (whole 128-byte lines).
template <int NR, bool OPEN, bool TROLE, class KM, class KC, bool PRE = false, int LPR = 8,
          class RKT = RkLds>
__device__ __forceinline__ void octet_job(const KC& kc, const tg_batch& b,
                                          const uint32_t* __restrict__ order, uint64_t t0,
                                          uint32_t recw, const RKT& rkT, uint32_t sbox,
                                          const KM& km, uint32_t tid = threadIdx.x) {
    static_assert(LPR == 8 || LPR == 16 || LPR == 32 || LPR == 64, "lanes per record");
    static_assert(LPR == 8 || LPR == 32 || !TROLE, "the T-table role runs octets or pairs");
    constexpr uint32_t kM = LPR - 1, kS = LPR == 8 ? 3 : LPR == 16 ? 4 : LPR == 32 ? 5 : 6;
    const uint32_t* rk = kc.rk();
    // payload loads and stores with the non-temporal hint: read or written
    // once, they no longer push the tables, key rows and per-key material out
    // of L2 (single key: AES-128-GCM seal / open -1.6 / -1.3 %,
    // profiles/r05/r5l/; key table: config 4 +1.5 %, FETCH_SIZE -4 to -6 %,
    // r5k/)
    constexpr bool kNt = true;
    // the bitsliced role's short last batches on a T-table half (key-table
    // hybrid: its bitsliced waves get the job key's rotated copy too)
    constexpr bool kShortT = !TROLE && LPR == 32 && std::is_same<RKT, RkTab>::value;
#if !defined(TG_KT_SHORT_MAX)
#define TG_KT_SHORT_MAX 5   // A/B builds: 7 / 8 measured 0.5 % slower (profiles/r05/r5v/)
#endif
    constexpr uint32_t kShortMax = TG_KT_SHORT_MAX;
    RoleProbe pr;   // (measurement build TG_ROLE_PROBE; otherwise empty)
    if constexpr (LPR == 8) pr.start();
    const uint32_t lane = tid & 63u;
    const uint32_t l = lane & kM;
    const uint64_t t = t0 + (lane >> kS);
    const bool valid = t < b.n;
    const uint64_t i = valid ? (order ? gld(order, t) : t) : 0;
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
    const uint32_t nfull = len >> 4, tail = len & 15, nc = (len + 15) >> 4, na = (alen + 15) >> 4;
    const uint32_t rho = (l + nc + 1u) & kM;   // this lane's ciphertext blocks: rho + LPR v
    const uint32_t recb = recw + (lane >> kS) * 128u;
    // rows 0-1 after round 1's SubBytes, behind the (64 / LPR) records' planes
    const uint32_t rsub = recw + (64u >> kS) * 128u + (lane >> kS) * 64u;
    const uint32_t lane4 = ((lane & 31u) << 2) | kTeBase;
    CtrCache cc = {0, 0, 0, 0};
    if (TROLE) {
        cc = ctr_cache<NR>(lane4, rkT, nv);
    } else {   // the record's first-state planes 4 l .. 4 l + 3 (nonce ^ rk0 spread to bytes)
        const uint32_t u[4] = {nv.x ^ rk[0], nv.y ^ rk[1], nv.z ^ rk[2], rk[3]};
        const uint32_t e = 4 * (l & 7u);
        const uint4 rp = make_uint4(bs8::rec_plane(u, e), bs8::rec_plane(u, e + 1),
                                    bs8::rec_plane(u, e + 2), bs8::rec_plane(u, e + 3));
        if (l < 8) lds_st128(recb + 16u * l, rp);   // read back by the same wave (in order per wave)
        __builtin_amdgcn_wave_barrier();
        // rows 0 and 1 hold no counter byte below 2^16 (bs8::encrypt, sub01):
        // their round-1 SubBytes once per record, lane l % 2 doing row l % 2
        uint32_t r[8];
        const uint4 a = lds_u128(recb + 32u * (l & 1u)), c = lds_u128(recb + 32u * (l & 1u) + 16u);
        r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = c.x; r[5] = c.y; r[6] = c.z; r[7] = c.w;
        bs::sbox(r);
        if (l < 2) {
            lds_st128(rsub + 32u * l, make_uint4(r[0], r[1], r[2], r[3]));
            lds_st128(rsub + 32u * l + 16u, make_uint4(r[4], r[5], r[6], r[7]));
        }
        __builtin_amdgcn_wave_barrier();
    }
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint32_t nvl = nc > rho ? (nc - rho + kM) >> kS : 0u;         // blocks of this lane
    const uint32_t nfl = nfull > rho ? (nfull - rho + kM) >> kS : 0u;   // full ones
    const uint32_t nbatch = wave_max_u32((nvl + 7u) >> 3);
    // batches in which every valid lane of the wave has all eight blocks full
    // (any alignment: the fast path's accesses are gload16u / gstore16u)
    const uint32_t nfast = wave_min_u32(valid ? nfl >> 3 : 0xffffffffu);
    // per-slot precomputed keystream blocks: E_K(J0) at 2 t, the last block's
    // at 2 t + 1 when the record's last batch holds only that block
    const uint4* mt = kc.masks();

    // GHASH over this lane's AAD positions (aesgcm.py:69-79), zero-padded blocks
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t a = (l + na + nc + 1u) & kM; a < na; a += LPR) {
        const uint32_t m = alen - 16 * a < 16 ? alen - 16 * a : 16;
        y = kc.gmulx(y, load_partial(ad + 16 * a, m));
    }
    if constexpr (LPR == 8) pr.mark(0);

    // the bitsliced cipher leaves out the last round key (folded into the XOR)
    // (KeyPlanesVec: by a vector load, so consume()'s 3-input XORs take it
    // from VGPRs at full rate instead of from SGPRs at half rate)
    uint4 rkl = make_uint4(0, 0, 0, 0);
    if constexpr (!TROLE) {
        if constexpr (bs8::round_rows<KM>()) {
            const uint4 v = gload16(reinterpret_cast<const uint8_t*>(rk + 4 * NR) + km.zv);
            rkl = make_uint4(v.x ^ 0x63636363u, v.y ^ 0x63636363u, v.z ^ 0x63636363u, v.w ^ 0x63636363u);
        } else {
            rkl = make_uint4(rk[4 * NR] ^ 0x63636363u, rk[4 * NR + 1] ^ 0x63636363u,
                             rk[4 * NR + 2] ^ 0x63636363u, rk[4 * NR + 3] ^ 0x63636363u);
        }
    }
    // XOR + store of N consecutive slots j0 .. j0 + N - 1 (the keystream dies
    // block by block), then the GHASH chain over their inputs
    // pre: the slots' payload already loaded (fast path only), else nullptr
    auto consume = [&](const uint4* ks, uint32_t blk0, int j0, auto NN, const uint4* pre) {
        constexpr int N = decltype(NN)::value;
        if (blk0 < (nfast << (kS + 3))) {   // every valid lane of the wave has these blocks full
            if (valid) {
                uint4 d[N];
#pragma unroll
                for (int q = 0; q < N; ++q)
                    d[q] = pre ? pre[q]
                               : kNt ? gload16u_nt(in + 16u * (blk0 + LPR * (j0 + q)))
                                     : gload16u(in + 16u * (blk0 + LPR * (j0 + q)));
#pragma unroll
                for (int q = 0; q < N; ++q) {
                    const uint4 k = ks[q];
                    const uint4 c = make_uint4(xor3(d[q].x, k.x, rkl.x), xor3(d[q].y, k.y, rkl.y),
                                               xor3(d[q].z, k.z, rkl.z), xor3(d[q].w, k.w, rkl.w));
                    if constexpr (kNt)
                        gstore16u_nt(out + 16u * (blk0 + LPR * (j0 + q)), c);
                    else
                        gstore16u(out + 16u * (blk0 + LPR * (j0 + q)), c);
                    if (!OPEN) d[q] = c;
                }
#pragma unroll
                for (int q = 0; q < N; ++q) y = kc.gmulx(y, d[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint32_t blk = blk0 + LPR * (j0 + q);
                if (!valid || blk >= nc) continue;
                const uint4 k = ks[q];
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
                y = kc.gmulx(y, OPEN ? d : c);
            }
        }
    };
    for (uint32_t beta = 0; beta < nbatch; ++beta) {
        const uint32_t blk0 = rho + 8u * LPR * beta;   // block of slot j: blk0 + LPR j
        const uint32_t c0 = 2u + blk0;                  // its counter: c0 + LPR j
        // A batch in which no lane has more than one (four) of its blocks
        // left -- the last one of a record of 64 q + 1 blocks, e.g. a full TLS
        // 1.3 record's 16 385-byte inner plaintext -- runs one block per lane
        // (one T-table half) instead of eight (two).  Seal only on the
        // bitsliced waves: in the open kernel the extra path's registers
        // spill elsewhere and cost 2 % (profiles/r02/v66_one_block/).
        const bool one = !OPEN && __all(!valid || nvl <= 8u * beta + 1u);
        // the same batch when its one block per lane is the record's last and
        // the launch precomputed that block's keystream (mask kernels, slot
        // 2 t + 1): no cipher at all, either role.  Seal only: in the open
        // kernel the path cost registers (spills) and time
        // (profiles/r04/r4p/).
        if (!OPEN && mt && __all(!valid || nvl <= 8u * beta || (nvl == 8u * beta + 1u && blk0 == nc - 1u))) {
            uint4 ks[1] = {rkl};
            if (valid && nvl == 8u * beta + 1u) {
                // the lanes' rho mapping puts a lone last block on lane rho = 0,
                // i.e. nc = 8 LPR beta + 1: the slot the mask kernels wrote
#if defined(TG_DEBUG_ASSERT)
                assert(lone_last_block<LPR>(nc));
#endif
                ks[0] = xor4(gload16(reinterpret_cast<const uint8_t*>(mt + 2 * t + 1)), rkl);
            }
            consume(ks, blk0, 0, std::integral_constant<int, 1>(), nullptr);
        } else if (TROLE) {
            // through the 256-counter window cache when no lane of the wave
            // crosses a window in this batch (wave-uniform); two halves of four.
            // Octets: one window for the batch's counters c0 .. c0 + 56; pairs
            // (LPR 32): a window per half, c0 + 128 h .. c0 + 128 h + 96.
            const bool win = __all(((c0 ^ (c0 + 7u * LPR)) >> 8) == 0);
            const uint32_t k0w = rkT.get(0).w;
            const uint4 wc = LPR == 8 && win ? win_consts<NR>(lane4, rkT, cc, c0) : make_uint4(0, 0, 0, 0);
#if defined(TG_T_UNROLL)
#pragma unroll
#else
#pragma unroll 1
#endif
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && __all(!valid || nvl <= 8u * beta + 4u)) break;
                uint4 ks[4];
                // the half's payload is loaded before its keystream is computed
                // (1.3 / 0.6 % for seal / open, profiles/r02/v70_tprefetch/)
                uint4 dp[4];
                const bool fast = blk0 < (nfast << (kS + 3));
                if (fast && valid) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        dp[q] = kNt ? gload16u_nt(in + 16u * (blk0 + LPR * (4 * h + q)))
                                    : gload16u(in + 16u * (blk0 + LPR * (4 * h + q)));
                }
                if constexpr (LPR == 8) {
                    t_half<NR>(lane4, rkT, cc, c0, win, wc, k0w, h, ks);
                } else {
                    const uint32_t ch = c0 + 4u * LPR * h;
                    const bool winh = __all(((ch ^ (ch + 3u * LPR)) >> 8) == 0);
                    const uint4 wch = winh ? win_consts<NR>(lane4, rkT, cc, ch) : make_uint4(0, 0, 0, 0);
                    t_half<NR, LPR>(lane4, rkT, cc, c0, winh, wch, k0w, h, ks);
                }
                if constexpr (LPR == 8) pr.mark(1);
                consume(ks, blk0, 4 * h, std::integral_constant<int, 4>(), fast ? dp : nullptr);
                if constexpr (LPR == 8) pr.mark(2);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (!OPEN && one) {
            // slot 0 only: E_K(nonce || c0) byte-wise (the tag mask's path);
            // consume() XORs the last round key again
            const uint4 nvr = valid ? load_partial(b.nonce + 12 * i, 12) : make_uint4(0, 0, 0, 0);
            uint4 ks[1] = {xor4(aes_block_sb<NR>(rk, make_uint4(nvr.x, nvr.y, nvr.z, bswap32(c0)), sbox), rkl)};
            consume(ks, blk0, 0, std::integral_constant<int, 1>(), nullptr);
        } else if (kShortT && __all(!valid || nvl < 8u * beta + kShortMax)) {
            // bitsliced role, a record's last batch with fewer than
            // kShortMax blocks per lane: T-table halves (the T-table role's
            // code, its Te copies and rotated key) instead of eight bitsliced
            // blocks; the keystream is final, so the bitsliced
            // last-round-key term that consume() adds is added here once more
            // to cancel it
            const CtrCache cct = ctr_cache<NR>(lane4, rkT, nv);
#pragma unroll 1
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && __all(!valid || nvl <= 8u * beta + 4u)) break;
                const uint32_t ch = c0 + 4u * LPR * h;
                const bool winh = __all(((ch ^ (ch + 3u * LPR)) >> 8) == 0);
                const uint4 wch = winh ? win_consts<NR>(lane4, rkT, cct, ch) : make_uint4(0, 0, 0, 0);
                uint4 ks[4];
                t_half<NR, LPR>(lane4, rkT, cct, c0, winh, wch, rkT.get(0).w, h, ks);
#pragma unroll
                for (int q = 0; q < 4; ++q) ks[q] = xor4(ks[q], rkl);
                consume(ks, blk0, 4 * h, std::integral_constant<int, 4>(), nullptr);
            }
        } else {
            // counters of this batch below 2^16 (wave-uniform): rows 0-1
            // come in after round 1's SubBytes (bs8::encrypt sub01)
            const bool hi = (beta + 1u) >> (16 - (kS + 3));
            uint32_t s[4][8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint4 v = lds_u128((q < 4 && !hi ? rsub : recb) + 16u * q);
                s[q >> 1][4 * (q & 1) + 0] = v.x;
                s[q >> 1][4 * (q & 1) + 1] = v.y;
                s[q >> 1][4 * (q & 1) + 2] = v.z;
                s[q >> 1][4 * (q & 1) + 3] = v.w;
            }
            uint32_t lanec[kS + 3], kmask;
            bs8::lane_consts<kS>(c0, lanec, kmask);
#pragma unroll
            for (int bb = 0; bb < (int)kS + 3; ++bb) s[3 - (bb >> 3)][bb & 7] ^= lanec[bb];
            bs8::ctr_planes<kS + 3, 16, kS + 3>(s, kmask, beta);
            if (hi) bs8::ctr_planes<16, 32, kS + 3>(s, kmask, beta);
            // PRE: the batch's payload is loaded before the cipher runs, so
            // the XOR does not wait for HBM (32 VGPRs live across encrypt():
            // only at three waves per SIMD; at four the seal kernel spilled
            // 270 registers)
            uint4 dp[8];
            const bool pre = PRE && blk0 < (nfast << (kS + 3));
            if (pre && valid) {
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    dp[q] = kNt ? gload16u_nt(in + 16u * (blk0 + LPR * q)) : gload16u(in + 16u * (blk0 + LPR * q));
            }

            uint32_t w[4][8];
            bs8::encrypt<NR>(s, km, w, hi);
            uint4 ks[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) ks[j] = make_uint4(w[0][j], w[1][j], w[2][j], w[3][j]);
            if constexpr (LPR == 8) pr.mark(1);
            consume(ks, blk0, 0, std::integral_constant<int, 8>(), pre ? dp : nullptr);
            if constexpr (LPR == 8) pr.mark(2);
        }
    }
    if constexpr (LPR == 8) pr.mark(2);
#if defined(TG_ROLE_PROBE)
    uint32_t pblk = (valid && l == 0) ? nc : 0u;
    for (int m = 8; m < 64; m <<= 1) pblk += (uint32_t)__shfl_xor((int)pblk, m, 64);
#endif
    if (!__any(valid)) {
#if defined(TG_ROLE_PROBE)
        if constexpr (LPR == 8) pr.flush(TROLE, pblk);
#endif
        return;
    }
    // length block be64(8 alen) || be64(8 len) (aesgcm.py:64): the last position
    if (l == kM) {
        const uint64_t abits = (uint64_t)alen << 3, cbits = (uint64_t)len << 3;
        y = kc.gmulx(y, make_uint4(bswap32((uint32_t)(abits >> 32)), bswap32((uint32_t)abits),
                                     bswap32((uint32_t)(cbits >> 32)), bswap32((uint32_t)cbits)));
    }
    // E_K(J0) precomputed per slot (slot 2 t; hy_mask_kernel, kt_mask_kernel),
    // loaded here so the lift below covers the load
    uint4 mask = make_uint4(0, 0, 0, 0);
    if (mt && valid) mask = gload16(reinterpret_cast<const uint8_t*>(mt + 2 * t));
    // lift by H^(LPR - l) and XOR-reduce over the record's lanes
    uint4 yn = norm4(y);
    if (yn.x | yn.y | yn.z | yn.w) yn = gf128_mul(yn, kc.hpow(LPR - l));
#pragma unroll
    for (int m = 1; m < LPR; m <<= 1) yn = xor4(yn, shfl_xor4(yn, m));
    // tag = GHASH ^ E_K(J0), J0 = nonce || be32(1) (aesgcm.py:112-122)
    if (!mt) {
        if (valid) nv = load_partial(b.nonce + 12 * i, 12);   // reloaded: not held across the loop
        mask = TROLE ? aes_ctr<NR>(lane4, rkT, cc, 1u)
                     : aes_block_sb<NR>(rk, make_uint4(nv.x, nv.y, nv.z, bswap32(1u)), sbox);
    }
    const uint4 tag = xor4(norm4(yn), mask);
    const bool tag_aligned = aligned && tail == 0;
    if (!OPEN) {
        if (valid && l == 0) store16(out + len, tag, tag_aligned);
#if defined(TG_ROLE_PROBE)
        if constexpr (LPR == 8) {
            pr.mark(3);
            pr.flush(TROLE, pblk);
        }
#endif
        return;
    }
    // open: compare before releasing (aesgcm.py:148-149, constanttime.py:209-218)
    uint32_t diff = 0;
    if (valid && l == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status) gst(b.status, i, (uint8_t)(diff == 0));
    }
    diff = (uint32_t)__shfl((int)diff, (int)(lane & ~kM & 63u), 64);
    if (valid && diff) {   // a rejected record's plaintext is zeroed: each lane its own blocks
        // (rho from a fresh lane index: held until here, it was the open
        // kernel's last spill)
        const uint32_t rz = ((fresh_lane() & kM) + nc + 1u) & kM;
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t blk = rz; blk < nfull; blk += LPR) store16(out + 16u * blk, z, aligned);
        if (tail && (nfull & kM) == rz) store_partial(out + 16u * nfull, z, tail);
    }
#if defined(TG_ROLE_PROBE)
    if constexpr (LPR == 8) {
        pr.mark(3);
        pr.flush(TROLE, pblk);
    }
#endif
}

__device__ __forceinline__ void stage_sbox(uint32_t base) {
    if (threadIdx.x < 64) {   // S(x) = byte 1 of Te0[x]
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v |= ((c_te.te0[4 * threadIdx.x + q] >> 8) & 0xffu) << (8 * q);
        reinterpret_cast<uint32_t*>(g_lds_bs8)[base / 4 + threadIdx.x] = v;
    }
}

// All-bitsliced grid: one job per wave, kBs8Recs records per workgroup.
template <int NR, bool OPEN>
__global__ __launch_bounds__(kBs8Threads, 4) void gcm_bs8_kernel(const GcmKeyDev* __restrict__ key,
                                                                tg_batch b,
                                                                const uint32_t* __restrict__ order) {
    stage_ghash_rot(g_lds_bs8, key->ghash8, kBs8Jt);
    stage_sbox(kBs8Sbox);
    bs8::stage_lds_planes(kBs8Keys, key->bs8mask, NR);
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    octet_job<NR, OPEN, false>(SingleKeyCtx{key, kBs8Jt}, b, order,
                               (uint64_t)blockIdx.x * kBs8Recs + 8u * wave,
                               kBs8RecBase + wave * kRecArea, RkLds{0}, kBs8Sbox,
                               bs8::KeyPlanesLds{kBs8Keys});
}

// ---- hybrid persistent kernel: T-table waves beside bitsliced waves -------
// The T-table cipher is bound by LDS lookups with the VALU ~35 % busy, the
// bitsliced one by the VALU; one workgroup per CU runs both kinds of wave
// (waves 0 .. nt-1 T-table at raised priority, the rest bitsliced), each
// taking octet jobs (8 records) from a global queue until the batch is done,
// so the LDS and the VALU are busy at the same time.
// LDS: H^8 tables [0, 64K), Te0/Te2 copies [64K, 128K), S-box, then 1 KiB of
// record planes per wave.
// 1024 threads = 16 waves = 4 per SIMD at <= 128 VGPRs; 768 = 3 per SIMD
// at <= 168 VGPRs, which lets the bitsliced waves prefetch their payload
// (option hy_threads).
constexpr int kHyThreads = 1024;
constexpr uint32_t kHySbox = 2 * 65536;
constexpr uint32_t kHyRk = kHySbox + 256;               // 15 round keys (16 B each)
constexpr uint32_t kHyJt = kHyRk + 256;                 // gmul_rot lane-offset rows
constexpr uint32_t kHyKeys = kHyJt + 256;               // (unused: round 2's key-plane area)
constexpr uint32_t kHyRecBase = kHyKeys + 2048;
constexpr size_t kHyLds = kHyRecBase + (kHyThreads / 64) * kRecArea;   // for either size
static_assert(kTeBase == 65536, "Te block follows the GHASH tables");

// The batch descriptor is read from memory per job (bp): held in SGPRs
// across the persistent loop it would crowd out the ciphers' own scalars.
// The bitsliced waves read the MixColumns-folded round-key planes from the
// row layout at ``krows`` (compiler-scalarised loads: SGPR operands, 1.3 %
// faster than the plain planes and 3 % faster than LDS-staged ones, whose
// LDS reads compete with the T-table waves; profiles/r02/v58_fold_keys/,
// v25_hy_keys.txt).
#if defined(TG_TAIL_PROBE)   // measurement build: the persistent loop's end spread
__device__ unsigned long long g_tp[8] = {~0ull, 0, ~0ull, 0, 0, 0, 0, 0};
__device__ __forceinline__ void tail_probe_start() {
    if ((threadIdx.x & 63u) == 0) atomicMin(&g_tp[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void tail_probe_end(bool trole) {
    if ((threadIdx.x & 63u) == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMax(&g_tp[1], t);
        atomicMin(&g_tp[2], t);
        atomicAdd(&g_tp[3], t - g_tp[0]);
        atomicAdd(&g_tp[4], 1ull);
        atomicMax(&g_tp[trole ? 5 : 6], t);
    }
}
__global__ void tail_probe_print() {
    const unsigned long long t0 = g_tp[0];
    printf("TAIL_PROBE kernel_us %.1f first_end_us %.1f mean_end_us %.1f last_T_us %.1f last_bs_us %.1f waves %llu\n",
           (g_tp[1] - t0) / 100.0, (g_tp[2] - t0) / 100.0, g_tp[3] / (100.0 * g_tp[4]), (g_tp[5] - t0) / 100.0,
           (g_tp[6] - t0) / 100.0, g_tp[4]);
    g_tp[0] = ~0ull; g_tp[1] = 0; g_tp[2] = ~0ull; g_tp[3] = 0; g_tp[4] = 0; g_tp[5] = 0; g_tp[6] = 0;
}
#endif

// The thread index passes through an empty asm at the top of every job, so
// the per-lane values derived from it (lane fields, LDS row offsets of the
// rotated GHASH tables, T-table copy offsets) are recomputed per job instead
// of being hoisted out of the persistent loop and held across it -- where
// they were spilled to scratch.
// The index itself is rebuilt from the wave number (an SGPR) and the lane's
// mbcnt inside an asm, so no VGPR holds it across the loop either.
#if defined(TG_HY_HOIST)   // A/B builds: the compiler's hoisting (round 5)
__device__ __forceinline__ uint32_t hy_tid(uint32_t) { return threadIdx.x; }
#else
__device__ __forceinline__ uint32_t hy_tid(uint32_t wave) { return (wave << 6) | fresh_lane(); }
#endif
template <int NR, bool OPEN, int THREADS>
__global__ __launch_bounds__(THREADS) void gcm_hy_kernel(const GcmKeyDev* __restrict__ key,
                                                            const tg_batch* __restrict__ bp,
                                                            const uint32_t* __restrict__ order,
                                                            uint32_t* __restrict__ queue,
                                                            uint32_t nt, uint32_t prio,
                                                            const uint4* __restrict__ krows,
                                                            const uint4* __restrict__ rkrot,
                                                            const uint4* __restrict__ masks) {
    stage_ghash_rot(g_lds_bs8, key->ghash8, kHyJt);
    stage_te(reinterpret_cast<uint32_t*>(g_lds_bs8) + kTeBase / 4);
    stage_sbox(kHySbox);
    if (threadIdx.x < 4 * (NR + 1)) reinterpret_cast<uint32_t*>(g_lds_bs8)[kHyRk / 4 + threadIdx.x] = key->rk[threadIdx.x];
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#if defined(TG_TAIL_PROBE)
    tail_probe_start();
#endif
    const uint64_t njobs = (bp->n + 7) / 8;
    const uint32_t recw = kHyRecBase + wave * kRecArea;
#if defined(TG_ROLE_PROBE)
    const uint64_t rp_t0 = __builtin_amdgcn_s_memtime();
    uint64_t rp_grab = 0;
#define RP_GRAB_START const uint64_t rp_g0 = __builtin_amdgcn_s_memtime();
#define RP_GRAB_END rp_grab += __builtin_amdgcn_s_memtime() - rp_g0;
#else
#define RP_GRAB_START
#define RP_GRAB_END
#endif
    if (wave < nt) {
        if (prio) __builtin_amdgcn_s_setprio(1);
        const RkLds rk{kHyRk, rkrot};
        for (;;) {
            RP_GRAB_START
            uint32_t job = 0;
            if ((threadIdx.x & 63u) == 0) job = atomicAdd(queue, 1u);
            job = (uint32_t)__builtin_amdgcn_readfirstlane((int)job);
            RP_GRAB_END
            if (job >= njobs) break;
            asm volatile("" ::: "memory");
            const tg_batch b = *bp;
            const uint32_t tid = hy_tid(wave);
            const uint4 jw = lds_u128(kHyJt + ((tid & 15u) << 4));
            octet_job<NR, OPEN, true>(SingleKeyRowCtx{key, jw, masks, tid}, b, order, 8ull * job, recw, rk,
                                      kHySbox, bs8::KeyPlanesVmemFolded{{krows}}, tid);
        }
    } else {
        // The key rows by scalar loads (SGPR operands: the T gates issue at
        // half rate).  Vector loads into VGPRs (bs8::KeyPlanesVec) measured
        // seal equal and open 3 % slower (spills in the open kernel's loop,
        // profiles/r04/r4a/aes_ab.txt), so they are not used here.
        const RkLds none{0};
        for (;;) {
            RP_GRAB_START
            uint32_t job = 0;
            if ((threadIdx.x & 63u) == 0) job = atomicAdd(queue, 1u);
            job = (uint32_t)__builtin_amdgcn_readfirstlane((int)job);
            RP_GRAB_END
            if (job >= njobs) break;
            asm volatile("" ::: "memory");
            const tg_batch b = *bp;
            const uint32_t tid = hy_tid(wave);
            const uint4 jw = lds_u128(kHyJt + ((tid & 15u) << 4));
            octet_job<NR, OPEN, false, bs8::KeyPlanesVmemFolded, SingleKeyRowCtx, (THREADS < 1024)>(
                SingleKeyRowCtx{key, jw, masks, tid}, b, order, 8ull * job, recw, none, kHySbox,
                bs8::KeyPlanesVmemFolded{{krows}}, tid);
        }
    }
#if defined(TG_TAIL_PROBE)
    tail_probe_end(wave < nt);
#endif
#if defined(TG_ROLE_PROBE)
    if ((threadIdx.x & 63u) == 0) {
        const bool tr = wave < nt;
        atomicAdd(&g_rp[tr][4], (unsigned long long)rp_grab);
        atomicAdd(&g_rp[tr][7], (unsigned long long)(__builtin_amdgcn_s_memtime() - rp_t0));
        atomicAdd(&g_rp[tr][8], 1ull);
    }
#endif
#undef RP_GRAB_START
#undef RP_GRAB_END
}

// Stream-ordered setup of the hybrid kernel's scratch: the job counter and a
// device copy of the batch descriptor.
__global__ void hy_setup_kernel(tg_batch b, uint32_t* queue, tg_batch* bcopy) {
    if (threadIdx.x == 0) {
        *queue = 0;
        *bcopy = b;
    }
}

// E_K(J0) of every record of a single-key batch, by slot t (record order[t]
// or t): a persistent grid of one 1024-thread workgroup per CU, the Te0/Te2
// copies staged once per CU and the round keys in SGPRs, each lane a record
// at a time with the T-table cipher (aes_block).  The hybrid's waves read it
// at the end of each record instead of running a dependent 10- or 14-round
// chain per job (aesgcm.py:112-115).  (A lane per record with the byte-wise
// S-box cipher took 36 us per 2^20 records, profiles/r04/f2/.)
template <int NR>
__global__ __launch_bounds__(1024) void hy_mask_kernel(const GcmKeyDev* __restrict__ key, tg_batch b,
                                                       const uint32_t* __restrict__ order,
                                                       uint4* __restrict__ masks) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_bs8));
    RkRegs<NR> rk;
#pragma unroll
    for (int k = 0; k < 4 * (NR + 1); ++k) rk.w[k] = key->rk[k];
    __syncthreads();
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;   // Te block at LDS 0
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < b.n;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = order ? gld(order, t) : t;
        const uint4 nv = load_partial(b.nonce + 12 * i, 12);
        gstore16(reinterpret_cast<uint8_t*>(masks + 2 * t),
                 aes_block<NR>(lane4, rk, make_uint4(nv.x, nv.y, nv.z, bswap32(1u))));
        // a record whose last batch row (8 x 8 blocks) holds one block -- a
        // full TLS 1.3 record's 16 385-byte inner plaintext -- gets that
        // block's keystream too (counter 2 + nc - 1, octet_job's tail path)
        const uint32_t nc = (rec_len(b, i) + 15) >> 4;
        if (lone_last_block<8>(nc))
            gstore16(reinterpret_cast<uint8_t*>(masks + 2 * t + 1),
                     aes_block<NR>(lane4, rk, make_uint4(nv.x, nv.y, nv.z, bswap32(nc + 1u))));
    }
}

template <int NR, bool OPEN>
int launch_bs8(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    if (lds_attr((const void*)gcm_bs8_kernel<NR, OPEN>, (int)kBs8Lds)) return TG_EHIP;
    const uint64_t groups = (b.n + kBs8Recs - 1) / kBs8Recs;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_bs8_kernel<NR, OPEN>), dim3((unsigned)groups), dim3(kBs8Threads), kBs8Lds, s,
                       key, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// The mask and hybrid kernels of one launch_hy call, on its scratch.
template <int NR, bool OPEN>
int launch_hy_kernels(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order, uint32_t nt,
                      uint32_t prio, bool small, uint32_t* queue, tg_batch* bcopy, uint4* masks) {
    if (masks && b.n) {
        if (lds_attr((const void*)hy_mask_kernel<NR>, 65536)) return TG_EHIP;
        const uint64_t wgs = (b.n + 1023) / 1024, cus = (uint64_t)device_cus();
        const unsigned grid = (unsigned)(wgs < cus ? wgs : cus);   // persistent: at most one per CU
        hipLaunchKernelGGL((hy_mask_kernel<NR>), dim3(grid), dim3(1024), 65536, s, key, b, order, masks);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
    }
    const uint4* krows = reinterpret_cast<const uint4*>(key->bs8rows);
    const uint4* rkrot = reinterpret_cast<const uint4*>(key->rkrot);
    if (small)
        hipLaunchKernelGGL((gcm_hy_kernel<NR, OPEN, 768>), dim3((unsigned)device_cus()), dim3(768), kHyLds, s,
                           key, (const tg_batch*)bcopy, order, queue, nt, prio, krows, rkrot, masks);
    else
        hipLaunchKernelGGL((gcm_hy_kernel<NR, OPEN, 1024>), dim3((unsigned)device_cus()), dim3(1024), kHyLds,
                           s, key, (const tg_batch*)bcopy, order, queue, nt, prio, krows, rkrot, masks);
#if defined(TG_TAIL_PROBE)
    hipLaunchKernelGGL(tail_probe_print, dim3(1), dim3(1), 0, s);
#endif
#if defined(TG_ROLE_PROBE)
    hipLaunchKernelGGL(role_probe_print, dim3(1), dim3(1), 0, s);
#endif
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Options hy_t (T-table waves per workgroup; -1 none) and hy_prio (1: the
// T-table waves at raised priority) are measurement knobs.  Default: 10 of
// the 16 waves run the T-table cipher, all at normal priority -- 1.5 / 1.1 %
// faster seal / open than round 2's 8 at raised priority, every one of six
// alternating rounds (profiles/r03/hysw/); half of the 768-thread variant's.
template <int NR, bool OPEN>
int launch_hy(const GcmKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    if ((b.n + 7) / 8 > 0xffffffffull) return TG_EINVAL;
    const int t = opt(kOptHyT);
    const bool small = opt(kOptHyThreads) == 768;
    const int waves = small ? 12 : 16;
    if (t > waves) return TG_EINVAL;   // more T-table waves than the workgroup has
    // t < 0: bitsliced waves only (measurement)
    const uint32_t nt = t < 0 ? 0u : t > 0 && t <= waves ? (uint32_t)t : small ? 6u : 10u;
    const uint32_t prio = opt(kOptHyPrio) == 1 ? 1u : 0u;
    const void* fn = small ? (const void*)gcm_hy_kernel<NR, OPEN, 768> : (const void*)gcm_hy_kernel<NR, OPEN, 1024>;
    if (lds_attr(fn, (int)kHyLds)) return TG_EHIP;
    // The launch's scratch -- job counter and batch copy (256 bytes), then two
    // 16-byte keystream blocks per record (hy_mask_kernel) -- comes from the
    // per-launch scratch cache (api.hip stream_alloc: a buffer is reused once
    // the launches behind it have completed, or at once on the same stream)
    // and goes back behind the kernel: launches on different streams
    // (hipStreamPerThread included) never share it, and memory is bounded by
    // the launches in flight.  The key rows and rotated round keys come
    // with the key (GcmKeyDev::bs8rows, rkrot).
#if defined(TG_HY_NO_MASK)   // A/B builds: every wave computes its records' masks
    const uint64_t mrec = 0;
#else
    const uint64_t mrec = b.n;
#endif
    uint8_t* scratch = nullptr;
    if (stream_alloc((void**)&scratch, 256 + 32 * mrec, s)) return TG_EHIP;
    uint4* masks = mrec ? reinterpret_cast<uint4*>(scratch + 256) : nullptr;
    uint32_t* queue = reinterpret_cast<uint32_t*>(scratch);
    tg_batch* bcopy = reinterpret_cast<tg_batch*>(scratch + 64);
    hipLaunchKernelGGL(hy_setup_kernel, dim3(1), dim3(64), 0, s, b, queue, bcopy);
    int rc = hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    if (!rc) rc = launch_hy_kernels<NR, OPEN>(key, b, s, order, nt, prio, small, queue, bcopy, masks);
    if (stream_free(scratch, s) && !rc) rc = TG_EHIP;
    return rc;
}


// ---- key tables: key-grouped octet jobs on bitsliced waves ----------------
// A batch over a key table (config 4: many sessions, per-record key_idx) is
// planned into jobs of at most eight records of ONE key (tg_key_job_plan:
// sorted by key, then length descending).  A wave's job then has
// wave-uniform round keys and key planes (scalar loads from the key table and
// the per-key plane table) and one GHASH key: the wave builds 4-bit tables of
// that key's H^8 in its own 8 KiB of LDS (build_table4, ~700 VALU per lane;
// gmul4: 32 conflict-free lookups per block instead of the table-free
// multiply's ~650 VALU slots).  No Te tables (the LDS holds the GHASH
// copies), so every wave runs the bitsliced cipher.
//
// One job per wave, four waves per workgroup, no persistent loop: the jobs of
// a key are consecutive, so a persistent wave would rarely keep its key, and
// a loop around the job body made the compiler hoist its per-lane table and
// plane addresses and spill ~180 VGPRs.  The grid is sized for the most jobs
// a batch of n records over nkeys keys can have (ceil(c_k / 8) per key k:
// at most n / 8 + min(n, nkeys)); workgroups past the planned count exit at
// once.
constexpr int kKtThreads = 256;
constexpr int kKtWaves = kKtThreads / 64;
constexpr uint32_t kKtSbox = kKtWaves * 8192;            // after the per-wave tables
constexpr uint32_t kKtRecBase = kKtSbox + 256;           // kRecArea per wave (octet_job)
constexpr size_t kKtLds = kKtRecBase + kKtWaves * kRecArea;
constexpr int kKtPlaneWords = 15 * 32;                   // per key in the plane table

template <int NR, bool OPEN, int LPR>
__global__ __launch_bounds__(kKtThreads, 4) void gcm_kt_kernel(const GcmTableKey* __restrict__ keys,
                                                            const uint4* __restrict__ hpow,
                                                            const uint32_t* __restrict__ planes,
                                                            tg_batch b,
                                                            const uint32_t* __restrict__ order,
                                                            const uint32_t* __restrict__ jobpos,
                                                            const uint32_t* __restrict__ njobs_p,
                                                            const uint32_t* __restrict__ nlong_p) {
    const uint32_t njobs = *njobs_p;
    if (blockIdx.x * kKtWaves >= njobs) return;   // the whole workgroup (uniform)
    stage_sbox(kKtSbox);
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t job = blockIdx.x * kKtWaves + wave;
    if (job >= njobs) return;
    const uint32_t p0 = gld(jobpos, job), p1 = gld(jobpos, job + 1);
    // the plan's tail (slots >= *nlong) holds the records this kernel leaves
    // to the lane kernel: short ones and out-of-range key indices
    if (p0 >= *nlong_p) return;
    const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)gld(b.key_idx, gld(order, p0)));
    const uint32_t tab = 8192u * wave, recw = kKtRecBase + wave * kRecArea;
#if !defined(TG_KT_NO_BUILD)   // measurement build: tables left as they are (wrong tags)
    build_table4(tab, hpow[64u * k + LPR - 1u]);   // this wave's GHASH tables: the key's H^LPR
#endif
    __builtin_amdgcn_wave_barrier();
    b.n = p1;   // the job's slots are p0 .. p1 - 1 (at most 64 / LPR)
    octet_job<NR, OPEN, false, bs8::KeyPlanesVmemFolded, TableKeyCtx, false, LPR>(
        TableKeyCtx{keys[k].rk, hpow + 64u * k, tab}, b, order, p0, recw, RkLds{0}, kKtSbox,
        bs8::KeyPlanesVmemFolded{{reinterpret_cast<const uint4*>(planes + kKtPlaneWords * k)}});
}

// ---- key tables, long records: T-table waves beside bitsliced waves -------
// The single-key hybrid's two ciphers (gcm_hy_kernel) for a key table: one
// persistent workgroup of 11 waves per CU; waves 0 .. nt - 1 run the T-table
// cipher (Te0/Te2 copies at kTeBase, the job key's round keys by scalar
// loads, its rotated copy from the per-key ``rot`` table), the rest the
// bitsliced one (the key's folded plane rows).  A planned job is up to
// kKthGroup pairs of records of one key (tg_key_job_plan, 32 lanes per
// record, a pair per octet_job); a wave takes kKthChunk planned jobs at a
// time and rebuilds its 4-bit GHASH tables of the key's H^32 (8 KiB,
// build_table4) only when the key changes.  LDS (160 KiB):
// eight waves' tables below the Te block, three above it, the S-box and a
// 384-byte record area per wave (two records' first-state planes and their
// round-1 rows).  11 waves: the Te block and 11 tables fill the LDS (3 waves
// per SIMD on three SIMDs, 2 on the fourth; <= 168 VGPRs).
constexpr int kKthWaves = 11;
constexpr int kKthThreads = kKthWaves * 64;
constexpr uint32_t kKthSbox = 2 * 65536 + 3 * 8192;
constexpr uint32_t kKthRec = kKthSbox + 256;
constexpr uint32_t kKthRecArea = 384;                   // (64 / 32) x 128 + (64 / 32) x 64
constexpr size_t kKthLds = kKthRec + kKthWaves * kKthRecArea;
// A planned job holds up to kKthGroup pairs of one key (the plan's job size
// is 2 kKthGroup records): its waves run them pair by pair with one table
// build.  kKthChunk planned jobs per grab.
#if !defined(TG_KTH_GROUP)
// Round 5 (separate lane kernel, 2 048-byte split): 2 pairs of one key per
// grab 666.6-668.0 GiB/s, 1 pair (two planned per grab) 663.6-665.0, 4 pairs
// 657.7-659.9 (profiles/r05/r5x/).  Round 6, with the short records inside
// this kernel and the 1 024-byte split: 4 pairs 677.6-678.8 / 691.5-693.6
// against 675.3-675.5 / 689.6-689.8 for 2 on two boxes, 8 pairs 671.0
// (profiles/r06/g2/, g3/); 3 is refused by the plan (job sizes are powers
// of two).
#define TG_KTH_GROUP 4
#endif
constexpr uint32_t kKthGroup = TG_KTH_GROUP;
// jobs per grab (1 / 2 / 4 / 8: 607 / 614 / 610 / 590 GiB/s, profiles/r04/r4j)
constexpr uint32_t kKthChunk = kKthGroup == 1 ? 2 : 1;
constexpr int kKthTDefault = 7;
static_assert(kKthLds <= 163840, "key-table hybrid LDS");

__device__ __forceinline__ uint32_t kth_tab(uint32_t w) {
    return w < 8 ? w * 8192u : 2u * 65536u + (w - 8u) * 8192u;
}

// The thread index per pair from a fresh lane index, as in gcm_hy_kernel:
// 154 -> 142 VGPRs, config 4 +0.4 / +0.6 % in two alternations
// (profiles/r06/y3/c4_ab.txt).
#if defined(TG_KTH_HOIST)   // A/B builds: the compiler's hoisting (round 5)
#define KTH_TID(w) threadIdx.x
#else
#define KTH_TID(w) hy_tid(w)
#endif
template <int NR, bool OPEN>
__global__ __launch_bounds__(kKthThreads) void gcm_kth_kernel(const GcmTableKey* __restrict__ keys,
                                                             const uint4* __restrict__ hpow,
                                                             const uint32_t* __restrict__ planes,
                                                             const uint4* __restrict__ rot, tg_batch b,
                                                             const uint32_t* __restrict__ order,
                                                             const uint32_t* __restrict__ jobpos,
                                                             const uint32_t* __restrict__ njobs_p,
                                                             const uint32_t* __restrict__ nlong_p,
                                                             const uint4* __restrict__ masks,
                                                             const uint32_t* __restrict__ jobkey,
                                                             uint32_t* __restrict__ queue, uint32_t nt,
                                                             uint64_t nkeys, uint32_t lanes) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_bs8) + kTeBase / 4);
    stage_sbox(kKthSbox);
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t tab = kth_tab(wave), recw = kKthRec + wave * kKthRecArea;
    const uint32_t njobs = *njobs_p, nlong = *nlong_p;
    uint32_t cur = 0xffffffffu;   // the key whose tables this wave holds
    for (;;) {
        uint32_t j0 = 0;
        if ((threadIdx.x & 63u) == 0) j0 = atomicAdd(queue, kKthChunk);
        j0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)j0);
        if (j0 >= njobs) break;
        const uint32_t j1 = j0 + kKthChunk < njobs ? j0 + kKthChunk : njobs;
        // the chunk's job bounds and keys in one round of loads (jobkey: from
        // the plan, tg_key_job_plan), not a dependent jobpos -> order -> key_idx
        // chain per job
        // (chunk of two: the values by selects, so the loop body -- both
        // roles' code -- exists once)
        const uint32_t pa = gld(jobpos, j0), pb = gld(jobpos, j0 + 1u),
                       pc = kKthChunk > 1 && j0 + 2u <= njobs ? gld(jobpos, j0 + 2u) : 0u;
        const uint32_t ka = gld(jobkey, j0), kb = kKthChunk > 1 && j0 + 1u < njobs ? gld(jobkey, j0 + 1u) : 0u;
        bool tail = false;
        for (uint32_t q = 0; q < j1 - j0; ++q) {
            const uint32_t p0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(q ? pb : pa));
            const uint32_t p1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(q ? pc : pb));
            // the plan's tail (slots >= nlong) is the lane kernel's, and every
            // later job lies in it too
            if (p0 >= nlong) {
                tail = true;
                break;
            }
            const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)(q ? kb : ka));
            if (k != cur) {
                __builtin_amdgcn_wave_barrier();   // the previous job's lookups are done
#if !defined(TG_KT_NO_BUILD)   // measurement build: tables left as they are (wrong tags)
                build_table4(tab, hpow[64u * k + 31u]);
#endif
                cur = k;
                __builtin_amdgcn_wave_barrier();
            }
            const TableKeyCtx kc{keys[k].rk, hpow + 64u * k, tab, masks};
            const bs8::KeyPlanesVmemFolded km{{reinterpret_cast<const uint4*>(planes + kKtPlaneWords * k)}};
            for (uint32_t pp = p0; pp < p1; pp += 2u) {   // the planned job's pairs
                tg_batch bj = b;
                bj.n = pp + 2u < p1 ? pp + 2u : p1;   // the pair's slots are pp .. bj.n - 1
                const uint32_t tid = KTH_TID(wave);
                if (wave < nt)
                    octet_job<NR, OPEN, true, bs8::KeyPlanesVmemFolded, TableKeyCtx, false, 32, RkTab>(
                        kc, bj, order, pp, recw, RkTab{keys[k].rk, rot + 16u * k}, kKthSbox, km, tid);
                else
                    octet_job<NR, OPEN, false, bs8::KeyPlanesVmemFolded, TableKeyCtx, false, 32, RkTab>(
                        kc, bj, order, pp, recw, RkTab{keys[k].rk, rot + 16u * k}, kKthSbox, km, tid);
            }
        }
        if (tail) break;
    }
    // The short records -- plan slots [nlong, n) -- once the long jobs are all
    // taken: one record per lane, 64 per grab, T-table CTR and the table-free
    // GHASH of the lane kernel (gcm_lane.h gcm_record), the lane's 256-counter
    // window slot in this wave's GHASH table area (free from here on).  The
    // CUs then stay busy to the end instead of running a separate lane kernel
    // after the long one (round 6; TG_KTH_LANE_KERNEL: the separate kernel).
    if (lanes) {
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t lane4 = ((lane & 31u) << 2) | kTeBase, win = tab + 16u * lane;
        for (;;) {
            uint32_t c0 = 0;
            if (lane == 0) c0 = atomicAdd(queue + 1, 64u);
            c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)c0);
            if ((uint64_t)nlong + c0 >= b.n) break;
            const uint64_t t = (uint64_t)nlong + c0 + lane;
            if (t >= b.n) continue;
            const uint32_t i = gld(order, t), k = gld(b.key_idx, i);
            if (k >= nkeys) {   // skipped (open: status 0; tg_launch_zero_skipped clears it)
                if (OPEN && b.status) gst(b.status, i, (uint8_t)0);
                continue;
            }
            const GcmTableKey* kp = keys + k;
            RkRegs<NR> rk;   // this record's key: per-lane values
#pragma unroll
            for (int q = 0; q <= NR; ++q) {
                const uint4 v = gload16(reinterpret_cast<const uint8_t*>(kp->rk + 4 * q));
                rk.w[4 * q] = v.x; rk.w[4 * q + 1] = v.y; rk.w[4 * q + 2] = v.z; rk.w[4 * q + 3] = v.w;
            }
            const GhashClmul gh{gload16(reinterpret_cast<const uint8_t*>(kp->hn))};
            gcm_record<NR, OPEN, 1, RkRegs<NR>, GhashClmul, true>(b, i, lane4, rk, gh, win);
        }
    }
}

// E_K(J0) of every long record of a key-table plan, by plan slot (slots
// [0, nlong)): masks[2 t] = E_K(nonce || be32(1)) with the record's key
// (aesgcm.py:112-115).  A persistent grid of one 1024-thread workgroup per CU
// (the Te0/Te2 copies staged once per CU), each lane a record at a time with
// its key's round keys in VGPRs and the T-table cipher (aes_block).  The
// key-table hybrid reads it at the end of each record instead of running a
// dependent 10- or 14-round chain per record and wave.  (A lane per record
// with the byte-wise S-box cipher took 49 us per config-4 launch.)
template <int NR>
__global__ __launch_bounds__(1024) void kt_mask_kernel(const GcmTableKey* __restrict__ keys, tg_batch b,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ nlong_p,
                                                       uint4* __restrict__ masks) {
    stage_te(reinterpret_cast<uint32_t*>(g_lds_bs8));
    __syncthreads();
    const uint32_t lane4 = (threadIdx.x & 31u) << 2;   // Te block at LDS 0
    const uint64_t nlong = *nlong_p;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nlong;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t i = gld(order, t);
        const uint4 nv = load_partial(b.nonce + 12 * (uint64_t)i, 12);
        const uint4* kr = reinterpret_cast<const uint4*>(keys[gld(b.key_idx, i)].rk);
        RkRegs<NR> rk;   // this record's key: per-lane values
#pragma unroll
        for (int q = 0; q <= NR; ++q) {
            const uint4 v = gload16(reinterpret_cast<const uint8_t*>(kr + q));
            rk.w[4 * q] = v.x; rk.w[4 * q + 1] = v.y; rk.w[4 * q + 2] = v.z; rk.w[4 * q + 3] = v.w;
        }
        gstore16(reinterpret_cast<uint8_t*>(masks + 2 * t),
                 aes_block<NR>(lane4, rk, make_uint4(nv.x, nv.y, nv.z, bswap32(1u))));
        // a record whose last batch row (8 x 32 blocks) holds one block: that
        // block's keystream, counter 2 + nc - 1 (octet_job's tail path)
        const uint32_t nc = (rec_len(b, i) + 15) >> 4;
        if (lone_last_block<32>(nc))
            gstore16(reinterpret_cast<uint8_t*>(masks + 2 * t + 1),
                     aes_block<NR>(lane4, rk, make_uint4(nv.x, nv.y, nv.z, bswap32(nc + 1u))));
    }
}

// Per key, the T-table waves' rotated round keys: rot[16 k + r] = rotr8 of
// round key r (r = 0 .. nr, aes_round.h col_r), rot[16 k + nr + 1] = the
// plain last round key (t_half reads it after the rotated ones).
__global__ void kt_rot_kernel(const GcmTableKey* __restrict__ keys, uint64_t n, int nr, uint32_t* __restrict__ rot) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = t / 64;
    const int e = (int)(t % 64);
    if (k >= n) return;
    uint32_t w = 0;
    if (e < 4 * (nr + 1))
        w = rotl32(keys[k].rk[e], 24);
    else if (e < 4 * (nr + 2))
        w = keys[k].rk[e - 4];
    rot[64 * k + e] = w;
}

// Per key, the hybrid kernel's key rows (keymath.h bs8_row_word): the
// MixColumns-folded planes (keymath.h bs8_fold_word) of rounds 1 .. nr - 1 and
// the round-key planes of rounds 0 and nr, row (8 r + bit) = the four rows' words.
__global__ void kt_planes_kernel(const GcmTableKey* __restrict__ keys, uint64_t n, int nr,
                                 uint32_t* __restrict__ planes) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = t / kKtPlaneWords;
    const int e = (int)(t % kKtPlaneWords);
    if (k >= n) return;
    const int r = e >> 5, i = (e >> 3) & 3, bit = e & 7;
    const uint32_t w = e >= 32 * (nr + 1) ? 0u
                       : r >= 1 && r < nr ? bs8_fold_word(keys[k].rk, e) : bs8_mask_word(keys[k].rk, e);
    planes[k * kKtPlaneWords + 4 * (8 * r + bit) + i] = w;
}

// Key-table AES-GCM by record length (BASELINE config 4): records of at
// least ``split`` bytes run the key-grouped octet kernel (long_kernel
// kKtLongOctet) or the key-table wave-per-record kernel with per-wave 4-bit
// GHASH tables (kKtLongWave, aes_gcm.hip), the rest (and
// records whose key_idx is not below nkeys) the lane-per-record kernel
// (aes_gcm.hip gcm_table_vkernel) over the tail of the same plan, which the
// planner leaves sorted by length, longest first.  split 0: every in-range
// record takes the octet kernel; split ~0u: every record the lane kernel.
template <int NR, bool OPEN>
int launch_kth(const GcmTableKey* keys, const uint4* hpow, const uint32_t* planes, const uint4* rot,
               const tg_batch& b, hipStream_t s, const uint32_t* order, const uint32_t* jobpos,
               const uint32_t* njobs, const uint32_t* nlong, uint32_t* queue, uint4* masks,
               uint32_t* jobkey, uint64_t nkeys, bool lanes) {
    const int t = opt(kOptKtT);
    if (t < 0 || t > kKthWaves) return TG_EINVAL;
    const uint32_t nt = t ? (uint32_t)t : (uint32_t)kKthTDefault;
    if (lds_attr((const void*)gcm_kth_kernel<NR, OPEN>, (int)kKthLds)) return TG_EHIP;
    if (hipMemsetAsync(queue, 0, 8, s) != hipSuccess) return TG_EHIP;   // long jobs, lane records
#if defined(TG_KTH_NO_MASK)   // A/B builds: every wave computes its records' masks
    masks = nullptr;
#else
    if (lds_attr((const void*)kt_mask_kernel<NR>, 65536)) return TG_EHIP;
    const uint64_t wgs = (b.n + 1023) / 1024, cus = (uint64_t)device_cus();   // nlong <= n
    hipLaunchKernelGGL((kt_mask_kernel<NR>), dim3((unsigned)(wgs < cus ? wgs : cus)), dim3(1024), 65536, s, keys,
                       b, order, nlong, masks);
#endif
    hipLaunchKernelGGL((gcm_kth_kernel<NR, OPEN>), dim3((unsigned)device_cus()), dim3(kKthThreads), kKthLds, s,
                       keys, hpow, planes, rot, b, order, jobpos, njobs, nlong, masks, jobkey, queue, nt, nkeys,
                       lanes ? 1u : 0u);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

template <int NR, bool OPEN, int LPR>
int launch_kt_jobs(const GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, const uint32_t* planes,
                   const tg_batch& b, hipStream_t s, const uint32_t* order, const uint32_t* jobpos,
                   const uint32_t* njobs, const uint32_t* nlong) {
    if (lds_attr((const void*)gcm_kt_kernel<NR, OPEN, LPR>, (int)kKtLds)) return TG_EHIP;
    // jobs: at most ceil(c_k / R) per distinct key k of the long records (R =
    // 64 / LPR records per job), i.e. n / R + min(n, nkeys), plus the tail's
    // jobs (which exit at once)
    constexpr uint64_t R = 64 / LPR;
    const uint64_t maxjobs = (b.n + R - 1) / R + (nkeys < b.n ? nkeys : b.n) + 1;
    const uint64_t groups = (maxjobs + kKtWaves - 1) / kKtWaves;
    if (groups > 0x7fffffffull) return TG_EINVAL;
    hipLaunchKernelGGL((gcm_kt_kernel<NR, OPEN, LPR>), dim3((unsigned)groups), dim3(kKtThreads), kKtLds, s, keys,
                       hpow, planes, b, order, jobpos, njobs, nlong);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Key-table AES-GCM by record length (BASELINE config 4): records of at
// least ``split`` bytes run the key-grouped bitsliced kernel with lpr lanes
// per record (8: octet jobs of up to eight records of one key; 16 / 32 / 64:
// jobs of 4 / 2 / 1) or, with lpr 0, the key-table wave-per-record kernel
// with per-wave 4-bit GHASH tables (T-table AES, aes_gcm.hip); the rest (and
// records whose key_idx is not below nkeys) the lane-per-record kernel
// (aes_gcm.hip gcm_table_vkernel) over the tail of the same plan, which the
// planner leaves sorted by length, longest first.  split 0: every in-range
// record takes the long kernel; split ~0u: every record the lane kernel.
// The key-table hybrid (lpr 32, the default) runs the lane kernel's routine
// itself over those records once its long jobs are taken: a separate lane
// kernel ran 250-610 us alone after it (round 6, profiles/r06/z3/).  Beside
// the other long kernels the lane kernel runs on a helper stream of the
// caller's stream (api.hip helper_fork / helper_join: idle or last used by
// this caller, so two callers never chain through one helper).  Option
// kt_overlap -1: one stream.
template <int NR, bool OPEN>
int launch_kt(const GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, const uint32_t* planes,
              const uint4* rot, const tg_batch& b, hipStream_t s, uint32_t split, int lpr, bool hybrid) {
    if (b.n == 0) return TG_OK;
    if (b.n > 0xfffffffeull || !b.key_idx) return TG_EINVAL;
    if (lpr != 0 && lpr != 8 && lpr != 16 && lpr != 32 && lpr != 64) return TG_EINVAL;
    // the key-table hybrid plans groups of kKthGroup pairs (gcm_kth_kernel)
    const uint32_t jobsz = lpr ? (64u / (uint32_t)lpr) * (lpr == 32 && hybrid ? kKthGroup : 1u) : 1u;
    size_t plan = 0;
    int rc = tg_key_job_plan(b.key_idx, b.len, b.fixed_len, b.n, nkeys, split, jobsz, nullptr, nullptr,
                             nullptr, nullptr, nullptr, &plan, s);
    if (rc) return rc;
    const size_t so = (b.n * 4 + 255) & ~(size_t)255, sj = ((b.n + 1) * 4 + 255) & ~(size_t)255;
    // the key-table hybrid's per-slot tag masks (kt_mask_kernel) after the plan
    const size_t sm = hybrid && lpr == 32 ? b.n * 32 + (b.n + 1) * 4 : 0;   // + the jobs' keys
    const size_t po = (so + sj + 256 + plan + 255) & ~(size_t)255;
    uint8_t* buf = nullptr;
    if (stream_alloc((void**)&buf, po + sm, s)) return TG_EHIP;
    uint32_t* order = reinterpret_cast<uint32_t*>(buf);
    uint32_t* jobpos = reinterpret_cast<uint32_t*>(buf + so);
    uint32_t* njobs = reinterpret_cast<uint32_t*>(buf + so + sj);
    uint32_t* nlong = njobs + 1;
    uint32_t* jobkey = sm ? reinterpret_cast<uint32_t*>(buf + po + b.n * 32) : nullptr;
    rc = tg_key_job_plan(b.key_idx, b.len, b.fixed_len, b.n, nkeys, split, jobsz, order, jobpos, njobs, nlong,
                         buf + so + sj + 256, &plan, s, jobkey);
    // The short records (plan slots [nlong, n)): the key-table hybrid takes
    // them itself once its long jobs are taken (gcm_kth_kernel).  With the
    // other long kernels they go to the lane kernel, on a helper stream forked
    // after the plan and joined before the scratch goes back (its records are
    // disjoint from the long kernel's; option kt_overlap -1: one stream).
#if defined(TG_KTH_LANE_KERNEL)   // A/B builds: the separate lane kernel beside the hybrid
    const bool kth_lanes = false;
#else
    const bool kth_lanes = hybrid && lpr == 32 && split != 0xffffffffu;
#endif
    hipStream_t s2 = nullptr;
    if (!rc && split != 0xffffffffu && !kth_lanes && opt(kOptKtOverlap) >= 0) rc = helper_fork(s, &s2);
    if (!rc && split != 0xffffffffu) {
        switch (lpr) {
            case 0:   // the long records one per wavefront (plan slots [0, nlong))
                rc = tg_launch_gcm_table_wave(keys, nkeys, hpow, NR, b, OPEN, s, true, order, nlong);
                break;
            case 8: rc = launch_kt_jobs<NR, OPEN, 8>(keys, nkeys, hpow, planes, b, s, order, jobpos, njobs, nlong); break;
            case 16: rc = launch_kt_jobs<NR, OPEN, 16>(keys, nkeys, hpow, planes, b, s, order, jobpos, njobs, nlong); break;
            case 32:
                rc = hybrid ? launch_kth<NR, OPEN>(keys, hpow, planes, rot, b, s, order, jobpos, njobs, nlong,
                                                   njobs + 16, reinterpret_cast<uint4*>(buf + po), jobkey, nkeys,
                                                   kth_lanes)
                            : launch_kt_jobs<NR, OPEN, 32>(keys, nkeys, hpow, planes, b, s, order, jobpos, njobs,
                                                           nlong);
                break;
            default: rc = launch_kt_jobs<NR, OPEN, 64>(keys, nkeys, hpow, planes, b, s, order, jobpos, njobs, nlong); break;
        }
    }
    if (!rc && !kth_lanes) rc = tg_launch_gcm_table_lane(keys, nkeys, NR, b, OPEN, s2 ? s2 : s, order, nlong);
    // rejoin (also after a failed launch: the scratch must outlive both streams' work)
    if (s2 && helper_join(s2, s) && !rc) rc = TG_EHIP;
    if (stream_free(buf, s)) return TG_EHIP;
    return rc;
}

}  // namespace
}  // namespace tg

int tg_launch_gcm_hy(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                     hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch_hy<10, true>(key, b, s, order) : tg::launch_hy<10, false>(key, b, s, order);
    if (rounds == 14)
        return open ? tg::launch_hy<14, true>(key, b, s, order) : tg::launch_hy<14, false>(key, b, s, order);
    return TG_EINVAL;
}

int tg_launch_gcm_bs8(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                      hipStream_t s, const uint32_t* order) {
    if (rounds == 10)
        return open ? tg::launch_bs8<10, true>(key, b, s, order) : tg::launch_bs8<10, false>(key, b, s, order);
    if (rounds == 14)
        return open ? tg::launch_bs8<14, true>(key, b, s, order) : tg::launch_bs8<14, false>(key, b, s, order);
    return TG_EINVAL;
}

int tg_launch_gcm_kt(const tg::GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, const uint32_t* planes,
                     const uint4* rot, int rounds, const tg_batch& b, bool open, hipStream_t s, uint32_t split,
                     int lpr, bool hybrid) {
    if (rounds == 10)
        return open ? tg::launch_kt<10, true>(keys, nkeys, hpow, planes, rot, b, s, split, lpr, hybrid)
                    : tg::launch_kt<10, false>(keys, nkeys, hpow, planes, rot, b, s, split, lpr, hybrid);
    if (rounds == 14)
        return open ? tg::launch_kt<14, true>(keys, nkeys, hpow, planes, rot, b, s, split, lpr, hybrid)
                    : tg::launch_kt<14, false>(keys, nkeys, hpow, planes, rot, b, s, split, lpr, hybrid);
    return TG_EINVAL;
}

int tg_launch_kt_planes(const tg::GcmTableKey* keys, uint64_t n, int rounds, uint32_t* planes,
                        uint4* rot, hipStream_t s) {
    const uint64_t total = n * tg::kKtPlaneWords;
    hipLaunchKernelGGL(tg::kt_planes_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, keys, n,
                       rounds, planes);
    if (hipGetLastError() != hipSuccess) return TG_EHIP;
    hipLaunchKernelGGL(tg::kt_rot_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, keys, n,
                       rounds, reinterpret_cast<uint32_t*>(rot));
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}
