// chacha_poly.hip -- batched ChaCha20-Poly1305 seal/open for gfx950 (CDNA4).
//
// Restates CHACHA20_POLY1305.seal/open (tlslite/utils/chacha20_poly1305.py:
// 48-94) over ChaCha (chacha.py:98-153) and Poly1305 (poly1305.py:32-48),
// one TLS record per lane, pure 32-bit VALU work (no tables, no LDS):
//
//   * the one-time Poly1305 key is ChaCha block 0 (chacha20_poly1305.py:35-38),
//     the payload uses blocks 1.. (chacha20_poly1305.py:58);
//   * each 64-byte keystream block is XORed with four 16-byte loads and its
//     four ciphertext blocks go straight into the Poly1305 accumulator, so
//     mac_data = aad || pad || ct || pad || le64 || le64 (:60-63) is never
//     materialised;
//   * Poly1305 runs in 32-bit limbs with 32x32->64 multiply-adds (the wave
//     kernel's striped Horner keeps five 26-bit limbs).
#include <cstdlib>

#include "common.h"
#include "options.h"
#include "poly1305.h"

namespace tg {
namespace {

#if !defined(TG_CHACHA_THREADS)   // measurement builds may override the workgroup size
#define TG_CHACHA_THREADS 256
#endif
#if !defined(TG_CHACHA_MINW)      // ... and the waves per SIMD of the lane kernel (VGPR budget)
#define TG_CHACHA_MINW 4
#endif
constexpr int kChachaThreads = TG_CHACHA_THREADS;

#define QR(a, b, c, d)                                  \
    a += b; d ^= a; d = rotl32(d, 16);                  \
    c += d; b ^= c; b = rotl32(b, 12);                  \
    a += b; d ^= a; d = rotl32(d, 8);                   \
    c += d; b ^= c; b = rotl32(b, 7);

// ChaCha.chacha_block (chacha.py:98-109): 10 double rounds + feed-forward.
__device__ __forceinline__ void chacha_block(const uint32_t (&k)[8], uint32_t ctr, uint32_t n0,
                                             uint32_t n1, uint32_t n2, uint32_t (&o)[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3];
    uint32_t x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
    uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        QR(x0, x4, x8, x12);
        QR(x1, x5, x9, x13);
        QR(x2, x6, x10, x14);
        QR(x3, x7, x11, x15);
        QR(x0, x5, x10, x15);
        QR(x1, x6, x11, x12);
        QR(x2, x7, x8, x13);
        QR(x3, x4, x9, x14);
    }
    o[0] = x0 + 0x61707865u; o[1] = x1 + 0x3320646eu;
    o[2] = x2 + 0x79622d32u; o[3] = x3 + 0x6b206574u;
    o[4] = x4 + k[0]; o[5] = x5 + k[1]; o[6] = x6 + k[2]; o[7] = x7 + k[3];
    o[8] = x8 + k[4]; o[9] = x9 + k[5]; o[10] = x10 + k[6]; o[11] = x11 + k[7];
    o[12] = x12 + ctr; o[13] = x13 + n0; o[14] = x14 + n1; o[15] = x15 + n2;
}
#undef QR

// The 64-byte blocks of a record.  Software-pipelined one block deep: while
// block j is XORed and fed to Poly1305, the keystream of block j+1 is
// generated and the payload of block j+1 is in flight, so seal's Poly1305
// chain (which needs the ciphertext) overlaps the next block's 20 rounds.
// Leaves in ks the keystream of block nfull+1 (the partial tail, if any).
// ALIGNED records use 16-byte vector loads and stores with no branches.
template <bool OPEN, bool ALIGNED>
__device__ __forceinline__ void full_blocks(const uint32_t (&k)[8], uint4 nv, const uint8_t* in,
                                            uint8_t* out, uint32_t j0, uint32_t nfull, Poly32& p,
                                            uint32_t (&ks)[16]) {
    if (j0 >= nfull) return;
    uint4 d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = load16(in + 64 * j0 + 16 * q, ALIGNED);
    for (uint32_t j = j0; j < nfull; ++j) {
        // m = the Poly1305 input of block j (ciphertext: c for seal, d for open)
        uint4 m[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 c = make_uint4(d[q].x ^ ks[4 * q], d[q].y ^ ks[4 * q + 1],
                                       d[q].z ^ ks[4 * q + 2], d[q].w ^ ks[4 * q + 3]);
            store16(out + 64 * j + 16 * q, c, ALIGNED);
            m[q] = OPEN ? d[q] : c;
        }
        // payload of block j+1 in flight (the last iteration re-reads block j: in bounds)
        const uint32_t jn = j + 1 < nfull ? j + 1 : j;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = load16(in + 64 * jn + 16 * q, ALIGNED);
        chacha_block(k, j + 2, nv.x, nv.y, nv.z, ks);
#pragma unroll
        for (int q = 0; q < 4; ++q) poly_block(p, m[q]);
    }
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max_octet(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
        v = w > v ? w : v;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Per-wave LDS: a 64-record x 128-byte tile -- row r = the record of lane r,
// holding one aligned pair of 64-byte blocks (one 128-byte HBM line) -- and
// the records' in/out base pointers.  Chunk c of row r sits at 16-byte slot
// c ^ ((r >> 1) & 7) ^ 4 (r & 1): ds_read_b128 serves 16 lanes per LDS cycle
// over the 16 slots of a 256-byte bank row (rows r and r + 1 share one) and
// ds_write_b128 8 consecutive lanes over 8 slots of 128 bytes, so with this
// swizzle the row-wise reads and writes (lane r, row r) and the coalesced
// ones (8 lanes per row) are all conflict-free.  Round 2's c ^ ((r >> 1) & 7)
// put lanes 2k and 2k + 1 of a row-wise write on one slot: 21 % of the LDS
// cycles were bank conflicts (profiles/r02/v75/pmc_chacha_summary.txt).
struct WaveTile {
    uint4 row[64][8];
    uint4 ptr[64];  // {in lo, in hi, out lo, out hi}
    uint4 skey[64]; // each lane's Poly1305 s, parked across the tile loop (chacha_kernel)
};
constexpr int kWavesPerGroup = kChachaThreads / 64;

__device__ __forceinline__ uint32_t swz(uint32_t r, uint32_t c) {
    return c ^ ((r >> 1) & 7u) ^ ((r & 1u) << 2);
}


// Blocks [0, jmin) of all 64 records of a wave (every record has >= jmin full
// blocks and 16-byte aligned buffers).  HBM traffic goes through the tile in
// whole 128-byte lines: coalesced instruction q of row group g moves chunk
// lane % 8 of the block pair of record 32 g + 8 q + lane / 8, i.e. 8 records
// x 128 contiguous bytes (a half-line per record and instruction read the
// other half after it had left L2: 1.3x the algorithmic HBM bytes,
// profiles/r02/v27/traffic.json).  Rows 0-31 (group A) take the pairs
// (p, p + 1), p even, at iteration p; rows 32-63 (group B) run one block
// behind (block b at iteration b + 1), so each iteration moves one group's
// pair in and the other group's finished pair out -- 4 load and 4 store
// instructions, as with 64-byte rows.  The keystream/Poly1305 pipeline is
// the same as full_blocks(); a lane's next keystream block is b + 1.
template <bool OPEN>
__device__ __forceinline__ void tiled_blocks(WaveTile& t, uint32_t lane,
                                             const uint32_t (&k)[8], uint4 nv, uint32_t jmin,
                                             Poly32& p, uint32_t (&ks)[16]) {
    const uint32_t grp = lane >> 5, cq = lane & 7u, rq = lane >> 3;
    // the coalesced ops of group g's pair starting at block p0 (even)
    auto load_pair = [&](uint32_t g, uint32_t p0, uint4 (&R)[4]) {
        // unconditional: a chunk past the tile's blocks re-reads block 0 of
        // its record (rows without a record of their own read a valid row's),
        // so no branch leaves a load into R pending on some paths only
        const uint32_t off = p0 + (cq >> 2) < jmin ? 64 * p0 + 16 * cq : 16 * (cq & 3u);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            const uint4 pr = t.ptr[r];
            const uint8_t* src = reinterpret_cast<const uint8_t*>(((uint64_t)pr.y << 32) | pr.x);
#if defined(TG_CHACHA_NO_IO)   // measurement build (tools/build_variant.sh): no HBM access
            R[q] = make_uint4(pr.x + off, pr.y, pr.x ^ off, q);
            (void)src;
#else
            R[q] = gload16(src + off);
#endif
        }
    };
    auto put_pair = [&](uint32_t g, const uint4 (&R)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            t.row[r][swz(r, cq)] = R[q];
        }
    };
    auto store_pair = [&](uint32_t g, uint32_t p0) {
        const uint32_t blk = p0 + (cq >> 2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            const uint4 v = t.row[r][swz(r, cq)];
            const uint4 pr = t.ptr[r];
            uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)pr.w << 32) | pr.z);
#if !defined(TG_CHACHA_NO_IO)
            if (blk < jmin && dst) gstore16(dst + 64 * p0 + 16 * cq, v);
#else
            if (blk < jmin && dst && v.x == 0x12345678u && v.y == 0x9abcdef0u) gstore16(dst, v);
#endif
        }
    };
    // The pair finished in iteration i is stored at the top of iteration
    // i + 1: its rows are read before put_pair overwrites them and the global
    // stores go out right after it, so the next iteration's vmcnt(0) (loads
    // and stores share the counter) waits for stores issued a whole
    // iteration earlier instead of one ChaCha block earlier.
    auto flush_pair = [&](uint32_t g, uint32_t p0, const uint4 (&S)[4]) {
        const uint32_t blk = p0 + (cq >> 2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            const uint4 pr = t.ptr[r];
            uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)pr.w << 32) | pr.z);
#if !defined(TG_CHACHA_NO_IO)
            if (blk < jmin && dst) gstore16(dst + 64 * p0 + 16 * cq, S[q]);
#else
            if (blk < jmin && dst && S[q].x == 0x12345678u && S[q].y == 0x9abcdef0u) gstore16(dst, S[q]);
#endif
        }
    };
    auto read_pair = [&](uint32_t g, uint4 (&S)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            S[q] = t.row[r][swz(r, cq)];
        }
    };
    uint4 R[4];
    load_pair(0, 0, R);
    for (uint32_t i = 0; i <= jmin; ++i) {
        // group A's pair (i, i + 1) at even i, group B's (i - 1, i) at odd i
        const uint32_t g = i & 1u;
        // the pair finished in iteration i - 1: group A's (i - 2, i - 1) at
        // even i >= 2, group B's (i - 3, i - 2) at odd i >= 3
        const bool fl = (i >= 2 && !(i & 1u)) || (i >= 3 && (i & 1u));
        const uint32_t fg = i & 1u, fp = (i & 1u) ? i - 3 : i - 2;
        uint4 S[4];
        if (fl) read_pair(fg, S);
        put_pair(g, R);   // past the last pair: the group's rows are free (read above)
        if (fl) flush_pair(fg, fp, S);
        __builtin_amdgcn_wave_barrier();
        load_pair((i + 1) & 1u, i + 1 - ((i + 1) & 1u), R);
        const uint32_t b = i - grp;                 // this lane's block
        const bool act = i >= grp && b < jmin;
        uint4 m[4];
        if (act) {
            // the row's four chunks are read together and written back
            // together: one LDS round trip instead of four dependent ones
            const uint32_t h = 4 * (b & 1u);
            uint4 d[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) d[c] = t.row[lane][swz(lane, h + c)];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint4 ct = make_uint4(d[c].x ^ ks[4 * c], d[c].y ^ ks[4 * c + 1], d[c].z ^ ks[4 * c + 2],
                                            d[c].w ^ ks[4 * c + 3]);
                t.row[lane][swz(lane, h + c)] = ct;
                m[c] = OPEN ? d[c] : ct;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (act) {
            chacha_block(k, b + 2, nv.x, nv.y, nv.z, ks);
#pragma unroll
            for (int c = 0; c < 4; ++c) poly_block(p, m[c]);
        }
    }
    // the pair finished in the last iteration (i = jmin)
    if (jmin & 1u) {
        store_pair(0, jmin - 1);
    } else if (jmin >= 2) {
        store_pair(1, jmin - 2);
    }
    // group B's last pair when jmin is odd (its block jmin - 1 ran at iteration jmin)
    if (jmin & 1u) store_pair(1, jmin - 1);
}

// tiled_blocks with the tile filled by LDS-DMA (global_load_lds_dwordx4): no
// VGPR round trip and no ds_write for the loads.  A DMA instruction writes
// 1 KiB lane-linearly (lane x -> slot x % 8 of row 8 q + x / 8), so the swizzle
// goes on the source address: the lane landing in slot s of row r fetches
// chunk s ^ ((r >> 1) & 7).  A group's next pair is fetched right after its
// finished pair has been read out of the rows (after the row pass of the
// iteration that completes it), so it has the next ChaCha block to land;
// the wait for it is the first LDS read of the next iteration.
template <bool OPEN>
__device__ __forceinline__ void tiled_blocks_dma(WaveTile& t, uint32_t lane,
                                                 const uint32_t (&k)[8], uint4 nv, uint32_t jmin,
                                                 Poly32& p, uint32_t (&ks)[16]) {
    const uint32_t grp = lane >> 5, cq = lane & 7u, rq = lane >> 3;
    auto fetch_pair = [&](uint32_t g, uint32_t p0, const uint4 (&P)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            const uint32_t c = swz(r, cq);          // the chunk that lands in slot cq
            const uint32_t off = p0 + (c >> 2) < jmin ? 64 * p0 + 16 * c : 16 * (c & 3u);
#if defined(TG_CHACHA_ILV)   // measurement build: the group's lines interleaved (wrong bytes, same volume)
            const uint4 b0 = t.ptr[32 * g];
            const uint8_t* src = reinterpret_cast<const uint8_t*>(((uint64_t)b0.y << 32) | b0.x) +
                                 ((p0 >> 1) * 32u + 8u * q + rq) * 128u + 16u * c;
            (void)off;
#else
            const uint8_t* src = reinterpret_cast<const uint8_t*>(((uint64_t)P[q].y << 32) | P[q].x) + off;
#endif
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)src,
                (__attribute__((address_space(3))) void*)(&t.row[32 * g + 8 * q][0]),
                16, 0, 0);
        }
    };
    auto ptrs = [&](uint32_t g, uint4 (&P)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) P[q] = t.ptr[32 * g + 8 * q + rq];
    };
    // read group g's finished pair (blocks p0, p0 + 1), store it, fetch the next
    auto turn = [&](uint32_t g, uint32_t p0) {
        uint4 P[4], S[4];
        ptrs(g, P);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = 32 * g + 8 * q + rq;
            S[q] = t.row[r][swz(r, cq)];
        }
        const uint32_t blk = p0 + (cq >> 2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#if defined(TG_CHACHA_ILV)
            const uint4 b0 = t.ptr[32 * g];
            uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)b0.w << 32) | b0.z);
            if (blk < jmin && dst) gstore16(dst + ((p0 >> 1) * 32u + 8u * q + rq) * 128u + 16u * cq, S[q]);
#else
            uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)P[q].w << 32) | P[q].z);
            if (blk < jmin && dst) gstore16(dst + 64 * p0 + 16 * cq, S[q]);
#endif
        }
        if (p0 + 2 < jmin) fetch_pair(g, p0 + 2, P);
    };
    {
        uint4 P[4];
        ptrs(0, P);
        fetch_pair(0, 0, P);
        ptrs(1, P);
        fetch_pair(1, 0, P);
    }
    for (uint32_t i = 0; i <= jmin; ++i) {
        const uint32_t b = i - grp;                 // this lane's block
        const bool act = i >= grp && b < jmin;
        uint4 m[4];
        if (act) {
            const uint32_t h = 4 * (b & 1u);
            uint4 d[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) d[c] = t.row[lane][swz(lane, h + c)];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint4 ct = make_uint4(d[c].x ^ ks[4 * c], d[c].y ^ ks[4 * c + 1], d[c].z ^ ks[4 * c + 2],
                                            d[c].w ^ ks[4 * c + 3]);
                t.row[lane][swz(lane, h + c)] = ct;
                m[c] = OPEN ? d[c] : ct;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // group A finished block i, group B block i - 1 (wave-uniform)
        if (i < jmin && ((i & 1u) || i + 1 == jmin)) turn(0, i & ~1u);
        if (i >= 1 && (((i - 1) & 1u) || i == jmin)) turn(1, (i - 1) & ~1u);
        __builtin_amdgcn_wave_barrier();
        if (act) {
            chacha_block(k, b + 2, nv.x, nv.y, nv.z, ks);
#pragma unroll
            for (int c = 0; c < 4; ++c) poly_block(p, m[c]);
        }
    }
}

// A key-table record whose key_idx is not below nkeys is skipped (open:
// status 0): its row still serves the wave's coalesced transfers, with its
// output pointer cleared so the tile never stores it.
template <bool OPEN, bool MULTIKEY, int MINW, bool DMA>
__global__ __launch_bounds__(kChachaThreads, MINW) void chacha_kernel(
    const ChachaKeyDev* __restrict__ keys, uint64_t nkeys, tg_batch b, const uint32_t* __restrict__ order) {
    __shared__ WaveTile tiles[kWavesPerGroup];
    const uint64_t i_raw = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave_base = i_raw - lane;
    if (wave_base >= b.n) return;  // whole wave idle (uniform)
    // Lanes past the end of the batch stay alive to serve the wave's
    // coalesced transfers, but work on a clamped record and never store.
    const uint64_t t = i_raw < b.n ? i_raw : b.n - 1;
    uint64_t i = order ? order[t] : t;   // planner.hip: records longest first
    uint32_t ki = 0;
    if (MULTIKEY) {
        ki = b.key_idx[i];
        if (ki >= nkeys) {
            if (OPEN && b.status && i_raw < b.n) b.status[i] = 0;
            ki = 0;
        }
    }
    const bool valid = i_raw < b.n && (!MULTIKEY || b.key_idx[i] < nkeys);
    uint32_t k[8];
    const ChachaKeyDev* kp = keys + ki;
#pragma unroll
    for (int w = 0; w < 8; ++w) k[w] = kp->k[w];

    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    // the tile stores a row only with a non-null output pointer
    uint8_t* const tile_out = valid ? out : nullptr;

    Poly32 p;   // radix 2^32 (poly1305.h)
    {
        uint32_t otk[16];
        chacha_block(k, 0, nv.x, nv.y, nv.z, otk);  // poly1305_key_gen
        poly_init(p, otk);
    }

    for (uint32_t off = 0; off < alen; off += 16) {
        uint32_t m = alen - off < 16 ? alen - off : 16;
        poly_block(p, load_partial(ad + off, m));
    }

    const uint32_t nfull = len >> 6;
    uint32_t ks[16];
    chacha_block(k, 1, nv.x, nv.y, nv.z, ks);
    // Coalesced tile path for the blocks every record of the wave has.  Rows
    // of lanes without a record of their own (past the batch, or a skipped
    // key) load from the first valid lane's record, which has >= jmin blocks.
    const uint64_t vmask = __ballot(valid);
    const uint32_t jmin = (vmask && __all(!valid || aligned)) ? wave_min(valid ? nfull : 0xffffffffu) : 0;
    uint32_t j0 = 0;
    if (jmin > 0) {
        WaveTile& t = tiles[threadIdx.x >> 6];
        const int src = __ffsll((unsigned long long)vmask) - 1;
        const uint32_t in_lo = (uint32_t)__shfl((int)(uint32_t)(uintptr_t)in, src, 64);
        const uint32_t in_hi = (uint32_t)__shfl((int)(uint32_t)((uintptr_t)in >> 32), src, 64);
        const uint8_t* tile_in = valid ? in : reinterpret_cast<const uint8_t*>(((uint64_t)in_hi << 32) | in_lo);
        t.ptr[lane] = make_uint4((uint32_t)(uintptr_t)tile_in, (uint32_t)((uintptr_t)tile_in >> 32),
                                 (uint32_t)(uintptr_t)tile_out, (uint32_t)((uintptr_t)tile_out >> 32));
        t.skey[lane] = make_uint4(p.p0, p.p1, p.p2, p.p3);
        __builtin_amdgcn_wave_barrier();
        if (DMA)
            tiled_blocks_dma<OPEN>(t, lane, k, nv, jmin, p, ks);
        else
            tiled_blocks<OPEN>(t, lane, k, nv, jmin, p, ks);
        j0 = jmin;
        const uint4 sk = t.skey[lane];
        p.p0 = sk.x; p.p1 = sk.y; p.p2 = sk.z; p.p3 = sk.w;
    }
#if !defined(TG_CHACHA_KEEP_FIELDS)
    // The record's index and fields are read again here instead of being kept
    // live across the tile loop, which does not use them: holding them cost
    // 9 (seal) / 12 (open) VGPRs of spills to scratch, i.e. a private segment
    // and runtime scratch memory for every queue the kernel runs on
    // (profiles/r06/x10/stream_mem.jsonl).  The index goes through an empty asm
    // so the compiler cannot reuse the loads above (and keep their results).
    {
        uint64_t tr = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        tr = tr < b.n ? tr : b.n - 1;
        __asm__ volatile("" : "+v"(tr));
        i = order ? order[tr] : tr;
        in = rec_in(b, i);
        out = rec_out(b, i);
        len = rec_len(b, i);
        alen = rec_aad_len(b, i);
    }
#endif
    if (valid) {
        if (aligned) {
            full_blocks<OPEN, true>(k, nv, in, out, j0, nfull, p, ks);
        } else {
            full_blocks<OPEN, false>(k, nv, in, out, j0, nfull, p, ks);
        }
    }
    if (!valid) return;
    const uint32_t rem = len - 64 * nfull;
    if (rem) {  // ks already holds keystream block nfull + 1
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (16u * q < rem) {
                uint32_t m = rem - 16 * q < 16 ? rem - 16 * q : 16;
                uint4 d = load_partial(in + 64 * nfull + 16 * q, m);
                uint4 c = mask_tail(make_uint4(d.x ^ ks[4 * q], d.y ^ ks[4 * q + 1],
                                               d.z ^ ks[4 * q + 2], d.w ^ ks[4 * q + 3]), m);
                store_partial(out + 64 * nfull + 16 * q, c, m);
                poly_block(p, OPEN ? d : c);
            }
        }
    }
    // le64(len(aad)) || le64(len(ct))
    poly_block(p, make_uint4(alen, 0, len, 0));
    const uint4 tag = poly_finish(p);
    const bool tag_aligned = aligned && (len & 15) == 0;
    if (!OPEN) {
        store16(out + len, tag, tag_aligned);
        return;
    }
    const uint4 exp = load16(in + len, tag_aligned);
    const uint32_t diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
    if (b.status) b.status[i] = diff == 0;
    if (diff) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t q = 0; q < (len >> 4); ++q) store16(out + 16 * q, z, aligned);
        if (len & 15) store_partial(out + (len & ~15u), z, len & 15);
    }
}

// ---- wave-per-record kernel (small batches and the per-record calls) ----
// One record per wavefront (or W waves, S = 64 W threads): thread t takes the
// payload ChaCha blocks t, t + S, t + 2S, ... (counters 1 + q) and runs
// Poly1305's Horner over its ciphertext 16-byte blocks, multiplying by
// r^(4S - 4) across the gaps; since acc = sum_k m_k r^(M-k) over the M blocks
// of mac_data, each thread's value is lifted by r^(blocks after its last one)
// (square and multiply in the same 26-bit limbs) and the partials are summed
// by a shuffle tree (and across the record's waves through LDS).  Thread 0
// adds the AAD blocks (lifted by r^(nc+1)) and the length block (times r).
// W waves per record: W = 1 four records per 256-thread workgroup, W = 4 / 16
// one record per 256 / 1024-thread workgroup (batches that leave CUs idle,
// the per-record calls).
template <int W>
constexpr int chacha_wave_threads() { return W == 16 ? 1024 : 256; }

// MULTIKEY: a key table (record i uses keys[key_idx[i]]; an index not below
// nkeys skips the record, open status 0 -- the record group exits together).
template <bool OPEN, int W, bool MULTIKEY>
__global__ __launch_bounds__(chacha_wave_threads<W>()) void chacha_wave_kernel(
    const ChachaKeyDev* __restrict__ keys, uint64_t nkeys, tg_batch b) {
    constexpr uint32_t S = 64u * W;            // segments (threads) per record
    __shared__ F5 s_part[W];
    __shared__ uint32_t s_diff;
    const uint64_t i = (uint64_t)blockIdx.x * (chacha_wave_threads<W>() / S) +
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / S));   // wave-uniform
    if (i >= b.n) return;   // whole record group (uniform)
    const uint32_t lane = threadIdx.x & (S - 1u);
    const ChachaKeyDev* kp = keys;
    if (MULTIKEY) {
        const uint32_t ki = (uint32_t)__builtin_amdgcn_readfirstlane((int)gld(b.key_idx, i));
        if (ki >= nkeys) {   // uniform over the record group
            if (OPEN && b.status && lane == 0) b.status[i] = 0;
            return;
        }
        kp = keys + ki;
    }
    uint32_t k[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) k[w] = kp->k[w];
    const uint8_t* in = rec_in(b, i);
    uint8_t* out = rec_out(b, i);
    const uint32_t len = rec_len(b, i);
    const uint8_t* ad = rec_aad(b, i);
    const uint32_t alen = rec_aad_len(b, i);
    const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    Poly p;
    {
        uint32_t otk[16];
        chacha_block(k, 0, nv.x, nv.y, nv.z, otk);   // poly1305_key_gen (every lane)
        poly_init(p, otk);
    }
    const F5 r = {p.r0, p.r1, p.r2, p.r3, p.r4};
    const uint32_t nc = (len + 15) >> 4, nf = len >> 4, tail = len & 15;
    const uint32_t nq = (len + 63) >> 6;
    // thread seg takes the ChaCha blocks q = seg + S j, so each load / store
    // instruction of a wave covers 4 KiB of consecutive bytes; between two of
    // its blocks the Horner value skips the other threads' 4 (S - 1) Poly1305
    // blocks: h <- h r^(4S - 4)
    F5 rgap = {0, 0, 0, 0, 0};
    uint32_t cb = 0;                                 // end of the thread's last block
    for (uint32_t q = lane; q < nq; q += S) {        // chacha20_poly1305.py:58-63
        stripe_gap<S>(p, r, q, lane, rgap);
        uint32_t ks[16];
        chacha_block(k, 1 + q, nv.x, nv.y, nv.z, ks);
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            const uint32_t c = 4 * q + sb;
            const uint4 kv = make_uint4(ks[4 * sb], ks[4 * sb + 1], ks[4 * sb + 2], ks[4 * sb + 3]);
            if (c < nf) {
                const uint4 d = load16(in + 16 * c, aligned);
                const uint4 ct = xor4(d, kv);
                store16(out + 16 * c, ct, aligned);
                poly_block(p, OPEN ? d : ct);
            } else if (c == nf && tail) {
                const uint4 d = load_partial(in + 16 * c, tail);
                const uint4 ct = mask_tail(xor4(d, kv), tail);
                store_partial(out + 16 * c, ct, tail);
                poly_block(p, OPEN ? d : ct);
            }
        }
        cb = 4 * q + 4 < nc ? 4 * q + 4 : nc;
    }
    // lift: h r^(blocks after the thread's last one, incl. the length block)
    F5 z = stripe_lift(p, r, cb, nc - cb + 1);
    if (lane == 0) {
        Poly pa = p;                                 // the AAD (mac_data starts with it)
        pa.h0 = pa.h1 = pa.h2 = pa.h3 = pa.h4 = 0;
        for (uint32_t off = 0; off < alen; off += 16) {
            const uint32_t m = alen - off < 16 ? alen - off : 16;
            poly_block(pa, load_partial(ad + off, m));
        }
        z = fnorm_add(z, fmul(F5{pa.h0, pa.h1, pa.h2, pa.h3, pa.h4}, fpow(r, nc + 1)));
        Poly pl = pa;                                // le64(alen) || le64(len), times r
        pl.h0 = pl.h1 = pl.h2 = pl.h3 = pl.h4 = 0;
        poly_block(pl, make_uint4(alen, 0, len, 0));
        z = fnorm_add(z, F5{pl.h0, pl.h1, pl.h2, pl.h3, pl.h4});
    }
    z = stripe_sum<W>(z, s_part, lane, 0);
    p.h0 = z.h0; p.h1 = z.h1; p.h2 = z.h2; p.h3 = z.h3; p.h4 = z.h4;
    const uint4 tag = poly_finish(p);                // poly1305.py:47-48
    const bool tag_aligned = aligned && (len & 15) == 0;
    if (!OPEN) {
        if (lane == 0) store16(out + len, tag, tag_aligned);
        return;
    }
    uint32_t diff = 0;
    if (lane == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status) b.status[i] = diff == 0;
        if (W > 1) s_diff = diff;
    }
    if (W > 1) {
        __syncthreads();
        diff = s_diff;
    } else {
        diff = (uint32_t)__shfl((int)diff, 0, 64);
    }
    if (diff) {                                      // chacha20_poly1305.py:90-91
        const uint4 zz = make_uint4(0, 0, 0, 0);
        for (uint32_t c = lane; c < nf; c += S) store16(out + 16 * c, zz, aligned);
        if (tail && lane == 0) store_partial(out + 16 * nf, zz, tail);
    }
}

// ---- octet kernel: eight lanes per record, no LDS tile --------------------
// (chacha_variant 6.)  Lane l of a record's octet takes
// the ChaCha blocks b = l, l + 8, ... (counter b + 1): for a fixed load or
// store instruction the octet's lanes touch 8 x 16 bytes of one 512-byte
// stretch of the record, and the four instructions of a block complete its
// 128-byte lines back to back -- no LDS round trip, no wave barriers.
// Poly1305 runs per lane over the lane's own blocks (poly1305.h octet
// striping: r within a block, r^29 across the other lanes' blocks, the lift
// and the octet sum at the end), in 26-bit limbs.  The one-time key and the
// powers of r come from chacha_otk_kernel (one lane per record, before).
// Lane 0 of the octet also runs the AAD blocks, which precede its block 0
// in mac_data (chacha20_poly1305.py:60-63).
constexpr int kOctetThreads = 256;
#if !defined(TG_OCTET_NT)   // A/B builds: non-temporal payload loads and stores
#define TG_OCTET_NT 0
#endif

// Block 0 of every record (poly1305_key_gen, chacha20_poly1305.py:35-38):
// r clamped, its powers and s, by slot t (record order[t] or t).
__global__ __launch_bounds__(256) void chacha_otk_kernel(const ChachaKeyDev* __restrict__ key, tg_batch b,
                                                         const uint32_t* __restrict__ order,
                                                         OctetPoly* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= b.n) return;
    const uint64_t i = order ? gld(order, t) : t;
    uint32_t k[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) k[w] = key->k[w];
    const uint4 nv = load_partial(b.nonce + 12 * i, 12);
    uint32_t otk[16];
    chacha_block(k, 0, nv.x, nv.y, nv.z, otk);
    Poly p;
    poly_init(p, otk);
    OctetPoly o;
    octet_powers(F5{p.r0, p.r1, p.r2, p.r3, p.r4}, o);
    o.s[0] = p.p0; o.s[1] = p.p1; o.s[2] = p.p2; o.s[3] = p.p3;
    o.pad[0] = o.pad[1] = 0;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&o);
    uint8_t* dst = reinterpret_cast<uint8_t*>(out + t);
#pragma unroll
    for (int q = 0; q < 9; ++q) gstore16(dst + 16 * q, make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]));
}

template <bool OPEN>
__global__ __launch_bounds__(kOctetThreads, 4) void chacha_octet_kernel(const ChachaKeyDev* __restrict__ key,
                                                                        tg_batch b,
                                                                        const uint32_t* __restrict__ order,
                                                                        const OctetPoly* __restrict__ pw) {
    const uint32_t lane = threadIdx.x & 63u, l = lane & 7u;
    const uint64_t t = ((uint64_t)blockIdx.x * kOctetThreads + threadIdx.x) >> 3;
    const uint64_t wave_first = ((uint64_t)blockIdx.x * kOctetThreads + (threadIdx.x & ~63u)) >> 3;
    if (wave_first >= b.n) return;   // whole wave idle (uniform)
    const bool valid = t < b.n;
    const uint64_t i = valid ? (order ? gld(order, t) : t) : 0;
    uint32_t k[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) k[w] = key->k[w];
    uint32_t len = 0, alen = 0;
    const uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    const uint8_t* ad = nullptr;
    uint4 nv = make_uint4(0, 0, 0, 0);
    const uint32_t* pwt = reinterpret_cast<const uint32_t*>(pw + (valid ? t : 0));
    if (valid) {
        len = rec_len(b, i);
        alen = rec_aad_len(b, i);
        in = rec_in(b, i);
        out = rec_out(b, i);
        ad = rec_aad(b, i);
        nv = load_partial(b.nonce + 12 * i, 12);
    }
    const OctetPoly* op = reinterpret_cast<const OctetPoly*>(pwt);
    const Mul26 R = mul26(f5_at(op->r)), R29 = mul26(f5_at(op->r29));
    const uint32_t nch = (len + 63) >> 6;        // 64-byte chunks (ChaCha blocks) of the payload
    const uint32_t nfull = len >> 6;             // full ones
    F5 h = {0, 0, 0, 0, 0};
    if (l == 0) {   // mac_data starts with the AAD (chacha20_poly1305.py:60)
        for (uint32_t off = 0; off < alen; off += 16) {
            const uint32_t m = alen - off < 16 ? alen - off : 16;
            fblock(h, load_partial(ad + off, m), R);
        }
    }
    // steps: the wave's longest record (uniform loop count)
    const uint32_t steps = wave_max_octet((nch + 7u) >> 3);
    uint4 m[4];            // the previous block's Poly1305 input (seal: ct; open: the input)
    bool pend = false;     // m holds a full block whose Horner is not done yet
    for (uint32_t s = 0; s < steps; ++s) {
        const uint32_t blk = 8u * s + l;
        const bool have = blk < nch;
        const bool full = blk < nfull;
        // unconditional loads (a lane without a full block reads its slot's
        // OctetPoly instead): loads under a divergent branch made the compiler
        // wait for them at the branch's end, before the keystream
        const uint8_t* src = full ? in + 64u * blk : reinterpret_cast<const uint8_t*>(pwt);
        uint4 d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = TG_OCTET_NT ? gload16u_nt(src + 16u * q) : gload16u(src + 16u * q);
        uint32_t ks[16];
        chacha_block(k, blk + 1u, nv.x, nv.y, nv.z, ks);
        // the previous block's Horner (ends with the jump over the other
        // lanes' blocks, or with r when that block was the lane's last)
        if (pend) {
            const Mul26& RL = have ? R29 : R;
            fblock(h, m[0], R);
            fblock(h, m[1], R);
            fblock(h, m[2], R);
            fblock(h, m[3], RL);
            pend = false;
        }
        if (full) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 c = make_uint4(d[q].x ^ ks[4 * q], d[q].y ^ ks[4 * q + 1], d[q].z ^ ks[4 * q + 2],
                                           d[q].w ^ ks[4 * q + 3]);
                if (TG_OCTET_NT)
                    gstore16u_nt(out + 64u * blk + 16u * q, c);
                else
                    gstore16u(out + 64u * blk + 16u * q, c);
                m[q] = OPEN ? d[q] : c;
            }
            pend = true;
        } else if (have) {   // the record's partial last block: the lane's last
            const uint32_t rem = len - 64u * blk;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (16u * q < rem) {
                    const uint32_t mm = rem - 16u * q < 16u ? rem - 16u * q : 16u;
                    const uint4 dd = load_partial(in + 64u * blk + 16u * q, mm);
                    const uint4 c = mask_tail(make_uint4(dd.x ^ ks[4 * q], dd.y ^ ks[4 * q + 1], dd.z ^ ks[4 * q + 2],
                                                         dd.w ^ ks[4 * q + 3]), mm);
                    store_partial(out + 64u * blk + 16u * q, c, mm);
                    fblock(h, OPEN ? dd : c, R);
                }
            }
        }
    }
    if (pend) {   // the lane's last block was full
        fblock(h, m[0], R);
        fblock(h, m[1], R);
        fblock(h, m[2], R);
        fblock(h, m[3], R);
    }
    // lift and sum over the octet; lane 0 adds the length block
    const uint32_t nc = (len + 15) >> 4;
    const uint32_t mlast = nch ? nc - 4u * (nch - 1u) : 0u;
    h = octet_lift(h, octet_lift_exp(l, nch, mlast), op->r, op->r2, op->r4, op->r8, op->r16);
    h = octet_sum(h);
    // le64(len(aad)) || le64(len(ct)) (chacha20_poly1305.py:62-63)
    fblock(h, make_uint4(alen, 0, len, 0), R);
    const uint4 tag = octet_finish(h, op->s);
    const bool tag_aligned = ((((uintptr_t)in | (uintptr_t)out) & 15) == 0) && (len & 15) == 0;
    if (!valid) return;
    if (!OPEN) {
        if (l == 0) store16(out + len, tag, tag_aligned);
        return;
    }
    uint32_t diff = 0;
    if (l == 0) {
        const uint4 exp = load16(in + len, tag_aligned);
        diff = (exp.x ^ tag.x) | (exp.y ^ tag.y) | (exp.z ^ tag.z) | (exp.w ^ tag.w);
        if (b.status) gst(b.status, i, (uint8_t)(diff == 0));
    }
    diff = (uint32_t)__shfl((int)diff, (int)(lane & ~7u), 64);
    if (diff) {   // chacha20_poly1305.py:90-91: each lane zeroes its own blocks
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t blk = l; blk < nch; blk += 8) {
            const uint32_t rem = len - 64u * blk;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (16u * q < rem) store_partial(out + 64u * blk + 16u * q, z, rem - 16u * q < 16u ? rem - 16u * q : 16u);
        }
    }
}

// Up to this many records a batch runs one record per wavefront (see the
// GCM launcher; at 16 KiB the kernels meet between 2^15 and 2^16 records:
// profiles/r01/v21_smallbatch.txt).
constexpr uint64_t kWaveMaxRecords = 49152;

template <bool OPEN, bool MULTIKEY>
int launch_w(const ChachaKeyDev* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    const uint64_t blocks = (b.n + kChachaThreads - 1) / kChachaThreads;
    if (blocks > 0x7fffffffull) return TG_EINVAL;
    if (opt(kOptChachaVariant) == 4)   // register-staged tile fill
        hipLaunchKernelGGL((chacha_kernel<OPEN, MULTIKEY, TG_CHACHA_MINW, false>), dim3((unsigned)blocks), dim3(kChachaThreads),
                           0, s, keys, nkeys, b, order);
    else                                // LDS-DMA tile fill
        hipLaunchKernelGGL((chacha_kernel<OPEN, MULTIKEY, TG_CHACHA_MINW, true>), dim3((unsigned)blocks), dim3(kChachaThreads),
                           0, s, keys, nkeys, b, order);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// Option chacha_variant (tests and measurement): 0 = auto (wave per record
// up to kWaveMaxRecords records, else lane per record at 4 waves per SIMD,
// i.e. <= 128 VGPRs, tile filled by LDS-DMA; 5 and 6 waves per SIMD measured
// slower), 3 = wave per record, 4 = lane per record with the register-staged
// tile fill (1.5 % slower, profiles/r03/chacha_dma_nt_ab.txt), 5 = lane per
// record (LDS-DMA fill).
bool wave_path(uint64_t n) {
    const int v = opt(kOptChachaVariant);
    return v == 3 || (v == 0 && n <= kWaveMaxRecords);
}

// The octet kernel (single key): the one-time keys and powers of r into
// per-launch scratch (api.hip stream_alloc), then the records.
template <bool OPEN>
int launch_octet(const ChachaKeyDev* key, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    const uint64_t groups = (b.n + (kOctetThreads / 8) - 1) / (kOctetThreads / 8);
    if (groups > 0x7fffffffull) return TG_EINVAL;
    OctetPoly* pw = nullptr;
    if (stream_alloc((void**)&pw, sizeof(OctetPoly) * b.n, s)) return TG_EHIP;
    hipLaunchKernelGGL(chacha_otk_kernel, dim3((unsigned)((b.n + 255) / 256)), dim3(256), 0, s, key, b, order, pw);
    int rc = hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    if (!rc) {
        hipLaunchKernelGGL((chacha_octet_kernel<OPEN>), dim3((unsigned)groups), dim3(kOctetThreads), 0, s, key, b,
                           order, pw);
        rc = hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    }
    if (stream_free(pw, s) && !rc) rc = TG_EHIP;
    return rc;
}

template <bool OPEN, bool MULTIKEY>
int launch(const ChachaKeyDev* keys, uint64_t nkeys, const tg_batch& b, hipStream_t s, const uint32_t* order) {
    const int v = opt(kOptChachaVariant);
    if (v != 0 && v != 3 && v != 4 && v != 5 && v != 6) return TG_EINVAL;
    // 6: the octet kernel for every single-key batch (key tables: the lane kernel)
    if (v == 6 && !MULTIKEY) return launch_octet<OPEN>(keys, b, s, order);
    if (wave_path(b.n)) {
        // waves per record as in the GCM launcher (aes_gcm.hip waves_per_record)
        const int o = opt(kOptWavesPerRecord);
        const int w = o ? o : b.n <= 512 ? 4 : 1;   // profiles/r01/v21_smallbatch.txt
        const uint64_t groups = w == 1 ? (b.n + 3) / 4 : b.n;
        if (groups > 0x7fffffffull) return TG_EINVAL;
        if (w == 16)
            hipLaunchKernelGGL((chacha_wave_kernel<OPEN, 16, MULTIKEY>), dim3((unsigned)groups), dim3(1024), 0,
                               s, keys, nkeys, b);
        else if (w == 4)
            hipLaunchKernelGGL((chacha_wave_kernel<OPEN, 4, MULTIKEY>), dim3((unsigned)groups), dim3(256), 0, s,
                               keys, nkeys, b);
        else if (w == 1)
            hipLaunchKernelGGL((chacha_wave_kernel<OPEN, 1, MULTIKEY>), dim3((unsigned)groups), dim3(256), 0, s,
                               keys, nkeys, b);
        else
            return TG_EINVAL;
        return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
    }
    return launch_w<OPEN, MULTIKEY>(keys, nkeys, b, s, order);
}

// RecordLayer._getNonce (recordlayer.py:522-534) for a run of sequence numbers.
__global__ void nonce_kernel(int mode, uint4 iv, uint64_t seq0, uint64_t n, uint8_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t seq = seq0 + i;
    const uint32_t hi = bswap32((uint32_t)(seq >> 32)), lo = bswap32((uint32_t)seq);
    uint32_t w0, w1, w2;
    if (mode == 0) {          // iv12 xor (0^4 || be64(seq))
        w0 = iv.x; w1 = iv.y ^ hi; w2 = iv.z ^ lo;
    } else {                  // iv4 || be64(seq)
        w0 = iv.x; w1 = hi; w2 = lo;
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out + 12 * i);
    if ((((uintptr_t)out) & 3) == 0) {
        o[0] = w0; o[1] = w1; o[2] = w2;
    } else {
        store_partial(out + 12 * i, make_uint4(w0, w1, w2, 0), 12);
    }
}

}  // namespace
}  // namespace tg

bool tg_chacha_wave_path(uint64_t n) { return tg::wave_path(n); }

int tg_launch_chacha(const tg::ChachaKeyDev* keys, uint64_t nkeys, const tg_batch& b, bool open, hipStream_t s,
                     const uint32_t* order) {
    const bool multi = b.key_idx != nullptr;
    if (open)
        return multi ? tg::launch<true, true>(keys, nkeys, b, s, order)
                     : tg::launch<true, false>(keys, nkeys, b, s, order);
    return multi ? tg::launch<false, true>(keys, nkeys, b, s, order)
                 : tg::launch<false, false>(keys, nkeys, b, s, order);
}

int tg_launch_nonces(int mode, const uint8_t* iv_host, uint64_t seq0, uint64_t n, uint8_t* out,
                     hipStream_t s) {
    uint32_t w[3] = {0, 0, 0};
    const int ivlen = mode == 0 ? 12 : 4;
    for (int k = 0; k < ivlen; ++k) w[k >> 2] |= (uint32_t)iv_host[k] << (8 * (k & 3));
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(tg::nonce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, mode,
                       make_uint4(w[0], w[1], w[2], 0), seq0, n, out);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}
