// planner.hip -- processing order for batches of mixed record lengths.
//
// The batch kernels give each record one lane, so a wave takes as long as
// its longest record.  With mixed lengths (BASELINE config 4: Zipf 64 B -
// 16 KiB) almost every wave of 64 random records holds a 16 KiB one and the
// lanes of the short ones idle.  Launching the records longest first, in the
// order of a descending radix sort of their lengths (rocPRIM, on the stream
// of the launch), gives every wave records of nearly equal length; the
// kernels read record order[t] for thread t.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "common.h"

// scratch == nullptr: *bytes = what a batch of n needs.  Layout: sorted keys
// (n u32) | rocPRIM temporary storage.
int tg_length_order(const uint32_t* len, uint64_t n, uint32_t* order, void* scratch, size_t* bytes,
                    hipStream_t s) {
    size_t tmp = 0;
    rocprim::counting_iterator<uint32_t> iota(0);
    if (rocprim::radix_sort_pairs_desc(nullptr, tmp, len, (uint32_t*)nullptr, iota, (uint32_t*)nullptr,
                                       (size_t)n, 0, 32, s) != hipSuccess)
        return TG_EHIP;
    const size_t keys = (n * sizeof(uint32_t) + 255) & ~(size_t)255;
    if (!scratch) {
        *bytes = keys + tmp;
        return TG_OK;
    }
    if (*bytes < keys + tmp) return TG_EINVAL;
    uint32_t* keys_out = static_cast<uint32_t*>(scratch);
    void* t = static_cast<uint8_t*>(scratch) + keys;
    if (rocprim::radix_sort_pairs_desc(t, tmp, len, keys_out, iota, order, (size_t)n, 0, 32, s) !=
        hipSuccess)
        return TG_EHIP;
    return TG_OK;
}

// ---- open over a key table: records with an out-of-range key_idx ---------
// The AEAD kernels skip such a record (status 0, never reading past the
// table); this pass zeroes its plaintext output over len[i] bytes, as for a
// rejected record (include/tlsgpu.h: a status-0 record's plaintext is zero).
// One thread per record; the common case (every index in range) reads the
// key index and exits.
namespace {
__global__ void zero_skipped_kernel(tg_batch b, uint64_t nkeys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n || b.key_idx[i] < nkeys) return;
    uint8_t* o = tg::rec_out(b, i);
    const uint32_t L = tg::rec_len(b, i);
    uint32_t k = 0;
    for (; k < L && (((uintptr_t)(o + k)) & 3u); ++k) o[k] = 0;
    for (; k + 4 <= L; k += 4) *reinterpret_cast<uint32_t*>(o + k) = 0u;
    for (; k < L; ++k) o[k] = 0;
}
}  // namespace

int tg_launch_zero_skipped(const tg_batch& b, uint64_t nkeys, hipStream_t s) {
    if (b.n == 0 || !b.key_idx) return TG_OK;
    hipLaunchKernelGGL(zero_skipped_kernel, dim3((unsigned)((b.n + 255) / 256)), dim3(256), 0, s, b, nkeys);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// ---- key-grouped octet jobs (key-table AES-GCM, aes_gcm_bs8.hip) ---------
// The records of a key-table batch sorted by (key, length descending), then
// cut into jobs of at most eight consecutive records of one key, so that a
// wavefront runs a whole job with one key (its round keys and key planes
// wave-uniform, one GHASH table per wave) and records of similar length.
namespace {

// Sort key: (key, length descending); records shorter than ``split`` or with
// a key index not below nkeys get the tail key nkeys (sorted last, by length).
// Packed as g << LB | (max - L) in a K: with a 32-bit K the length keeps LB =
// 32 - bits(nkeys) bits (longer records sort as equal, which only loosens the
// longest-first order among them), so the radix sort makes 4 passes over
// 32-bit keys instead of 8 over 64-bit ones (config 4: nkeys = 65 536, LB =
// 15, every TLS record length fits).
template <class K>
__global__ void kjp_keys(const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ len,
                         uint32_t fixed_len, uint64_t n, uint64_t nkeys, uint32_t split, int lb,
                         K* __restrict__ ck, uint32_t* __restrict__ nlong) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) *nlong = (uint32_t)n;   // no tail unless kjp_tail finds one
    if (t >= n) return;
    const uint32_t L = len ? len[t] : fixed_len;
    const uint32_t k = key_idx[t];
    const uint64_t g = (k >= nkeys || L < split) ? nkeys : k;
    const uint64_t lmax = lb >= 32 ? 0xffffffffull : (1ull << lb) - 1u;
    const uint64_t Lc = L < lmax ? L : lmax;
    ck[t] = (K)((g << lb) | (lmax - Lc));
}

template <class K>
__global__ void kjp_tail(const K* __restrict__ ck, uint64_t n, uint64_t nkeys, int lb,
                         uint32_t* __restrict__ nlong) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if ((uint64_t)(ck[t] >> lb) == nkeys && (t == 0 || (uint64_t)(ck[t - 1] >> lb) != nkeys))
        *nlong = (uint32_t)t;
}

template <class K>
__global__ void kjp_group_starts(const K* __restrict__ ck, uint64_t n, int lb, uint32_t* __restrict__ g) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    g[t] = (t == 0 || (ck[t] >> lb) != (ck[t - 1] >> lb)) ? (uint32_t)t : 0u;
}

__global__ void kjp_job_starts(const uint32_t* __restrict__ gs, uint64_t n, uint32_t jobsz,
                               uint32_t* __restrict__ js) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    js[t] = (((uint32_t)t - gs[t]) & (jobsz - 1u)) == 0 ? 1u : 0u;
}

__global__ void kjp_scatter(const uint32_t* __restrict__ js, const uint32_t* __restrict__ jx, uint64_t n,
                            uint32_t* __restrict__ jobpos, uint32_t* __restrict__ njobs) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    if (js[t]) jobpos[jx[t] - 1] = (uint32_t)t;
    if (t == n - 1) {
        *njobs = jx[t];
        jobpos[jx[t]] = (uint32_t)n;
    }
}

// Per job of the radix plan, the key of its records: jobkey[j] =
// key_idx[order[jobpos[j]]] for the long jobs, ~0 for the tail's.
__global__ void kjp_jobkey(const uint32_t* __restrict__ jobpos, const uint32_t* __restrict__ njobs_p,
                           const uint32_t* __restrict__ nlong_p, const uint32_t* __restrict__ order,
                           const uint32_t* __restrict__ key_idx, uint32_t* __restrict__ jobkey) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *njobs_p) return;
    const uint32_t p0 = jobpos[j];
    jobkey[j] = p0 < *nlong_p ? key_idx[order[p0]] : 0xffffffffu;
}

int bit_width(uint64_t v) {
    int b = 0;
    while (v) {
        ++b;
        v >>= 1;
    }
    return b;
}

// The plan with K-wide sort keys (see kjp_keys).
template <class K>
int key_job_plan(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                 uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                 uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s, int lb);

size_t ru256(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace

namespace {
// ---- the same plan by counting (round 6) ---------------------------------
// The radix-sorted plan above costs config 4 a 32-bit sort of the whole batch:
// 20 rocPRIM launches, 175 of the 313 us between an op's start and its
// long-record kernel (profiles/r06/y9/c4_plan_timeline.txt).  With at most
// kBucketMaxKeys keys the same plan takes six launches: a memset, counts per
// key group and per tail length (atomics), a two-launch scan, a scatter,
// and a pass that puts each key's records longest first (one thread per key,
// insertion sort in place) and writes the job starts.  Records within a key
// group or a tail length come out of the scatter in any order; a key with more
// than kBucketSortMax long records keeps that order, which costs the long
// kernel some lanes, not correctness (every record is independent).
constexpr uint32_t kTailBuckets = 4096;    // tail lengths, clamped at 4 095, longest first
constexpr uint32_t kBucketSortMax = 64;
constexpr uint64_t kBucketMaxKeys = 1ull << 17;   // above: the radix plan (64-bit keys)
constexpr uint32_t kBpThreads = 1024, kBpPer = 8;   // records per workgroup: 8 192

__device__ __forceinline__ uint32_t tail_bucket(uint32_t L) {
    return kTailBuckets - 1u - (L < kTailBuckets - 1u ? L : kTailBuckets - 1u);
}

// The tail (short records, bad key indices) has few distinct lengths -- 32 in
// config 4 -- so its counts and cursors go through a per-workgroup LDS
// histogram and one global atomic per (workgroup, length): counting straight
// into global counters serialised 578 087 atomics on 32 addresses (2.1 ms).
// The long records' counters are per key (config 4: ~7 records a key).
__global__ __launch_bounds__(kBpThreads) void kbp_count(const uint32_t* __restrict__ key_idx,
                                                        const uint32_t* __restrict__ len, uint32_t fixed_len,
                                                        uint64_t n, uint64_t nkeys, uint32_t split,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ tcnt) {
    __shared__ uint32_t h[kTailBuckets];
    for (uint32_t b = threadIdx.x; b < kTailBuckets; b += kBpThreads) h[b] = 0;
    __syncthreads();
    for (uint32_t r = 0; r < kBpPer; ++r) {
        const uint64_t t = (uint64_t)blockIdx.x * (kBpThreads * kBpPer) + r * kBpThreads + threadIdx.x;
        if (t >= n) break;
        const uint32_t L = len ? len[t] : fixed_len;
        const uint32_t k = key_idx[t];
        if (k < nkeys && L >= split)
            atomicAdd(&cnt[k], 1u);
        else
            atomicAdd(&h[tail_bucket(L)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kTailBuckets; b += kBpThreads)
        if (h[b]) atomicAdd(&tcnt[b], h[b]);
}

// The counters' exclusive scans over many workgroups, in two launches:
// kbp_sums reduces each 1 024-entry block (key counters, then the tail's
// length counters) to its entries and jobs; kbp_offsets gives each block its
// base from the sums before it and scans the block (coalesced loads and
// stores, a shuffle scan per wave, the waves' totals through LDS).  The key
// counters become start[g] (and the scatter's cursors), their job counts
// ceil(c / jobsz) jstart[g]; the tail's counters become cursors from nlong.
// (One workgroup scanning all of it took 55-116 us: one CU's memory pipe.)
constexpr uint32_t kScanBlock = 1024;

__device__ __forceinline__ void block_sum2(uint32_t& a, uint32_t& j, uint32_t* s_a, uint32_t* s_b) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += (uint32_t)__shfl_xor((int)a, o, 64);
        j += (uint32_t)__shfl_xor((int)j, o, 64);
    }
    if (lane == 0) {
        s_a[w] = a;
        s_b[w] = j;
    }
    __syncthreads();
    a = 0;
    j = 0;
    for (uint32_t q = 0; q < kScanBlock / 64u; ++q) {
        a += s_a[q];
        j += s_b[q];
    }
}

__global__ __launch_bounds__(kScanBlock) void kbp_sums(const uint32_t* __restrict__ cnt, uint64_t nkeys,
                                                       const uint32_t* __restrict__ tcnt, uint32_t nbl, uint32_t jobsz,
                                                       uint32_t* __restrict__ sums) {
    __shared__ uint32_t s_a[kScanBlock / 64u], s_b[kScanBlock / 64u];
    const uint32_t b = blockIdx.x;
    const bool tail = b >= nbl;
    const uint64_t e = (uint64_t)(tail ? b - nbl : b) * kScanBlock + threadIdx.x;
    const uint32_t v = tail ? (e < kTailBuckets ? tcnt[e] : 0u) : (e < nkeys ? cnt[e] : 0u);
    uint32_t a = v, j = (v + jobsz - 1u) / jobsz;
    block_sum2(a, j, s_a, s_b);
    if (threadIdx.x == 0) {
        sums[2 * b] = a;
        sums[2 * b + 1] = j;
    }
}

__global__ __launch_bounds__(kScanBlock) void kbp_offsets(uint32_t* __restrict__ cnt, uint64_t nkeys,
                                                          uint32_t* __restrict__ tcnt, uint32_t nbl, uint32_t ntb,
                                                          const uint32_t* __restrict__ sums, uint64_t n,
                                                          uint32_t jobsz, uint32_t* __restrict__ start,
                                                          uint32_t* __restrict__ jstart, uint32_t* __restrict__ jobpos,
                                                          uint32_t* __restrict__ njobs, uint32_t* __restrict__ nlong) {
    __shared__ uint32_t s_a[kScanBlock / 64u], s_b[kScanBlock / 64u];
    const uint32_t b = blockIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const bool tail = b >= nbl;
    // bases: the long blocks before this one (all of them for a tail block,
    // plus the tail blocks before it); nl / jl: the long totals
    uint32_t ba = 0, bj = 0, nl = 0, jl = 0;
    for (uint32_t q = lane; q < nbl + ntb; q += 64u) {
        const uint32_t sa = sums[2 * q], sj = sums[2 * q + 1];
        if (q < nbl) {
            nl += sa;
            jl += sj;
        }
        if (q < b && (q < nbl || tail)) {
            ba += sa;
            bj += sj;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ba += (uint32_t)__shfl_xor((int)ba, o, 64);
        bj += (uint32_t)__shfl_xor((int)bj, o, 64);
        nl += (uint32_t)__shfl_xor((int)nl, o, 64);
        jl += (uint32_t)__shfl_xor((int)jl, o, 64);
    }
    // (for a tail block ba already holds all long entries: its base is nlong
    // plus the tail blocks before it; the tail's job counts are not kept)
    const uint64_t e = (uint64_t)(tail ? b - nbl : b) * kScanBlock + threadIdx.x;
    const bool in = tail ? e < kTailBuckets : e < nkeys;
    const uint32_t v = in ? (tail ? tcnt[e] : cnt[e]) : 0u, vj = (v + jobsz - 1u) / jobsz;
    uint32_t ia = v, ij = vj;
#pragma unroll
    for (uint32_t o = 1; o < 64u; o <<= 1) {   // inclusive scan over the wave
        const uint32_t xa = (uint32_t)__shfl_up((int)ia, o, 64), xj = (uint32_t)__shfl_up((int)ij, o, 64);
        if (lane >= o) {
            ia += xa;
            ij += xj;
        }
    }
    if (lane == 63u) {
        s_a[w] = ia;
        s_b[w] = ij;
    }
    __syncthreads();
    for (uint32_t q = 0; q < w; ++q) {
        ba += s_a[q];
        bj += s_b[q];
    }
    if (in) {
        const uint32_t pa = ba + ia - v;
        if (tail) {
            tcnt[e] = pa;   // the scatter's cursor
        } else {
            start[e] = pa;
            cnt[e] = pa;
            jstart[e] = bj + ij - vj;
        }
    }
    if (b == 0 && threadIdx.x == 0) {
        start[nkeys] = nl;
        jstart[nkeys] = jl;
        const uint32_t tail_jobs = ((uint32_t)n - nl + jobsz - 1u) / jobsz;
        *nlong = nl;
        *njobs = jl + tail_jobs;
        jobpos[jl + tail_jobs] = (uint32_t)n;
    }
}

__global__ __launch_bounds__(kBpThreads) void kbp_scatter(const uint32_t* __restrict__ key_idx,
                                                          const uint32_t* __restrict__ len, uint32_t fixed_len,
                                                          uint64_t n, uint64_t nkeys, uint32_t split,
                                                          uint32_t* __restrict__ cur, uint32_t* __restrict__ tcur,
                                                          uint32_t* __restrict__ order) {
    __shared__ uint32_t h[kTailBuckets];
    uint32_t rank[kBpPer], bk[kBpPer];
    for (uint32_t b = threadIdx.x; b < kTailBuckets; b += kBpThreads) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kBpPer; ++r) {   // long records straight to their key; the tail's local ranks
        const uint64_t t = (uint64_t)blockIdx.x * (kBpThreads * kBpPer) + r * kBpThreads + threadIdx.x;
        bk[r] = 0xffffffffu;
        if (t >= n) continue;
        const uint32_t L = len ? len[t] : fixed_len;
        const uint32_t k = key_idx[t];
        if (k < nkeys && L >= split) {
            order[atomicAdd(&cur[k], 1u)] = (uint32_t)t;
        } else {
            bk[r] = tail_bucket(L);
            rank[r] = atomicAdd(&h[bk[r]], 1u);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kTailBuckets; b += kBpThreads)   // this workgroup's range per length
        if (h[b]) h[b] = atomicAdd(&tcur[b], h[b]);
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kBpPer; ++r) {
        const uint64_t t = (uint64_t)blockIdx.x * (kBpThreads * kBpPer) + r * kBpThreads + threadIdx.x;
        if (bk[r] != 0xffffffffu) order[h[bk[r]] + rank[r]] = (uint32_t)t;
    }
}

// A key's N or fewer records longest first (ties by record index), loaded at
// once and sorted in registers by an odd-even transposition network: static
// indices, so no scratch.  Empty places (length 0, index ~0) sort last.
template <uint32_t N>
__device__ __forceinline__ void kbp_sort_small(uint32_t* __restrict__ order, const uint32_t* __restrict__ len,
                                               uint32_t s0, uint32_t m) {
    uint32_t x[N], lx[N];
#pragma unroll
    for (uint32_t a = 0; a < N; ++a) x[a] = order[s0 + (a < m ? a : m - 1u)];   // unconditional loads
#pragma unroll
    for (uint32_t a = 0; a < N; ++a) lx[a] = len[x[a]];
#pragma unroll
    for (uint32_t a = 0; a < N; ++a)
        if (a >= m) {
            x[a] = 0xffffffffu;
            lx[a] = 0u;
        }
#pragma unroll
    for (uint32_t r = 0; r < N; ++r) {
#pragma unroll
        for (uint32_t a = r & 1u; a + 1u < N; a += 2u) {
            const bool sw = lx[a + 1] > lx[a] || (lx[a + 1] == lx[a] && x[a + 1] < x[a]);
            const uint32_t xa = x[a], la = lx[a];
            x[a] = sw ? x[a + 1] : xa;
            lx[a] = sw ? lx[a + 1] : la;
            x[a + 1] = sw ? xa : x[a + 1];
            lx[a + 1] = sw ? la : lx[a + 1];
        }
    }
#pragma unroll
    for (uint32_t a = 0; a < N; ++a)
        if (a < m) order[s0 + a] = x[a];
}

// One thread per key: its long records longest first (up to 8, 16 or 32 in
// registers, up to kBucketSortMax by insertion in place), then its jobs'
// first slots; the tail's jobs by grid stride.
__global__ __launch_bounds__(256) void kbp_finish(const uint32_t* __restrict__ start, const uint32_t* __restrict__ jstart,
                           const uint32_t* __restrict__ len, uint64_t nkeys, uint32_t jobsz,
                           uint32_t* __restrict__ order, uint32_t* __restrict__ jobpos,
                           const uint32_t* __restrict__ njobs, const uint32_t* __restrict__ nlong,
                           uint32_t* __restrict__ jobkey) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nkeys) {
        const uint32_t s0 = start[t], m = start[t + 1] - s0;
        if (len && m > 1u) {
            if (m <= 8u) {
                kbp_sort_small<8>(order, len, s0, m);
            } else if (m <= 16u) {
                kbp_sort_small<16>(order, len, s0, m);
            } else if (m <= 32u) {
                kbp_sort_small<32>(order, len, s0, m);
            } else if (m <= kBucketSortMax) {
                for (uint32_t a = 1; a < m; ++a) {   // insertion sort, in place
                    const uint32_t x = order[s0 + a], lx = len[x];
                    uint32_t b = a;
                    while (b > 0) {
                        const uint32_t y = order[s0 + b - 1u], ly = len[y];
                        if (ly > lx || (ly == lx && y < x)) break;
                        order[s0 + b] = y;
                        --b;
                    }
                    order[s0 + b] = x;
                }
            }
        }
        const uint32_t j0 = jstart[t];
        for (uint32_t q = 0; q * jobsz < m; ++q) {
            jobpos[j0 + q] = s0 + q * jobsz;
            if (jobkey) jobkey[j0 + q] = (uint32_t)t;
        }
    }
    const uint32_t jl = jstart[nkeys], nl = *nlong, jt = *njobs - jl;
    for (uint64_t q = t; q < jt; q += (uint64_t)gridDim.x * blockDim.x) {
        jobpos[jl + q] = nl + (uint32_t)q * jobsz;
        if (jobkey) jobkey[jl + q] = 0xffffffffu;
    }
}

int key_job_plan_counting(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                          uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                          uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s,
                          uint32_t* jobkey) {
    // [key counters | tail counters | start | jstart], each 256-byte aligned
    // (the scan reads the counters 16 bytes at a time)
    const size_t bk = ru256(nkeys * 4), bc = bk + ru256(kTailBuckets * 4), bs = ru256((nkeys + 1) * 4);
    const size_t need = bc + 2 * bs + ru256(8 * ((nkeys + kScanBlock - 1) / kScanBlock + kTailBuckets / kScanBlock));
    if (!scratch) {
        *bytes = need;
        return TG_OK;
    }
    if (*bytes < need || n == 0) return TG_EINVAL;
    uint8_t* p = static_cast<uint8_t*>(scratch);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(p);
    uint32_t* tcnt = reinterpret_cast<uint32_t*>(p + bk);
    uint32_t* start = reinterpret_cast<uint32_t*>(p + bc);
    uint32_t* jstart = reinterpret_cast<uint32_t*>(p + bc + bs);
    if (hipMemsetAsync(cnt, 0, bc, s) != hipSuccess) return TG_EHIP;
    const unsigned blocks = (unsigned)((n + kBpThreads * kBpPer - 1) / (kBpThreads * kBpPer));
    hipLaunchKernelGGL(kbp_count, dim3(blocks), dim3(kBpThreads), 0, s, key_idx, len, fixed_len, n, nkeys, split, cnt,
                       tcnt);
    const uint32_t nbl = (uint32_t)((nkeys + kScanBlock - 1) / kScanBlock), ntb = kTailBuckets / kScanBlock;
    uint32_t* sums = reinterpret_cast<uint32_t*>(p + bc + 2 * bs);
    hipLaunchKernelGGL(kbp_sums, dim3(nbl + ntb), dim3(kScanBlock), 0, s, cnt, nkeys, tcnt, nbl, jobsz, sums);
    hipLaunchKernelGGL(kbp_offsets, dim3(nbl + ntb), dim3(kScanBlock), 0, s, cnt, nkeys, tcnt, nbl, ntb, sums, n, jobsz,
                       start, jstart, jobpos, njobs, nlong);
    hipLaunchKernelGGL(kbp_scatter, dim3(blocks), dim3(kBpThreads), 0, s, key_idx, len, fixed_len, n, nkeys, split,
                       cnt, tcnt, order);
    const uint64_t fthreads = nkeys > n / jobsz ? nkeys : n / jobsz + 1;
    hipLaunchKernelGGL(kbp_finish, dim3((unsigned)((fthreads + 255) / 256)), dim3(256), 0, s, start, jstart, len, nkeys,
                       jobsz, order, jobpos, njobs, nlong, jobkey);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

}  // namespace

// scratch == nullptr: *bytes = what a batch of n needs.  Outputs: order[n]
// (record index per slot), jobpos[n + 1] (first slot of job j; jobpos[njobs]
// = n), *njobs and *nlong (device): slots [0, nlong) hold the records of at
// least ``split`` bytes with key_idx < nkeys, grouped by key, longest first
// within a key, cut into jobs of at most jobsz records; slots [nlong, n) the
// rest, longest first.  n < 2^32.  Up to kBucketMaxKeys keys the plan comes
// from counting (key_job_plan_counting), otherwise from a radix sort.
int tg_key_job_plan(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                    uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                    uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s,
                    uint32_t* jobkey) {
    if (jobsz == 0 || (jobsz & (jobsz - 1u))) return TG_EINVAL;
#if !defined(TG_PLAN_RADIX)   // A/B builds: the radix-sorted plan at any key count
    if (nkeys <= kBucketMaxKeys && n < 0xffffffffull)
        return key_job_plan_counting(key_idx, len, fixed_len, n, nkeys, split, jobsz, order, jobpos, njobs, nlong,
                                     scratch, bytes, s, jobkey);
#endif
    // 32-bit keys when the key index (tail marker nkeys included) leaves at
    // least 15 bits for the length: 2^14 + 256, the longest TLS record, fits
    const int kb = bit_width(nkeys);
    const int rc = kb <= 17 ? key_job_plan<uint32_t>(key_idx, len, fixed_len, n, nkeys, split, jobsz, order, jobpos,
                                                     njobs, nlong, scratch, bytes, s, 32 - kb)
                            : key_job_plan<uint64_t>(key_idx, len, fixed_len, n, nkeys, split, jobsz, order, jobpos,
                                                     njobs, nlong, scratch, bytes, s, 32);
    if (rc || !scratch || !jobkey) return rc;
    // every job holds at least one plan slot, so njobs <= n
    hipLaunchKernelGGL(kjp_jobkey, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, s, jobpos, njobs, nlong, order,
                       key_idx, jobkey);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

namespace {
template <class K>
int key_job_plan(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                 uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                 uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s, int lb) {
    rocprim::counting_iterator<uint32_t> iota(0);
    const int kbits = lb + bit_width(nkeys);   // significant bits of the sort key
    size_t t_sort = 0, t_max = 0, t_sum = 0;
    if (rocprim::radix_sort_pairs(nullptr, t_sort, (K*)nullptr, (K*)nullptr, iota, (uint32_t*)nullptr, (size_t)n,
                                  0, kbits, s) != hipSuccess ||
        rocprim::inclusive_scan(nullptr, t_max, (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                                rocprim::maximum<uint32_t>(), s) != hipSuccess ||
        rocprim::inclusive_scan(nullptr, t_sum, (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n,
                                rocprim::plus<uint32_t>(), s) != hipSuccess)
        return TG_EHIP;
    const size_t bk = ru256(n * sizeof(K)), b32 = ru256(n * 4);
    size_t tmp = t_sort > t_max ? t_sort : t_max;
    tmp = tmp > t_sum ? tmp : t_sum;
    const size_t need = 2 * bk + 3 * b32 + ru256(tmp);
    if (!scratch) {
        *bytes = need;
        return TG_OK;
    }
    if (*bytes < need || n == 0) return TG_EINVAL;
    uint8_t* p = static_cast<uint8_t*>(scratch);
    K* ck = reinterpret_cast<K*>(p);
    K* ck_sorted = reinterpret_cast<K*>(p + bk);
    uint32_t* g = reinterpret_cast<uint32_t*>(p + 2 * bk);
    uint32_t* gs = reinterpret_cast<uint32_t*>(p + 2 * bk + b32);
    uint32_t* js = reinterpret_cast<uint32_t*>(p + 2 * bk + 2 * b32);
    void* t = p + 2 * bk + 3 * b32;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL((kjp_keys<K>), dim3(blocks), dim3(256), 0, s, key_idx, len, fixed_len, n, nkeys, split, lb,
                       ck, nlong);
    size_t ts = t_sort;
    if (rocprim::radix_sort_pairs(t, ts, ck, ck_sorted, iota, order, (size_t)n, 0, kbits, s) != hipSuccess)
        return TG_EHIP;
    hipLaunchKernelGGL((kjp_tail<K>), dim3(blocks), dim3(256), 0, s, ck_sorted, n, nkeys, lb, nlong);
    hipLaunchKernelGGL((kjp_group_starts<K>), dim3(blocks), dim3(256), 0, s, ck_sorted, n, lb, g);
    size_t tm = t_max;
    if (rocprim::inclusive_scan(t, tm, g, gs, (size_t)n, rocprim::maximum<uint32_t>(), s) != hipSuccess)
        return TG_EHIP;
    hipLaunchKernelGGL(kjp_job_starts, dim3(blocks), dim3(256), 0, s, gs, n, jobsz, js);
    uint32_t* jx = g;   // reused: the group starts are no longer needed
    size_t tp = t_sum;
    if (rocprim::inclusive_scan(t, tp, js, jx, (size_t)n, rocprim::plus<uint32_t>(), s) != hipSuccess)
        return TG_EHIP;
    hipLaunchKernelGGL(kjp_scatter, dim3(blocks), dim3(256), 0, s, js, jx, n, jobpos, njobs);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}
}  // namespace
