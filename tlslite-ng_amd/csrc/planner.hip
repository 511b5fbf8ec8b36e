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

// scratch == nullptr: *bytes = what a batch of n needs.  Outputs: order[n]
// (record index per slot), jobpos[n + 1] (first slot of job j; jobpos[njobs]
// = n), *njobs and *nlong (device): slots [0, nlong) hold the records of at
// least ``split`` bytes with key_idx < nkeys, grouped by key, longest first
// within a key, cut into jobs of at most jobsz records; slots [nlong, n) the
// rest, longest first.  n < 2^32.
int tg_key_job_plan(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                    uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                    uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s) {
    if (jobsz == 0 || (jobsz & (jobsz - 1u))) return TG_EINVAL;
    // 32-bit keys when the key index (tail marker nkeys included) leaves at
    // least 15 bits for the length: 2^14 + 256, the longest TLS record, fits
    const int kb = bit_width(nkeys);
    if (kb <= 17)
        return key_job_plan<uint32_t>(key_idx, len, fixed_len, n, nkeys, split, jobsz, order, jobpos, njobs,
                                      nlong, scratch, bytes, s, 32 - kb);
    return key_job_plan<uint64_t>(key_idx, len, fixed_len, n, nkeys, split, jobsz, order, jobpos, njobs, nlong,
                                  scratch, bytes, s, 32);
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
