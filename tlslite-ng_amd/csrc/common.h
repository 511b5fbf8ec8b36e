// common.h -- shared device helpers and key layouts for libtlsgpu.
//
// Layout of one AES-GCM key in HBM (GcmKeyDev) and the per-record accessors
// used by every kernel.  All record data is handled as little-endian 32-bit
// words of the wire bytes, so a 16-byte block is one uint4 load and no byte
// swapping happens on the hot path (GHASH tables are built in the same byte
// layout on the host, see host.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "keymath.h"
#include "tlsgpu.h"

namespace tg {

// Measurement builds (tools/build_variant.sh -D...) that return wrong bytes or
// differ from the product in their memory behaviour.  A translation unit
// compiled with one of these flags registers itself at load time; tg_version()
// then carries a "MEASUREMENT BUILD" marker and tlsgpu.load() refuses the
// library unless TLSGPU_ALLOW_MEASUREMENT_BUILD=1.
void note_measurement_build(const char* flag);
#if defined(TG_CHACHA_NO_IO) || defined(TG_CHACHA_ILV) || defined(TG_KT_NO_GHASH) || \
    defined(TG_KT_NO_BUILD) || defined(TG_NT_IO) || defined(TG_TAIL_PROBE) || defined(TG_ROLE_PROBE)
namespace {
struct MeasurementMark {
    MeasurementMark() {
#if defined(TG_CHACHA_NO_IO)
        note_measurement_build("TG_CHACHA_NO_IO");
#endif
#if defined(TG_CHACHA_ILV)
        note_measurement_build("TG_CHACHA_ILV");
#endif
#if defined(TG_KT_NO_GHASH)
        note_measurement_build("TG_KT_NO_GHASH");
#endif
#if defined(TG_KT_NO_BUILD)
        note_measurement_build("TG_KT_NO_BUILD");
#endif
#if defined(TG_NT_IO)
        note_measurement_build("TG_NT_IO");
#endif
#if defined(TG_TAIL_PROBE)
        note_measurement_build("TG_TAIL_PROBE");
#endif
#if defined(TG_ROLE_PROBE)
        note_measurement_build("TG_ROLE_PROBE");
#endif
    }
} g_measurement_mark;
}  // namespace
#endif

// The lane's index within its wave, computed inside an asm: the compiler can
// neither hoist it out of a loop nor reuse an earlier copy, so the values
// derived from it are recomputed where they are used instead of being held in
// VGPRs across long loops (the persistent kernels spilled such values).
__device__ __forceinline__ uint32_t fresh_lane() {
    uint32_t l;
    __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// 16 tables x 256 entries x 16 bytes: M_j[b] = b * x^(8j) * H, so that
// X * H = XOR_j M_j[byte_j(X)] (GCM bit order, aesgcm.py:8-14).
constexpr int kGhashEntries = 16 * 256;

struct GcmKeyDev {
    uint32_t rk[60];       // round keys as LE words of the key-schedule bytes
    uint32_t rounds;       // 10 (AES-128) or 14 (AES-256)
    uint32_t pad[3];
    uint4 ghash[kGhashEntries];
    uint4 hpow[2048];      // H^1 .. H^kHPow, normal order (gcm_wave_kernel)
    uint4 ghash64[kGhashEntries];   // the 8-bit tables of H^64 (gcm_wave_kernel's stride)
    uint4 ghash8[kGhashEntries];    // the 8-bit tables of H^8 (gcm_bs8_kernel's stride)
    // 8-block bitsliced AES (aes_bs8.h): round-key plane (r, i, b) at (4 r + i) 8 + b
    uint32_t bs8mask[15 * 32];
    // the hybrid kernel's key material, built with the key: the bitsliced
    // waves' key rows (keymath.h bs8_row_word) and the T-table waves' rotated
    // round keys (rkrot_word)
    uint32_t bs8rows[15 * 32];
    uint32_t rkrot[64];
};

// Powers of H for the wave-per-record kernel: hpow[e - 1] = H^e in normal
// polynomial order (coefficient of x^i at bit i of the 128-bit value, word 0
// first) for e = 1 .. kHPow.
constexpr int kHPow = 2048;

// Entry e of the 8-bit GHASH tables of G as a uint4 (keymath.h
// ghash_table_words): built on the device by keysetup.hip and by the
// self-test (selftest.hip); host.cpp's builder gives the same tables.
__host__ __device__ inline uint4 ghash_table_entry(const uint32_t hv[4], int e) {
    uint32_t w[4];
    ghash_table_words(hv, e, w);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// One entry of an AES-GCM key table (many sessions in one batch): the round
// keys and H = E_K(0) in normal polynomial order (see GhashClmul).
struct GcmTableKey {
    uint32_t rk[60];
    uint32_t hn[4];
};

// One AES key (AES-CCM): the round keys; a key table is an array of these.
struct AesKeyDev {
    uint32_t rk[60];
    uint32_t pad[4];
};

struct ChachaKeyDev {
    uint32_t k[8];         // key as LE words (chacha.py:101, _bytearray_to_words)
};

// 16-byte global accesses through pointers the compiler cannot place (read
// back from LDS or from a descriptor in memory): without the address space it
// emits FLAT instructions, which also count on lgkmcnt, so every LDS wait
// would wait for the HBM access too.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(TG_NT_IO)   // measurement build (tools/build_variant.sh): non-temporal record I/O
    const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)p);
#else
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)p;
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return uint4();
#endif
}
__device__ __forceinline__ void gstore16(uint8_t* p, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(TG_NT_IO)
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (__attribute__((address_space(1))) u32x4*)p);
#else
    *(__attribute__((address_space(1))) u32x4*)p = u32x4{v.x, v.y, v.z, v.w};
#endif
#endif
}

// The same at any byte address: one global_load/store_dwordx4 with the byte
// offset (amdhsa runs gfx9 in unaligned-access mode), instead of 16 byte
// accesses -- records behind a 5-byte TLS header are never 16-byte aligned.
typedef u32x4 u32x4_u1 __attribute__((aligned(1)));
__device__ __forceinline__ uint4 gload16u(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(TG_NT_IO)
    const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4_u1*)p);
#else
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4_u1*)p;
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return uint4();
#endif
}
__device__ __forceinline__ void gstore16u(uint8_t* p, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
#if defined(TG_NT_IO)
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (__attribute__((address_space(1))) u32x4_u1*)p);
#else
    *(__attribute__((address_space(1))) u32x4_u1*)p = u32x4{v.x, v.y, v.z, v.w};
#endif
#endif
}

// gload16u / gstore16u with the non-temporal hint: payload that is read or
// written once and should not push other data out of L2 (aes_gcm_bs8.hip
// octet_job: the key material and GHASH rows it re-reads every batch stay
// resident).
__device__ __forceinline__ uint4 gload16u_nt(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4_u1*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return uint4();
#endif
}
__device__ __forceinline__ void gstore16u_nt(uint8_t* p, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (__attribute__((address_space(1))) u32x4_u1*)p);
#endif
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t v, int c) {
    return __builtin_amdgcn_alignbit(v, v, 32 - c);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) {
    return __builtin_bswap32(v);
}

// p[i] of a global array (batch metadata behind descriptor pointers).
template <class T>
__device__ __forceinline__ T gld(const T* p, uint64_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(1))) T*)p)[i];
#else
    return p[i];
#endif
}
template <class T>
__device__ __forceinline__ void gst(T* p, uint64_t i, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
    ((__attribute__((address_space(1))) T*)p)[i] = v;
#else
    p[i] = v;
#endif
}

__device__ __forceinline__ const uint8_t* rec_in(const tg_batch& b, uint64_t i) {
    return b.in + (b.in_off ? gld(b.in_off, i) : i * b.in_stride);
}
__device__ __forceinline__ uint8_t* rec_out(const tg_batch& b, uint64_t i) {
    return b.out + (b.out_off ? gld(b.out_off, i) : i * b.out_stride);
}
__device__ __forceinline__ uint32_t rec_len(const tg_batch& b, uint64_t i) {
    return b.len ? gld(b.len, i) : b.fixed_len;
}
__device__ __forceinline__ const uint8_t* rec_aad(const tg_batch& b, uint64_t i) {
    return b.aad + (b.aad_off ? gld(b.aad_off, i) : i * b.aad_stride);
}
__device__ __forceinline__ uint32_t rec_aad_len(const tg_batch& b, uint64_t i) {
    return b.aad_len ? gld(b.aad_len, i) : b.fixed_aad_len;
}

// Record memory is global.  The record pointers come out of the batch
// descriptor, so the compiler cannot place them and would emit FLAT accesses
// (which also count on lgkmcnt: an LDS wait then waits for HBM too); these
// helpers address global memory explicitly.
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(1))) uint8_t* gptr_c;
typedef __attribute__((address_space(1))) uint8_t* gptr;
#else
typedef const uint8_t* gptr_c;
typedef uint8_t* gptr;
#endif

// n (<= 16) bytes from p, zero-padded, as 4 LE words.  Fully unrolled with
// compile-time word indices so nothing is placed in scratch.
__device__ __forceinline__ uint4 load_partial(const uint8_t* p, uint32_t n) {
    const gptr_c g = (gptr_c)p;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
        if (k < n) w[k >> 2] |= (uint32_t)g[k] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_partial(uint8_t* p, uint4 v, uint32_t n) {
    const gptr g = (gptr)p;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
        if (k < n) g[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// Full 16-byte block; the vector form when the record is 16-byte aligned.
__device__ __forceinline__ uint4 load16(const uint8_t* p, bool aligned) {
    return aligned ? gload16(p) : gload16u(p);
}

__device__ __forceinline__ void store16(uint8_t* p, uint4 v, bool aligned) {
    if (aligned) {
        gstore16(p, v);
    } else {
        gstore16u(p, v);
    }
}

__device__ __forceinline__ uint4 mask_tail(uint4 v, uint32_t n) {
    // keep the first n (< 16) bytes of a block, zero the rest
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int keep = (int)n - 4 * k;
        uint32_t m = keep >= 4 ? 0xffffffffu : (keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u));
        w[k] &= m;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// The session-independent part of an HKDF-Expand-Label call (keysetup.hip):
// info || 0x01 and its SHA padding, as big-endian 32-bit words of the message
// blocks that follow the (K ^ ipad) block.
struct HkdfMsg {
    uint32_t nblocks;     // SHA-256: 64-byte blocks (16 words); SHA-384: 128-byte (32 words)
    uint32_t outlen;      // bytes kept of T(1), <= hash length
    uint32_t words[64];
};

// Per-call device scratch of the record-framing entry points (records.hip).
struct RecScratch {
    uint64_t* in_abs;     // AEAD input address per record (open)
    uint64_t* out_abs;    // AEAD output address per record
    uint32_t* len;        // AEAD payload length (inner plaintext / ciphertext)
    uint8_t* nonce;       // 12 B per record
    uint8_t* aad;         // 16 B stride, 5 or 13 used
    uint32_t* aad_len;
    uint8_t* st;          // framing status from prep (open)
    uint8_t* aead_st;     // AEAD open status
    uint8_t* dummy;       // 32 zero bytes: AEAD input of publicly-invalid records
};

// The per-slot keystream precompute of the AES-GCM octet / pair jobs
// (aes_gcm_bs8.hip): a record of nc blocks whose last batch row (8 blocks of
// each of its LPR lanes) holds only its last block -- nc % (8 LPR) == 1, e.g.
// a full TLS 1.3 record's 16 385-byte inner plaintext -- gets that block's
// keystream at mask slot 2 t + 1 (hy_mask_kernel: LPR 8, kt_mask_kernel: LPR
// 32), and octet_job's seal path reads it exactly then.  One definition for
// the writers and the reader.
template <int LPR>
__host__ __device__ constexpr bool lone_last_block(uint32_t nc) {
    return nc % (8u * LPR) == 1u;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for ``fn`` on the current
// device, once per (function, device); thread-safe (api.hip).  0 or TG_EHIP.
int lds_attr(const void* fn, int bytes);

// Per-launch device scratch for launches on stream ``s``: stream_alloc takes
// a buffer of at least ``bytes`` from a process-wide cache (reused once the
// launches that last used it have completed, or at once by the next launch
// on the same stream), stream_free hands it back behind the work queued on
// ``s`` (api.hip).  0, TG_EHIP, or TG_EINVAL for a pointer not from
// stream_alloc.
int stream_alloc(void** p, size_t bytes, hipStream_t s);
int stream_free(void* p, hipStream_t s);
void scratch_totals(uint64_t* bytes, uint64_t* buffers);   // tg_scratch_info
void scratch_trim(size_t keep);                             // tg_scratch_trim

// A helper stream beside caller stream ``s`` (api.hip pool): helper_fork
// takes one (idle, or last used by ``s``) and makes it wait for the work
// queued on ``s`` so far; *h = nullptr when ``s`` belongs to another device
// than the current one (run everything on ``s`` then).  helper_join makes
// ``s`` wait for the helper's work and gives the helper back.  0 or TG_EHIP.
int helper_fork(hipStream_t s, hipStream_t* h);
int helper_join(hipStream_t h, hipStream_t s);
void helper_totals(uint64_t* streams, uint64_t* busy);

// Compute units of the current device (grid size of the persistent kernels),
// looked up once per device.
inline int device_cus() {
    // one entry per device, filled by whichever thread gets there first;
    // every thread would store the same value, but the entries are atomics so
    // concurrent tg_seal / tg_open calls on one handle are race-free
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int v = cache[dev].load(std::memory_order_relaxed);
    if (!v) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        cache[dev].store(cus, std::memory_order_relaxed);
        v = cus;
    }
    return v;
}

}  // namespace tg

// Launchers implemented in the kernel files (host side).
// order: NULL, or the processing order of the records (planner.hip): thread
// t of a lane-per-record kernel handles record order[t].
int tg_launch_gcm(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                  hipStream_t s, const uint32_t* order = nullptr);
// The 8-block bitsliced single-key kernel and the hybrid T-table + bitsliced
// persistent kernel (aes_gcm_bs8.hip).
int tg_launch_gcm_hy(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                     hipStream_t s, const uint32_t* order);
int tg_launch_gcm_bs8(const tg::GcmKeyDev* key, int rounds, const tg_batch& b, bool open,
                      hipStream_t s, const uint32_t* order);
// hpow[64 k + e - 1] = H_k^e (normal order), e = 1..64, for the n keys.
int tg_launch_table_hpow(const tg::GcmTableKey* keys, uint64_t n, uint4* hpow, hipStream_t s);
int tg_length_order(const uint32_t* len, uint64_t n, uint32_t* order, void* scratch, size_t* bytes,
                    hipStream_t s);
// Open over a key table: zero the output of every record whose key_idx is not
// below nkeys (the AEAD kernels skip it with status 0; planner.hip).
int tg_launch_zero_skipped(const tg_batch& b, uint64_t nkeys, hipStream_t s);
// Key-grouped jobs of a key-table batch (planner.hip): records of at least
// ``split`` bytes with key_idx < nkeys in front, grouped by key and cut into
// jobs of at most jobsz (a power of two) records of one key; the rest
// behind them from slot *nlong on, longest first.  jobkey (optional, n + 1
// entries): each job's key, ~0 for the tail's jobs.
int tg_key_job_plan(const uint32_t* key_idx, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                    uint64_t nkeys, uint32_t split, uint32_t jobsz, uint32_t* order, uint32_t* jobpos,
                    uint32_t* njobs, uint32_t* nlong, void* scratch, size_t* bytes, hipStream_t s,
                    uint32_t* jobkey = nullptr);
// Key-table AES-GCM (aes_gcm_bs8.hip launch_kt): records of at least
// ``split`` bytes through the key-grouped octet kernel (planes = per-key
// bitsliced key rows, MixColumns-folded, tg_launch_kt_planes; hpow = the keys'
// H^1..H^64), the others through the lane kernel.
// lpr: lanes per record of the key-grouped bitsliced kernel for the long
// records (8, 16, 32 or 64), or 0 for the wave-per-record T-table kernel
// with per-wave 4-bit GHASH tables.  hybrid (lpr 32 only): the long records on
// the persistent T-table + bitsliced kernel (rot = the keys' rotated round
// keys, tg_launch_kt_planes).
int tg_launch_gcm_kt(const tg::GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, const uint32_t* planes,
                     const uint4* rot, int rounds, const tg_batch& b, bool open, hipStream_t s, uint32_t split,
                     int lpr, bool hybrid);
// The key-table lane kernel over slots [*first, n) of ``order`` (first NULL:
// all of them) and the key-table wave-per-record kernel (aes_gcm.hip).
int tg_launch_gcm_table_lane(const tg::GcmTableKey* keys, uint64_t nkeys, int rounds, const tg_batch& b,
                             bool open, hipStream_t s, const uint32_t* order, const uint32_t* first);
// t4: GHASH through per-wave 4-bit tables of H^64 (else table-free); plan
// slots [0, *count) of ``order`` (NULL: every record, in order).
int tg_launch_gcm_table_wave(const tg::GcmTableKey* keys, uint64_t nkeys, const uint4* hpow, int rounds,
                             const tg_batch& b, bool open, hipStream_t s, bool t4,
                             const uint32_t* order = nullptr, const uint32_t* count = nullptr);
// The key table's bitsliced key rows (planes) and the T-table waves' rotated
// round keys (rot, 16 x 16 bytes per key).
int tg_launch_kt_planes(const tg::GcmTableKey* keys, uint64_t n, int rounds, uint32_t* planes,
                        uint4* rot, hipStream_t s);
int tg_launch_ccm(const tg::AesKeyDev* keys, uint64_t nkeys, int rounds, int taglen,
                  const tg_batch& b, bool open, hipStream_t s);
// Whether a single-key batch of n records runs the wave-per-record kernel
// (no length planning needed then).
bool tg_gcm_wave_path(uint64_t n);
bool tg_chacha_wave_path(uint64_t n);
int tg_launch_chacha(const tg::ChachaKeyDev* keys, uint64_t nkeys, const tg_batch& b, bool open, hipStream_t s,
                     const uint32_t* order = nullptr);
int tg_launch_records_prep(const tg_records& r, bool seal, bool aes, int taglen,
                           const tg::RecScratch& s, hipStream_t st);
int tg_launch_records_finish(const tg_records& r, const tg::RecScratch& s, hipStream_t st);
int tg_launch_hkdf(int hashlen, const tg::HkdfMsg& msg, const uint8_t* secrets, uint64_t n,
                   uint8_t* out, hipStream_t s);
int tg_launch_aes_setup(int keylen, int layout, const uint8_t* keys, uint64_t n, void* out,
                        hipStream_t s);
int tg_launch_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
                     const uint64_t* dst_off, uint64_t n, hipStream_t s);
int tg_launch_nonces(int mode, const uint8_t* iv_host, uint64_t seq0, uint64_t n, uint8_t* out,
                     hipStream_t s);
