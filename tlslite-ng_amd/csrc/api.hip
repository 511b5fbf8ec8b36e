// api.hip -- the C ABI of libtlsgpu.so (declared in include/tlsgpu.h).
//
// Host side of the engine: key objects (AES key schedule and GHASH tables
// built once per key, like AESGCM.__init__ at tlslite/utils/aesgcm.py:27-57),
// the per-record drop-in entry points that the ctypes objects behind
// tlsgpu.cipherfactory call for every record (recordlayer.py:558, :821), and
// the device-pointer batch entry points.  No exceptions cross the ABI.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "aes_bs8.h"
#include "common.h"
#include "host.h"
#include "options.h"
#include "tlsgpu.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(TG_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                        __FILE__, __LINE__);                                          \
    } while (0)

using tg::host::le32;

// host.cpp fills the GcmKeyDev image without HIP types: same layout.
#define TG_SAME_OFFSET(m) \
    static_assert(offsetof(tg::GcmKeyDev, m) == offsetof(tg::host::GcmKeyImage, m), #m)
static_assert(sizeof(tg::GcmKeyDev) == sizeof(tg::host::GcmKeyImage), "GcmKeyDev image size");
TG_SAME_OFFSET(rounds);
TG_SAME_OFFSET(ghash);
TG_SAME_OFFSET(hpow);
TG_SAME_OFFSET(ghash64);
TG_SAME_OFFSET(ghash8);
TG_SAME_OFFSET(bs8mask);
TG_SAME_OFFSET(bs8rows);
TG_SAME_OFFSET(rkrot);
#undef TG_SAME_OFFSET

}  // namespace

// Staging of one per-record call in flight: a mapped pinned buffer, its
// device twin (option stage_copy) and a stream.  A key keeps a pool of them:
// a call takes a free slot (or makes one) and gives it back, so calls on
// copies of one AEAD object (copy.copy shares the handle, recordlayer.py:262,
// :913) from several threads never share a buffer -- ctypes releases the GIL
// around every call.
struct Stage {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
};

struct tg_key {
    int alg;
    size_t keylen;
    size_t nkeys;
    int device;
    int rounds;
    int taglen;             // 16, or 8 for AES-CCM_8
    void* dev_key;          // GcmKeyDev / GcmTableKey[nkeys] (AES-GCM),
                            // AesKeyDev[nkeys] (AES-CCM), ChachaKeyDev[nkeys]
    std::mutex stage_mu;    // guards the two lists
    std::vector<Stage*> stages;        // every slot of this key
    std::vector<Stage*> free_stages;   // the idle ones (never trimmed before destroy)
};

namespace {

int select_device(const tg_key* k) {
    int cur = -1;
    HIP_TRY(hipGetDevice(&cur));
    if (cur != k->device) HIP_TRY(hipSetDevice(k->device));
    return TG_OK;
}

void free_stage(Stage* st) {
    if (st->h) (void)hipHostFree(st->h);
    if (st->d) (void)hipFree(st->d);
    if (st->stream) (void)hipStreamDestroy(st->stream);
    delete st;
}

// A free staging slot of this key (a new one if all are in use).  Returns
// TG_OK with *out set, or the error code recorded by fail() (TG_ENOMEM for
// host memory, TG_EHIP when the stream cannot be created).
int take_stage(tg_key* k, Stage** out) {
    {
        std::lock_guard<std::mutex> g(k->stage_mu);
        if (!k->free_stages.empty()) {
            *out = k->free_stages.back();
            k->free_stages.pop_back();
            return TG_OK;
        }
    }
    Stage* st = new (std::nothrow) Stage();
    if (!st) return fail(TG_ENOMEM, "out of host memory");
    hipError_t e = hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete st;
        return fail(TG_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> g(k->stage_mu);
    k->stages.push_back(st);
    *out = st;
    return TG_OK;
}

// A slot given back stays with the key until tg_key_destroy: the pool is as
// large as the most calls the key has had in flight at once, so bursts of
// concurrent calls reuse their slots instead of destroying streams and
// freeing pinned memory (which can synchronise the device) after each burst
// (ADVICE r04).
void give_stage(tg_key* k, Stage* st) {
    std::lock_guard<std::mutex> g(k->stage_mu);
    k->free_stages.push_back(st);
}

int ensure_stage(Stage* st, size_t bytes) {
    if (bytes <= st->cap) return TG_OK;
    size_t cap = st->cap ? st->cap : 65536;
    while (cap < bytes) cap *= 2;
    if (st->h) (void)hipHostFree(st->h);
    if (st->d) (void)hipFree(st->d);
    st->h = nullptr;
    st->d = nullptr;
    st->cap = 0;
    HIP_TRY(hipHostMalloc((void**)&st->h, cap, hipHostMallocMapped));
    HIP_TRY(hipMalloc((void**)&st->d, cap));
    st->cap = cap;
    return TG_OK;
}

bool is_ccm(int alg) { return alg == TG_AES_CCM || alg == TG_AES_CCM_8; }

// A multi-key AES-GCM allocation: GcmTableKey[nkeys], then the 64 GHASH
// powers of each key (gcm_table_wave_kernel, gcm_kt_kernel), then the 15 x 32
// bitsliced key-plane words of each key, MixColumns-folded, in the hybrid
// kernel's row layout (gcm_kt_kernel, kt_planes_kernel), then 16 rotated
// round-key words x 4 per key (gcm_kth_kernel's T-table waves, kt_rot_kernel).
constexpr size_t kTableHpowBytes = 64 * sizeof(uint4);
constexpr size_t kTablePlaneBytes = 15 * 32 * sizeof(uint32_t);
constexpr size_t kTableRotBytes = 16 * sizeof(uint4);
uint4* table_hpow(const tg_key* k) {
    return reinterpret_cast<uint4*>(static_cast<uint8_t*>(k->dev_key) +
                                    sizeof(tg::GcmTableKey) * k->nkeys);
}
uint32_t* table_planes(const tg_key* k) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(table_hpow(k)) +
                                       kTableHpowBytes * k->nkeys);
}
uint4* table_rot(const tg_key* k) {
    return reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(table_planes(k)) + kTablePlaneBytes * k->nkeys);
}

// The table's derived arrays on the device: H^1..H^64 and the key planes.
int table_derive(tg_key* k, hipStream_t s) {
    const auto* keys = static_cast<const tg::GcmTableKey*>(k->dev_key);
    int rc = tg_launch_table_hpow(keys, k->nkeys, table_hpow(k), s);
    if (!rc) rc = tg_launch_kt_planes(keys, k->nkeys, k->rounds, table_planes(k), table_rot(k), s);
    return rc;
}

size_t dev_key_bytes(const tg_key* k) {
    if (k->alg == TG_CHACHA20_POLY1305) return sizeof(tg::ChachaKeyDev) * k->nkeys;
    if (is_ccm(k->alg)) return sizeof(tg::AesKeyDev) * k->nkeys;
    return k->nkeys > 1 ? (sizeof(tg::GcmTableKey) + kTableHpowBytes + kTablePlaneBytes + kTableRotBytes) * k->nkeys
                        : sizeof(tg::GcmKeyDev);
}

// Batches that run a lane-per-record kernel (more records than the
// wave-per-record kernels take) with per-record lengths run longest first
// (planner.hip): a wave then holds records of nearly one length instead of
// idling behind its longest.
constexpr uint64_t kPlanMinRecords = 2049;

// Key-table AES-GCM: records of at least this many bytes take the
// key-grouped octet kernel, shorter ones the lane kernel (option kt_split).
constexpr uint32_t kKtSplitDefault = 2048;
// With the short records inside the key-table hybrid (its lane loop runs
// beside the long jobs instead of after them) the split moves down.  With two
// pairs per planned job: config 4 674-676 GiB/s at 1 024 against 663-668 at
// 2 048 (profiles/r06/s2/); with four (TG_KTH_GROUP): 694.5-696.7 at 1 536,
// 694.3-694.6 at 1 280, 693.1-693.8 at 1 792, 690.4 at 2 048, 688.4-689.1 at
// 1 024, 681 at 768 (profiles/r06/s4/, s5/).
constexpr uint32_t kKtSplitFused = 1536;
// Small key-table batches -- at most this many records, or one length with
// at most this many bytes in all -- run one record per wavefront (the wave
// kernel, table-free GHASH, no plan): 0.014 / 0.023 / 0.099 ms for 1 / 2 048 /
// 16 384 records of 1 KiB against 0.23 / 0.32 / 0.34 ms planned, and 0.11
// against 0.21 ms for 2 048 records of 16 KiB (profiles/r04/r4w/).
constexpr uint64_t kKtWaveMaxRecords = 2048;
constexpr uint64_t kKtWaveMaxBytes = 16ull << 20;

int launch_kernels(tg_key* k, const tg_batch& b, bool open, hipStream_t s, const uint32_t* order) {
    if (k->alg == TG_AES_GCM)
        return tg_launch_gcm(static_cast<const tg::GcmKeyDev*>(k->dev_key), k->rounds, b, open, s, order);
    return tg_launch_chacha(static_cast<const tg::ChachaKeyDev*>(k->dev_key), k->nkeys, b, open, s, order);
}

// Key-table AES-GCM (option gcm_table_variant): 0 = auto (small batches one
// record per wavefront, see kKtWaveMaxRecords; otherwise a length split at
// kt_split: the long records on the kernel kt_lpr picks -- 0 = default,
// 8 / 16 / 32 / 64 lanes per record on the key-grouped bitsliced kernel, -1
// the wave-per-record T-table kernel with 4-bit GHASH tables -- the rest on
// the lane kernel, one plan); 1 = the lane kernel for every record; 5 = the
// wave-per-record kernel, table-free GHASH, no plan; 6 = the wave-per-record
// kernel with 4-bit tables for every record; 14 = the octet kernel (8 lanes
// per record) for every record.
constexpr int kKtLprDefault = 32;

int launch_gcm_table(tg_key* k, const tg_batch& b, bool open, hipStream_t s) {
    const auto* keys = static_cast<const tg::GcmTableKey*>(k->dev_key);
    uint32_t split;
    const int o = tg::opt(tg::kOptKtLpr);
    int lpr = o == 0 ? kKtLprDefault : o < 0 ? 0 : o;
    switch (tg::opt(tg::kOptGcmTableVariant)) {
        case 0: {
            const int sp = tg::opt(tg::kOptKtSplit);
            split = sp > 0 ? (uint32_t)sp
                  : lpr == 32 && tg::opt(tg::kOptKtHybrid) >= 0 ? kKtSplitFused : kKtSplitDefault;
            // small batches (unless the split or the long-record kernel is forced)
            if (sp == 0 && o == 0 &&
                (b.n <= kKtWaveMaxRecords || (!b.len && b.n * (uint64_t)b.fixed_len <= kKtWaveMaxBytes)))
                return tg_launch_gcm_table_wave(keys, k->nkeys, table_hpow(k), k->rounds, b, open, s, false);
            break;
        }
        case 1: split = 0xffffffffu; break;
        case 5: return tg_launch_gcm_table_wave(keys, k->nkeys, table_hpow(k), k->rounds, b, open, s, false);
        case 6: split = 0; lpr = 0; break;
        case 14: split = 0; lpr = 8; break;
        default: return TG_EINVAL;
    }
    // One length for every record, below the split (or option no_plan): every
    // record is the lane kernel's and a length order is moot, so no plan --
    // its sort, scans and stream-ordered allocation are pure latency for small
    // multi-session batches (profiles/r04/r4w/).
    if (split != 0 && ((!b.len && b.fixed_len < split) || tg::opt(tg::kOptNoPlan)))
        return tg_launch_gcm_table_lane(keys, k->nkeys, k->rounds, b, open, s, nullptr, nullptr);
    // the long records (lpr 32) on the T-table + bitsliced kernel unless
    // kt_hybrid = -1 (the bitsliced-only key-grouped kernel)
    const bool hybrid = lpr == 32 && tg::opt(tg::kOptKtHybrid) >= 0;
    return tg_launch_gcm_kt(keys, k->nkeys, table_hpow(k), table_planes(k), table_rot(k), k->rounds, b, open, s,
                            split, lpr, hybrid);
}

// The order and the sort's scratch come from the per-launch scratch cache
// (stream_alloc / stream_free), so batches in flight on other streams never
// share them.
int launch(tg_key* k, const tg_batch& b, bool open, hipStream_t s) {
    if (is_ccm(k->alg))
        return tg_launch_ccm(static_cast<const tg::AesKeyDev*>(k->dev_key), k->nkeys, k->rounds, k->taglen,
                             b, open, s);
    if (k->alg == TG_AES_GCM && k->nkeys > 1) return launch_gcm_table(k, b, open, s);
    // (ChaCha key tables take the wave kernel too: chacha_wave_kernel<.., MULTIKEY>)
    const bool wave = (k->nkeys == 1 && k->alg == TG_AES_GCM && tg_gcm_wave_path(b.n)) ||
                      (k->alg == TG_CHACHA20_POLY1305 && tg_chacha_wave_path(b.n));
    if (!b.len || b.n < kPlanMinRecords || wave || b.n > 0xffffffffull || tg::opt(tg::kOptNoPlan))
        return launch_kernels(k, b, open, s, nullptr);
    size_t scratch = 0;
    int rc = tg_length_order(b.len, b.n, nullptr, nullptr, &scratch, s);
    if (rc) return rc;
    const size_t obytes = (b.n * sizeof(uint32_t) + 255) & ~(size_t)255;
    uint8_t* buf = nullptr;
    if (tg::stream_alloc((void**)&buf, obytes + scratch, s)) return fail(TG_EHIP, "scratch allocation failed");
    uint32_t* order = reinterpret_cast<uint32_t*>(buf);
    rc = tg_length_order(b.len, b.n, order, buf + obytes, &scratch, s);
    if (!rc) rc = launch_kernels(k, b, open, s, order);
    (void)tg::stream_free(buf, s);
    return rc;
}

size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

// The record's round trip through one staging slot (single()).
int single_staged(tg_key* k, Stage* st, const uint8_t* nonce, const uint8_t* aad, size_t aadlen,
                  const uint8_t* in, size_t inlen, uint8_t* out, bool open, size_t len, size_t outlen,
                  size_t o_aad, size_t o_in, size_t o_out, size_t o_st, size_t total) {
    int rc = ensure_stage(st, total);
    if (rc) return rc;
    memcpy(st->h, nonce, 12);
    if (aadlen) memcpy(st->h + o_aad, aad, aadlen);
    if (inlen) memcpy(st->h + o_in, in, inlen);
    // Zero copy by default: the kernel reads and writes the mapped pinned
    // staging buffer over PCIe, so a record costs one launch and one
    // synchronisation instead of two copies more (option stage_copy: copy
    // through device memory instead).
    const bool copy = tg::opt(tg::kOptStageCopy) != 0;
    uint8_t* base = st->d;
    if (!copy) {
        void* dp = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dp, st->h, 0));
        base = static_cast<uint8_t*>(dp);
    } else {
        HIP_TRY(hipMemcpyAsync(st->d, st->h, o_out, hipMemcpyHostToDevice, st->stream));
    }
    tg_batch b;
    memset(&b, 0, sizeof(b));
    b.n = 1;
    b.in = base + o_in;
    b.fixed_len = (uint32_t)len;
    b.fixed_aad_len = (uint32_t)aadlen;
    b.out = base + o_out;
    b.nonce = base;
    b.aad = base + o_aad;
    b.status = open ? base + o_st : nullptr;
    if ((rc = launch(k, b, open, st->stream))) return fail(rc, "kernel launch failed");
    if (copy)
        HIP_TRY(hipMemcpyAsync(st->h + o_out, st->d + o_out, total - o_out, hipMemcpyDeviceToHost, st->stream));
    HIP_TRY(hipStreamSynchronize(st->stream));
    if (open) {
        const int ok = st->h[o_st] == 1;
        if (ok && len) memcpy(out, st->h + o_out, len);
        if (!ok && len) memset(out, 0, len);
        return ok;
    }
    memcpy(out, st->h + o_out, outlen);
    return TG_OK;
}

// One record through the staging buffers: [nonce | aad | input | output | status]
int single(tg_key* k, const uint8_t* nonce, size_t noncelen, const uint8_t* aad, size_t aadlen,
           const uint8_t* in, size_t inlen, uint8_t* out, bool open) {
    if (!k) return fail(TG_EINVAL, "null key");
    if (k->nkeys != 1) return fail(TG_EINVAL, "per-record calls need a single-key handle");
    if (noncelen != 12) return fail(TG_ENONCE, "Bad nonce length");
    if ((aadlen && !aad) || (inlen && !in)) return fail(TG_EINVAL, "null buffer");
    const size_t T = (size_t)k->taglen;
    if (open && inlen < T) {   // aesgcm.py:135-136, chacha20_poly1305.py:76-77, aesccm.py:120-123
        return 0;
    }
    const size_t len = open ? inlen - T : inlen;
    if (len > 0xffffffffull || aadlen > 0xffffffffull) return fail(TG_EINVAL, "record too long");
    if (is_ccm(k->alg) && len >= (1ull << 28) - 32) return fail(TG_EINVAL, "CCM record too long");
    const size_t o_aad = 16, o_in = align16(o_aad + aadlen), o_out = align16(o_in + inlen);
    const size_t outlen = open ? len : len + T;
    const size_t o_st = align16(o_out + outlen), total = o_st + 16;
    int rc = select_device(k);
    if (rc) return rc;
    Stage* st = nullptr;
    if ((rc = take_stage(k, &st))) return rc;
    rc = single_staged(k, st, nonce, aad, aadlen, in, inlen, out, open, len, outlen, o_aad, o_in, o_out,
                       o_st, total);
    give_stage(k, st);
    return rc;
}

int batch(tg_key* k, const tg_batch* b, void* stream, bool open) {
    if (!k || !b) return fail(TG_EINVAL, "null argument");
    if (b->n == 0) return TG_OK;
    if (!b->in || !b->out || !b->nonce) return fail(TG_EINVAL, "null device buffer");
    if (!b->aad && (b->aad_len || b->fixed_aad_len)) return fail(TG_EINVAL, "null aad");
    if (k->nkeys > 1 && !b->key_idx) return fail(TG_EINVAL, "key table needs key_idx");
    if (k->nkeys == 1 && b->key_idx) return fail(TG_EINVAL, "key_idx given for a single key");
    int rc = select_device(k);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null stream
    if ((rc = launch(k, *b, open, s))) return fail(rc, "kernel launch failed: %s",
                                                   hipGetErrorString(hipGetLastError()));
    if (open && k->nkeys > 1 && (rc = tg_launch_zero_skipped(*b, k->nkeys, s)))
        return fail(rc, "zeroing skipped records failed");
    return TG_OK;
}

// Stream-ordered scratch for the record-framing calls.
struct ScratchAlloc {
    void* base = nullptr;
    hipStream_t s = nullptr;
    ~ScratchAlloc() {
        if (base) (void)tg::stream_free(base, s);
    }
};

int records_scratch(uint64_t n, hipStream_t st, ScratchAlloc& a, tg::RecScratch& s) {
    const size_t per = 8 + 8 + 4 + 12 + 16 + 4 + 1 + 1;
    const size_t bytes = per * n + 64 + 64;
    a.s = st;
    if (tg::stream_alloc(&a.base, bytes, st)) return fail(TG_EHIP, "scratch allocation failed");
    uint8_t* p = static_cast<uint8_t*>(a.base);
    s.in_abs = reinterpret_cast<uint64_t*>(p); p += 8 * n;
    s.out_abs = reinterpret_cast<uint64_t*>(p); p += 8 * n;
    s.aad = p; p += 16 * n;
    s.len = reinterpret_cast<uint32_t*>(p); p += 4 * n;
    s.aad_len = reinterpret_cast<uint32_t*>(p); p += 4 * n;
    s.nonce = p; p += 12 * n;
    s.st = p; p += n;
    s.aead_st = p; p += n;
    p = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(p) + 63) & ~uintptr_t(63));
    s.dummy = p;
    HIP_TRY(hipMemsetAsync(s.dummy, 0, 32, st));
    return TG_OK;
}

int records(tg_key* k, const tg_records* r, void* stream, bool seal) {
    if (!k || !r) return fail(TG_EINVAL, "null argument");
    if (r->n == 0) return TG_OK;
    if (k->nkeys != 1) return fail(TG_EINVAL, "record framing needs a single-key handle");
    if (r->version != TG_TLS12 && r->version != TG_TLS13)
        return fail(TG_EINVAL, "version must be TG_TLS12 or TG_TLS13");
    // _getNonce (recordlayer.py:522-534) then asserts a 12-byte nonce (:556):
    // TLS 1.3 XORs a 12-byte IV; TLS 1.2 AES-GCM / AES-CCM append the 8-byte
    // sequence number to a 4-byte IV; TLS 1.2 ChaCha XORs a 12-byte IV (RFC
    // 7905) or appends to a 4-byte one (draft-00).
    {
        const bool chacha = k->alg == TG_CHACHA20_POLY1305;
        const uint32_t ivl = r->fixed_iv_len;
        const bool ok = r->version == TG_TLS13 ? ivl == 12 : chacha ? (ivl == 12 || ivl == 4) : ivl == 4;
        if (!ok)
            return fail(TG_EINVAL, "fixed IV of %u bytes gives no 12-byte nonce for this suite "
                        "(TLS 1.3: 12; TLS 1.2 AES: 4; TLS 1.2 ChaCha: 12 or 4)", ivl);
    }
    if (!r->data || !r->data_off || !r->data_len || !r->ctype || !r->wire || !r->wire_off ||
        !r->wire_len || (!seal && !r->status))
        return fail(TG_EINVAL, "null device array");
    int rc = select_device(k);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    ScratchAlloc alloc;
    tg::RecScratch s;
    if ((rc = records_scratch(r->n, st, alloc, s))) return rc;
    const bool aes = k->alg != TG_CHACHA20_POLY1305;   // "aes" in name (recordlayer.py:561, :783)
    if ((rc = tg_launch_records_prep(*r, seal, aes, k->taglen, s, st)))
        return fail(rc, "framing launch failed");
    tg_batch b;
    memset(&b, 0, sizeof(b));
    b.n = r->n;
    b.len = s.len;
    b.nonce = s.nonce;
    b.aad = s.aad;
    b.aad_stride = 16;
    b.aad_len = s.aad_len;
    b.out_off = s.out_abs;          // absolute addresses: out base NULL
    if (seal) {
        b.in = r->data;
        b.in_off = r->data_off;
    } else {
        b.in_off = s.in_abs;
        b.status = s.aead_st;
    }
    if ((rc = launch(k, b, !seal, st))) return fail(rc, "AEAD launch failed");
    if (!seal && (rc = tg_launch_records_finish(*r, s, st))) return fail(rc, "finish launch failed");
    return TG_OK;
}

// Validate (alg, keylen, nkeys) and allocate a handle with its stream.
int new_key(int alg, size_t keylen, size_t nkeys, tg_key** out) {
    *out = nullptr;
    if (alg == TG_AES_GCM || is_ccm(alg)) {
        // AssertionError in AESGCM.__init__ (aesgcm.py:37-38) and AESCCM.__init__ (aesccm.py:22-30)
        if (keylen != 16 && keylen != 32) return fail(TG_EKEYLEN, "AES key must be 16 or 32 bytes");
    } else if (alg == TG_CHACHA20_POLY1305) {
        if (keylen != 32) return fail(TG_EKEYLEN, "Key must be 256 bit long");
    } else {
        return fail(TG_EINVAL, "unknown algorithm %d", alg);
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    tg_key* k = new (std::nothrow) tg_key();
    if (!k) return fail(TG_ENOMEM, "out of host memory");
    k->alg = alg;
    k->keylen = keylen;
    k->nkeys = nkeys;
    k->taglen = alg == TG_AES_CCM_8 ? 8 : 16;
    k->rounds = alg == TG_CHACHA20_POLY1305 ? 0 : (keylen == 16 ? 10 : 14);
    k->device = dev;
    *out = k;
    return TG_OK;
}

// HkdfLabel (cryptomath.py:155-173) || 0x01, SHA-padded after one key block.
int hkdf_message(int hashlen, const uint8_t* label, size_t labellen, const uint8_t* ctx,
                 size_t ctxlen, size_t outlen, tg::HkdfMsg& msg) {
    uint8_t m[256];
    size_t n = 0;
    if (6 + labellen > 255 || ctxlen > 255) return fail(TG_EINVAL, "label or context too long");
    m[n++] = (uint8_t)(outlen >> 8);                     // addTwo(length)
    m[n++] = (uint8_t)outlen;
    m[n++] = (uint8_t)(6 + labellen);                    // addVarSeq("tls13 " + label, 1, 1)
    memcpy(m + n, "tls13 ", 6);
    n += 6;
    if (n + labellen + 2 + ctxlen > 200) return fail(TG_EINVAL, "label or context too long");
    memcpy(m + n, label, labellen);
    n += labellen;
    m[n++] = (uint8_t)ctxlen;                            // addVarSeq(hashValue, 1, 1)
    if (ctxlen) memcpy(m + n, ctx, ctxlen);
    n += ctxlen;
    m[n++] = 1;                                          // HKDF_expand block counter x = 1
    const size_t block = hashlen == 32 ? 64 : 128, lenfield = hashlen == 32 ? 8 : 16;
    const uint64_t bits = (uint64_t)(block + n) * 8;     // the (K ^ ipad) block comes first
    size_t total = (n + 1 + lenfield + block - 1) / block * block;
    if (total > sizeof(msg.words)) return fail(TG_EINVAL, "label or context too long");
    uint8_t buf[256] = {0};
    memcpy(buf, m, n);
    buf[n] = 0x80;
    for (int k = 0; k < 8; ++k) buf[total - 1 - k] = (uint8_t)(bits >> (8 * k));
    memset(&msg, 0, sizeof(msg));
    msg.nblocks = (uint32_t)(total / block);
    msg.outlen = (uint32_t)outlen;
    for (size_t w = 0; w < total / 4; ++w)
        msg.words[w] = ((uint32_t)buf[4 * w] << 24) | ((uint32_t)buf[4 * w + 1] << 16) |
                       ((uint32_t)buf[4 * w + 2] << 8) | buf[4 * w + 3];
    return TG_OK;
}

}  // namespace

namespace tg {

int lds_attr(const void* fn, int bytes) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;   // (kernel, device)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TG_EHIP;
    std::lock_guard<std::mutex> g(mu);
    if (done.count({fn, dev})) return TG_OK;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
        return TG_EHIP;
    done.insert({fn, dev});
    return TG_OK;
}

// Per-launch scratch (common.h stream_alloc / stream_free): a process-wide
// list of device buffers, each free for reuse once the event recorded behind
// its last launch has completed.  A buffer released on a stream is taken
// again at once only by the next launch on that same stream handle -- never
// through hipStreamPerThread, whose handle names a different stream in each
// thread -- and that launch's stream also waits for
// the buffer's event, so a handle that a destroyed stream left behind and a
// new stream took over cannot reuse a buffer whose work is still pending
// (on the stream that recorded the event the wait orders
// nothing new).  So memory is bounded by the launches in flight, not by the
// streams a caller has ever used.  (The device memory pool of
// hipMallocAsync measured 4.7 MB more per stream used, without reuse across
// streams: profiles/r05/r5b.)  Idle buffers are freed by tg_scratch_trim,
// and by stream_alloc itself once the cache holds more than kScratchHigh
// bytes.
namespace {
struct ScratchBuf {
    void* p = nullptr;
    size_t cap = 0;
    int dev = -1;
    hipEvent_t done = nullptr;   // recorded behind the buffer's last launch
    hipStream_t last = nullptr;  // the stream of that launch
    bool busy = false;           // between stream_alloc and stream_free
};
std::mutex g_scratch_mu;
std::vector<ScratchBuf>& scratch_list() {
    static std::vector<ScratchBuf>* v = new std::vector<ScratchBuf>();   // outlives static teardown
    return *v;
}
// hipStreamPerThread names a different stream in each thread.  The null
// stream does not: this library is built without per-thread default
// streams, so 0 is the device's legacy default stream, one per device (and
// buffers and helpers are kept per device).  Round 6 treated 0 as
// per-thread too: every key-table batch on the default stream then created a
// new helper stream while the last one's work was in flight (config 4
// 657 -> 547 GiB/s, profiles/r06/f2/bench_c4.json).
bool per_thread_handle(hipStream_t s) { return s == hipStreamPerThread; }
constexpr size_t kScratchHigh = (size_t)8 << 30;

// Frees idle buffers whose last launch has completed until the cache holds
// at most ``keep`` bytes, largest first (g_scratch_mu held).  hipFree of an
// idle buffer waits for nothing: its event has completed.
void trim_locked(size_t keep) {
    auto& v = scratch_list();
    size_t total = 0;
    for (const auto& b : v) total += b.cap;
    while (total > keep) {
        size_t best = v.size();
        for (size_t i = 0; i < v.size(); ++i) {
            const ScratchBuf& b = v[i];
            if (b.busy || (b.done && hipEventQuery(b.done) != hipSuccess)) continue;
            if (best == v.size() || b.cap > v[best].cap) best = i;
        }
        if (best == v.size()) return;   // everything left is in use
        int cur = 0;
        const bool switch_dev = hipGetDevice(&cur) == hipSuccess && cur != v[best].dev;
        if (switch_dev) (void)hipSetDevice(v[best].dev);
        (void)hipFree(v[best].p);
        if (v[best].done) (void)hipEventDestroy(v[best].done);
        if (switch_dev) (void)hipSetDevice(cur);
        total -= v[best].cap;
        v.erase(v.begin() + (std::ptrdiff_t)best);
    }
}
}  // namespace

int stream_alloc(void** p, size_t bytes, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TG_EHIP;
    if (!bytes) bytes = 1;
    std::lock_guard<std::mutex> g(g_scratch_mu);
    auto& v = scratch_list();
    ScratchBuf* pick = nullptr;
    bool pick_pending = false;
    for (auto& b : v) {
        if (b.busy || b.dev != dev || b.cap < bytes) continue;
        const bool complete = !b.done || hipEventQuery(b.done) == hipSuccess;
        const bool ordered = b.last == s && !per_thread_handle(s);
        if (complete || ordered) {
            if (!pick || b.cap < pick->cap) {
                pick = &b;
                pick_pending = !complete;
            }
        }
    }
    if (!pick) {
        size_t total = 0;
        for (const auto& b : v) total += b.cap;
        if (total + bytes > kScratchHigh) trim_locked(kScratchHigh > bytes ? kScratchHigh - bytes : 0);
        ScratchBuf nb;
        nb.cap = bytes < (1u << 20) ? (size_t)1 << 20 : (bytes + 0xfffff) & ~(size_t)0xfffff;
        nb.dev = dev;
        if (hipMalloc(&nb.p, nb.cap) != hipSuccess) return TG_EHIP;
        if (hipEventCreateWithFlags(&nb.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipFree(nb.p);
            return TG_EHIP;
        }
        v.push_back(nb);
        pick = &v.back();
    } else if (pick_pending && hipStreamWaitEvent(s, pick->done, 0) != hipSuccess) {
        return TG_EHIP;
    }
    pick->busy = true;
    *p = pick->p;
    return TG_OK;
}

void scratch_totals(uint64_t* bytes, uint64_t* buffers) {
    std::lock_guard<std::mutex> g(g_scratch_mu);
    *bytes = 0;
    *buffers = scratch_list().size();
    for (const auto& b : scratch_list()) *bytes += b.cap;
}

// The event is recorded first: only once the record has succeeded is the
// buffer reusable.  If it fails the buffer stays busy (leaked, never handed
// out behind a stale event) and the caller gets TG_EHIP.
int stream_free(void* p, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_scratch_mu);
    for (auto& b : scratch_list()) {
        if (b.p != p) continue;
        if (hipEventRecord(b.done, s) != hipSuccess) return TG_EHIP;
        b.busy = false;
        b.last = s;
        return TG_OK;
    }
    return TG_EINVAL;
}

// Helper streams (common.h helper_fork / helper_join): a process-wide pool.
// A launch that runs a second kernel beside its main one (the key-table
// short records, aes_gcm_bs8.hip launch_kt) takes a helper of its device and
// priority class that is idle -- its last join has completed -- or that
// its own stream used last, so independent callers never queue behind each
// other's helper work (round 5 had one helper per device shared
// by every caller).  A caller at raised priority gets a helper at its own
// priority; any other caller one at the lowest priority (the short records
// fill the CUs the long kernel's tail leaves idle, profiles/r05/r5z/).
namespace {
struct HelperStream {
    hipStream_t h = nullptr;
    int dev = -1;
    int prio = 0;
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t last = nullptr;
    bool busy = false;
};
std::mutex g_helper_mu;
std::vector<HelperStream>& helper_list() {
    static std::vector<HelperStream>* v = new std::vector<HelperStream>();
    return *v;
}
}  // namespace

int helper_fork(hipStream_t s, hipStream_t* out) {
    *out = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TG_EHIP;
    // the caller's stream on another device than the current one: no helper
    hipDevice_t sd = 0;
    if (hipStreamGetDevice(s, &sd) == hipSuccess && (int)sd != dev) return TG_OK;
    int least = 0, greatest = 0, sp = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
    if (hipStreamGetPriority(s, &sp) != hipSuccess) sp = 0;
    // priorities: lower numbers run first; 0 is the default
    const int prio = sp < 0 && least != greatest ? sp : least;
    std::lock_guard<std::mutex> g(g_helper_mu);
    auto& v = helper_list();
    HelperStream* pick = nullptr;
    for (auto& x : v) {
        if (x.busy || x.dev != dev || x.prio != prio) continue;
        if ((x.last == s && !per_thread_handle(s)) || hipEventQuery(x.join) == hipSuccess) {
            pick = &x;
            break;
        }
    }
    if (!pick) {
        HelperStream x;
        x.dev = dev;
        x.prio = prio;
        if (hipStreamCreateWithPriority(&x.h, hipStreamNonBlocking, prio) != hipSuccess) return TG_EHIP;
        if (hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&x.join, hipEventDisableTiming) != hipSuccess) {
            if (x.fork) (void)hipEventDestroy(x.fork);
            (void)hipStreamDestroy(x.h);
            return TG_EHIP;
        }
        v.push_back(x);
        pick = &v.back();
    }
    if (hipEventRecord(pick->fork, s) != hipSuccess || hipStreamWaitEvent(pick->h, pick->fork, 0) != hipSuccess)
        return TG_EHIP;
    pick->busy = true;
    *out = pick->h;
    return TG_OK;
}

int helper_join(hipStream_t h, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_helper_mu);
    for (auto& x : helper_list()) {
        if (x.h != h || !x.busy) continue;
        // on failure the helper stays busy: never handed out behind a join
        // event that does not cover its work
        if (hipEventRecord(x.join, h) != hipSuccess || hipStreamWaitEvent(s, x.join, 0) != hipSuccess)
            return TG_EHIP;
        x.busy = false;
        x.last = s;
        return TG_OK;
    }
    return TG_EINVAL;
}

void helper_totals(uint64_t* streams, uint64_t* busy) {
    std::lock_guard<std::mutex> g(g_helper_mu);
    *streams = helper_list().size();
    *busy = 0;
    for (const auto& x : helper_list()) *busy += x.busy;
}

// Frees every idle helper whose work has completed, and idle scratch
// buffers down to ``keep`` bytes (tg_scratch_trim).
void scratch_trim(size_t keep) {
    {
        std::lock_guard<std::mutex> g(g_scratch_mu);
        trim_locked(keep);
    }
    std::lock_guard<std::mutex> g(g_helper_mu);
    auto& v = helper_list();
    for (size_t i = 0; i < v.size();) {
        HelperStream& x = v[i];
        if (x.busy || hipEventQuery(x.join) != hipSuccess || hipStreamQuery(x.h) != hipSuccess) {
            ++i;
            continue;
        }
        (void)hipStreamDestroy(x.h);
        (void)hipEventDestroy(x.fork);
        (void)hipEventDestroy(x.join);
        v.erase(v.begin() + (std::ptrdiff_t)i);
    }
}

// tg_version()'s text; a measurement build appends its flags (common.h).
static std::string& version_text() {
    static std::string v = "tlsgpu 0.1.0 (gfx950)";
    return v;
}

void note_measurement_build(const char* flag) {
    std::string& v = version_text();
    if (v.find("MEASUREMENT BUILD") == std::string::npos) v += " MEASUREMENT BUILD (not the product):";
    v += " ";
    v += flag;
}

}  // namespace tg

extern "C" {

const char* tg_version(void) { return tg::version_text().c_str(); }

const char* tg_last_error(void) { return g_err.c_str(); }

int tg_device_count(int* count) {
    if (!count) return fail(TG_EINVAL, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(TG_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return TG_OK;
}

int tg_set_option(const char* name, int value) {
    const int o = tg::opt_index(name);
    if (o < 0) return fail(TG_EINVAL, "unknown option %s", name ? name : "(null)");
    tg::opt_set(static_cast<tg::Opt>(o), value);
    return TG_OK;
}

int tg_get_option(const char* name, int* value) {
    const int o = tg::opt_index(name);
    if (o < 0 || !value) return fail(TG_EINVAL, "unknown option %s", name ? name : "(null)");
    *value = tg::opt(static_cast<tg::Opt>(o));
    return TG_OK;
}

int tg_init(int device) {
    int n = 0;
    int rc = tg_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n) return fail(TG_ENODEV, "device %d not present (%d)", device, n);
    HIP_TRY(hipSetDevice(device));
    return TG_OK;
}

int tg_key_create(int alg, const uint8_t* keys, size_t keylen, size_t nkeys, tg_key** out) {
    if (!out || !keys || nkeys == 0) return fail(TG_EINVAL, "null argument");
    tg_key* k = nullptr;
    int rc = new_key(alg, keylen, nkeys, &k);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    if (is_ccm(alg)) {
        tg::AesKeyDev* hk = new (std::nothrow) tg::AesKeyDev[nkeys];
        if (!hk) rc = fail(TG_ENOMEM, "out of host memory");
        if (!rc) {
            for (size_t i = 0; i < nkeys; ++i) {
                memset(&hk[i], 0, sizeof(hk[i]));
                k->rounds = tg::host::aes_round_words(keys + keylen * i, keylen, hk[i].rk, nullptr);
            }
            const size_t bytes = sizeof(tg::AesKeyDev) * nkeys;
            e = hipMalloc(&k->dev_key, bytes);
            if (e == hipSuccess) e = hipMemcpy(k->dev_key, hk, bytes, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(TG_EHIP, "key upload: %s", hipGetErrorString(e));
            memset(hk, 0, sizeof(tg::AesKeyDev) * nkeys);
            delete[] hk;
        }
    } else if (alg == TG_AES_GCM && nkeys > 1) {
        tg::GcmTableKey* hk = new (std::nothrow) tg::GcmTableKey[nkeys];
        if (!hk) rc = fail(TG_ENOMEM, "out of host memory");
        if (!rc) {
            for (size_t i = 0; i < nkeys; ++i) {
                memset(&hk[i], 0, sizeof(hk[i]));
                k->rounds = tg::host::aes_round_words(keys + keylen * i, keylen, hk[i].rk, hk[i].hn);
            }
            const size_t bytes = sizeof(tg::GcmTableKey) * nkeys;
            e = hipMalloc(&k->dev_key, dev_key_bytes(k));
            if (e == hipSuccess) e = hipMemcpy(k->dev_key, hk, bytes, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(TG_EHIP, "key upload: %s", hipGetErrorString(e));
            if (!rc && table_derive(k, nullptr)) rc = fail(TG_EHIP, "key powers launch failed");
            if (!rc && (e = hipDeviceSynchronize()) != hipSuccess)
                rc = fail(TG_EHIP, "key powers: %s", hipGetErrorString(e));
            memset(hk, 0, sizeof(tg::GcmTableKey) * nkeys);
            delete[] hk;
        }
    } else if (alg == TG_AES_GCM) {
        auto* hk = new (std::nothrow) tg::host::GcmKeyImage();
        if (!hk) rc = fail(TG_ENOMEM, "out of host memory");
        if (!rc) {
            tg::host::gcm_key_image(keys, keylen, hk);   // key length checked by new_key
            k->rounds = (int)hk->rounds;
            e = hipMalloc(&k->dev_key, sizeof(tg::GcmKeyDev));
            if (e == hipSuccess) e = hipMemcpy(k->dev_key, hk, sizeof(tg::GcmKeyDev), hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(TG_EHIP, "key upload: %s", hipGetErrorString(e));
            memset(hk, 0, sizeof(*hk));
            delete hk;
        }
    } else {
        tg::ChachaKeyDev* hk = new (std::nothrow) tg::ChachaKeyDev[nkeys];
        if (!hk) rc = fail(TG_ENOMEM, "out of host memory");
        if (!rc) {
            for (size_t i = 0; i < nkeys; ++i)
                for (int w = 0; w < 8; ++w) hk[i].k[w] = le32(keys + 32 * i + 4 * w);
            const size_t bytes = sizeof(tg::ChachaKeyDev) * nkeys;
            e = hipMalloc(&k->dev_key, bytes);
            if (e == hipSuccess) e = hipMemcpy(k->dev_key, hk, bytes, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(TG_EHIP, "key upload: %s", hipGetErrorString(e));
            memset(hk, 0, sizeof(tg::ChachaKeyDev) * nkeys);
            delete[] hk;
        }
    }
    if (rc) {
        tg_key_destroy(k);
        return rc;
    }
    *out = k;
    return TG_OK;
}

int tg_key_create_device(int alg, const uint8_t* keys, size_t keylen, size_t nkeys,
                         tg_key** out, void* stream) {
    if (!out || !keys || nkeys == 0) return fail(TG_EINVAL, "null argument");
    tg_key* k = nullptr;
    int rc = new_key(alg, keylen, nkeys, &k);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t bytes = dev_key_bytes(k);
    hipError_t e = hipMalloc(&k->dev_key, bytes);
    if (e != hipSuccess) {
        rc = fail(TG_EHIP, "key alloc: %s", hipGetErrorString(e));
    } else if (alg == TG_CHACHA20_POLY1305) {   // ChachaKeyDev is the raw key bytes (LE words)
        e = hipMemcpyAsync(k->dev_key, keys, 32 * nkeys, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) rc = fail(TG_EHIP, "key copy: %s", hipGetErrorString(e));
    } else {
        const int layout = is_ccm(alg) ? 2 : (nkeys > 1 ? 1 : 0);
        rc = tg_launch_aes_setup((int)keylen, layout, keys, nkeys, k->dev_key, st);
        if (!rc && layout == 1) rc = table_derive(k, st);
        if (rc) rc = fail(rc, "key setup launch failed");
    }
    if (!rc && (e = hipStreamSynchronize(st)) != hipSuccess)
        rc = fail(TG_EHIP, "key setup: %s", hipGetErrorString(e));
    if (rc) {
        tg_key_destroy(k);
        return rc;
    }
    *out = k;
    return TG_OK;
}

int tg_hkdf_expand_label(int hashlen, const uint8_t* secrets, uint64_t n, const uint8_t* label,
                         size_t labellen, const uint8_t* context, size_t ctxlen, size_t outlen,
                         uint8_t* out, void* stream) {
    if (hashlen != 32 && hashlen != 48) return fail(TG_EINVAL, "hash length must be 32 or 48");
    if (outlen == 0 || outlen > (size_t)hashlen)
        return fail(TG_EINVAL, "output length must be 1..%d", hashlen);
    if ((labellen && !label) || (ctxlen && !context)) return fail(TG_EINVAL, "null label");
    if (n == 0) return TG_OK;
    if (!secrets || !out) return fail(TG_EINVAL, "null device buffer");
    tg::HkdfMsg msg;
    int rc = hkdf_message(hashlen, label, labellen, context, ctxlen, outlen, msg);
    if (rc) return rc;
    rc = tg_launch_hkdf(hashlen, msg, secrets, n, out, static_cast<hipStream_t>(stream));
    return rc ? fail(rc, "hkdf launch failed") : TG_OK;
}


int tg_key_destroy(tg_key* k) {
    if (!k) return TG_OK;
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != k->device) (void)hipSetDevice(k->device);
    // Batches may still be running on caller streams (tg_seal_batch and
    // friends take any stream): wait for the whole device before the key
    // material is scrubbed and released, so no launch ever reads a zeroed or
    // freed schedule.
    (void)hipDeviceSynchronize();
    if (k->dev_key) {
        // scrub key material before release
        (void)hipMemset(k->dev_key, 0, dev_key_bytes(k));
        (void)hipFree(k->dev_key);
    }
    for (Stage* st : k->stages) free_stage(st);   // no call may be in flight on k any more
    if (cur >= 0 && cur != k->device) (void)hipSetDevice(cur);
    delete k;
    return TG_OK;
}

int tg_key_info(const tg_key* k, int* alg, size_t* keylen, size_t* nkeys) {
    if (!k) return fail(TG_EINVAL, "null key");
    if (alg) *alg = k->alg;
    if (keylen) *keylen = k->keylen;
    if (nkeys) *nkeys = k->nkeys;
    return TG_OK;
}

int tg_key_taglen(const tg_key* k) {
    if (!k) return fail(TG_EINVAL, "null key");
    return k->taglen;
}

int tg_seal(tg_key* k, const uint8_t* nonce, size_t noncelen, const uint8_t* aad, size_t aadlen,
            const uint8_t* pt, size_t len, uint8_t* out) {
    if (!out) return fail(TG_EINVAL, "null output");
    return single(k, nonce, noncelen, aad, aadlen, pt, len, out, false);
}

int tg_open(tg_key* k, const uint8_t* nonce, size_t noncelen, const uint8_t* aad, size_t aadlen,
            const uint8_t* in, size_t inlen, uint8_t* pt) {
    if (!pt && k && inlen > (size_t)k->taglen) return fail(TG_EINVAL, "null output");
    return single(k, nonce, noncelen, aad, aadlen, in, inlen, pt, true);
}

int tg_seal_batch(tg_key* k, const tg_batch* b, void* stream) { return batch(k, b, stream, false); }

int tg_open_batch(tg_key* k, const tg_batch* b, void* stream) { return batch(k, b, stream, true); }

int tg_seal_records(tg_key* k, const tg_records* r, void* stream) {
    return records(k, r, stream, true);
}

int tg_open_records(tg_key* k, const tg_records* r, void* stream) {
    return records(k, r, stream, false);
}

int tg_make_nonces(int mode, const uint8_t* iv, size_t ivlen, uint64_t seq0, uint64_t n,
                   uint8_t* out, void* stream) {
    if (!iv || !out) return fail(TG_EINVAL, "null argument");
    if (!((mode == 0 && ivlen == 12) || (mode == 1 && ivlen == 4)))
        return fail(TG_EINVAL, "mode %d needs a %d-byte iv", mode, mode == 0 ? 12 : 4);
    if (n == 0) return TG_OK;
    int rc = tg_launch_nonces(mode, iv, seq0, n, out, static_cast<hipStream_t>(stream));
    return rc ? fail(rc, "nonce kernel launch failed") : TG_OK;
}

int tg_malloc(void** p, size_t bytes) {
    if (!p) return fail(TG_EINVAL, "null argument");
    HIP_TRY(hipMalloc(p, bytes ? bytes : 1));
    return TG_OK;
}

int tg_free(void* p) {
    if (p) HIP_TRY(hipFree(p));
    return TG_OK;
}

int tg_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (!bytes) return TG_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return TG_OK;
}

int tg_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    if (!bytes) return TG_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return TG_OK;
}

int64_t tg_scan_records(const uint8_t* buf, size_t len, uint32_t max_body, uint64_t* off,
                        uint32_t* rlen, size_t max_n, size_t* consumed) {
    if (!consumed || (len && !buf) || (max_n && (!off || !rlen)))
        return fail(TG_EINVAL, "null argument");
    tg::host::ScanError err{};
    const int64_t k = tg::host::scan_records(buf, len, max_body, off, rlen, max_n, consumed, &err);
    if (k >= 0) return k;
    if (err.code == 1) return fail(TG_EHEADER, "record %zu: content type %u", err.index, err.value);
    return fail(TG_EOVERFLOW, "record %zu: %u > %u bytes", err.index, err.value, max_body);
}

int tg_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
              const uint64_t* dst_off, uint64_t n, void* stream) {
    if (n && (!src || !src_off || !len || !dst || !dst_off)) return fail(TG_EINVAL, "null argument");
    if (n == 0) return TG_OK;
    int rc = tg_launch_gather(src, src_off, len, dst, dst_off, n, static_cast<hipStream_t>(stream));
    return rc ? fail(rc, "gather kernel launch failed") : TG_OK;
}

int tg_host_copy(void* dst, const void* src, size_t bytes, int nthreads) {
    if (bytes && (!dst || !src)) return fail(TG_EINVAL, "null buffer");
    tg::host::parallel_copy(dst, src, bytes, nthreads);
    return TG_OK;
}

int tg_host_copy_rows(void* dst, size_t dst_stride, const void* src, size_t src_stride, size_t row_bytes,
                      size_t rows, int nthreads) {
    if (rows && row_bytes && (!dst || !src)) return fail(TG_EINVAL, "null buffer");
    if (rows > 1 && (dst_stride < row_bytes || src_stride < row_bytes)) return fail(TG_EINVAL, "stride below row");
    tg::host::parallel_copy_rows(static_cast<uint8_t*>(dst), dst_stride, static_cast<const uint8_t*>(src),
                                 src_stride, row_bytes, rows, nthreads);
    return TG_OK;
}

int tg_scratch_info(uint64_t* bytes, uint64_t* buffers) {
    if (!bytes || !buffers) return fail(TG_EINVAL, "null argument");
    tg::scratch_totals(bytes, buffers);
    return TG_OK;
}

int tg_scratch_trim(uint64_t keep_bytes) {
    tg::scratch_trim((size_t)keep_bytes);
    return TG_OK;
}

int tg_helper_info(uint64_t* streams, uint64_t* busy) {
    if (!streams || !busy) return fail(TG_EINVAL, "null argument");
    tg::helper_totals(streams, busy);
    return TG_OK;
}

int tg_stream_sync(void* stream) {
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return TG_OK;
}

}  // extern "C"
