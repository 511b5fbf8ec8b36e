// records.hip -- TLS record framing around the AEAD kernels (SURVEY.md
// section 8(f) row 1), restating tlslite/recordlayer.py:
//   _getNonce           :522-534  (fixed IV xor seq, or fixed IV || seq)
//   _encryptThenSeal    :536-565  (AAD; TLS 1.2 AES-GCM explicit nonce)
//   sendRecord          :606-617  (TLS 1.3 inner content type + zero padding)
//   _decryptAndUnseal   :780-824  (publicly-invalid checks, AAD, open)
//   _tls13_de_pad       :863-884  (strip padding, recover the content type)
// Seal: a per-record prep kernel appends the TLS 1.3 inner tail in place,
// writes the header / explicit nonce into the wire buffer and builds the
// nonce and AAD rows; the AEAD kernel then reads the fragment and writes
// ct || tag straight into the wire record (no payload copy).  Open: prep
// parses and checks headers, the AEAD kernel writes the plaintext straight
// into the data buffer, and a finish kernel de-pads and settles the status.
#include "common.h"

namespace tg {
namespace {

constexpr int kRecThreads = 256;
constexpr uint8_t kAppData = 23;

__device__ __forceinline__ void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

__device__ __forceinline__ void put_be64(uint8_t* p, uint64_t v) {
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = (uint8_t)(v >> (56 - 8 * k));
}

// RecordLayer._getNonce: XOR form for TLS 1.3 and for ChaCha with a 12-byte
// fixed IV (RFC 7905); concatenation form otherwise (TLS 1.2 AES-GCM).
__device__ __forceinline__ void rec_nonce(const tg_records& r, bool xor_form, uint64_t seq,
                                          uint8_t* out) {
    if (xor_form) {
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const uint8_t s = k < 4 ? 0 : (uint8_t)(seq >> (8 * (11 - k)));
            out[k] = r.fixed_iv[k] ^ s;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) out[k] = r.fixed_iv[k];
        put_be64(out + 4, seq);
    }
}

// rec_nonce as three little-endian words of its 12 bytes, for one aligned
// row store instead of twelve byte stores (the prep kernels' rows are
// 4-byte aligned: RecScratch).
__device__ __forceinline__ uint32_t iv_word(const tg_records& r, int q) {
    return (uint32_t)r.fixed_iv[4 * q] | ((uint32_t)r.fixed_iv[4 * q + 1] << 8) |
           ((uint32_t)r.fixed_iv[4 * q + 2] << 16) | ((uint32_t)r.fixed_iv[4 * q + 3] << 24);
}
__device__ __forceinline__ void rec_nonce_row(const tg_records& r, bool xor_form, uint64_t seq, uint32_t* out) {
    // be64(seq) as the LE words of bytes 4..11
    const uint32_t hi = bswap32((uint32_t)(seq >> 32)), lo = bswap32((uint32_t)seq);
    if (xor_form) {
        out[0] = iv_word(r, 0);
        out[1] = iv_word(r, 1) ^ hi;
        out[2] = iv_word(r, 2) ^ lo;
    } else {
        out[0] = iv_word(r, 0);
        out[1] = hi;
        out[2] = lo;
    }
}

__global__ void seal_prep(tg_records r, bool aes, uint32_t taglen, RecScratch s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= r.n) return;
    const bool tls13 = r.version == TG_TLS13;
    const uint64_t seq = r.seq0 + i;
    const uint32_t L = r.data_len[i];
    const uint8_t ct = r.ctype[i];
    uint8_t* d = r.data + r.data_off[i];
    uint32_t inner = L;
    if (tls13) {  // TLSInnerPlaintext = content || type || zeros (sendRecord :606-617)
        const uint32_t pad = r.pad_len ? r.pad_len[i] : 0;
        d[L] = ct;
        for (uint32_t k = 0; k < pad; ++k) d[L + 1 + k] = 0;
        inner = L + 1 + pad;
    }
    const uint32_t explicit_len = (!tls13 && aes) ? 8 : 0;
    const uint32_t body = explicit_len + inner + taglen;
    uint8_t* w = r.wire + r.wire_off[i];
    w[0] = tls13 ? kAppData : ct;   // TLS 1.3 hides the type (:614)
    w[1] = 3;
    w[2] = 3;
    put_be16(w + 3, body);
    if (explicit_len) put_be64(w + 5, seq);   // explicit nonce = seq (:561-563)
    r.wire_len[i] = 5 + body;
    s.out_abs[i] = (uint64_t)(uintptr_t)(w + 5 + explicit_len);
    s.len[i] = inner;
    rec_nonce_row(r, tls13 || (!aes && r.fixed_iv_len == 12), seq, reinterpret_cast<uint32_t*>(s.nonce + 12 * i));
    // the AAD row as one 16-byte store (LE words of its bytes, zero-padded)
    uint4 a;
    if (tls13) {  // AAD = the record header, length = inner + tag (:546-552)
        a = make_uint4((tls13 ? kAppData : ct) | (3u << 8) | (3u << 16) | ((body >> 8) << 24), body & 0xffu, 0, 0);
        s.aad_len[i] = 5;
    } else {      // seq || type || version || length (:540-545)
        a = make_uint4(bswap32((uint32_t)(seq >> 32)), bswap32((uint32_t)seq),
                       (uint32_t)ct | (3u << 8) | (3u << 16) | (((L >> 8) & 0xffu) << 24), L & 0xffu);
        s.aad_len[i] = 13;
    }
    *reinterpret_cast<uint4*>(s.aad + 16 * i) = a;
}

__global__ void open_prep(tg_records r, bool aes, uint32_t taglen, RecScratch s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= r.n) return;
    const bool tls13 = r.version == TG_TLS13;
    const uint64_t seq = r.seq0 + i;
    const uint8_t* w = r.wire + r.wire_off[i];
    const uint32_t wl = r.wire_len[i];
    const uint32_t buf_len = wl >= 5 ? wl - 5 : 0;
    uint8_t st = TG_REC_OK;
    const uint32_t explicit_len = (!tls13 && aes) ? 8 : 0;
    if (wl < 5 || explicit_len > buf_len) st = TG_REC_TRUNCATED;           // :787-789
    else if (buf_len - explicit_len < taglen) st = TG_REC_TRUNCATED;       // :797-799
    const uint8_t type = wl >= 1 ? w[0] : 0;
    const uint32_t limit = r.recv_limit ? r.recv_limit : 16384u;
    // RecordSocket.recv (:219-222) refuses the header before any decryption
    if (st == TG_REC_OK && (buf_len > limit + 2048u || (tls13 && buf_len > limit + 256u)))
        st = TG_REC_OVERFLOW;
    if (st == TG_REC_OK && tls13) {
        const uint32_t ver = ((uint32_t)w[1] << 8) | w[2];
        const uint32_t hlen = ((uint32_t)w[3] << 8) | w[4];
        if (type != kAppData) st = TG_REC_BAD_TYPE;                        // :809-812
        else if (ver != 0x0303) st = TG_REC_BAD_VERSION;                   // :813-815
        else if (hlen != buf_len) st = TG_REC_LENGTH;                      // :816-817
    }
    s.st[i] = st;
    const uint32_t ct_len = st == TG_REC_OK ? buf_len - explicit_len - taglen : 0;
    s.len[i] = ct_len;
    // invalid records run the AEAD over an empty message with a dummy tag
    s.in_abs[i] = st == TG_REC_OK ? (uint64_t)(uintptr_t)(w + 5 + explicit_len)
                                  : (uint64_t)(uintptr_t)s.dummy;
    s.out_abs[i] = (uint64_t)(uintptr_t)(r.data + r.data_off[i]);
    uint8_t* n = s.nonce + 12 * i;
    if (explicit_len && st == TG_REC_OK) {   // fixed IV || explicit nonce (:790)
        for (int k = 0; k < 4; ++k) n[k] = r.fixed_iv[k];
        for (int k = 0; k < 8; ++k) n[4 + k] = w[5 + k];
    } else {
        rec_nonce(r, tls13 || (!aes && r.fixed_iv_len == 12), seq, n);
    }
    uint8_t* a = s.aad + 16 * i;
    if (tls13) {
        for (int k = 0; k < 5; ++k) a[k] = k < (int)wl ? w[k] : 0;   // header.write() (:819)
        s.aad_len[i] = 5;
    } else {
        put_be64(a, seq);                    // :801-806
        a[8] = type;
        a[9] = 3;
        a[10] = 3;
        put_be16(a + 11, ct_len);
        s.aad_len[i] = 13;
    }
}

__global__ void open_finish(tg_records r, RecScratch s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= r.n) return;
    const bool tls13 = r.version == TG_TLS13;
    uint8_t st = s.st[i];
    if (st == TG_REC_OK && s.aead_st[i] != 1) st = TG_REC_BAD_MAC;         // :822-823
    uint32_t plen = 0;
    uint8_t type = 0;
    const uint32_t limit = r.recv_limit ? r.recv_limit : 16384u;
    if (st == TG_REC_OK && tls13 && s.len[i] > limit + 1u) st = TG_REC_OVERFLOW;   // :974-975
    if (st == TG_REC_OK) {
        const uint32_t ct_len = s.len[i];
        if (tls13) {  // last non-zero byte is the content type (:863-884)
            const uint8_t* d = r.data + r.data_off[i];
            uint32_t pos = ct_len;
            while (pos > 0 && d[pos - 1] == 0) --pos;
            if (pos == 0) {
                st = TG_REC_NO_CONTENT_TYPE;
            } else {
                type = d[pos - 1];
                plen = pos - 1;
            }
        } else {
            type = r.wire[r.wire_off[i]];
            plen = ct_len;
        }
        if (st == TG_REC_OK && plen > limit) st = TG_REC_OVERFLOW;                  // :980-981
    }
    r.data_len[i] = plen;
    r.ctype[i] = type;
    r.status[i] = st;
}

// tg_gather: one workgroup per range; 16-byte vector copies when source and
// destination are co-aligned, otherwise bytes.  Coalesced: consecutive
// threads move consecutive 16-byte pieces of the range.
__global__ void gather_kernel(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                              const uint32_t* __restrict__ len, uint8_t* __restrict__ dst,
                              const uint64_t* __restrict__ dst_off) {
    const uint64_t i = blockIdx.x;
    const uint8_t* s = src + src_off[i];
    uint8_t* d = dst + dst_off[i];
    const uint32_t L = len[i];
    const uint32_t mis = (uint32_t)((uintptr_t)s & 15u);
    if (mis == ((uintptr_t)d & 15u)) {
        const uint32_t head = mis ? (16u - mis < L ? 16u - mis : L) : 0u;
        for (uint32_t k = threadIdx.x; k < head; k += blockDim.x) d[k] = s[k];
        const uint32_t nvec = (L - head) >> 4;
        const uint4* sv = reinterpret_cast<const uint4*>(s + head);
        uint4* dv = reinterpret_cast<uint4*>(d + head);
        for (uint32_t k = threadIdx.x; k < nvec; k += blockDim.x) dv[k] = sv[k];
        for (uint32_t k = head + 16u * nvec + threadIdx.x; k < L; k += blockDim.x) d[k] = s[k];
    } else {
        for (uint32_t k = threadIdx.x; k < L; k += blockDim.x) d[k] = s[k];
    }
}

}  // namespace
}  // namespace tg

int tg_launch_records_prep(const tg_records& r, bool seal, bool aes, int taglen,
                           const tg::RecScratch& s, hipStream_t st) {
    const uint64_t blocks = (r.n + tg::kRecThreads - 1) / tg::kRecThreads;
    if (seal)
        hipLaunchKernelGGL(tg::seal_prep, dim3((unsigned)blocks), dim3(tg::kRecThreads), 0, st, r,
                           aes, (uint32_t)taglen, s);
    else
        hipLaunchKernelGGL(tg::open_prep, dim3((unsigned)blocks), dim3(tg::kRecThreads), 0, st, r,
                           aes, (uint32_t)taglen, s);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

int tg_launch_records_finish(const tg_records& r, const tg::RecScratch& s, hipStream_t st) {
    const uint64_t blocks = (r.n + tg::kRecThreads - 1) / tg::kRecThreads;
    hipLaunchKernelGGL(tg::open_finish, dim3((unsigned)blocks), dim3(tg::kRecThreads), 0, st, r, s);
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

int tg_launch_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
                     const uint64_t* dst_off, uint64_t n, hipStream_t s) {
    for (uint64_t i0 = 0; i0 < n; i0 += 0x7fffffffull) {   // grid.x limit
        const uint64_t k = n - i0 < 0x7fffffffull ? n - i0 : 0x7fffffffull;
        hipLaunchKernelGGL(tg::gather_kernel, dim3((unsigned)k), dim3(256), 0, s, src, src_off + i0,
                           len + i0, dst, dst_off + i0);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
    }
    return TG_OK;
}
