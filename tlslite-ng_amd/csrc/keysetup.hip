// keysetup.hip -- bulk TLS 1.3 key setup on the device (SURVEY.md section 8(f)
// row 4): many sessions' traffic keys and IVs derived and expanded in one
// pass, so a key table never round-trips through the host.
//
//   hkdf_kernel      HKDF-Expand-Label (tlslite/utils/cryptomath.py:155-173,
//                    HKDF_expand :146-153 with secureHMAC :128-132) of one
//                    secret per lane, SHA-256 or SHA-384, output <= one hash
//                    block (every record-layer use: "key", "iv",
//                    "traffic upd", "finished"; recordlayer.py:1268-1344).
//                    The HkdfLabel message (info || 0x01 and its SHA padding)
//                    is the same for every session, so the host lays it out
//                    once and each lane only hashes its own key blocks.
//   aes_setup_kernel AES key expansion (rijndael.py:922-993) per key, plus
//                    H = E_K(0^128) for GCM (aesgcm.py:45) in the layout the
//                    GCM kernels read (GcmKeyDev / GcmTableKey) or the CCM
//                    layout (AesKeyDev).
//   ghash_table_kernel  the 64 KiB single-key GHASH tables from H (the same
//                    tables api.hip builds on the host).
#include "aes_bs8.h"
#include "common.h"

namespace tg {
namespace {

// ---------------------------------------------------------------- SHA-2 --
__constant__ uint32_t c_k256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

__constant__ uint64_t c_k512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

struct Sha256 {
    using word = uint32_t;
    static constexpr int kHash = 32, kStateOut = 8;
    __device__ static void init(word s[8]) {
        const word iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = iv[k];
    }
    __device__ static void compress(word s[8], const word m[16]) {
        word w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = m[k];
        word a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            if (t >= 16) {
                const word w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                w[t & 15] += (rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3)) + w[(t - 7) & 15] +
                             (rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10));
            }
            const word t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                            c_k256[t] + w[t & 15];
            const word t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    }
};

struct Sha384 {
    using word = uint64_t;
    static constexpr int kHash = 48, kStateOut = 6;
    __device__ static void init(word s[8]) {
        const word iv[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                            0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                            0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = iv[k];
    }
    __device__ static void compress(word s[8], const word m[16]) {
        word w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = m[k];
        word a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
        for (int t = 0; t < 80; ++t) {
            if (t >= 16) {
                const word w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                w[t & 15] += (rotr64(w15, 1) ^ rotr64(w15, 8) ^ (w15 >> 7)) + w[(t - 7) & 15] +
                             (rotr64(w2, 19) ^ rotr64(w2, 61) ^ (w2 >> 6));
            }
            const word t1 = h + (rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41)) +
                            ((e & f) ^ (~e & g)) + c_k512[t] + w[t & 15];
            const word t2 = (rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39)) +
                            ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    }
};

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

template <class H>
__device__ __forceinline__ typename H::word load_be(const uint8_t* p) {
    if constexpr (sizeof(typename H::word) == 4) {
        return be32(p);
    } else {
        return ((uint64_t)be32(p) << 32) | be32(p + 4);
    }
}

// HMAC(secret, info || 0x01) truncated to outlen: HKDF_expand's first block
// T(1) (cryptomath.py:146-153), which is all of it for outlen <= hash length.
template <class H>
__global__ __launch_bounds__(256) void hkdf_kernel(tg::HkdfMsg msg, const uint8_t* __restrict__ secrets, uint64_t n,
                            uint8_t* __restrict__ out) {
    using W = typename H::word;
    constexpr int WB = sizeof(W);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* sec = secrets + (uint64_t)H::kHash * i;
    W key[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) key[k] = k * WB < H::kHash ? load_be<H>(sec + k * WB) : W(0);
    const W ipad = (W)0x3636363636363636ull, opad = (W)0x5c5c5c5c5c5c5c5cull;
    W st[8], blk[16];
    // inner: H((K ^ ipad) || info || 0x01)
    H::init(st);
#pragma unroll
    for (int k = 0; k < 16; ++k) blk[k] = key[k] ^ ipad;
    H::compress(st, blk);
    for (uint32_t b = 0; b < msg.nblocks; ++b) {   // uniform message blocks
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if constexpr (WB == 4) {
                blk[k] = msg.words[16 * b + k];
            } else {
                blk[k] = ((uint64_t)msg.words[32 * b + 2 * k] << 32) | msg.words[32 * b + 2 * k + 1];
            }
        }
        H::compress(st, blk);
    }
    // outer: H((K ^ opad) || inner digest), one padded block
    W inner[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) inner[k] = st[k];
    H::init(st);
#pragma unroll
    for (int k = 0; k < 16; ++k) blk[k] = key[k] ^ opad;
    H::compress(st, blk);
    constexpr int dw = H::kStateOut;                       // digest words
#pragma unroll
    for (int k = 0; k < 16; ++k) blk[k] = k < dw ? inner[k] : W(0);
    blk[dw] = (W)1 << (8 * WB - 1);                        // 0x80 terminator
    blk[15] = (W)((16 * WB + H::kHash) * 8);               // bit length of block + digest
    H::compress(st, blk);
    uint8_t* o = out + (uint64_t)msg.outlen * i;
    for (uint32_t k = 0; k < msg.outlen; ++k) {
        const W wv = st[k / WB];
        o[k] = (uint8_t)(wv >> (8 * (WB - 1 - (k % WB))));
    }
}

// ------------------------------------------------------- AES key schedule --
constexpr uint8_t xtime8(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

struct SboxTable {
    uint8_t s[256];
};

constexpr SboxTable make_sbox() {
    uint8_t exp[256] = {};
    uint8_t log[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {
        exp[i] = x;
        log[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime8(x));
    }
    SboxTable t = {};
    for (int v = 0; v < 256; ++v) {
        uint8_t inv = v ? exp[(255 - log[v]) % 255] : 0;
        uint8_t s = inv, r = inv;
        for (int k = 0; k < 4; ++k) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s = (uint8_t)(s ^ r);
        }
        t.s[v] = (uint8_t)(s ^ 0x63);
    }
    return t;
}

__constant__ SboxTable c_sbox = make_sbox();

__device__ __forceinline__ uint32_t sub_word(const uint8_t* sb, uint32_t w) {
    return (uint32_t)sb[w & 0xff] | ((uint32_t)sb[(w >> 8) & 0xff] << 8) |
           ((uint32_t)sb[(w >> 16) & 0xff] << 16) | ((uint32_t)sb[w >> 24] << 24);
}

// FIPS-197 key expansion (rijndael.py:922-993); words are LE words of the
// key-schedule bytes (the layout every AES kernel reads).
template <int NK>
__device__ __forceinline__ void expand_key(const uint8_t* sb, const uint8_t* key, uint32_t rk[60]) {
    constexpr int NR = NK + 6, TOTAL = 4 * (NR + 1);
#pragma unroll
    for (int k = 0; k < NK; ++k)
        rk[k] = (uint32_t)key[4 * k] | ((uint32_t)key[4 * k + 1] << 8) |
                ((uint32_t)key[4 * k + 2] << 16) | ((uint32_t)key[4 * k + 3] << 24);
    uint32_t rcon = 1;
#pragma unroll
    for (int k = NK; k < TOTAL; ++k) {
        uint32_t t = rk[k - 1];
        if (k % NK == 0) {
            t = sub_word(sb, (t >> 8) | (t << 24)) ^ rcon;   // SubWord(RotWord(t)) ^ Rcon
            rcon = xtime8((uint8_t)rcon);
        } else if (NK > 6 && k % NK == 4) {
            t = sub_word(sb, t);
        }
        rk[k] = rk[k - NK] ^ t;
    }
#pragma unroll
    for (int k = TOTAL; k < 60; ++k) rk[k] = 0;
}

// E_K(0^128) bytewise (SubBytes, ShiftRows, MixColumns) -> H as 4 LE words.
template <int NR>
__device__ __forceinline__ void aes_zero_block(const uint8_t* sb, const uint32_t rk[60], uint32_t h[4]) {
    uint8_t s[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = (uint8_t)(rk[k >> 2] >> (8 * (k & 3)));
#pragma unroll
    for (int r = 1; r <= NR; ++r) {
        uint8_t t[16];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int row = 0; row < 4; ++row) t[4 * c + row] = sb[s[4 * ((c + row) & 3) + row]];
        if (r != NR) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint8_t* a = t + 4 * c;
                const uint8_t all = (uint8_t)(a[0] ^ a[1] ^ a[2] ^ a[3]), a0 = a[0];
                a[0] = (uint8_t)(a[0] ^ all ^ xtime8((uint8_t)(a[0] ^ a[1])));
                a[1] = (uint8_t)(a[1] ^ all ^ xtime8((uint8_t)(a[1] ^ a[2])));
                a[2] = (uint8_t)(a[2] ^ all ^ xtime8((uint8_t)(a[2] ^ a[3])));
                a[3] = (uint8_t)(a[3] ^ all ^ xtime8((uint8_t)(a[3] ^ a0)));
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) s[k] = (uint8_t)(t[k] ^ (rk[4 * r + (k >> 2)] >> (8 * (k & 3))));
    }
#pragma unroll
    for (int w = 0; w < 4; ++w)
        h[w] = (uint32_t)s[4 * w] | ((uint32_t)s[4 * w + 1] << 8) | ((uint32_t)s[4 * w + 2] << 16) |
               ((uint32_t)s[4 * w + 3] << 24);
}

// out layouts: 0 = GcmKeyDev (single key), 1 = GcmTableKey[n], 2 = AesKeyDev[n]
template <int NK, int LAYOUT>
__global__ void aes_setup_kernel(const uint8_t* __restrict__ keys, uint64_t n, void* out) {
    __shared__ uint8_t sb[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) sb[k] = c_sbox.s[k];
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    constexpr int NR = NK + 6;
    uint32_t rk[60];
    expand_key<NK>(sb, keys + 4 * NK * i, rk);
    if (LAYOUT == 2) {
        AesKeyDev* o = static_cast<AesKeyDev*>(out) + i;
#pragma unroll
        for (int k = 0; k < 60; ++k) o->rk[k] = rk[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) o->pad[k] = 0;
        return;
    }
    uint32_t h[4];
    aes_zero_block<NR>(sb, rk, h);
    if (LAYOUT == 1) {
        GcmTableKey* o = static_cast<GcmTableKey*>(out) + i;
#pragma unroll
        for (int k = 0; k < 60; ++k) o->rk[k] = rk[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) o->hn[k] = __builtin_bswap32(__builtin_bitreverse32(h[k]));
        return;
    }
    GcmKeyDev* o = static_cast<GcmKeyDev*>(out);   // n == 1
#pragma unroll
    for (int k = 0; k < 60; ++k) o->rk[k] = rk[k];
    o->rounds = NR;
#pragma unroll
    for (int k = 0; k < 3; ++k) o->pad[k] = 0;
    o->ghash[0] = make_uint4(h[0], h[1], h[2], h[3]);   // H parked in entry (0, 0), see below
}

// M_j[b] = XOR of H * x^(8j + t) over the bits t (MSB first) of b, in the
// block byte layout (api.hip build_ghash_tables; aesgcm.py:8-14 bit order).
// Entry (0, 0) = 0 holds H on entry and is left alone here (every thread reads
// it); the launcher zeroes it afterwards, stream-ordered.

__global__ void ghash_table_kernel(GcmKeyDev* key) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;   // entry j * 256 + b
    if (e == 0 || e >= kGhashEntries) return;
    const uint4 hw = key->ghash[0];                         // H as LE words of its bytes
    const uint32_t hv[4] = {hw.x, hw.y, hw.z, hw.w};
    key->ghash[e] = ghash_table_entry(hv, e);
}

// GcmKeyDev::ghash64: the same tables for H^64 (after hpow_kernel).
__global__ void ghash64_table_kernel(GcmKeyDev* key) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGhashEntries) return;
    const uint4 p = key->hpow[63];                          // normal order -> byte layout
    const uint32_t hv[4] = {gcm_word_to_norm(p.x), gcm_word_to_norm(p.y), gcm_word_to_norm(p.z),
                            gcm_word_to_norm(p.w)};
    key->ghash64[e] = ghash_table_entry(hv, e);
}

// GcmKeyDev::ghash8: the same tables for H^8 (after hpow_kernel).
__global__ void ghash8_table_kernel(GcmKeyDev* key) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGhashEntries) return;
    const uint4 p = key->hpow[7];
    const uint32_t hv[4] = {gcm_word_to_norm(p.x), gcm_word_to_norm(p.y), gcm_word_to_norm(p.z),
                            gcm_word_to_norm(p.w)};
    key->ghash8[e] = ghash_table_entry(hv, e);
}

// GcmKeyDev::hpow: thread e computes H^(e+1) by square and multiply from H,
// which aes_setup_kernel parked in ghash[0] (the table kernel leaves entry 0
// alone and the launcher zeroes it after this kernel, stream-ordered).
__global__ void hpow_kernel(GcmKeyDev* key) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kHPow) return;
    const uint4 hw = key->ghash[0];
    const uint32_t hn[4] = {gcm_word_to_norm(hw.x), gcm_word_to_norm(hw.y), gcm_word_to_norm(hw.z),
                            gcm_word_to_norm(hw.w)};
    uint32_t r[4] = {1, 0, 0, 0}, x[4] = {hn[0], hn[1], hn[2], hn[3]};
    for (uint32_t n = (uint32_t)e + 1; n; n >>= 1) {
        if (n & 1) gf_mul_norm(r, x, r);
        if (n > 1) gf_mul_norm(x, x, x);
    }
    key->hpow[e] = make_uint4(r[0], r[1], r[2], r[3]);
}

// GcmKeyDev::bs8mask from the round keys (after aes_setup_kernel, layout 0):
// 32 (NR + 1) <= 480 planes.
__global__ void bs_mask_kernel(GcmKeyDev* key) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int nr = (int)key->rounds;
    if (e < 32 * (nr + 1)) key->bs8mask[e] = bs8::mask_word(key->rk, e);
    if (e < 15 * 32) key->bs8rows[e] = bs8_row_word(key->rk, nr, e);   // the hybrid's key rows
    if (e < 64) key->rkrot[e] = rkrot_word(key->rk, nr, e);
}

}  // namespace
}  // namespace tg

int tg_launch_hkdf(int hashlen, const tg::HkdfMsg& msg, const uint8_t* secrets, uint64_t n,
                   uint8_t* out, hipStream_t s) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (hashlen == 32)
        hipLaunchKernelGGL(tg::hkdf_kernel<tg::Sha256>, dim3(blocks), dim3(256), 0, s, msg, secrets,
                           n, out);
    else if (hashlen == 48)
        hipLaunchKernelGGL(tg::hkdf_kernel<tg::Sha384>, dim3(blocks), dim3(256), 0, s, msg, secrets,
                           n, out);
    else
        return TG_EINVAL;
    return hipGetLastError() == hipSuccess ? TG_OK : TG_EHIP;
}

// layout: 0 = GcmKeyDev (n == 1, GHASH tables built too), 1 = GcmTableKey, 2 = AesKeyDev
int tg_launch_aes_setup(int keylen, int layout, const uint8_t* keys, uint64_t n, void* out,
                        hipStream_t s) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
#define TG_AES_SETUP(NK, L)                                                                        \
    hipLaunchKernelGGL((tg::aes_setup_kernel<NK, L>), dim3(blocks), dim3(256), 0, s, keys, n, out)
    if (keylen == 16) {
        if (layout == 0) TG_AES_SETUP(4, 0);
        else if (layout == 1) TG_AES_SETUP(4, 1);
        else TG_AES_SETUP(4, 2);
    } else if (keylen == 32) {
        if (layout == 0) TG_AES_SETUP(8, 0);
        else if (layout == 1) TG_AES_SETUP(8, 1);
        else TG_AES_SETUP(8, 2);
    } else {
        return TG_EINVAL;
    }
#undef TG_AES_SETUP
    if (hipGetLastError() != hipSuccess) return TG_EHIP;
    if (layout == 0) {
        tg::GcmKeyDev* k = static_cast<tg::GcmKeyDev*>(out);
        hipLaunchKernelGGL(tg::ghash_table_kernel, dim3(tg::kGhashEntries / 256), dim3(256), 0, s, k);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
        hipLaunchKernelGGL(tg::hpow_kernel, dim3((tg::kHPow + 255) / 256), dim3(256), 0, s, k);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
        hipLaunchKernelGGL(tg::ghash64_table_kernel, dim3(tg::kGhashEntries / 256), dim3(256), 0, s, k);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
        hipLaunchKernelGGL(tg::ghash8_table_kernel, dim3(tg::kGhashEntries / 256), dim3(256), 0, s, k);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
        hipLaunchKernelGGL(tg::bs_mask_kernel, dim3((15 * 32 + 255) / 256), dim3(256), 0, s, k);
        if (hipGetLastError() != hipSuccess) return TG_EHIP;
        if (hipMemsetAsync(&k->ghash[0], 0, sizeof(uint4), s) != hipSuccess) return TG_EHIP;
    }
    return TG_OK;
}
