// host_check.cpp -- CPU check of libtlsgpu's host half (csrc/host.cpp) built
// with -fsanitize=address,undefined by tests/test_host_sanitize.py.
//
//   host_check keys        AES FIPS-197 C.1-C.3 known answers; the GHASH
//                          table builder against keymath.h's per-entry
//                          restatement; the GcmKeyDev image (powers of H,
//                          tables of H^8 / H^64, key planes) against their
//                          definitions; bad key lengths.
//   host_check scan        record scanner cases from stdin (see read_case),
//                          each in an exactly-sized heap buffer so any read
//                          past the end trips ASan; one result line per case
//                          for the Python restatement of RecordSocket.recv.
//   host_check canary      a deliberate heap over-read (must abort under ASan).
//   host_check fuzz N S    N random / truncated / oversize header streams
//                          (seed S) through the scanner with invariant checks.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <thread>
#include <vector>

#include "host.h"
#include "keymath.h"

using namespace tg;

static int g_fail = 0;
#define CHECK(c, ...)                         \
    do {                                      \
        if (!(c)) {                           \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);     \
            fprintf(stderr, "\n");            \
            ++g_fail;                         \
        }                                     \
    } while (0)

static void unhex(const char* s, uint8_t* out) {
    for (size_t i = 0; s[2 * i]; ++i) {
        unsigned v = 0;
        sscanf(s + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
}

static int check_keys() {
    // FIPS-197 Appendix C: plaintext 00112233..ff, key 000102..
    const char* want[3] = {"69c4e0d86a7b0430d8cdb78070b4c55a", "dda97ca4864cdfe06eaf70a0ec0d7191",
                           "8ea2b7ca516745bfeafc49904b496089"};
    uint8_t pt[16], key[32], ct[16], exp[16];
    for (int i = 0; i < 16; ++i) pt[i] = (uint8_t)(0x11 * i);
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)i;
    for (int v = 0; v < 3; ++v) {
        const size_t kl = 16 + 8 * v;
        uint8_t* rk = (uint8_t*)malloc(240);
        const int nr = host::aes_expand(key, kl, rk);
        CHECK(nr == 10 + 2 * v, "rounds %d", nr);
        // exact-size copy: encryption may read only the 16 (nr + 1) schedule bytes
        uint8_t* rk2 = (uint8_t*)malloc(16 * (nr + 1));
        memcpy(rk2, rk, 16 * (nr + 1));
        host::aes_encrypt(rk2, nr, pt, ct);
        unhex(want[v], exp);
        CHECK(memcmp(ct, exp, 16) == 0, "FIPS-197 C.%d", v + 1);
        free(rk);
        free(rk2);
    }
    uint8_t rk[240];
    CHECK(host::aes_expand(key, 20, rk) == -1, "keylen 20 accepted");
    uint32_t rkw[60], hn[4];
    CHECK(host::aes_round_words(key, 0, rkw, hn) == -1, "keylen 0 accepted");

    std::mt19937_64 rng(7);
    auto* table = new uint32_t[16 * 256][4];
    for (int t = 0; t < 6; ++t) {
        uint8_t h[16];
        for (int i = 0; i < 16; ++i) h[i] = t == 0 ? 0 : t == 1 ? (i == 0 ? 0x80 : 0) : (uint8_t)rng();
        host::ghash_tables(h, table);
        uint32_t hv[4];
        for (int w = 0; w < 4; ++w) hv[w] = host::le32(h + 4 * w);
        for (int e = 0; e < 16 * 256; ++e) {
            uint32_t w[4];
            ghash_table_words(hv, e, w);
            CHECK(memcmp(w, table[e], 16) == 0, "ghash table H#%d entry %d", t, e);
            if (memcmp(w, table[e], 16)) break;
        }
    }
    delete[] table;

    for (int v = 0; v < 2; ++v) {
        const size_t kl = v ? 32 : 16;
        for (int i = 0; i < 32; ++i) key[i] = (uint8_t)rng();
        auto* img = new host::GcmKeyImage;
        CHECK(host::gcm_key_image(key, kl, img) == 0, "gcm_key_image");
        const int nr = (int)img->rounds;
        uint32_t rw[60];
        CHECK(host::aes_round_words(key, kl, rw, hn) == nr, "rounds");
        CHECK(memcmp(rw, img->rk, sizeof(rw)) == 0, "round words");
        CHECK(memcmp(hn, img->hpow[0], 16) == 0, "H^1");
        uint32_t p[4];
        for (int e : {1, 7, 63, 64, 1000, 2047}) {
            gf_mul_norm(img->hpow[e - 1], hn, p);
            CHECK(memcmp(p, img->hpow[e], 16) == 0, "H^%d", e + 1);
        }
        // the tables of H^8 and H^64 from the powers
        for (int which = 0; which < 2; ++which) {
            const uint32_t* pw = img->hpow[which ? 63 : 7];
            uint32_t hv[4];
            for (int w = 0; w < 4; ++w) hv[w] = gcm_word_to_norm(pw[w]);
            const uint32_t(*tab)[4] = which ? img->ghash64 : img->ghash8;
            for (int e = 0; e < 16 * 256; e += 97) {
                uint32_t w[4];
                ghash_table_words(hv, e, w);
                CHECK(memcmp(w, tab[e], 16) == 0, "H^%d table entry %d", which ? 64 : 8, e);
            }
        }
        for (int e = 0; e < 32 * (nr + 1); ++e)
            CHECK(img->bs8mask[e] == bs8_mask_word(img->rk, e), "bs8mask %d", e);
        // the hybrid kernel's rows: plane (r, i, bit) at word 4 (8 r + bit) + i,
        // folded for the middle rounds; the rotated round keys
        for (int e = 0; e < 32 * (nr + 1); ++e) {
            const int r = e >> 5, i = (e >> 3) & 3, bit = e & 7;
            const uint32_t want = r >= 1 && r < nr ? bs8_fold_word(img->rk, e) : bs8_mask_word(img->rk, e);
            CHECK(img->bs8rows[4 * (8 * r + bit) + i] == want, "bs8rows %d", e);
        }
        for (int w = 4 * 8 * (nr + 1); w < 15 * 32; ++w) CHECK(img->bs8rows[w] == 0, "bs8rows tail %d", w);
        for (int w = 0; w < 4 * (nr + 2); ++w) {
            const uint32_t want = w < 4 * (nr + 1) ? ((img->rk[w] >> 8) | (img->rk[w] << 24)) : img->rk[w - 4];
            CHECK(img->rkrot[w] == want, "rkrot %d", w);
        }
        delete img;
    }
    return g_fail;
}

// One scanner case on stdin: u32 max_body, u32 max_n, u32 len, then len bytes
// (all little-endian).  Output: "ok <k> <consumed> <off>:<len> ..." or
// "err <code> <index> <value>".
static bool read_case(uint32_t* max_body, uint32_t* max_n, std::vector<uint8_t>* buf) {
    uint32_t hdr[3];
    if (fread(hdr, 4, 3, stdin) != 3) return false;
    *max_body = hdr[0];
    *max_n = hdr[1];
    buf->resize(hdr[2]);
    return hdr[2] == 0 || fread(buf->data(), 1, hdr[2], stdin) == hdr[2];
}

static int run_scan(const uint8_t* data, size_t len, uint32_t max_body, size_t max_n, bool print) {
    uint8_t* exact = len ? (uint8_t*)malloc(len) : nullptr;
    if (len) memcpy(exact, data, len);
    uint64_t* off = max_n ? (uint64_t*)malloc(max_n * sizeof(uint64_t)) : nullptr;
    uint32_t* rl = max_n ? (uint32_t*)malloc(max_n * sizeof(uint32_t)) : nullptr;
    size_t consumed = 12345;
    host::ScanError err{};
    const int64_t k = host::scan_records(exact, len, max_body, off, rl, max_n, &consumed, &err);
    if (k >= 0) {
        CHECK((size_t)k <= max_n, "k %lld > max_n", (long long)k);
        uint64_t pos = 0;
        for (int64_t i = 0; i < k; ++i) {   // contiguous, in bounds, headers valid
            CHECK(off[i] == pos, "record %lld offset", (long long)i);
            CHECK(rl[i] >= 5 && rl[i] - 5 <= max_body, "record %lld length", (long long)i);
            pos += rl[i];
            CHECK(pos <= len, "record %lld past the end", (long long)i);
        }
        CHECK(consumed == pos, "consumed %zu != %llu", consumed, (unsigned long long)pos);
        if (print) {
            printf("ok %lld %zu", (long long)k, consumed);
            for (int64_t i = 0; i < k; ++i) printf(" %llu:%u", (unsigned long long)off[i], rl[i]);
            printf("\n");
        }
    } else {
        CHECK(err.code == 1 || err.code == 2, "error code %d", err.code);
        if (print) printf("err %d %zu %u\n", err.code, err.index, err.value);
    }
    free(exact);
    free(off);
    free(rl);
    return g_fail;
}

static int check_scan() {
    uint32_t max_body, max_n;
    std::vector<uint8_t> buf;
    while (read_case(&max_body, &max_n, &buf)) run_scan(buf.data(), buf.size(), max_body, max_n, true);
    return g_fail;
}

static int fuzz(long iters, uint64_t seed) {
    std::mt19937_64 rng(seed);
    std::vector<uint8_t> b;
    for (long it = 0; it < iters; ++it) {
        b.clear();
        const int nrec = (int)(rng() % 12);
        static const uint32_t limits[5] = {16384, 16384 + 256, 16384 + 2048, 0, 100};
        const uint32_t max_body = limits[rng() % 5];
        for (int r = 0; r < nrec; ++r) {
            const int kind = (int)(rng() % 16);
            uint32_t body = kind < 3 ? (uint32_t)(rng() % 65536)              // any 16-bit length
                                     : kind < 5 ? max_body + (uint32_t)(rng() % 3)   // at / over the limit
                                                : (uint32_t)(rng() % 300);
            if (body > 65535) body = 65535;
            const uint8_t type = kind == 15 ? (uint8_t)rng() : (uint8_t)(20 + rng() % 5);
            b.push_back(type);
            b.push_back(3);
            b.push_back((uint8_t)(rng() % 5));
            b.push_back((uint8_t)(body >> 8));
            b.push_back((uint8_t)body);
            const size_t pay = kind == 6 ? rng() % (body + 1) : body;          // short payload
            b.resize(b.size() + pay, (uint8_t)r);   // payload bytes do not matter to the scanner
        }
        if (!b.empty() && rng() % 3 == 0) b.resize(rng() % b.size());           // truncated stream
        const size_t max_n = rng() % 4 == 0 ? rng() % 4 : 64;
        run_scan(b.data(), b.size(), max_body, max_n, false);
        if (g_fail) return g_fail;
    }
    printf("fuzz %ld cases ok\n", iters);
    return g_fail;
}

// tg::host::parallel_copy(_rows) (hostcopy.cpp) into exactly-sized heap
// buffers: every split (one row by bytes, rows contiguous and strided, 1 to
// 12 threads, sizes around the 1 MiB chunk and 4 KiB boundaries) against a
// plain memcpy, from two threads at once so the shared pool serves both.
static int check_copy() {
    std::mt19937_64 rng(99);
    int fails = 0;
    auto one = [&](uint64_t seed) {
        std::mt19937_64 r(seed);
        int f = 0;
        for (int it = 0; it < 40; ++it) {
            const size_t rows = r() % 3 == 0 ? 1 : 1 + r() % 700;
            const size_t row = rows == 1 ? (r() % 2 ? (1u << 20) * (1 + r() % 5) + r() % 9000 : r() % 70000)
                                         : 1 + r() % 20000;
            const size_t ss = row + (r() % 2 ? 0 : r() % 64), ds = row + (r() % 2 ? 0 : r() % 64);
            const size_t slen = rows ? (rows - 1) * ss + row : 0, dlen = rows ? (rows - 1) * ds + row : 0;
            std::vector<uint8_t> src(slen), dst(dlen, 0xee), want(dlen, 0xee);
            for (auto& x : src) x = (uint8_t)r();
            for (size_t q = 0; q < rows; ++q) memcpy(want.data() + q * ds, src.data() + q * ss, row);
            const int nt = 1 + (int)(r() % 12);
            tg::host::parallel_copy_rows(dst.data(), ds, src.data(), ss, row, rows, nt);
            if (dst != want) {
                printf("copy mismatch rows %zu row %zu threads %d\n", rows, row, nt);
                ++f;
            }
        }
        return f;
    };
    int f1 = 0;
    std::thread t([&] { f1 = one(rng()); });
    fails += one(rng());
    t.join();
    fails += f1;
    if (!fails) printf("copy ok\n");
    return fails;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !strcmp(argv[1], "copy")) return check_copy() ? 1 : 0;
    if (argc >= 2 && !strcmp(argv[1], "keys")) {
        const int f = check_keys();
        if (!f) printf("keys ok\n");
        return f ? 1 : 0;
    }
    if (argc >= 2 && !strcmp(argv[1], "scan")) return check_scan() ? 1 : 0;
    if (argc >= 2 && !strcmp(argv[1], "canary")) {   // the sanitizer is live: a 1-byte over-read
        uint8_t* p = (uint8_t*)malloc(5);
        memset(p, 23, 5);
        volatile int v = p[5 + (argc > 9)];
        free(p);
        return v == 0 ? 3 : 4;
    }
    if (argc >= 4 && !strcmp(argv[1], "fuzz")) return fuzz(atol(argv[2]), strtoull(argv[3], 0, 10)) ? 1 : 0;
    fprintf(stderr, "usage: host_check keys | scan < cases | fuzz N SEED\n");
    return 2;
}
