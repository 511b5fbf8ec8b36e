/*
 * tlsgpu.h -- C ABI of the MI355X TLS record-layer AEAD engine (libtlsgpu.so).
 *
 * This is the drop-in boundary for tlslite-ng's bulk-cipher path.  The
 * reference binds AEAD objects through tlslite/utils/cipherfactory.py
 * (createAESGCM :81-100, createCHACHA20 :144-159) and calls
 * obj.seal(nonce, plaintext, data) / obj.open(nonce, ciphertext, data)
 * (tlslite/utils/aesgcm.py:101,126; tlslite/utils/chacha20_poly1305.py:48,68)
 * once per record from tlslite/recordlayer.py:558 (_encryptThenSeal) and
 * :821 (_decryptAndUnseal).  The ctypes objects in tlsgpu/ (see
 * INTEGRATION.md) bind exactly the functions below.
 *
 * Conventions: plain pointers and sizes, no exceptions across the ABI, every
 * function returns an int status (TG_OK = 0, negative = error; tg_open
 * returns 1 = authentic / 0 = rejected).  A key handle is bound to the device
 * current when it was created.  tg_seal / tg_open may be called on one handle
 * from several threads at once (each call takes its own staging slot: copies
 * of an AEAD object share the handle, recordlayer.py:262, :913);
 * tg_key_destroy must not race with calls on the same handle.  Batch entry
 * points take DEVICE pointers and are ordered on the given HIP stream (NULL =
 * the null stream).
 */
#ifndef TLSGPU_H
#define TLSGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

#define TG_OK 0
#define TG_EINVAL (-22)      /* bad argument (NULL pointer, bad size) */
#define TG_EKEYLEN (-2)      /* key length: AssertionError (aesgcm.py:37-38) /
                                ValueError (chacha20_poly1305.py:21-22) */
#define TG_ENONCE (-3)       /* nonce length != 12: ValueError
                                (aesgcm.py:107-108, chacha20_poly1305.py:53-54) */
#define TG_ENOMEM (-12)
#define TG_EHIP (-5)         /* a HIP runtime call failed; see tg_last_error() */
#define TG_ENODEV (-19)      /* no GPU visible */

/* Algorithms (the reference's cipher .name values). */
#define TG_AES_GCM 0          /* "aes128gcm" (16-byte key) / "aes256gcm" (32) */
#define TG_CHACHA20_POLY1305 1 /* "chacha20-poly1305" (32-byte key) */
#define TG_AES_CCM 2          /* "aes128ccm" / "aes256ccm": 16-byte tag
                                 (aesccm.py:11-155, cipherfactory.py:102-121) */
#define TG_AES_CCM_8 3        /* "aes128ccm_8" / "aes256ccm_8": 8-byte tag
                                 (cipherfactory.py:123-142) */

typedef struct tg_key tg_key;

/* Library / device. */
const char* tg_version(void);
const char* tg_last_error(void);           /* thread-local message of the last error */
int tg_device_count(int* count);
int tg_init(int device);                   /* hipSetDevice for the calling thread */

/* Kernel-selection options (process-wide; tests and measurement -- the
 * engine's own choice is value 0 everywhere).  Each starts from its TLSGPU_*
 * environment variable, read once at first use:
 *   gcm_variant        0 auto, 6 wave per record, 14 bitsliced octet,
 *                      15 hybrid octet, 16 T-table lane per record
 *   gcm_table_variant  0 auto (<= 2048 records, or one length with <= 16 MiB
 *                      in all: wave per record without a plan; else the
 *                      length split), 1 lane, 5 wave per record,
 *                      6 wave per record with 4-bit GHASH tables,
 *                      14 key-grouped octet
 *   kt_split           key-table length split in bytes (0 = 2048)
 *   kt_lpr             key-table long records: lanes per record of the
 *                      key-grouped bitsliced kernel (8 / 16 / 32 / 64; 0 =
 *                      32), -1 = the wave-per-record T-table kernel
 *   kt_hybrid, kt_t    key-table long records at 32 lanes per record: 0 =
 *                      the persistent T-table + bitsliced kernel, -1 = the
 *                      bitsliced key-grouped kernel; its T-table waves (0 =
 *                      7 of 11, at most 11)
 *   kt_overlap         key tables: the short records' lane kernel on a
 *                      helper stream of the caller's stream beside the long
 *                      records' kernel (0 = on, -1 = both on the caller's
 *                      stream)
 *   chacha_variant     0 auto, 3 wave per record, 4 lane per record with
 *                      the register-staged tile, 5 lane per record with the
 *                      LDS-DMA tile (auto's choice for large batches),
 *                      6 eight lanes per record (octets, single key)
 *   ccm_variant        0 auto, 1 lane full rounds, 2 wave, 3 lane, 4 hybrid
 *                      (bitsliced keystream + T-table MAC waves, single key),
 *                      5 / 6 / 7 / 8 lane with the payload 1 / 2 / 4 / 8
 *                      blocks ahead (auto's single-key choice: 4)
 *   ccm_hy_t           T-table waves of the CCM hybrid (0 = 4 of 12, -1 none)
 *   waves_per_record   0 auto, 1 / 4 / 16
 *   no_plan            1 = no length-sorted launch order
 *   stage_copy         1 = per-record calls copy through device memory
 *   hy_t, hy_prio      hybrid AES-GCM kernel: T-table waves (0 = auto: 10
 *                      of 16, -1 = none; more than the workgroup's waves
 *                      fails the launch with TG_EINVAL), 1 = T-table waves
 *                      at raised priority
 *   hy_threads         hybrid AES-GCM workgroup: 0 = 1024, or 768
 * An unknown name is TG_EINVAL; a variant a launcher does not know makes
 * its launches fail with TG_EINVAL. */
int tg_set_option(const char* name, int value);
int tg_get_option(const char* name, int* value);

/* Keys -- replaces python_aesgcm.new (python_aesgcm.py:10-11) and
 * python_chacha20_poly1305.new (python_chacha20_poly1305.py:9-11): expands the
 * AES round keys and the GHASH tables for H = E_K(0) (aesgcm.py:27-57) on the
 * host and uploads them once.  nkeys > 1 builds a key table indexed by
 * tg_batch.key_idx (many sessions in one batch). */
int tg_key_create(int alg, const uint8_t* keys, size_t keylen, size_t nkeys,
                  tg_key** out);
/* tg_key_destroy waits for the device (batches on any stream may still read
 * the key), then scrubs and frees the key material. */
int tg_key_destroy(tg_key* k);
int tg_key_info(const tg_key* k, int* alg, size_t* keylen, size_t* nkeys);

/* Tag length of a key's algorithm: 16, or 8 for TG_AES_CCM_8.  Below, "T"
 * is this length. */
int tg_key_taglen(const tg_key* k);
/* Per-record drop-in, HOST buffers (synchronous).
 * tg_seal: out receives ct || tag (len + T bytes) -- AESGCM.seal /
 *   CHACHA20_POLY1305.seal / AESCCM.seal.
 * tg_open: in = ct || tag (inlen bytes); pt receives inlen - T bytes.
 *   Returns 1 when the tag verifies, 0 when the record is rejected (the
 *   reference's None: bad tag, or inlen < T), negative on error.
 *   On rejection pt is zeroed, never left holding unauthenticated bytes. */
int tg_seal(tg_key* k, const uint8_t* nonce, size_t noncelen,
            const uint8_t* aad, size_t aadlen, const uint8_t* pt, size_t len,
            uint8_t* out);
int tg_open(tg_key* k, const uint8_t* nonce, size_t noncelen,
            const uint8_t* aad, size_t aadlen, const uint8_t* in, size_t inlen,
            uint8_t* pt);

/* Batch of records, DEVICE pointers.  Record i:
 *   payload  in  + (in_off  ? in_off[i]  : i * in_stride),  len[i] bytes
 *            (seal: plaintext; open: ciphertext, followed by its T-byte tag)
 *   output   out + (out_off ? out_off[i] : i * out_stride)
 *            (seal: ct || tag, len[i] + T bytes; open: pt, len[i] bytes)
 *   nonce    nonce + 12 * i (12 bytes)
 *   aad      aad + (aad_off ? aad_off[i] : i * aad_stride),
 *            aad_len ? aad_len[i] : fixed_aad_len bytes
 *   key      key table entry key_idx ? key_idx[i] : 0; key_idx[i] must be
 *            below the table's nkeys -- a record with an index out of range
 *            is skipped (never read past the table; open: status[i] = 0
 *            and its plaintext output zeroed, as a rejected record's)
 *   status   open only: status[i] = 1 authentic / 0 rejected (pt zeroed)
 * len == NULL means every record is fixed_len bytes.  Offsets with 16-byte
 * alignment take the vector path; any alignment is accepted.
 * Records are independent; nothing is ordered between them.  AES-CCM records
 * must be shorter than 2^28 - 32 bytes (the 3-byte CCM counter; TLS records
 * are at most 2^14 + 256). */
typedef struct tg_batch {
    uint64_t n;
    const uint8_t* in;
    const uint64_t* in_off;
    uint64_t in_stride;
    const uint32_t* len;
    uint32_t fixed_len;
    uint32_t fixed_aad_len;
    uint8_t* out;
    const uint64_t* out_off;
    uint64_t out_stride;
    const uint8_t* nonce;
    const uint8_t* aad;
    const uint64_t* aad_off;
    uint64_t aad_stride;
    const uint32_t* aad_len;
    const uint32_t* key_idx;
    uint8_t* status;
} tg_batch;

int tg_seal_batch(tg_key* k, const tg_batch* b, void* stream);
int tg_open_batch(tg_key* k, const tg_batch* b, void* stream);

/* Build per-record 12-byte nonces on the device from a connection's fixed IV
 * and sequence numbers, as RecordLayer._getNonce does (recordlayer.py:522-534):
 *   mode 0 (TLS 1.3 / RFC ChaCha): nonce_i = iv12 xor (0^4 || be64(seq0 + i))
 *   mode 1 (TLS 1.2 AES-GCM / AES-CCM, draft ChaCha):
 *          nonce_i = iv4 || be64(seq0 + i)
 * out: device, 12 * n bytes. */
int tg_make_nonces(int mode, const uint8_t* iv, size_t ivlen, uint64_t seq0,
                   uint64_t n, uint8_t* out, void* stream);

/* TLS record framing on the device -- the callers either side of the AEAD in
 * tlslite/recordlayer.py: _getNonce (:522-534), _encryptThenSeal (:536-565,
 * AAD, TLS 1.2 AES-GCM / AES-CCM explicit nonce), sendRecord (:606-617, TLS 1.3 inner
 * content type + zero padding, 5-byte header), _decryptAndUnseal (:780-824,
 * publicly-invalid checks) and _tls13_de_pad (:863-884).  Record i has
 * sequence number seq0 + i.  All arrays are DEVICE pointers.
 *   seal: fragment data + data_off[i], data_len[i] bytes, content type
 *         ctype[i]; TLS 1.3 appends ctype[i] and pad_len[i] zero bytes IN
 *         PLACE after the fragment (the data buffer needs that much slack),
 *         then writes the whole record (header || [explicit nonce] || ct ||
 *         tag) at wire + wire_off[i] and its size to wire_len[i].
 *   open: wire record (header included) at wire + wire_off[i], wire_len[i]
 *         bytes; plaintext goes to data + data_off[i] (room for the inner
 *         plaintext), its length to data_len[i], the (inner) content type to
 *         ctype[i], and a TG_REC_* code to status[i].
 * For the vector path place records so the payload after the header (and
 * TLS 1.2 AES explicit nonce) is 16-byte aligned.  The tag is T bytes. */
#define TG_TLS12 0x0303
#define TG_TLS13 0x0304
#define TG_REC_OK 0
#define TG_REC_BAD_MAC 1        /* TLSBadRecordMAC (recordlayer.py:822-823) */
#define TG_REC_TRUNCATED 2      /* "Truncated nonce" / "Truncated tag" (:788-789, :797-799) */
#define TG_REC_LENGTH 3         /* "Length mismatch" (:816-817) */
#define TG_REC_BAD_TYPE 4       /* TLSUnexpectedMessage, encrypted non-app-data (:809-812) */
#define TG_REC_BAD_VERSION 5    /* TLSIllegalParameterException (:813-815) */
#define TG_REC_NO_CONTENT_TYPE 6 /* malformed inner plaintext (:880-882) */
#define TG_REC_OVERFLOW 7       /* TLSRecordOverflow: header length over the limit
                                   (RecordSocket.recv :219-222), TLS 1.3 inner
                                   plaintext over limit + 1 (:974-975), plaintext
                                   over limit (:980-981) */

typedef struct tg_records {
    uint64_t n;
    uint32_t version;           /* TG_TLS12 or TG_TLS13 */
    uint32_t fixed_iv_len;      /* 4 (TLS 1.2 AES-GCM / AES-CCM) or 12 */
    uint8_t fixed_iv[12];
    uint32_t recv_limit;        /* open: recv_record_limit (0 = 2^14, recordlayer.py:56) */
    uint64_t seq0;
    uint8_t* data;
    const uint64_t* data_off;
    uint32_t* data_len;
    uint8_t* ctype;
    const uint32_t* pad_len;    /* seal, TLS 1.3 only; NULL = no padding */
    uint8_t* wire;
    const uint64_t* wire_off;
    uint32_t* wire_len;
    uint8_t* status;            /* open */
} tg_records;

int tg_seal_records(tg_key* k, const tg_records* r, void* stream);
int tg_open_records(tg_key* k, const tg_records* r, void* stream);

/* Bulk TLS 1.3 key setup on the device -- the
 * per-session work of RecordLayer.calcTLS1_3PendingState
 * (recordlayer.py:1268-1323) and _calcTLS1_3KeyUpdate (:1325-1350) for many
 * sessions at once, all buffers DEVICE pointers.
 * tg_hkdf_expand_label: out[i] = HKDF-Expand-Label(secrets[i], label,
 *   context, outlen) (cryptomath.py:155-173, HKDF_expand :146-153, HMAC
 *   :128-132) for i < n; hashlen 32 (SHA-256) or 48 (SHA-384) is both the
 *   PRF and the secret size; 1 <= outlen <= hashlen (every record-layer use:
 *   "key", "iv", "traffic upd", "finished").  Secrets at hashlen * i, outputs
 *   at outlen * i.
 * tg_key_create_device: tg_key_create with the keys (nkeys x keylen) already
 *   in device memory: the AES key schedule, H = E_K(0) and the GHASH tables
 *   are built by kernels on `stream` (synchronised before returning), so
 *   derived keys never visit the host. */
int tg_hkdf_expand_label(int hashlen, const uint8_t* secrets, uint64_t n, const uint8_t* label,
                         size_t labellen, const uint8_t* context, size_t ctxlen, size_t outlen,
                         uint8_t* out, void* stream);
int tg_key_create_device(int alg, const uint8_t* keys, size_t keylen, size_t nkeys,
                         tg_key** out, void* stream);
/* Host ingest pipeline (tlsgpu/ingest.py) -- the
 * batched counterpart of RecordSocket (recordlayer.py:35-237).
 * tg_scan_records (HOST memory, no GPU): walk the 5-byte record headers
 *   (RecordHeader3, RecordSocket._recvHeader :169-205) of the wire bytes
 *   buf[0, len): record k starts at off[k] and spans rlen[k] = 5 + body bytes.
 *   Stops at the first incomplete record or after max_n records; *consumed =
 *   the bytes of the complete records.  Returns the record count, or
 *   TG_EOVERFLOW if a header declares body > max_body (TLSRecordOverflow,
 *   RecordSocket.recv :225-229: recv_record_limit + 2048, TLS 1.3 + 256) and
 *   TG_EHEADER for a first byte that is no TLS content type (20..24; the
 *   reference would try SSLv2 framing there).  Records before the bad header
 *   are reported through *consumed and off/rlen (the return value is then
 *   negative, so count them by *consumed).
 * tg_gather (DEVICE memory): for i < n copy len[i] bytes from
 *   src + src_off[i] to dst + dst_off[i] (pack aligned wire records into
 *   one contiguous stream and back).  off/len arrays in device memory. */
#define TG_EOVERFLOW (-75)
#define TG_EHEADER (-71)
int64_t tg_scan_records(const uint8_t* buf, size_t len, uint32_t max_body, uint64_t* off,
                        uint32_t* rlen, size_t max_n, size_t* consumed);
int tg_gather(const uint8_t* src, const uint64_t* src_off, const uint32_t* len, uint8_t* dst,
              const uint64_t* dst_off, uint64_t n, void* stream);
/* tg_host_copy / tg_host_copy_rows (HOST memory, no GPU): the ingest
 *   pipeline's copies between callers' buffers and pinned staging, split over
 *   up to nthreads threads (the caller plus a shared pool of workers;
 *   nthreads <= 0 = min(8, hardware threads)).  rows: row r of row_bytes
 *   bytes goes from src + r * src_stride to dst + r * dst_stride.  Regions
 *   must not overlap.  Returns TG_OK or TG_EINVAL (NULL with a non-zero
 *   size). */
int tg_host_copy(void* dst, const void* src, size_t bytes, int nthreads);
int tg_host_copy_rows(void* dst, size_t dst_stride, const void* src, size_t src_stride, size_t row_bytes,
                      size_t rows, int nthreads);
/* Self-test entry points (TEST-ONLY, not on the record path): run the
 * engine's device Poly1305 / GHASH arithmetic on raw messages, HOST buffers,
 * synchronous, so the reference's known answers reach the exact device code
 * of the AEAD kernels (the reference's Poly1305 / GHASH have no entry point of
 * their own: poly1305.py:32-48 Poly1305.create_tag, aesgcm.py:60-79
 * AESGCM._auth with a zero tag mask).
 * tg_selftest_poly1305: tags[i] = Poly1305(keys[i] (32 B), msgs + off[i],
 *   len[i] bytes) with RFC padding; mode 0 = the lane Horner of the batch
 *   kernel, 1 / 2 / 3 = the wave-striped Horner of the wave-per-record
 *   kernel with 1 / 4 / 16 waves per message, 4 = the octet striping of the
 *   octet kernel (eight lanes per message, chacha_variant 6).
 * tg_selftest_ghash: out[i] = GHASH_H(aad_i, ct_i) (h: n x 16 B, GCM byte
 *   order); mode 0 = 8-bit tables, 1 = 8-bit tables 8 rows in flight,
 *   2 = conflict-free rotated tables, 3 = table-free carry-less multiply,
 *   4 = octet stride-H^8 + lift (aes_gcm_bs8.hip), 5 = wave stride-H^64 +
 *   lift (gcm_wave_kernel), 6 = octet stride-H^8 through a wave's 4-bit
 *   tables (the key-table octet kernel). */
int tg_selftest_poly1305(int mode, const uint8_t* keys, const uint8_t* msgs, const uint64_t* off,
                         const uint32_t* len, uint64_t n, uint8_t* tags);
int tg_selftest_ghash(int mode, const uint8_t* h, const uint8_t* aad, const uint64_t* aad_off,
                      const uint32_t* aad_len, const uint8_t* ct, const uint64_t* ct_off,
                      const uint32_t* ct_len, uint64_t n, uint8_t* out);

/* Diagnostics: the per-launch scratch the library holds (the buffers of
 * its scratch cache, all devices) -- bounded by the launches in flight, not
 * by the streams a caller has used.  Test and monitoring use.
 * A batch call borrows a scratch buffer and gives it back behind its work
 * on the caller's stream; the next call on the same stream handle may take
 * it again at once, and that call's stream then waits for the buffer's
 * last work, so a stream destroyed with work pending and a new stream that
 * receives its handle stay correct.
 * tg_scratch_trim: frees cached scratch buffers whose work has completed
 *   until at most keep_bytes remain, and every idle helper stream (the
 *   second stream a key-table batch runs its short records on).  The cache
 *   also trims itself before it grows past 8 GiB.
 * tg_helper_info: helper streams the library holds, and how many a batch
 *   is using right now (one per caller stream in flight, at most). */
int tg_scratch_info(uint64_t* bytes, uint64_t* buffers);
int tg_scratch_trim(uint64_t keep_bytes);
int tg_helper_info(uint64_t* streams, uint64_t* busy);

/* Device memory helpers so a ctypes host needs no other GPU runtime. */
int tg_malloc(void** p, size_t bytes);
int tg_free(void* p);
int tg_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int tg_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int tg_stream_sync(void* stream);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif
#ifdef __cplusplus
}
#endif
#endif
