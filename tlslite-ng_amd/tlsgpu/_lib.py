"""ctypes binding of libtlsgpu.so (include/tlsgpu.h).

The product path.  There is no fallback: if the HIP library is missing or no
GPU is visible, the calls raise -- nothing here routes through a CPU
implementation.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtlsgpu.so")

TG_OK = 0
TG_EINVAL = -22
TG_EKEYLEN = -2
TG_ENONCE = -3
TG_ENOMEM = -12
TG_EHIP = -5
TG_ENODEV = -19
TG_EOVERFLOW = -75
TG_EHEADER = -71

TG_AES_GCM = 0
TG_CHACHA20_POLY1305 = 1
TG_AES_CCM = 2
TG_AES_CCM_8 = 3

# Every function include/tlsgpu.h declares (checked by tests/test_abi.py).
EXPORTS = ("tg_version", "tg_last_error", "tg_device_count", "tg_init", "tg_key_create",
           "tg_key_destroy", "tg_key_info", "tg_key_taglen", "tg_seal", "tg_open", "tg_seal_batch",
           "tg_open_batch", "tg_make_nonces", "tg_malloc", "tg_free", "tg_memcpy_h2d",
           "tg_memcpy_d2h", "tg_stream_sync", "tg_seal_records", "tg_open_records",
           "tg_hkdf_expand_label", "tg_key_create_device", "tg_scan_records", "tg_gather",
           "tg_selftest_poly1305", "tg_selftest_ghash", "tg_set_option", "tg_get_option",
           "tg_scratch_info", "tg_scratch_trim", "tg_helper_info", "tg_host_copy", "tg_host_copy_rows")

TG_TLS12 = 0x0303
TG_TLS13 = 0x0304
# per-record status of tg_open_records (include/tlsgpu.h TG_REC_*)
REC_STATUS = {0: "ok", 1: "bad_record_mac", 2: "truncated", 3: "length_mismatch",
              4: "unexpected_content_type", 5: "illegal_version", 6: "no_content_type",
              7: "record_overflow"}


class TgBatch(ctypes.Structure):
    """``struct tg_batch`` (include/tlsgpu.h)."""
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("inp", ctypes.c_void_p),
        ("in_off", ctypes.c_void_p),
        ("in_stride", ctypes.c_uint64),
        ("len", ctypes.c_void_p),
        ("fixed_len", ctypes.c_uint32),
        ("fixed_aad_len", ctypes.c_uint32),
        ("out", ctypes.c_void_p),
        ("out_off", ctypes.c_void_p),
        ("out_stride", ctypes.c_uint64),
        ("nonce", ctypes.c_void_p),
        ("aad", ctypes.c_void_p),
        ("aad_off", ctypes.c_void_p),
        ("aad_stride", ctypes.c_uint64),
        ("aad_len", ctypes.c_void_p),
        ("key_idx", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
    ]


class TgRecords(ctypes.Structure):
    """``struct tg_records`` (include/tlsgpu.h)."""
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("version", ctypes.c_uint32),
        ("fixed_iv_len", ctypes.c_uint32),
        ("fixed_iv", ctypes.c_uint8 * 12),
        ("recv_limit", ctypes.c_uint32),
        ("seq0", ctypes.c_uint64),
        ("data", ctypes.c_void_p),
        ("data_off", ctypes.c_void_p),
        ("data_len", ctypes.c_void_p),
        ("ctype", ctypes.c_void_p),
        ("pad_len", ctypes.c_void_p),
        ("wire", ctypes.c_void_p),
        ("wire_off", ctypes.c_void_p),
        ("wire_len", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
    ]


class TlsGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libtlsgpu error %d: %s" % (code, msg))
        self.code = code


_lib = None


def load():
    """Load libtlsgpu.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # TLSGPU_LIB: an alternative build of the same library (A/B kernel
    # measurements in tools/, never set by the package itself)
    path = os.environ.get("TLSGPU_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise OSError("libtlsgpu.so not built (run __graft_entry__.build() or "
                      "make -C tlslite-ng_amd/csrc): %s" % path)
    l = ctypes.CDLL(path)
    p, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    l.tg_version.restype = ctypes.c_char_p
    l.tg_version.argtypes = []
    l.tg_last_error.restype = ctypes.c_char_p
    l.tg_last_error.argtypes = []
    l.tg_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    l.tg_init.argtypes = [i]
    l.tg_key_create.argtypes = [i, p, sz, sz, ctypes.POINTER(ctypes.c_void_p)]
    l.tg_key_destroy.argtypes = [p]
    l.tg_key_info.argtypes = [p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(sz),
                              ctypes.POINTER(sz)]
    l.tg_key_taglen.argtypes = [p]
    l.tg_seal.argtypes = [p, p, sz, p, sz, p, sz, p]
    l.tg_open.argtypes = [p, p, sz, p, sz, p, sz, p]
    l.tg_seal_batch.argtypes = [p, ctypes.POINTER(TgBatch), p]
    l.tg_open_batch.argtypes = [p, ctypes.POINTER(TgBatch), p]
    l.tg_make_nonces.argtypes = [i, p, sz, u64, u64, p, p]
    l.tg_seal_records.argtypes = [p, ctypes.POINTER(TgRecords), p]
    l.tg_open_records.argtypes = [p, ctypes.POINTER(TgRecords), p]
    l.tg_hkdf_expand_label.argtypes = [i, p, u64, p, sz, p, sz, sz, p, p]
    l.tg_key_create_device.argtypes = [i, p, sz, sz, ctypes.POINTER(ctypes.c_void_p), p]
    l.tg_malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), sz]
    l.tg_free.argtypes = [p]
    l.tg_memcpy_h2d.argtypes = [p, p, sz, p]
    l.tg_memcpy_d2h.argtypes = [p, p, sz, p]
    l.tg_stream_sync.argtypes = [p]
    l.tg_scan_records.argtypes = [p, sz, ctypes.c_uint32, p, p, sz, ctypes.POINTER(sz)]
    l.tg_gather.argtypes = [p, p, p, p, p, u64, p]
    l.tg_selftest_poly1305.argtypes = [i, p, p, p, p, u64, p]
    l.tg_selftest_ghash.argtypes = [i, p, p, p, p, p, p, p, u64, p]
    l.tg_set_option.argtypes = [ctypes.c_char_p, i]
    l.tg_get_option.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    l.tg_scratch_info.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    # round-6 entry points; an older build under TLSGPU_LIB (A/B timing of a
    # previous round's library) has none of them and loads without
    if os.environ.get("TLSGPU_LIB") is None or hasattr(l, "tg_host_copy"):
        l.tg_scratch_trim.argtypes = [ctypes.c_uint64]
        l.tg_host_copy.argtypes = [p, p, sz, i]
        l.tg_host_copy_rows.argtypes = [p, sz, p, sz, sz, sz, i]
        l.tg_helper_info.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    for name in EXPORTS:
        if name not in ("tg_version", "tg_last_error"):
            if os.environ.get("TLSGPU_LIB") is not None and not hasattr(l, name):
                continue   # an older build under TLSGPU_LIB (A/B timing)
            getattr(l, name).restype = ctypes.c_int
    l.tg_scan_records.restype = ctypes.c_int64
    ver = l.tg_version().decode()
    if "MEASUREMENT BUILD" in ver and os.environ.get("TLSGPU_ALLOW_MEASUREMENT_BUILD") != "1":
        # a library built with a measurement-only flag (tools/build_variant.sh)
        # may return wrong ciphertext or tags: never let it pass as the product
        raise OSError("refusing %s: %s (set TLSGPU_ALLOW_MEASUREMENT_BUILD=1 for a measurement run)"
                      % (path, ver))
    _lib = l
    return l


def check(rc):
    """Raise TlsGpuError for a negative status, return rc otherwise."""
    if rc < 0:
        msg = load().tg_last_error()
        raise TlsGpuError(rc, msg.decode() if msg else "")
    return rc


def set_option(name, value):
    """Set a process-wide kernel-selection option (include/tlsgpu.h
    tg_set_option: gcm_variant, gcm_table_variant, kt_split, chacha_variant,
    ccm_variant, waves_per_record, no_plan, stage_copy, hy_t, hy_prio)."""
    check(load().tg_set_option(name.encode(), int(value)))


def get_option(name):
    v = ctypes.c_int(0)
    check(load().tg_get_option(name.encode(), ctypes.byref(v)))
    return v.value


class options(object):
    """``with tlsgpu.options(gcm_variant=14): ...`` sets options for the block
    and restores the previous values after it (tests force kernels this way)."""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_option(k, v)
        return False


def scratch_info():
    """(bytes, buffers) of per-launch scratch the library holds (tg_scratch_info)."""
    b, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(load().tg_scratch_info(ctypes.byref(b), ctypes.byref(n)))
    return b.value, n.value


def scratch_trim(keep_bytes=0):
    """Free idle launch scratch down to ``keep_bytes`` and idle helper streams (tg_scratch_trim)."""
    check(load().tg_scratch_trim(int(keep_bytes)))


def helper_info():
    """(helper streams held, helper streams in use) (tg_helper_info)."""
    s, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(load().tg_helper_info(ctypes.byref(s), ctypes.byref(b)))
    return s.value, b.value


def device_count():
    n = ctypes.c_int(0)
    rc = load().tg_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
