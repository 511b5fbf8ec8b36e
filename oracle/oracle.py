"""ctypes front-end of the C oracle (``oracle/aead_oracle.c``).

TEST INFRASTRUCTURE ONLY.  Imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- as the checker, never as the
thing measured or shipped.  The product library (``libtlsgpu.so``) neither
links nor calls it.

Each function mirrors the object method of the reference it restates:
``gcm_seal``/``gcm_open`` = ``AESGCM.seal/open`` (tlslite/utils/aesgcm.py:101,126),
``chacha_seal``/``chacha_open`` = ``CHACHA20_POLY1305.seal/open``
(tlslite/utils/chacha20_poly1305.py:48,68), ``ccm_seal``/``ccm_open`` =
``AESCCM.seal/open`` (tlslite/utils/aesccm.py:85,115), including the error conventions
(``ValueError`` on a bad nonce, ``None`` on a rejected record).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    """Compile the oracle with gcc (``oracle/Makefile``)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        l = ctypes.CDLL(_LIB_PATH)
        sz = ctypes.c_size_t
        p = ctypes.c_void_p
        l.oracle_gcm_seal.argtypes = [p, sz, p, sz, p, sz, p, sz, p]
        l.oracle_gcm_open.argtypes = [p, sz, p, sz, p, sz, p, sz, p]
        l.oracle_chacha_seal.argtypes = [p, sz, p, sz, p, sz, p, sz, p]
        l.oracle_chacha_open.argtypes = [p, sz, p, sz, p, sz, p, sz, p]
        l.oracle_ccm_seal.argtypes = [p, sz, sz, p, sz, p, sz, p, sz, p]
        l.oracle_ccm_open.argtypes = [p, sz, sz, p, sz, p, sz, p, sz, p]
        l.oracle_aes_encrypt_block.argtypes = [p, sz, p, p]
        l.oracle_chacha20_xor.argtypes = [p, p, ctypes.c_uint32, p, sz, p]
        l.oracle_chacha20_xor.restype = ctypes.c_int
        l.oracle_poly1305.argtypes = [p, p, sz, p]
        l.oracle_poly1305.restype = None
        l.oracle_batch.argtypes = [ctypes.c_int, ctypes.c_int, p, sz, p, p, p, p,
                                   p, p, p, p, p, p, p, sz, ctypes.c_int]
        l.oracle_selfcheck.argtypes = [sz, ctypes.c_uint64]
        l.oracle_ghash.argtypes = [p, p, sz, p, sz, p]
        l.oracle_ghash.restype = None
        _lib = l
    return _lib


def _buf(b):
    b = bytes(b)
    return b, ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b else None


def _seal(fn, key, nonce, pt, aad):
    key, aad, pt, nonce = bytes(key), bytes(aad), bytes(pt), bytes(nonce)
    out = ctypes.create_string_buffer(len(pt) + 16)
    rc = fn(key, len(key), nonce, len(nonce), aad, len(aad), pt, len(pt), out)
    if rc == -1:
        raise ValueError("Bad nonce length")
    if rc == -2:
        raise AssertionError("Bad key length")
    return bytearray(out.raw)


def _open(fn, key, nonce, ct, aad):
    key, aad, ct, nonce = bytes(key), bytes(aad), bytes(ct), bytes(nonce)
    out = ctypes.create_string_buffer(max(len(ct) - 16, 1))
    rc = fn(key, len(key), nonce, len(nonce), aad, len(aad), ct, len(ct), out)
    if rc == -1:
        raise ValueError("Bad nonce length")
    if rc == -2:
        raise AssertionError("Bad key length")
    if rc == 0:
        return None
    return bytearray(out.raw[:len(ct) - 16])


def gcm_seal(key, nonce, pt, aad=b""):
    return _seal(lib().oracle_gcm_seal, key, nonce, pt, aad)


def gcm_open(key, nonce, ct, aad=b""):
    return _open(lib().oracle_gcm_open, key, nonce, ct, aad)


def chacha_seal(key, nonce, pt, aad=b""):
    return _seal(lib().oracle_chacha_seal, key, nonce, pt, aad)


def chacha_open(key, nonce, ct, aad=b""):
    return _open(lib().oracle_chacha_open, key, nonce, ct, aad)


def ccm_seal(key, nonce, pt, aad=b"", taglen=16):
    key, aad, pt, nonce = bytes(key), bytes(aad), bytes(pt), bytes(nonce)
    out = ctypes.create_string_buffer(len(pt) + taglen)
    rc = lib().oracle_ccm_seal(key, len(key), taglen, nonce, len(nonce), aad, len(aad), pt,
                               len(pt), out)
    if rc == -1:
        raise ValueError("Bad nonce length")
    if rc == -2:
        raise AssertionError("Bad key length")
    return bytearray(out.raw)


def ccm_open(key, nonce, ct, aad=b"", taglen=16):
    key, aad, ct, nonce = bytes(key), bytes(aad), bytes(ct), bytes(nonce)
    out = ctypes.create_string_buffer(max(len(ct) - taglen, 1))
    rc = lib().oracle_ccm_open(key, len(key), taglen, nonce, len(nonce), aad, len(aad), ct,
                               len(ct), out)
    if rc == -1:
        raise ValueError("Bad nonce length")
    if rc == -2:
        raise AssertionError("Bad key length")
    if rc == 0:
        return None
    return bytearray(out.raw[:len(ct) - taglen])


def aes_block(key, block):
    key, block = bytes(key), bytes(block)
    out = ctypes.create_string_buffer(16)
    if lib().oracle_aes_encrypt_block(key, len(key), block, out):
        raise ValueError("bad key length")
    return bytearray(out.raw)


def chacha20_xor(key, nonce, counter, data):
    data = bytes(data)
    out = ctypes.create_string_buffer(max(len(data), 1))
    lib().oracle_chacha20_xor(bytes(key), bytes(nonce), counter, data, len(data), out)
    return bytearray(out.raw[:len(data)])


def poly1305(key, data):
    data = bytes(data)
    out = ctypes.create_string_buffer(16)
    lib().oracle_poly1305(bytes(key), data, len(data), out)
    return bytearray(out.raw)


def ghash(h, aad, ct):
    """GHASH_H(aad, ct) incl. the length block (``AESGCM._auth`` before the
    tag mask, aesgcm.py:60-67) for a 16-byte big-endian H."""
    h, aad, ct = bytes(h), bytes(aad), bytes(ct)
    out = ctypes.create_string_buffer(16)
    lib().oracle_ghash(h, aad, len(aad), ct, len(ct), out)
    return bytearray(out.raw)


def selfcheck(n=20000, seed=0x5eed):
    """Mismatches between the oracle's fast forms and the reference's own
    formulations (``oracle_selfcheck``: T-table AES vs byte-wise rounds,
    byte-wise vs nibble-wise GHASH multiply) over ``n`` random cases."""
    return lib().oracle_selfcheck(n, seed)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def batch(alg, op, keys, nonces, aad, aad_off, aad_len, inp, in_off, inlen,
          out_size, out_off, key_idx=None, nthreads=1, out=None):
    """Numpy batch form (see ``oracle_batch`` in aead_oracle.h).

    ``alg``: "aesgcm", "chacha", "aesccm" or "aesccm8"; ``op``: "seal" or
    "open".  Returns ``(out, status)``; ``status`` is None for seal.
    ``out``: an optional uint8 buffer of at least ``out_size`` bytes to write
    into (reused across chunks by the whole-batch checks, so the threads do
    not fault in fresh pages on every call).
    """
    a = {"aesgcm": 0, "chacha": 1, "aesccm": 2, "aesccm8": 3}[alg]
    o = {"seal": 0, "open": 1}[op]
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    keylen = keys.shape[-1] if keys.ndim > 1 else keys.size
    n = len(inlen)
    if out is None:
        out = np.zeros(out_size, dtype=np.uint8)
    elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < out_size:
        raise ValueError("out must be a contiguous uint8 buffer of >= out_size bytes")
    status = np.zeros(n, dtype=np.uint8) if o == 1 else None
    args = [np.ascontiguousarray(x) for x in (nonces, aad, inp)]
    offs = [np.ascontiguousarray(x, dtype=np.uint64) for x in (aad_off, in_off, out_off)]
    lens = [np.ascontiguousarray(x, dtype=np.uint32) for x in (aad_len, inlen)]
    kidx = None if key_idx is None else np.ascontiguousarray(key_idx, dtype=np.uint32)
    rc = lib().oracle_batch(a, o, _ptr(keys), keylen, _ptr(kidx), _ptr(args[0]),
                            _ptr(args[1]), _ptr(offs[0]), _ptr(lens[0]), _ptr(args[2]),
                            _ptr(offs[1]), _ptr(lens[1]), _ptr(out), _ptr(offs[2]),
                            _ptr(status), n, nthreads)
    if rc:
        raise ValueError("oracle_batch failed")
    return out, status
