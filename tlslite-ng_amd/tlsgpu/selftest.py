"""Test-only front-end of the self-test entry points (include/tlsgpu.h
tg_selftest_poly1305 / tg_selftest_ghash): the engine's device Poly1305 and
GHASH arithmetic on raw messages, so the reference's known answers can be
checked against the exact device code the AEAD kernels use.  Not part of the
record path.
"""
import ctypes

import numpy as np

from . import _lib

POLY_MODES = {0: "lane Horner (batch kernel)", 1: "wave-striped, 1 wave",
              2: "wave-striped, 4 waves", 3: "wave-striped, 16 waves",
              4: "octet-striped, 8 lanes (octet kernel)"}
GHASH_MODES = {0: "8-bit tables", 1: "8-bit tables, 8 rows in flight", 2: "rotated tables",
               3: "table-free clmul", 4: "octet H^8 stride + lift", 5: "wave H^64 stride + lift",
               6: "octet H^8 stride, 4-bit wave tables (key-table octet kernel)"}


def _pack(msgs):
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bytes(m) for m in msgs) or b"\0", dtype=np.uint8).copy()
    return blob, offs, lens


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def poly1305(mode, keys, msgs):
    """Poly1305 tags (bytes) of msgs[i] under keys[i] (32 bytes each)."""
    lib = _lib.load()
    n = len(msgs)
    k = np.frombuffer(b"".join(bytes(x) for x in keys), dtype=np.uint8).copy()
    blob, offs, lens = _pack(msgs)
    out = np.zeros(16 * n, dtype=np.uint8)
    _lib.check(lib.tg_selftest_poly1305(mode, _ptr(k), _ptr(blob), _ptr(offs), _ptr(lens), n, _ptr(out)))
    return [out[16 * i:16 * i + 16].tobytes() for i in range(n)]


def ghash(mode, hs, aads, cts):
    """GHASH_H(aad, ct) (bytes) per item; hs: 16-byte H values (GCM order)."""
    lib = _lib.load()
    n = len(hs)
    h = np.frombuffer(b"".join(bytes(x) for x in hs), dtype=np.uint8).copy()
    ab, ao, al = _pack(aads)
    cb, co, cl = _pack(cts)
    out = np.zeros(16 * n, dtype=np.uint8)
    _lib.check(lib.tg_selftest_ghash(mode, _ptr(h), _ptr(ab), _ptr(ao), _ptr(al), _ptr(cb), _ptr(co),
                                     _ptr(cl), n, _ptr(out)))
    return [out[16 * i:16 * i + 16].tobytes() for i in range(n)]
