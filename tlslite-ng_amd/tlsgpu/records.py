"""TLS record framing on the device (tg_seal_records / tg_open_records).

The callers either side of the AEAD in tlslite/recordlayer.py, for a batch
of consecutive records of one connection direction (record i has sequence
number ``seq0 + i``):

* seal: fragment + content type (+ TLS 1.3 zero padding) -> wire record
  ``header || [TLS 1.2 AES-GCM/CCM explicit nonce] || ciphertext || tag``
  (``sendRecord`` :606-617, ``_encryptThenSeal`` :536-565, ``_getNonce``
  :522-534);
* open: wire record -> plaintext, content type and a per-record status
  mirroring the reference's exceptions (``_decryptAndUnseal`` :780-824,
  ``_tls13_de_pad`` :863-884).

All buffers are device tensors (or raw device pointers).  For seal, each
fragment needs ``1 + pad`` bytes of slack after it (TLS 1.3 writes the inner
content type and padding there in place).
"""
import ctypes

from . import _lib
from .batch import _handle, _ptr, _stream

TLS12 = _lib.TG_TLS12
TLS13 = _lib.TG_TLS13
STATUS = _lib.REC_STATUS


def _records(n, version, fixed_iv, seq0, data, data_off, data_len, ctype, wire, wire_off,
             wire_len, pad_len=None, status=None, recv_limit=0):
    r = _lib.TgRecords()
    r.n = int(n)
    r.recv_limit = int(recv_limit)
    r.version = int(version)
    iv = bytes(fixed_iv)
    if len(iv) not in (4, 12):
        raise ValueError("fixed IV must be 4 or 12 bytes")
    r.fixed_iv_len = len(iv)
    for k, b in enumerate(iv):
        r.fixed_iv[k] = b
    r.seq0 = int(seq0)
    r.data = _ptr(data, "data")
    r.data_off = _ptr(data_off, "data_off")
    r.data_len = _ptr(data_len, "data_len")
    r.ctype = _ptr(ctype, "ctype")
    r.pad_len = _ptr(pad_len, "pad_len")
    r.wire = _ptr(wire, "wire")
    r.wire_off = _ptr(wire_off, "wire_off")
    r.wire_len = _ptr(wire_len, "wire_len")
    r.status = _ptr(status, "status")
    return r


def seal_records(key, version, fixed_iv, seq0, n, data, data_off, data_len, ctype, wire,
                 wire_off, wire_len, pad_len=None, stream=None):
    """Frame and seal ``n`` records; ``wire_len`` receives each record's size."""
    dk = _handle(key)
    r = _records(n, version, fixed_iv, seq0, data, data_off, data_len, ctype, wire, wire_off,
                 wire_len, pad_len=pad_len)
    _lib.check(dk._lib.tg_seal_records(dk.handle, ctypes.byref(r), _stream(stream)))


def open_records(key, version, fixed_iv, seq0, n, wire, wire_off, wire_len, data, data_off,
                 data_len, ctype, status, stream=None, recv_limit=0):
    """Check, open and de-frame ``n`` wire records; per-record ``status`` codes
    are in ``STATUS`` (0 = ok).  ``recv_limit``: the connection's
    recv_record_limit (0 = 2^14, recordlayer.py:56)."""
    dk = _handle(key)
    r = _records(n, version, fixed_iv, seq0, data, data_off, data_len, ctype, wire, wire_off,
                 wire_len, status=status, recv_limit=recv_limit)
    _lib.check(dk._lib.tg_open_records(dk.handle, ctypes.byref(r), _stream(stream)))
