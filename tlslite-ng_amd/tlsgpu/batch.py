"""Device-resident batch entry points (tg_seal_batch / tg_open_batch).

The per-record objects in ``aead.py`` keep the reference's call pattern (one
synchronous seal/open per record, recordlayer.py:558, :821); throughput comes
from handing the engine a whole batch of records that already sit in HBM.
Buffers are anything with a device address: a ``torch`` CUDA tensor (torch is
only plumbing here: allocation, streams, distributed), or a raw ``int``
pointer from ``tlsgpu.device_alloc``.

Record i of a batch (include/tlsgpu.h, ``struct tg_batch``):
  payload  ``inp + in_off[i]`` (or ``i * in_stride``), ``lens[i]`` bytes
  output   ``out + out_off[i]`` (or ``i * out_stride``); seal writes ct||tag
  nonce    ``nonces + 12 i``
  aad      ``aad + aad_off[i]`` (or ``i * aad_stride``), ``aad_len[i]`` bytes
  key      ``key_idx[i]`` into a key table (multi-session batches)
"""
import ctypes

from . import _lib
from .aead import _DeviceKey, _HipAEAD


def _ptr(x, what):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if hasattr(x, "is_cuda") and not x.is_cuda:
            raise ValueError("%s must live in device memory" % what)
        if hasattr(x, "is_contiguous") and not x.is_contiguous():
            raise ValueError("%s must be contiguous" % what)
        return x.data_ptr()
    raise TypeError("%s: expected a device tensor or pointer, got %r" % (what, type(x)))


def _stream(stream):
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except ImportError:
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


ALG_CODES = {"aesgcm": _lib.TG_AES_GCM, "aesccm": _lib.TG_AES_CCM,
             "aesccm_8": _lib.TG_AES_CCM_8, "chacha20-poly1305": _lib.TG_CHACHA20_POLY1305}


class KeyTable(object):
    """Many session keys of one algorithm, indexed by ``key_idx`` in a batch."""

    def __init__(self, alg, keys):
        keys = [bytes(k) for k in keys]
        if not keys or len(set(len(k) for k in keys)) != 1:
            raise ValueError("keys must be a non-empty list of equal-length keys")
        self.alg = alg
        self.nkeys = len(keys)
        self.keylen = len(keys[0])
        self.tagLength = 8 if alg == "aesccm_8" else 16
        self._dkey = _DeviceKey(ALG_CODES[alg], b"".join(keys), len(keys))

    @classmethod
    def from_device(cls, alg, keys, nkeys, keylen, stream=None):
        """Key table from ``nkeys`` x ``keylen`` key bytes already in device
        memory (tg_key_create_device: schedule, H and tables built on the GPU)."""
        t = cls.__new__(cls)
        t.alg, t.nkeys, t.keylen = alg, int(nkeys), int(keylen)
        t.tagLength = 8 if alg == "aesccm_8" else 16
        t._dkey = _DeviceKey(ALG_CODES[alg], None, t.nkeys, device_keys=_ptr(keys, "keys"),
                             keylen=t.keylen, stream=_stream(stream))
        return t


def _handle(key):
    if isinstance(key, _HipAEAD):
        return key._dkey
    if isinstance(key, KeyTable):
        return key._dkey
    raise TypeError("key must be a tlsgpu AEAD object or KeyTable")


def make_batch(n, inp, out, nonces, aad=None, lens=None, fixed_len=0, in_off=None,
               in_stride=0, out_off=None, out_stride=0, aad_off=None, aad_stride=0,
               aad_len=None, fixed_aad_len=0, key_idx=None, status=None):
    b = _lib.TgBatch()
    b.n = int(n)
    b.inp = _ptr(inp, "inp")
    b.in_off = _ptr(in_off, "in_off")
    b.in_stride = int(in_stride)
    b.len = _ptr(lens, "lens")
    b.fixed_len = int(fixed_len)
    b.fixed_aad_len = int(fixed_aad_len)
    b.out = _ptr(out, "out")
    b.out_off = _ptr(out_off, "out_off")
    b.out_stride = int(out_stride)
    b.nonce = _ptr(nonces, "nonces")
    b.aad = _ptr(aad, "aad")
    b.aad_off = _ptr(aad_off, "aad_off")
    b.aad_stride = int(aad_stride)
    b.aad_len = _ptr(aad_len, "aad_len")
    b.key_idx = _ptr(key_idx, "key_idx")
    b.status = _ptr(status, "status")
    return b


def seal_batch(key, batch, stream=None):
    """Seal every record of ``batch`` (a TgBatch from make_batch); async on ``stream``."""
    dk = _handle(key)
    _lib.check(dk._lib.tg_seal_batch(dk.handle, ctypes.byref(batch), _stream(stream)))


def open_batch(key, batch, stream=None):
    """Open every record; ``batch.status`` receives 1 (authentic) / 0 (rejected)."""
    dk = _handle(key)
    if not batch.status:
        raise ValueError("open_batch needs a status buffer")
    _lib.check(dk._lib.tg_open_batch(dk.handle, ctypes.byref(batch), _stream(stream)))


def make_nonces(iv, seq0, n, out, tls13=True, stream=None):
    """Per-record nonces on the device, as RecordLayer._getNonce
    (recordlayer.py:522-534): iv xor seq (TLS 1.3) or iv4 || seq (TLS 1.2)."""
    iv = bytes(iv)
    _lib.check(_lib.load().tg_make_nonces(0 if tls13 else 1, iv, len(iv), int(seq0), int(n),
                                          _ptr(out, "out"), _stream(stream)))
