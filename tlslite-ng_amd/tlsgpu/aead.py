"""AEAD objects with the reference's object contract, backed by libtlsgpu.

``HipAESGCM``, ``HipAESCCM`` and ``HipCHACHA20_POLY1305`` expose exactly what
tlslite/recordlayer.py reads from an AEAD:
``isBlockCipher``, ``isAEAD``, ``name``, ``implementation``, ``nonceLength``,
``tagLength``, ``key``, ``seal(nonce, plaintext, data) -> ct||tag`` and
``open(nonce, ciphertext, data) -> plaintext or None``, with the error
conventions of tlslite/utils/aesgcm.py:27-154 (AssertionError on a bad key
length, ValueError on a bad nonce length), tlslite/utils/aesccm.py:11-149
(the same, with an 8- or 16-byte tag) and
tlslite/utils/chacha20_poly1305.py:19-94 (ValueError on either).  Objects are
stateless per call and survive ``copy.copy`` (recordlayer.py:262, :913):
copies share one refcounted device key.
"""
import ctypes

from . import _lib


class _DeviceKey(object):
    """Refcounted owner of one ``tg_key`` handle (freed when unreferenced)."""

    def __init__(self, alg, key, nkeys=1, device_keys=None, keylen=0, stream=None):
        lib = _lib.load()
        self._lib = lib
        self.handle = ctypes.c_void_p()
        if device_keys is not None:   # keys already in HBM (tg_key_create_device)
            _lib.check(lib.tg_key_create_device(alg, device_keys, keylen, nkeys,
                                                ctypes.byref(self.handle), stream))
            return
        raw = bytes(key)
        _lib.check(lib.tg_key_create(alg, raw, len(raw) // nkeys, nkeys,
                                     ctypes.byref(self.handle)))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self._lib.tg_key_destroy(h)
            self.handle = None


def _as_bytes(b):
    return b if isinstance(b, bytes) else bytes(b)


class _HipAEAD(object):
    _alg = None

    isBlockCipher = False
    isAEAD = True
    nonceLength = 12
    tagLength = 16

    def __init__(self, key, implementation="hip"):
        self.implementation = implementation
        self.key = key
        self._dkey = _DeviceKey(self._alg, key)

    def seal(self, nonce, plaintext, data):
        """Encrypt and authenticate; returns ``ciphertext || tag``."""
        if len(nonce) != 12:
            raise ValueError(self._nonce_msg)
        pt = _as_bytes(plaintext)
        aad = _as_bytes(data)
        out = ctypes.create_string_buffer(len(pt) + self.tagLength)
        _lib.check(self._dkey._lib.tg_seal(self._dkey.handle, _as_bytes(nonce), 12, aad,
                                           len(aad), pt, len(pt), out))
        return bytearray(out.raw)

    def open(self, nonce, ciphertext, data):
        """Verify then decrypt; returns the plaintext or None."""
        if len(nonce) != 12:
            raise ValueError(self._nonce_msg)
        T = self.tagLength
        if len(ciphertext) < T:
            return None
        ct = _as_bytes(ciphertext)
        aad = _as_bytes(data)
        out = ctypes.create_string_buffer(max(len(ct) - T, 1))
        rc = _lib.check(self._dkey._lib.tg_open(self._dkey.handle, _as_bytes(nonce), 12, aad,
                                                len(aad), ct, len(ct), out))
        if rc != 1:
            return None
        return bytearray(out.raw[:len(ct) - T])


class HipAESGCM(_HipAEAD):
    """Drop-in for ``AESGCM`` (tlslite/utils/aesgcm.py:21)."""
    _alg = _lib.TG_AES_GCM
    _nonce_msg = "Bad nonce length"

    def __init__(self, key, implementation="hip"):
        if len(key) == 16:
            self.name = "aes128gcm"
        elif len(key) == 32:
            self.name = "aes256gcm"
        else:
            raise AssertionError()
        super(HipAESGCM, self).__init__(key, implementation)


class HipAESCCM(_HipAEAD):
    """Drop-in for ``AESCCM`` (tlslite/utils/aesccm.py:11): ``tag_length`` 16
    (``aes128ccm`` / ``aes256ccm``) or 8 (``aes128ccm_8`` / ``aes256ccm_8``)."""
    _nonce_msg = "Bad nonce length"

    def __init__(self, key, implementation="hip", tag_length=16):
        # aesccm.py:22-30: any other key / tag combination is an AssertionError
        if len(key) == 16 and tag_length == 8:
            self.name = "aes128ccm_8"
        elif len(key) == 16 and tag_length == 16:
            self.name = "aes128ccm"
        elif len(key) == 32 and tag_length == 8:
            self.name = "aes256ccm_8"
        else:
            assert len(key) == 32 and tag_length == 16
            self.name = "aes256ccm"
        self.tagLength = tag_length
        self._alg = _lib.TG_AES_CCM if tag_length == 16 else _lib.TG_AES_CCM_8
        super(HipAESCCM, self).__init__(key, implementation)


class HipCHACHA20_POLY1305(_HipAEAD):
    """Drop-in for ``CHACHA20_POLY1305`` (tlslite/utils/chacha20_poly1305.py:17)."""
    _alg = _lib.TG_CHACHA20_POLY1305
    _nonce_msg = "Nonce must be 96 bit long"
    name = "chacha20-poly1305"

    def __init__(self, key, implementation="hip"):
        if len(key) != 32:
            raise ValueError("Key must be 256 bit long")
        super(HipCHACHA20_POLY1305, self).__init__(key, implementation)
