"""Factory functions mirroring tlslite/utils/cipherfactory.py for the AEADs.

``createAESGCM``, ``createAESCCM``, ``createAESCCM_8`` and ``createCHACHA20``
(all ``(key, implList=None)``) keep the reference's selection rule
(cipherfactory.py:81-100, :102-121, :123-142, :144-159): walk
``implList`` in order, return the first implementation that is available,
raise ``NotImplementedError`` if none is.  This package provides the ``"hip"``
implementation; the reference's ``"openssl"``/``"pycrypto"``/``"python"``
backends live in tlslite itself, so when this module is spliced into the
reference those names fall through to the reference's own
factory.  Standing alone, the default list is ``["hip"]``.
"""
from .aead import HipAESCCM, HipAESGCM, HipCHACHA20_POLY1305

#: implementation names this package can build
CIPHER_IMPLEMENTATIONS = ("hip",)


def _available():
    from . import _lib
    try:
        return _lib.device_count() > 0
    except OSError:
        return False


def createAESGCM(key, implList=None):
    """Create a new AES-GCM object (16- or 32-byte ``bytearray`` key)."""
    if implList is None:
        implList = ["hip"]
    for impl in implList:
        if impl == "hip" and _available():
            return HipAESGCM(key, "hip")
    raise NotImplementedError()


def createAESCCM(key, implList=None):
    """Create a new AES-CCM object with a 16-byte tag (16- or 32-byte key)."""
    if implList is None:
        implList = ["hip"]
    for impl in implList:
        if impl == "hip" and _available():
            return HipAESCCM(key, "hip")
    raise NotImplementedError()


def createAESCCM_8(key, implList=None):
    """Create a new AES-CCM object with an 8-byte tag (16- or 32-byte key)."""
    if implList is None:
        implList = ["hip"]
    for impl in implList:
        if impl == "hip" and _available():
            return HipAESCCM(key, "hip", 8)
    raise NotImplementedError()


def createCHACHA20(key, implList=None):
    """Create a new ChaCha20-Poly1305 object (32-byte ``bytearray`` key)."""
    if implList is None:
        implList = ["hip"]
    for impl in implList:
        if impl == "hip" and _available():
            return HipCHACHA20_POLY1305(key, "hip")
    raise NotImplementedError()
