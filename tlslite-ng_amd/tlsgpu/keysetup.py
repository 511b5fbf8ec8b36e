"""Bulk TLS 1.3 key setup on the device.

What ``RecordLayer.calcTLS1_3PendingState`` (tlslite/recordlayer.py:1268-1323)
and ``_calcTLS1_3KeyUpdate`` (:1325-1350) do for one connection, done for many
sessions in one launch:

* ``hkdf_expand_label``  -- ``HKDF_expand_label`` (cryptomath.py:155-173) of a
  batch of secrets (``tg_hkdf_expand_label``);
* ``traffic_keys``       -- write key + fixed IV of every session from its
  traffic secret, and the key table built from those keys without leaving
  HBM (``tg_key_create_device``);
* ``key_update``         -- the "traffic upd" step of a TLS 1.3 KeyUpdate.

Secrets, keys and IVs are device tensors (uint8, one row per session).
"""
from . import _lib
from .batch import KeyTable, _ptr, _stream

# TLS 1.3 suites (constants.py): AEAD, key length, PRF hash length
# (recordlayer.py _getCipherSettings :1022-1079, sha384PrfSuites).
TLS13_SUITES = {
    0x1301: ("aesgcm", 16, 32),             # TLS_AES_128_GCM_SHA256
    0x1302: ("aesgcm", 32, 48),             # TLS_AES_256_GCM_SHA384
    0x1303: ("chacha20-poly1305", 32, 32),  # TLS_CHACHA20_POLY1305_SHA256
    0x1304: ("aesccm", 16, 32),             # TLS_AES_128_CCM_SHA256
    0x1305: ("aesccm_8", 16, 32),           # TLS_AES_128_CCM_8_SHA256
}


def _torch():
    import torch
    return torch


def hkdf_expand_label(secrets, label, context, length, hashlen, out=None, stream=None):
    """``HKDF_expand_label(secret_i, label, context, length)`` for every row of
    ``secrets`` (n x hashlen device bytes); returns / fills ``out`` (n x length)."""
    torch = _torch()
    n = secrets.numel() // hashlen
    if out is None:
        out = torch.empty((n, length), dtype=torch.uint8, device=secrets.device)
    label, context = bytes(label), bytes(context)
    _lib.check(_lib.load().tg_hkdf_expand_label(hashlen, _ptr(secrets, "secrets"), n, label,
                                                len(label), context or None, len(context),
                                                length, _ptr(out, "out"), _stream(stream)))
    return out


def traffic_keys(cipher_suite, secrets, stream=None):
    """Per-session write keys and fixed IVs from traffic secrets, as
    calcTLS1_3PendingState derives them (recordlayer.py:1291-1312).

    Returns ``(KeyTable, keys, ivs)``: the key table (built on the device),
    the raw keys (n x key length) and the IVs (n x 12)."""
    alg, keylen, hashlen = TLS13_SUITES[cipher_suite]
    keys = hkdf_expand_label(secrets, b"key", b"", keylen, hashlen, stream=stream)
    ivs = hkdf_expand_label(secrets, b"iv", b"", 12, hashlen, stream=stream)
    table = KeyTable.from_device(alg, keys, keys.shape[0], keylen, stream=stream)
    return table, keys, ivs


def key_update(cipher_suite, secrets, stream=None):
    """The next application traffic secrets (``_calcTLS1_3KeyUpdate``,
    recordlayer.py:1333-1336): HKDF-Expand-Label(secret, "traffic upd", "", Hash.length)."""
    hashlen = TLS13_SUITES[cipher_suite][2]
    return hkdf_expand_label(secrets, b"traffic upd", b"", hashlen, hashlen, stream=stream)
