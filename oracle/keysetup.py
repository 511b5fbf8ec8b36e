"""CPU restatement of tlslite-ng's TLS 1.3 key derivation -- TEST INFRASTRUCTURE.

Checker for tg_hkdf_expand_label / tg_key_create_device (keysetup.hip).
Follows tlslite/utils/cryptomath.py: secureHMAC :128-132 (hmac + hashlib),
HKDF_expand :146-153, HKDF_expand_label :155-173; and the per-suite use in
tlslite/recordlayer.py calcTLS1_3PendingState :1268-1323 / _calcTLS1_3KeyUpdate
:1325-1349.  Pinned against tests/golden/keys.json (the RFC 8448 values of
unit_tests/test_tls1_3_vectors.py and outputs of the reference itself,
tests/golden/make_golden_keys.py).
"""
import hashlib
import hmac
import struct

SUITES = {0x1301: ("aesgcm", 16, "sha256"), 0x1302: ("aesgcm", 32, "sha384"),
          0x1303: ("chacha20-poly1305", 32, "sha256"), 0x1304: ("aesccm", 16, "sha256"),
          0x1305: ("aesccm_8", 16, "sha256")}


def hkdf_expand(prk, info, length, algorithm):
    """cryptomath.py:146-153: T(i) = HMAC(PRK, T(i-1) || info || i)."""
    size = hashlib.new(algorithm).digest_size
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(bytes(prk), t + bytes(info) + bytes([i]), algorithm).digest()
        out += t
        i += 1
    return out[:length]


def hkdf_label(label, context, length):
    """HkdfLabel (cryptomath.py:167-170): be16(length) || <tls13 label> || <context>."""
    full = b"tls13 " + bytes(label)
    return struct.pack(">H", length) + bytes([len(full)]) + full + bytes([len(context)]) + \
        bytes(context)


def hkdf_expand_label(secret, label, context, length, algorithm):
    return hkdf_expand(secret, hkdf_label(label, context, length), length, algorithm)


def traffic_keys(suite, secret):
    """(key, iv) of one direction, calcTLS1_3PendingState :1291-1312."""
    _, keylen, prf = SUITES[suite]
    return (hkdf_expand_label(secret, b"key", b"", keylen, prf),
            hkdf_expand_label(secret, b"iv", b"", 12, prf))


def key_update(suite, secret):
    """_calcTLS1_3KeyUpdate :1333-1336."""
    prf = SUITES[suite][2]
    return hkdf_expand_label(secret, b"traffic upd", b"", hashlib.new(prf).digest_size, prf)
