"""CPU restatement of tlslite-ng's AEAD record framing -- TEST INFRASTRUCTURE.

Checker for tg_seal_records / tg_open_records.  Follows
tlslite/recordlayer.py: _getNonce :522-534, _encryptThenSeal :536-565,
sendRecord :606-617 (TLS 1.3 inner plaintext), _decryptAndUnseal :780-824,
_tls13_de_pad :863-884, and the record-size limits of RecordSocket.recv
:219-222 and recvRecord :974-981 (TLSRecordOverflow).  Pinned against tests/golden/records.json, which
the reference RecordLayer itself produced (tests/golden/make_golden_records.py).
Status codes are include/tlsgpu.h TG_REC_*.
"""
from . import oracle

OK, BAD_MAC, TRUNCATED, LENGTH, BAD_TYPE, BAD_VERSION, NO_CONTENT_TYPE, OVERFLOW = range(8)
RECV_LIMIT = 2 ** 14   # recv_record_limit (recordlayer.py:56)
APP_DATA = 23


def taglen(alg):
    return 8 if alg.endswith("ccm_8") else 16


def _pair(alg):
    if alg.startswith("chacha"):
        return oracle.chacha_seal, oracle.chacha_open
    if "ccm" in alg:   # AESCCM (aesccm.py), tag 16 or 8
        t = taglen(alg)
        return (lambda k, n, p, a: oracle.ccm_seal(k, n, p, a, t),
                lambda k, n, c, a: oracle.ccm_open(k, n, c, a, t))
    return oracle.gcm_seal, oracle.gcm_open


def nonce(version, alg, iv, seq):
    iv = bytes(iv)
    if version == "tls13" or (alg.startswith("chacha") and len(iv) == 12):
        pad = bytes(4) + int(seq).to_bytes(8, "big")
        return bytes(a ^ b for a, b in zip(iv, pad))
    return iv[:4] + int(seq).to_bytes(8, "big")


def seal_record(version, alg, key, iv, seq, ctype, data, pad=0):
    seal, _ = _pair(alg)
    data = bytes(data)
    if version == "tls13":
        inner = data + bytes([ctype]) + bytes(pad)
        n = len(inner) + taglen(alg)
        hdr = bytes([APP_DATA, 3, 3, n >> 8, n & 0xff])
        return hdr + bytes(seal(key, nonce(version, alg, iv, seq), inner, hdr))
    aad = int(seq).to_bytes(8, "big") + bytes([ctype, 3, 3, len(data) >> 8, len(data) & 0xff])
    body = bytes(seal(key, nonce(version, alg, iv, seq), data, aad))
    if not alg.startswith("chacha"):
        body = int(seq).to_bytes(8, "big") + body
    return bytes([ctype, 3, 3, len(body) >> 8, len(body) & 0xff]) + body


def open_record(version, alg, key, iv, seq, wire, limit=RECV_LIMIT):
    """-> (status, content type, plaintext)"""
    _, open_ = _pair(alg)
    wire = bytes(wire)
    if len(wire) < 5:
        return TRUNCATED, 0, b""
    hdr, buf = wire[:5], wire[5:]
    # RecordSocket.recv refuses the header first (recordlayer.py:219-222)
    if len(buf) > limit + 2048 or (version == "tls13" and len(buf) > limit + 256):
        return OVERFLOW, 0, b""
    explicit = 8 if (version == "tls12" and not alg.startswith("chacha")) else 0
    if explicit > len(buf):
        return TRUNCATED, 0, b""
    if explicit:
        n = bytes(iv)[:4] + buf[:8]
        buf = buf[8:]
    else:
        n = nonce(version, alg, iv, seq)
    if len(buf) < taglen(alg):
        return TRUNCATED, 0, b""
    if version == "tls12":
        plen = len(buf) - taglen(alg)
        aad = int(seq).to_bytes(8, "big") + bytes([hdr[0], 3, 3, plen >> 8, plen & 0xff])
    else:
        if hdr[0] != APP_DATA:
            return BAD_TYPE, 0, b""
        if hdr[1:3] != b"\x03\x03":
            return BAD_VERSION, 0, b""
        if (hdr[3] << 8 | hdr[4]) != len(buf):
            return LENGTH, 0, b""
        aad = hdr
    pt = open_(key, n, buf, aad)
    if pt is None:
        return BAD_MAC, 0, b""
    pt = bytes(pt)
    if version == "tls12":
        if len(pt) > limit:                               # :980-981
            return OVERFLOW, 0, b""
        return OK, hdr[0], pt
    if len(pt) > limit + 1:                               # :974-975
        return OVERFLOW, 0, b""
    pos = len(pt)
    while pos > 0 and pt[pos - 1] == 0:
        pos -= 1
    if pos == 0:
        return NO_CONTENT_TYPE, 0, b""
    return OK, pt[pos - 1], pt[:pos - 1]
