"""Pin the framing oracle (oracle/records.py) to the reference RecordLayer's
own output (tests/golden/records.json, from make_golden_records.py)."""
import hashlib

import pytest

from vectors import detbytes, load
from oracle import records as R

CASES = load("records.json")


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_seal_matches_reference(ci):
    c = CASES[ci]
    key, iv = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"])
    for seq, r in enumerate(c["records"]):
        data = detbytes("rec-%d-%d" % (seq, r["len"]), r["len"])
        wire = R.seal_record(c["version"], c["alg"], key, iv, c["seq0"] + seq, r["ctype"], data,
                             r["pad"])
        assert len(wire) == r["wire_len"]
        assert hashlib.sha256(wire).hexdigest() == r["wire_sha256"]
        if "wire" in r:
            assert wire.hex() == r["wire"]
        st, ctype, pt = R.open_record(c["version"], c["alg"], key, iv, c["seq0"] + seq, wire)
        if r.get("recv", "ok") == "ok":
            assert (st, ctype, pt) == (R.OK, r["ctype"], bytes(data))
        else:   # what the reference receiver raised (make_golden_records.recv_status)
            assert r["recv"] == "TLSRecordOverflow" and st == R.OVERFLOW


def test_open_error_codes():
    c = [x for x in CASES if x["version"] == "tls13" and x["alg"] == "aes128gcm"][0]
    key, iv = bytes.fromhex(c["key"]), bytes.fromhex(c["iv"])
    wire = R.seal_record("tls13", "aes128gcm", key, iv, 0, 23, b"hello")
    assert R.open_record("tls13", "aes128gcm", key, iv, 1, wire)[0] == R.BAD_MAC
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, b"\x16" + wire[1:])[0] == R.BAD_TYPE
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, wire[:3] + b"\x00\x01" + wire[5:])[0] \
        == R.LENGTH
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, wire[:20])[0] == R.TRUNCATED
    zero = R.seal_record("tls13", "aes128gcm", key, iv, 0, 0, b"")   # inner plaintext all zero
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, zero)[0] == R.NO_CONTENT_TYPE


def test_record_limits():
    """TLSRecordOverflow (recordlayer.py:219-222, :974-981): TLS 1.3 headers
    over 2^14 + 256, inner plaintexts over 2^14 + 1; TLS 1.2 bodies over
    2^14 + 2048 and plaintexts over 2^14."""
    key, iv = bytes(16), bytes(12)
    ok = R.seal_record("tls13", "aes128gcm", key, iv, 0, 23, bytes(16384))
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, ok)[0] == R.OK
    big = R.seal_record("tls13", "aes128gcm", key, iv, 0, 23, bytes(16384), pad=1)
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, big)[0] == R.OVERFLOW
    hdr_big = R.seal_record("tls13", "aes128gcm", key, iv, 0, 23, bytes(16384), pad=300)
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, hdr_big)[0] == R.OVERFLOW
    assert R.open_record("tls13", "aes128gcm", key, iv, 0, big, limit=2 ** 14 + 1)[0] == R.OK
    t12 = R.seal_record("tls12", "aes128gcm", key, iv[:4], 0, 23, bytes(16385))
    assert R.open_record("tls12", "aes128gcm", key, iv[:4], 0, t12)[0] == R.OVERFLOW
    t12ok = R.seal_record("tls12", "aes128gcm", key, iv[:4], 0, 23, bytes(16384))
    assert R.open_record("tls12", "aes128gcm", key, iv[:4], 0, t12ok)[0] == R.OK
