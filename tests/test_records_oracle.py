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
        assert (st, ctype, pt) == (R.OK, r["ctype"], bytes(data))


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
