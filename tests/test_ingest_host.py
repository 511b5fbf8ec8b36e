"""Host side of the ingest pipeline (no GPU): tg_scan_records against a
restatement of RecordSocket._recvHeader / recv (recordlayer.py:169-237):
5-byte headers, the record length limits (TLSRecordOverflow), partial tails."""
import random

import pytest

from tlsgpu import ingest


def _walk(buf, max_body):
    """RecordSocket.recv restated: (records, consumed) or the exception."""
    pos, out = 0, []
    while len(buf) - pos >= 5:
        if buf[pos] not in (20, 21, 22, 23, 24):
            raise ingest.TLSIllegalParameterException()
        body = buf[pos + 3] << 8 | buf[pos + 4]
        if body > max_body:
            raise ingest.TLSRecordOverflow()
        if len(buf) - pos < 5 + body:
            break
        out.append((pos, 5 + body))
        pos += 5 + body
    return out, pos


def _stream(rng, n, max_body):
    b = bytearray()
    for _ in range(n):
        L = rng.choice([0, 1, 16, 17, 255, 1024, max_body, rng.randint(0, max_body)])
        b += bytes([rng.choice([20, 21, 22, 23, 24]), 3, 3, L >> 8, L & 0xff])
        b += bytes(rng.getrandbits(8) for _ in range(min(L, 64))) + bytes(max(0, L - 64))
    return b


@pytest.mark.parametrize("seed", range(6))
def test_scan_matches_restatement(seed):
    rng = random.Random(seed)
    max_body = (2 ** 14 + 256) if seed % 2 else (2 ** 14 + 2048)
    buf = _stream(rng, 40, max_body)
    for cut in (len(buf), len(buf) - 1, len(buf) - 4, len(buf) // 2, 3, 0):
        part = bytes(buf[:cut])
        assert ingest.scan_records(part, max_body) == _walk(part, max_body), cut


def test_scan_max_n():
    buf = _stream(random.Random(9), 10, 2 ** 14)
    recs, used = ingest.scan_records(buf, 2 ** 14 + 2048, max_n=3)
    want, _ = _walk(buf, 2 ** 14 + 2048)
    assert recs == want[:3] and used == sum(r[1] for r in want[:3])


def test_scan_overflow_and_bad_header():
    ok = bytes([23, 3, 3, 0, 4]) + b"abcd"
    big = bytes([23, 3, 3, 0x41, 0x01])           # 16641 > 2**14 + 256 (TLS 1.3 limit)
    with pytest.raises(ingest.TLSRecordOverflow):
        ingest.scan_records(ok + big + bytes(0x4101), 2 ** 14 + 256)
    assert ingest.scan_records(ok + big + bytes(0x4101), 2 ** 14 + 2048)[1] == 9 + 5 + 0x4101
    with pytest.raises(ingest.TLSIllegalParameterException):
        ingest.scan_records(ok + bytes([0x80, 3, 3, 0, 0]), 2 ** 14)
