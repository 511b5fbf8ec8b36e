"""GPU: the host ingest pipeline (tlsgpu/ingest.py).

RecordWriter output is compared record by record with the framing oracle
(oracle/records.py, pinned to the reference RecordLayer's wire bytes); the
RecordReader gets the wire stream back in socket-sized pieces and must return
the original fragments, then raise the reference's exceptions for a tampered
record and an oversized header; a socketpair round trip runs both ends
concurrently."""
import random
import socket
import threading

import numpy as np
import pytest

from oracle import records as orec
from vectors import detbytes

pytestmark = pytest.mark.gpu

SUITES = [("tls13", "aes128gcm", 16, 12), ("tls13", "chacha20-poly1305", 32, 12),
          ("tls12", "aes256gcm", 32, 4), ("tls12", "chacha20-poly1305", 32, 12),
          ("tls13", "aes128ccm", 16, 12)]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return t


@pytest.fixture(scope="module")
def tg(torch):
    import tlsgpu
    return tlsgpu


def _key(tg, alg, key):
    if alg.startswith("chacha"):
        return tg.HipCHACHA20_POLY1305(bytearray(key))
    if "ccm" in alg:
        return tg.HipAESCCM(bytearray(key))
    return tg.HipAESGCM(bytearray(key))


class Sink(object):
    def __init__(self):
        self.buf = bytearray()

    def sendall(self, mv):
        self.buf += bytes(mv)


def _messages(seed):
    rng = random.Random(seed)
    sizes = [0, 1, 15, 16, 2 ** 14 - 1, 2 ** 14, 2 ** 14 + 1, 3 * 2 ** 14 + 7, 100000]
    sizes += [rng.randint(0, 70000) for _ in range(12)]
    return [detbytes("ingest-%d-%d" % (seed, i), n) for i, n in enumerate(sizes)]


def _fragments(msgs, limit):
    out = []
    for m in msgs:
        if not m:
            out.append(b"")
        for p in range(0, len(m), limit):
            out.append(bytes(m[p:p + limit]))
    return out


@pytest.mark.parametrize("ver,alg,klen,ivlen", SUITES)
def test_writer_vs_oracle_and_reader_roundtrip(torch, tg, ver, alg, klen, ivlen):
    key = detbytes("ingest-key-" + alg, klen)
    iv = detbytes("ingest-iv-" + alg, ivlen)
    version = tg.TLS13 if ver == "tls13" else tg.TLS12
    pad = 3 if ver == "tls13" else 0
    # fragments shortened by the padding: the inner plaintext stays within
    # the 2^14 + 1 the receiver accepts (recordlayer.py:974-975)
    limit = 2 ** 14 - pad
    sink = Sink()
    w = tg.RecordWriter(sink, _key(tg, alg, key), version, iv, seq0=5, batch_records=7,
                        pad=pad, send_record_limit=limit)
    msgs = _messages(klen + ivlen)
    for m in msgs:
        w.write(m)
    w.flush()
    frags = _fragments(msgs, limit)
    want = b"".join(orec.seal_record(ver, alg, key, iv, 5 + i, 23, f, pad=pad)
                    for i, f in enumerate(frags))
    assert w.records_sent == len(frags)
    assert bytes(sink.buf) == want
    # reader: the same stream in uneven socket reads
    r = tg.RecordReader(_key(tg, alg, key), version, iv, seq0=5, batch_records=5)
    got, rng, pos = [], random.Random(1), 0
    while pos < len(want):
        k = rng.choice([1, 5, 100, 4096, 20000, 70000])
        r.feed(want[pos:pos + k])
        pos += k
        got.extend(r.records())
    assert [t for t, _ in got] == [23] * len(frags)
    assert [bytes(d) for _, d in got] == frags


def test_reader_errors(torch, tg):
    key, iv = detbytes("ingest-err", 16), detbytes("ingest-err-iv", 12)
    recs = [orec.seal_record("tls13", "aes128gcm", key, iv, i, 23, detbytes("e%d" % i, 300))
            for i in range(6)]
    bad = bytearray(recs[3])
    bad[-1] ^= 1
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv)
    r.feed(b"".join(recs[:3]) + bytes(bad) + b"".join(recs[4:]))
    ok = r.records()
    assert [bytes(d) for _, d in ok] == [bytes(detbytes("e%d" % i, 300)) for i in range(3)]
    from tlsgpu.ingest import TLSBadRecordMAC, TLSRecordOverflow
    with pytest.raises(TLSBadRecordMAC):
        r.records()
    r2 = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv)
    r2.feed(recs[0] + bytes([23, 3, 3, 0x41, 0x01]) + bytes(0x4101))   # > 2**14 + 256
    assert len(r2.records()) == 1
    with pytest.raises(TLSRecordOverflow):
        r2.records()


def test_socketpair_bulk(torch, tg):
    """Both ends over a real socket: 64 MiB of application data."""
    key, iv = detbytes("ingest-sock", 32), detbytes("ingest-sock-iv", 12)
    a, b = socket.socketpair()
    data = np.random.default_rng(3).integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    w = tg.RecordWriter(a, _key(tg, "chacha", key), tg.TLS13, iv, batch_records=512)

    def send():
        for p in range(0, len(data), 1 << 20):
            w.write(data[p:p + (1 << 20)])
        w.flush()
        a.shutdown(socket.SHUT_WR)

    t = threading.Thread(target=send)
    t.start()
    r = tg.RecordReader(_key(tg, "chacha", key), tg.TLS13, iv, batch_records=512)
    out = bytearray()
    while True:
        chunk = b.recv(1 << 20)
        if not chunk:
            break
        r.feed(chunk)
        for ct, d in r.records():
            assert ct == 23
            out += d
    t.join()
    a.close()
    b.close()
    assert out == data


def test_reader_refuses_oversized_inner_plaintext(torch, tg):
    """A TLS 1.3 record whose inner plaintext exceeds 2^14 + 1 (a full 2^14
    fragment with padding) is refused with TLSRecordOverflow after the
    records before it, as the reference's recvRecord does
    (recordlayer.py:974-975; tests/golden/records.json "recv")."""
    from tlsgpu.ingest import TLSRecordOverflow
    key, iv = detbytes("ingest-ovf", 16), detbytes("ingest-ovf-iv", 12)
    recs = [orec.seal_record("tls13", "aes128gcm", key, iv, i, 23, detbytes("o%d" % i, 16384),
                             pad=(3 if i == 2 else 0)) for i in range(4)]
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv)
    r.feed(b"".join(recs))
    ok = r.records()
    assert [bytes(d) for _, d in ok] == [bytes(detbytes("o%d" % i, 16384)) for i in range(2)]
    with pytest.raises(TLSRecordOverflow):
        r.records()


def _mixed_stream(key, iv, n, seed, bad=None):
    """n TLS 1.3 AES-128-GCM records, every fourth a handshake (22) record,
    sizes 0..2^14; ``bad``: index of a record with a flipped tag bit."""
    rng = random.Random(seed)
    recs, app = [], []
    for i in range(n):
        L = rng.choice([0, 1, 17, 300, 4096, 16384, rng.randint(0, 16384)])
        ct = 22 if i % 4 == 3 else 23
        pt = detbytes("mix-%d-%d" % (seed, i), L)
        r = bytearray(orec.seal_record("tls13", "aes128gcm", key, iv, i, ct, pt))
        if i == bad:
            r[-1] ^= 1
        recs.append(bytes(r))
        app.append(bytes(pt) if ct == 23 else b"")
    return recs, app


@pytest.mark.parametrize("out_kind", ["none", "pageable", "pinned"])
@pytest.mark.parametrize("batch", [2, 5, 1024])
def test_read_application_data_pipelined(torch, tg, out_kind, batch):
    """The bulk path over several pipelined slots: handshake records dropped,
    application data concatenated in order, whatever the socket read sizes
    and batch size (recordlayer.py:780-824 per record)."""
    key, iv = detbytes("bulk-key", 16), detbytes("bulk-iv", 12)
    recs, app = _mixed_stream(key, iv, 41, batch)
    wire, want = b"".join(recs), b"".join(app)
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
    if out_kind == "pinned":
        buf = torch.empty(len(want) + 64, dtype=torch.uint8).pin_memory().numpy()
    else:
        buf = np.zeros(len(want) + 64, np.uint8)
    got, pos, rng, fed = bytearray(), 0, random.Random(batch), 0
    while fed < len(wire):
        k = rng.choice([3, 700, 20000, 100000, 300000])
        r.feed(wire[fed:fed + k])
        fed += k
        if out_kind == "none":
            got += r.read_application_data()
        else:
            pos += len(r.read_application_data(out=memoryview(buf)[pos:]))
    if out_kind != "none":
        got = bytes(buf[:pos])
    assert bytes(got) == want


@pytest.mark.parametrize("batch", [2, 3, 1024])
def test_read_application_data_errors(torch, tg, batch):
    """A bad tag in a later pipelined batch: the application data before it is
    returned, TLSBadRecordMAC on the next call; an oversize header likewise
    raises TLSRecordOverflow after the records before it."""
    from tlsgpu.ingest import TLSBadRecordMAC, TLSRecordOverflow
    key, iv = detbytes("bulk-err", 16), detbytes("bulk-err-iv", 12)
    recs, app = _mixed_stream(key, iv, 12, 7, bad=9)
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
    r.feed(b"".join(recs))
    assert bytes(r.read_application_data()) == b"".join(app[:9])
    with pytest.raises(TLSBadRecordMAC):
        r.read_application_data()
    recs, app = _mixed_stream(key, iv, 6, 8)
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
    r.feed(b"".join(recs) + bytes([23, 3, 3, 0x41, 0x01]) + bytes(0x4101))
    assert bytes(r.read_application_data()) == b"".join(app)
    with pytest.raises(TLSRecordOverflow):
        r.read_application_data()
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
    r.feed(bytes([23, 3, 3, 0x41, 0x01]))
    with pytest.raises(TLSRecordOverflow):
        r.read_application_data()


@pytest.mark.parametrize("out_kind", ["pageable", "pinned"])
@pytest.mark.parametrize("batch", [2, 5, 1024])
def test_read_application_data_out_too_small_retry(torch, tg, out_kind, batch):
    """A caller buffer too small for the data is a ValueError that changes
    nothing: a retry with a large enough buffer returns exactly the bytes a
    first call with it would have (sequence numbers and the unread wire bytes
    are restored); the stream goes on after it, including a bad
    record's error at its place."""
    from tlsgpu.ingest import TLSBadRecordMAC
    key, iv = detbytes("small-out", 16), detbytes("small-out-iv", 12)
    recs, app = _mixed_stream(key, iv, 30, 3 + batch, bad=27)
    want = b"".join(app[:27])
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
    r.feed(b"".join(recs[:20]))
    first = len(b"".join(app[:20]))
    mk = (lambda n: torch.empty(n, dtype=torch.uint8).pin_memory().numpy()) if out_kind == "pinned" \
        else (lambda n: np.zeros(n, np.uint8))
    if first:
        small = mk(max(1, first // 3))
        with pytest.raises(ValueError):
            r.read_application_data(out=memoryview(small))
        with pytest.raises(ValueError):   # and again: still nothing consumed
            r.read_application_data(out=memoryview(small))
    big = mk(len(want) + 64)
    pos = len(r.read_application_data(out=memoryview(big)))
    assert bytes(big[:pos]) == b"".join(app[:20])
    r.feed(b"".join(recs[20:]))
    pos += len(r.read_application_data(out=memoryview(big)[pos:]))
    assert bytes(big[:pos]) == want
    with pytest.raises(TLSBadRecordMAC):
        r.read_application_data(out=memoryview(big)[pos:])


@pytest.mark.parametrize("ver,alg,klen,ivlen", SUITES[:3])
def test_writer_write_buffer_commit(torch, tg, ver, alg, klen, ivlen):
    """Zero-copy writes (write_buffer / commit): application data placed
    straight into the pinned slot gives the same wire bytes as write() -- the
    framing oracle's (oracle/records.py, pinned to the reference RecordLayer)
    -- and the two can be mixed."""
    key = detbytes("wb-key-" + alg, klen)
    iv = detbytes("wb-iv-" + alg, ivlen)
    version = tg.TLS13 if ver == "tls13" else tg.TLS12
    limit = 2 ** 14
    sink = Sink()
    w = tg.RecordWriter(sink, _key(tg, alg, key), version, iv, seq0=3, batch_records=6)
    msgs = _messages(3 * klen)
    frags = []
    for i, m in enumerate(msgs):
        if i % 2:
            w.write(m)
            frags += _fragments([m], limit)
            continue
        pos = 0
        while True:   # as much as the slot takes per commit (a socket recv_into loop)
            buf = w.write_buffer()
            k = min(len(buf), len(m) - pos)
            buf[:k] = m[pos:pos + k]
            w.commit(k)
            frags += _fragments([m[pos:pos + k]], limit)
            pos += k
            if pos >= len(m):
                break
    w.flush()
    want = b"".join(orec.seal_record(ver, alg, key, iv, 3 + i, 23, f) for i, f in enumerate(frags))
    assert w.records_sent == len(frags)
    assert bytes(sink.buf) == want
    with pytest.raises(ValueError):
        w.commit(10 ** 9)


@pytest.mark.parametrize("batch", [2, 5, 1024])
def test_read_application_data_with_data(torch, tg, batch):
    """read_application_data(out, data=...): the wire bytes handed to the call
    (copied batch by batch while the GPU opens the batches before) give the
    same application data as feed() + read, across uneven socket reads and
    records split between calls; recv_buffer / commit feeds in place."""
    key, iv = detbytes("data-key", 16), detbytes("data-iv", 12)
    recs, app = _mixed_stream(key, iv, 57, 11 + batch)
    wire, want = b"".join(recs), b"".join(app)
    for mode in ("data", "recv_buffer"):
        r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=batch)
        buf = torch.empty(len(want) + 64, dtype=torch.uint8).pin_memory().numpy()
        pos, rng, fed = 0, random.Random(batch), 0
        while fed < len(wire):
            k = rng.choice([3, 700, 20000, 100000, 300000, 10 ** 6])
            piece = wire[fed:fed + k]
            fed += k
            if mode == "data":
                pos += len(r.read_application_data(out=memoryview(buf)[pos:], data=piece))
            else:
                mv = r.recv_buffer(len(piece))
                mv[:len(piece)] = piece
                r.commit(len(piece))
                pos += len(r.read_application_data(out=memoryview(buf)[pos:]))
        assert bytes(buf[:pos]) == want, mode


def test_read_application_data_with_data_errors(torch, tg):
    """data= keeps the error contract: the application data before a bad tag,
    then TLSBadRecordMAC; a too-small ``out`` is a ValueError that consumes
    nothing of ``data`` (a retry with the same bytes and a larger buffer
    returns them)."""
    from tlsgpu.ingest import TLSBadRecordMAC
    key, iv = detbytes("data-err", 16), detbytes("data-err-iv", 12)
    recs, app = _mixed_stream(key, iv, 20, 5, bad=15)
    r = tg.RecordReader(_key(tg, "aesgcm", key), tg.TLS13, iv, batch_records=3)
    piece = b"".join(recs[:10])
    first = b"".join(app[:10])
    if first:
        small = np.zeros(max(1, len(first) // 3), np.uint8)
        with pytest.raises(ValueError):
            r.read_application_data(out=memoryview(small), data=piece)
    big = np.zeros(len(b"".join(app)) + 64, np.uint8)
    pos = len(r.read_application_data(out=memoryview(big), data=piece))
    assert bytes(big[:pos]) == first
    pos += len(r.read_application_data(out=memoryview(big)[pos:], data=b"".join(recs[10:])))
    assert bytes(big[:pos]) == b"".join(app[:15])
    with pytest.raises(TLSBadRecordMAC):
        r.read_application_data(out=memoryview(big)[pos:])
