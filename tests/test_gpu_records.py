"""GPU: device record framing (tg_seal_records / tg_open_records) against the
reference RecordLayer's wire bytes (tests/golden/records.json) and the
framing oracle (oracle/records.py)."""
import hashlib

import numpy as np
import pytest

from vectors import detbytes, load

pytestmark = pytest.mark.gpu

CASES = load("records.json")


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
        return tg.HipAESCCM(bytearray(key), tag_length=8 if alg.endswith("_8") else 16)
    return tg.HipAESGCM(bytearray(key))


def _tag(alg):
    return 8 if alg.endswith("ccm_8") else 16


def _hdr(version, alg):
    return 5 + (8 if version == "tls12" and not alg.startswith("chacha") else 0)


def _layout(lens, pads, hdr, aligned, tag=16):
    """data offsets (16-aligned, with slack for ctype + padding) and wire
    offsets (payload 16-aligned if ``aligned``, else packed back to back)."""
    data_off, wire_off, d, w = [], [], 0, 0
    for L, p in zip(lens, pads):
        data_off.append(d)
        d += (L + 1 + p + tag + 15) // 16 * 16
        if aligned:
            w = (w + hdr + 15) // 16 * 16 - hdr
        wire_off.append(w)
        w += hdr + L + 1 + p + tag
    return np.array(data_off, np.int64), np.array(wire_off, np.int64), d + 16, w + 64


def _run(torch, tg, version, alg, key, iv, seq0, ctypes_, datas, pads, aligned, tamper=None):
    n = len(datas)
    lens = [len(x) for x in datas]
    hdr = _hdr(version, alg)
    data_off, wire_off, dsz, wsz = _layout(lens, pads, hdr, aligned, _tag(alg))
    host = np.zeros(dsz, np.uint8)
    for o, x in zip(data_off, datas):
        host[o:o + len(x)] = np.frombuffer(bytes(x), np.uint8)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    data = dev(host)
    d_off, w_off = dev(data_off), dev(wire_off)
    d_len = dev(np.array(lens, np.int32))
    ctype = dev(np.array(ctypes_, np.uint8))
    pad = dev(np.array(pads, np.int32))
    wire = torch.zeros(wsz, dtype=torch.uint8, device="cuda")
    w_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    v = tg.TLS13 if version == "tls13" else tg.TLS12
    k = _key(tg, alg, key)
    tg.seal_records(k, v, iv, seq0, n, data, d_off, d_len, ctype, wire, w_off, w_len,
                    pad_len=pad if version == "tls13" else None)
    torch.cuda.synchronize()
    wh, wl = wire.cpu().numpy(), w_len.cpu().numpy()
    wires = [wh[o:o + l].tobytes() for o, l in zip(wire_off, wl)]
    # open them back into a fresh data buffer
    if tamper:
        for i, fn in tamper.items():
            nb = fn(wires[i])
            wh[wire_off[i]:wire_off[i] + len(nb)] = np.frombuffer(nb, np.uint8)
            wl[i] = len(nb)
    wire2 = dev(wh)
    w_len2 = dev(wl.astype(np.int32))
    out = torch.zeros(dsz, dtype=torch.uint8, device="cuda")
    o_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    o_ct = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 255, dtype=torch.uint8, device="cuda")
    tg.open_records(k, v, iv, seq0, n, wire2, w_off, w_len2, out, d_off, o_len, o_ct, st)
    torch.cuda.synchronize()
    oh = out.cpu().numpy()
    opened = [(int(s), int(c), oh[o:o + l].tobytes()) for s, c, o, l in
              zip(st.cpu().numpy(), o_ct.cpu().numpy(), data_off, o_len.cpu().numpy())]
    return wires, opened


@pytest.mark.parametrize("ci", range(len(CASES)))
@pytest.mark.parametrize("aligned", [True, False])
def test_reference_wire_bytes(torch, tg, ci, aligned):
    c = CASES[ci]
    recs = c["records"]
    datas = [bytes(detbytes("rec-%d-%d" % (s, r["len"]), r["len"])) for s, r in enumerate(recs)]
    wires, opened = _run(torch, tg, c["version"], c["alg"], bytes.fromhex(c["key"]),
                         bytes.fromhex(c["iv"]), c["seq0"], [r["ctype"] for r in recs], datas,
                         [r["pad"] for r in recs], aligned)
    for r, w, d, o in zip(recs, wires, datas, opened):
        assert len(w) == r["wire_len"]
        assert hashlib.sha256(w).hexdigest() == r["wire_sha256"], (c["version"], c["alg"])
        if r.get("recv", "ok") == "ok":
            assert o == (0, r["ctype"], d)
        else:   # the reference receiver raised TLSRecordOverflow (recordlayer.py:974-975)
            assert r["recv"] == "TLSRecordOverflow" and o[0] == 7, (c["version"], c["alg"], r["len"])


@pytest.mark.parametrize("version,alg,klen,ivlen", [
    ("tls13", "aes128gcm", 16, 12), ("tls13", "chacha20-poly1305", 32, 12),
    ("tls12", "aes256gcm", 32, 4), ("tls12", "chacha20-poly1305", 32, 12),
    ("tls13", "aes128ccm_8", 16, 12), ("tls12", "aes256ccm", 32, 4)])
def test_random_batch_vs_oracle_and_errors(torch, tg, version, alg, klen, ivlen):
    from oracle import records as R
    rng = np.random.default_rng(klen + ivlen)
    n = 300
    key, iv = rng.bytes(klen), rng.bytes(ivlen)
    lens = list(rng.integers(0, 16385 - 300, n))
    pads = [int(rng.integers(0, 256)) if version == "tls13" else 0 for _ in range(n)]
    ctypes_ = [int(x) for x in rng.choice([21, 22, 23], n)]
    datas = [rng.bytes(int(L)) for L in lens]
    seq0 = 2 ** 40 + 3
    tamper = {5: lambda w: w[:-1] + bytes([w[-1] ^ 1]),           # bad tag
              7: lambda w: w[:21] if version == "tls13" else w[:12]}  # truncated
    if version == "tls13":
        tamper[9] = lambda w: b"\x16" + w[1:]                         # wrong outer type
    wires, opened = _run(torch, tg, version, alg, key, iv, seq0, ctypes_, datas, pads, True,
                         tamper=tamper)
    for i in range(n):
        want = R.seal_record(version, alg, key, iv, seq0 + i, ctypes_[i], datas[i], pads[i])
        assert wires[i] == want, i
        if i in tamper:
            exp = R.open_record(version, alg, key, iv, seq0 + i, tamper[i](want))
            assert opened[i][0] == exp[0] != 0, (i, opened[i][0], exp[0])
        else:
            assert opened[i] == (0, ctypes_[i], datas[i]), i


def test_tls13_all_zero_inner_plaintext(torch, tg):
    """ctype 0 with an empty fragment: _tls13_de_pad finds no content type."""
    key, iv = bytes(16), bytes(12)
    _, opened = _run(torch, tg, "tls13", "aes128gcm", key, iv, 0, [0, 23], [b"", b"x"], [3, 0], True)
    assert opened[0][0] == 6 and opened[1] == (0, 23, b"x")


@pytest.mark.parametrize("version,alg,ivlen", [("tls12", "aes128gcm", 12), ("tls12", "aes128ccm", 12),
                                               ("tls13", "aes128gcm", 4),
                                               ("tls13", "chacha20-poly1305", 4)])
def test_fixed_iv_length_rejected(torch, tg, version, alg, ivlen):
    """A fixed IV that gives no 12-byte nonce is an error, as the reference's
    nonce-length assertion (recordlayer.py:522-534, :556): TLS 1.3 needs 12
    bytes, TLS 1.2 AES-GCM / AES-CCM 4 (fixedNonce || seq)."""
    import tlsgpu
    klen = 32 if alg.startswith("chacha") else 16
    k = _key(tg, alg, bytes(klen))
    z = lambda n, dt=torch.uint8: torch.zeros(n, dtype=dt, device="cuda")  # noqa: E731
    v = tg.TLS13 if version == "tls13" else tg.TLS12
    with pytest.raises(tlsgpu.TlsGpuError):
        tg.seal_records(k, v, bytes(ivlen), 0, 1, z(64), z(1, torch.int64), z(1, torch.int32),
                        z(1), z(128), z(1, torch.int64), z(1, torch.int32))


def test_record_limits_device(torch, tg):
    """TLSRecordOverflow cases on the device, as the framing oracle
    (recordlayer.py:219-222, :974-981): a TLS 1.3 record over 2^14 + 256 bytes
    (header), a TLS 1.3 inner plaintext of 2^14 + 2, a TLS 1.2 plaintext of
    2^14 + 1; the full 2^14 records beside them open."""
    from oracle import records as R
    key, iv = bytes(range(16)), bytes(range(12))
    datas = [bytes(16384), bytes(16384), bytes(16384), bytes(100)]
    pads = [0, 1, 300, 0]
    wires, opened = _run(torch, tg, "tls13", "aes128gcm", key, iv, 5, [23] * 4, datas, pads, True)
    assert [o[0] for o in opened] == [0, 7, 7, 0]
    for i in range(4):
        assert R.open_record("tls13", "aes128gcm", key, iv, 5 + i, wires[i])[0] == opened[i][0]
    wires, opened = _run(torch, tg, "tls12", "aes128gcm", key, iv[:4], 9, [23, 23],
                         [bytes(16385), bytes(16384)], [0, 0], True)
    assert [o[0] for o in opened] == [7, 0]


@pytest.mark.parametrize("n", [32768, 1 << 20])
def test_config5_full_shape_vs_oracle(torch, tg, n):
    """BASELINE configs[4] through the path bench.py --config c5 runs:
    tg_seal_records on n TLS 1.3 AES-128-GCM records of 16 384 application
    bytes (inner plaintext 16 385 = 64 q + 1 blocks: the hybrid kernel's
    one-block last batch), bench.py's layout (header at 128 k + 123, so the
    ciphertext starts on a 128-byte line), seq0 far from 0.  n >= 32 768 runs
    the hybrid octet kernel.  128 sampled wire records -- the first and the
    last among them -- equal the framing oracle's (recordlayer.py:592-641,
    :536-565 restated, pinned to the reference RecordLayer); every record
    opens back with status ok, content type 0x17 and its fragment.  At
    both sizes every record's header is 17 03 03 40 11 and its ciphertext
    and tag equal the C oracle's seal of fragment || 0x17 (tests/fullcheck.py,
    the whole batch)."""
    import bench
    from oracle import records as R
    L = bench.C5_APP
    DS, WS, H = bench.c5_layout(L)
    seq0 = 2 ** 40 + 12345
    key, iv = bytes(detbytes("c5-key", 16)), bytes(detbytes("c5-iv", 12))
    g = torch.Generator(device="cuda").manual_seed(0xc5)
    data = torch.randint(0, 256, (n * DS,), dtype=torch.uint8, device="cuda", generator=g)
    orig = data.view(n, DS)[:, :L].clone()
    data_off = torch.arange(n, dtype=torch.int64, device="cuda") * DS
    data_len = torch.full((n,), L, dtype=torch.int32, device="cuda")
    ctype = torch.full((n,), 0x17, dtype=torch.uint8, device="cuda")
    wire_off = torch.arange(n, dtype=torch.int64, device="cuda") * WS + H
    wire = torch.zeros(n * WS, dtype=torch.uint8, device="cuda")
    wire_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    k = tg.HipAESGCM(bytearray(key))
    tg.seal_records(k, tg.TLS13, iv, seq0, n, data, data_off, data_len, ctype, wire, wire_off,
                    wire_len)
    torch.cuda.synchronize()
    assert bool((wire_len == 5 + L + 1 + 16).all())
    samples = bench.c5_samples(data, wire, wire_len, bench.c5_pick(n), L)
    assert samples[0][0] == 0 and samples[-1][0] == n - 1 and len(samples) == 128
    for i, frag, w in samples:
        assert frag == orig[i].cpu().numpy().tobytes()
        assert w == R.seal_record("tls13", "aes128gcm", key, iv, seq0 + i, 0x17, frag), i
    import fullcheck
    from oracle import oracle as O
    hdr = torch.tensor([0x17, 3, 3, 0x40, 0x11], dtype=torch.uint8, device="cuda")
    assert bool((wire.view(n, WS)[:, H:H + 5] == hdr).all())
    recs, _ = fullcheck.check_all(
        torch, O, "aesgcm", np.frombuffer(key, np.uint8), orig.view(-1), np.arange(n) * L,
        np.full(n, L), wire, np.arange(n) * WS + H + 5, fullcheck.tls13_nonces(iv, seq0, n),
        hdr.cpu().numpy(), np.zeros(n), np.full(n, 5), inner_type=0x17)
    assert recs == n
    back = torch.zeros(n * DS, dtype=torch.uint8, device="cuda")
    o_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    o_ct = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 255, dtype=torch.uint8, device="cuda")
    tg.open_records(k, tg.TLS13, iv, seq0, n, wire, wire_off, wire_len, back, data_off, o_len, o_ct, st)
    torch.cuda.synchronize()
    assert int((st == 0).sum()) == n
    assert bool((o_ct == 0x17).all()) and bool((o_len == L).all())
    assert torch.equal(back.view(n, DS)[:, :L], orig)
    del data, orig, wire, back
    torch.cuda.empty_cache()
