"""GPU parity of AES-CCM / CCM_8: libtlsgpu against the
reference's fixtures (tests/golden/ccm.json, from make_golden_ccm.py) and the
C oracle, bit-exact, through the C ABI."""
import os

import numpy as np
import pytest

from vectors import FULL_HEX_MAX, detbytes, load, sha256hex, tls13_nonce

pytestmark = pytest.mark.gpu

CCM = load("ccm.json")
H = bytes.fromhex


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return t


@pytest.fixture(scope="module")
def tg(torch):
    import tlsgpu
    assert tlsgpu.device_count() > 0
    return tlsgpu


def _obj(tg, key, taglen):
    f = tg.createAESCCM if taglen == 16 else tg.createAESCCM_8
    return f(bytearray(key), ["hip"])


def _inputs(v):
    tag = "%s-%d-%d" % (v["alg"], v["len"], v["aadlen"])
    return (detbytes("key-" + tag, v["keylen"]), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, v["aadlen"]), detbytes("pt-" + tag, v["len"]))


def test_object_contract(tg):
    for klen, tl, name in ((16, 16, "aes128ccm"), (32, 16, "aes256ccm"), (16, 8, "aes128ccm_8"),
                           (32, 8, "aes256ccm_8")):
        o = _obj(tg, bytes(klen), tl)
        assert (o.name, o.tagLength, o.nonceLength, o.isAEAD, o.implementation) == \
            (name, tl, 12, True, "hip")
    with pytest.raises(AssertionError):          # aesccm.py:22-30
        tg.HipAESCCM(bytearray(24))
    with pytest.raises(AssertionError):
        tg.HipAESCCM(bytearray(16), tag_length=12)
    o = _obj(tg, bytes(16), 16)
    with pytest.raises(ValueError):
        o.seal(bytearray(11), bytearray(3), bytearray())
    assert o.open(bytearray(12), bytearray(15), bytearray()) is None   # < tag length
    assert _obj(tg, bytes(16), 8).open(bytearray(12), bytearray(7), bytearray()) is None


@pytest.mark.parametrize("i", range(len(CCM["kat"])))
def test_kat(tg, i):
    v = CCM["kat"][i]
    o = _obj(tg, H(v["key"]), v["taglen"])
    assert o.name == v["name"]
    got = o.seal(bytearray(H(v["nonce"])), bytearray(H(v["pt"])), bytearray(H(v["aad"])))
    assert got.hex() == v["ct_tag"]
    assert o.open(bytearray(H(v["nonce"])), got, bytearray(H(v["aad"]))) == bytearray(H(v["pt"]))


def test_golden_grid(tg):
    for v in CCM["vectors"]:
        key, nonce, aad, pt = _inputs(v)
        o = _obj(tg, key, v["taglen"])
        got = o.seal(nonce, pt, aad)
        tl = v["taglen"]
        assert got[-tl:].hex() == v["tag"], (v["alg"], v["len"], v["aadlen"])
        assert sha256hex(got[:-tl]) == v["ct_sha256"]
        if v["len"] <= FULL_HEX_MAX:
            assert got.hex() == v["ct_tag"]
        assert o.open(nonce, got, aad) == pt


def test_negative(tg):
    for v in CCM["negative"]:
        o = _obj(tg, H(v["key"]), v["taglen"])
        assert o.open(bytearray(H(v["nonce"])), bytearray(H(v["ct_tag"])),
                      bytearray(H(v["aad"]))) is None, (v["alg"], v["case"])


LEN_MIX = [0, 1, 15, 16, 17, 31, 63, 64, 65, 100, 255, 256, 1000, 1024, 1025, 4096,
           16383, 16384, 16385, 16400]


@pytest.mark.parametrize("klen,tl", [(16, 16), (32, 16), (16, 8), (32, 8)])
@pytest.mark.parametrize("align", [16, 1])
# auto / lane full rounds / wave per record / lane counter-window cache /
# hybrid (bitsliced keystream + T-table MAC; "4t": T-table waves only, "4b":
# bitsliced-keystream waves only) / lane with the payload 1 / 2 / 4 / 8 blocks ahead
@pytest.mark.parametrize("variant", ["0", "1", "2", "3", "4", "4t", "4b", "5", "6", "7", "8"])
def test_batch_ragged_vs_oracle(torch, tg, oracle_mod, klen, tl, align, variant):
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(klen * 11 + tl + align)
    # + long records: many 256-counter windows
    lens = LEN_MIX * 4 + list(rng.integers(0, 16401, 150)) + [65520, 65536, 70001]
    hb = HostBatch(lens, payload_seed=align + tl, align=align, aad_mode="random", tag=tl)
    key = rng.bytes(klen)
    hy_t = {"4t": 12, "4b": -1}.get(variant, 0)
    with tg.options(ccm_variant=int(variant[0]), ccm_hy_t=hy_t):
        run_seal_open(torch, tg, oracle_mod, hb, "aesccm" if tl == 16 else "aesccm8",
                      np.frombuffer(key, np.uint8), _obj(tg, key, tl), tamper=(3, 17, 100))


@pytest.mark.parametrize("klen,tl", [(16, 16), (32, 8)])
@pytest.mark.parametrize("align", [16, 1])
# wave per record / lane per record / hybrid (key tables: the lane kernel) /
# lane per record with the payload 4 blocks ahead
@pytest.mark.parametrize("variant", ["2", "3", "4", "7"])
def test_key_table_vs_oracle(torch, tg, oracle_mod, klen, tl, align, variant):
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(3 + klen + tl + align)
    lens = list(rng.integers(0, 4097, 700)) + [0, 1, 15, 16, 17, 16384, 16400]
    hb = HostBatch(lens, payload_seed=4, align=align, aad_mode="tls12", key_count=29, tag=tl)
    keys = [rng.bytes(klen) for _ in range(29)]
    table = tg.KeyTable("aesccm" if tl == 16 else "aesccm_8", keys)
    karr = np.frombuffer(b"".join(keys), np.uint8).reshape(29, klen)
    with tg.options(ccm_variant=int(variant)):
        run_seal_open(torch, tg, oracle_mod, hb, "aesccm" if tl == 16 else "aesccm8", karr, table,
                      tamper=(1, 500))


@pytest.mark.parametrize("bi", range(4))
def test_batch_fixtures(torch, tg, bi):
    """TLS 1.3 framed batches sealed by the reference (ccm.json ``batch``)."""
    b = CCM["batch"][bi]
    tl = b["taglen"]
    key, iv = H(b["key"]), H(b["iv"])
    recs = b["records"]
    n = len(recs)
    lens = np.array([r["len"] for r in recs], np.int32)
    stride = 16400 + 16
    host = np.zeros(n * stride, np.uint8)
    for k, r in enumerate(recs):
        host[k * stride:k * stride + r["len"]] = np.frombuffer(
            bytes(detbytes("ccm-batch-pt-%s-%d" % (b["alg"], r["seq"]), r["len"])), np.uint8)
    aad = np.concatenate([np.array([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff], np.uint8)
                          for L in lens])
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 0, n, nonces)
    out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    o = _obj(tg, key, tl)
    tg.seal_batch(o, tg.make_batch(n, dev(host), out, nonces, aad=dev(aad), lens=dev(lens),
                                   in_stride=stride, out_stride=stride, aad_stride=5,
                                   fixed_aad_len=5))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for k, r in enumerate(recs):
        rec = got[k * stride:k * stride + r["len"] + tl].tobytes()
        assert rec[-tl:].hex() == r["tag"], (b["alg"], k)
        assert sha256hex(rec[:-tl]) == r["ct_sha256"]
        assert bytes(tls13_nonce(iv, r["seq"])) == nonces[12 * k:12 * k + 12].cpu().numpy().tobytes()


@pytest.mark.parametrize("klen,tl", [(16, 16), (16, 8), (32, 16)])
def test_hybrid_counter_past_2_16(torch, tg, oracle_mod, klen, tl):
    """Hybrid kernel records over 1 MiB: counters from 2^16 on change rows
    0-1 of the counter block, so the bitsliced batches leave the per-record
    round-1 cache (aesccm.py:72-83 counter layout)."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(77 + tl + klen)
    lens = [1 << 20, (1 << 20) + 16, (1 << 20) + 1000, 1100007] + list(rng.integers(0, 3000, 60))
    hb = HostBatch(lens, payload_seed=6, align=16, aad_mode="tls13", tag=tl)
    key = rng.bytes(klen)
    with tg.options(ccm_variant=4, ccm_hy_t=-1):
        run_seal_open(torch, tg, oracle_mod, hb, "aesccm" if tl == 16 else "aesccm8",
                      np.frombuffer(key, np.uint8), _obj(tg, key, tl), tamper=(1, 7))


@pytest.mark.parametrize("variant", [0, 4])
def test_large_roundtrip_and_samples(torch, tg, oracle_mod, variant):
    """2^18 x 16 KiB AES-128-CCM records: seal -> open round trip, every
    record's ciphertext and tag against the threaded C oracle
    (tests/fullcheck.py), and 32 sampled records through its per-record
    entry point; variant 4 forces the hybrid kernel."""
    with tg.options(ccm_variant=variant):
        _large(torch, tg, oracle_mod)


def _large(torch, tg, oracle_mod):
    n, L, tl = 1 << 18, 16384, 16
    g = torch.Generator(device="cuda").manual_seed(0xcc)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    key = bytes(detbytes("ccm-large-key", 16))
    iv = detbytes("ccm-large-iv", 12)
    o = _obj(tg, key, tl)
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 0, n, nonces)
    hdr = bytes([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff])
    aad = torch.tensor(list(hdr), dtype=torch.uint8, device="cuda")
    sealed = torch.empty(n * (L + tl), dtype=torch.uint8, device="cuda")
    tg.seal_batch(o, tg.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                                   out_stride=L + tl, fixed_aad_len=5))
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tg.open_batch(o, tg.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L,
                                   in_stride=L + tl, out_stride=L, fixed_aad_len=5,
                                   status=status))
    torch.cuda.synchronize()
    assert int(status.sum()) == n
    assert torch.equal(back, inp)
    del back
    import fullcheck   # every record against the oracle (aesccm.py:85-113 restated)
    recs, _ = fullcheck.check_all(torch, oracle_mod, "aesccm", np.frombuffer(key, np.uint8), inp,
                                  np.arange(n) * L, np.full(n, L), sealed, np.arange(n) * (L + tl),
                                  fullcheck.tls13_nonces(iv, 0, n), np.frombuffer(hdr, np.uint8),
                                  np.zeros(n), np.full(n, 5), tag=tl)
    assert recs == n
    rng = np.random.default_rng(2)
    for i in np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 30)])):
        i = int(i)
        pt = inp[i * L:(i + 1) * L].cpu().numpy().tobytes()
        want = oracle_mod.ccm_seal(key, bytes(tls13_nonce(iv, i)), pt, hdr, tl)
        assert sealed[i * (L + tl):(i + 1) * (L + tl)].cpu().numpy().tobytes() == bytes(want), i
    del inp, sealed
    torch.cuda.empty_cache()
