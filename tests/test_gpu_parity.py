"""GPU parity: libtlsgpu (HIP, gfx950) against the reference's fixtures and
the C oracle, bit-exact.  Every call goes through the C ABI.
"""
import hashlib

import numpy as np
import pytest

from vectors import detbytes, load, tls13_aad, tls13_nonce

pytestmark = pytest.mark.gpu

KAT = load("kat.json")
VECS = load("aead_vectors.json")
NEG = load("negative.json")
BATCH = load("record_batch.json")
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


def _obj(tg, alg, key):
    key = bytearray(key)
    if alg.startswith("chacha"):
        return tg.createCHACHA20(key, ["hip"])
    return tg.createAESGCM(key, ["hip"])


def _inputs(v):
    tag = "%s-%d-%d" % (v["alg"], v["len"], v["aadlen"])
    return (detbytes("key-" + tag, v["keylen"]), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, v["aadlen"]), detbytes("pt-" + tag, v["len"]))


# ------------------------------------------------ per-record drop-in objects

def test_object_contract(tg):
    a = _obj(tg, "aes128gcm", bytes(16))
    assert (a.name, a.isAEAD, a.isBlockCipher, a.nonceLength, a.tagLength) == \
        ("aes128gcm", True, False, 12, 16)
    assert _obj(tg, "aes256gcm", bytes(32)).name == "aes256gcm"
    c = _obj(tg, "chacha20-poly1305", bytes(32))
    assert (c.name, c.implementation) == ("chacha20-poly1305", "hip")
    import copy
    c2 = copy.copy(c)
    del c
    assert c2.open(bytes(12), c2.seal(bytes(12), b"abc", b""), b"") == b"abc"
    with pytest.raises(ValueError):
        a.seal(bytearray(11), bytearray(16), bytearray(0))
    with pytest.raises(ValueError):
        c2.open(bytearray(16), bytearray(64), bytearray(0))
    assert a.open(bytearray(12), bytearray(15), bytearray(0)) is None


@pytest.mark.parametrize("i", range(len(KAT["aead"])))
def test_kat(tg, i):
    v = KAT["aead"][i]
    o = _obj(tg, v["alg"], H(v["key"]))
    got = o.seal(bytearray(H(v["nonce"])), bytearray(H(v["pt"])), bytearray(H(v["aad"])))
    assert got.hex() == v["ct_tag"]
    assert o.open(bytearray(H(v["nonce"])), got, bytearray(H(v["aad"]))) == bytearray(H(v["pt"]))


def test_golden_grid(tg):
    for v in VECS:
        key, nonce, aad, pt = _inputs(v)
        o = _obj(tg, v["alg"], key)
        sealed = o.seal(nonce, pt, aad)
        assert sealed[-16:].hex() == v["tag"], (v["alg"], v["len"], v["aadlen"])
        assert hashlib.sha256(bytes(sealed[:-16])).hexdigest() == v["ct_sha256"]
        assert o.open(nonce, sealed, aad) == pt


def test_negative(tg):
    for v in NEG:
        o = _obj(tg, v["alg"], H(v["key"]))
        assert o.open(bytearray(H(v["nonce"])), bytearray(H(v["ct_tag"])),
                      bytearray(H(v["aad"]))) is None, (v["alg"], v["case"])


# ----------------------------------------------------------- device batches

def _run_seal_open(torch, tg, oracle_mod, hb, alg, keys, key_obj, tamper=()):
    from batchpack import run_seal_open
    run_seal_open(torch, tg, oracle_mod, hb, alg, keys, key_obj, tamper)


LEN_MIX = [0, 1, 15, 16, 17, 31, 63, 64, 65, 100, 255, 256, 1000, 1024, 1025, 4096,
           16383, 16384, 16385, 16400]


@pytest.mark.parametrize("alg,klen", [("aesgcm", 16), ("aesgcm", 32), ("chacha", 32)])
@pytest.mark.parametrize("align", [16, 1])
def test_batch_ragged_vs_oracle(torch, tg, oracle_mod, alg, klen, align):
    from batchpack import HostBatch
    rng = np.random.default_rng(klen * 7 + align)
    lens = LEN_MIX * 6 + list(rng.integers(0, 16401, 200))
    hb = HostBatch(lens, payload_seed=align, align=align, aad_mode="random")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    _run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                   tamper=(3, 17, 100))


@pytest.mark.parametrize("alg,klen", [("chacha", 32), ("aesgcm", 16), ("aesgcm", 32)])
@pytest.mark.parametrize("align", [16, 1])
def test_key_table_vs_oracle(torch, tg, oracle_mod, alg, klen, align):
    """Many sessions in one batch (BASELINE config 4 shape): key_idx per record."""
    from batchpack import HostBatch
    rng = np.random.default_rng(5 + klen + align)
    lens = list(rng.integers(0, 4097, 700)) + [0, 1, 15, 16, 17, 16384, 16400]
    hb = HostBatch(lens, payload_seed=9, align=align, aad_mode="tls12", key_count=37)
    keys = [rng.bytes(klen) for _ in range(37)]
    table = tg.KeyTable("chacha20-poly1305" if alg == "chacha" else "aesgcm", keys)
    karr = np.frombuffer(b"".join(keys), np.uint8).reshape(37, klen)
    _run_seal_open(torch, tg, oracle_mod, hb, alg, karr, table, tamper=(1, 500))


def test_record_batch_fixtures(torch, tg):
    """The reference's own TLS 1.3 framed batches (tests/golden/record_batch.json)."""
    from batchpack import HostBatch
    for b in BATCH["batches"]:
        recs = b["records"]
        lens = [r["len"] for r in recs]
        hb = HostBatch(lens, align=16, iv=H(b["iv"]))
        for r in recs:
            o = int(hb.in_off[r["seq"]])
            hb.inp[o:o + r["len"]] = np.frombuffer(
                bytes(detbytes("batch-pt-%s-%d" % (b["alg"], r["seq"]), r["len"])), np.uint8)
        d = hb.to_device(torch)
        key = bytearray(H(b["key"]))
        obj = tg.HipCHACHA20_POLY1305(key) if b["alg"].startswith("chacha") else tg.HipAESGCM(key)
        tg.seal_batch(obj, hb.batch_kwargs(d))
        got = d["out"].cpu().numpy()
        for i, r in enumerate(recs):
            o, L = int(hb.out_off[i]), r["len"]
            assert got[o + L:o + L + 16].tobytes().hex() == r["tag"], (b["alg"], i)
            assert hashlib.sha256(got[o:o + L].tobytes()).hexdigest() == r["ct_sha256"]


def test_make_nonces(torch, tg):
    iv = detbytes("nonce-iv", 12)
    out = torch.zeros(12 * 1000, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 2 ** 40 - 7, 1000, out)
    got = out.cpu().numpy().tobytes()
    want = b"".join(bytes(tls13_nonce(iv, 2 ** 40 - 7 + i)) for i in range(1000))
    assert got == want
    tg.make_nonces(iv[:4], 5, 1000, out, tls13=False)
    got = out.cpu().numpy().tobytes()
    assert got == b"".join(bytes(iv[:4]) + (5 + i).to_bytes(8, "big") for i in range(1000))


def test_config1_digest(torch, tg):
    """BASELINE configs[0] through the device batch path: digest from the reference."""
    from vectors import config1_inputs
    key, iv, pts = config1_inputs()
    n = len(pts)
    inp = torch.from_numpy(np.frombuffer(b"".join(bytes(p) for p in pts), np.uint8).copy()).cuda()
    out = torch.zeros(n * 1040, dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 0, n, nonces)
    aad = torch.from_numpy(np.frombuffer(bytes(tls13_aad(1024)), np.uint8).copy()).cuda()
    obj = tg.HipCHACHA20_POLY1305(key)
    b = tg.make_batch(n, inp, out, nonces, aad=aad, fixed_len=1024, in_stride=1024,
                      out_stride=1040, aad_stride=0, fixed_aad_len=5)
    tg.seal_batch(obj, b)
    torch.cuda.synchronize()
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == \
        BATCH["config1"]["sealed_sha256"]
    # and the whole batch opens back to the plaintexts (chacha20_poly1305.py:68)
    back = torch.zeros_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tg.open_batch(obj, tg.make_batch(n, out, back, nonces, aad=aad, fixed_len=1024,
                                     in_stride=1040, out_stride=1024, aad_stride=0,
                                     fixed_aad_len=5, status=status))
    torch.cuda.synchronize()
    assert int(status.sum()) == n and torch.equal(back, inp)


# ------------------------------------------- full-size (BASELINE configs 2/3)

@pytest.mark.parametrize("alg", ["aesgcm", "chacha", "aesgcm-bs8", "chacha-regs", "aesgcm-stride",
                                 "chacha-stride", "chacha-octet", "chacha-octet-stride"])
def test_full_size_roundtrip_and_samples(torch, tg, oracle_mod, alg):
    """2^20 x 16 KiB records: every record's ciphertext and tag bit-exact
    against the threaded C oracle (tests/fullcheck.py, 2^16-record chunks),
    the seal -> open round trip on the whole batch, and 64 sampled records
    through the oracle's per-record entry point.
    aesgcm-bs8 forces the 8-block bitsliced kernel (gcm_variant 14),
    chacha-regs the register-staged tile fill (chacha_variant 4; the default
    fills it by LDS-DMA), chacha-octet the octet kernel (chacha_variant 6,
    eight lanes per record, no tile).  *-stride: sealed records at bench.py's stride,
    L + 16 rounded up to a 128-byte line (16 512 B), the layout the metric is
    measured on."""
    variant = 14 if alg == "aesgcm-bs8" else 0
    cv = 4 if alg == "chacha-regs" else 6 if alg.startswith("chacha-octet") else 0
    stride = 16512 if alg.endswith("-stride") else None
    alg = {"aesgcm-bs8": "aesgcm", "chacha-regs": "chacha", "aesgcm-stride": "aesgcm",
           "chacha-stride": "chacha", "chacha-octet": "chacha", "chacha-octet-stride": "chacha"}.get(alg, alg)
    with tg.options(gcm_variant=variant, chacha_variant=cv):
        _full_size(torch, tg, oracle_mod, alg, stride)


def _full_size(torch, tg, oracle_mod, alg, stride=None):
    n, L = 1 << 20, 16384
    SL = stride or L + 16
    g = torch.Generator(device="cuda").manual_seed(0x7715)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    key = bytes(detbytes("full-size-" + alg, 16 if alg == "aesgcm" else 32))
    iv = detbytes("full-size-iv", 12)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    sealed = torch.empty(n * SL, dtype=torch.uint8, device="cuda")
    tg.seal_batch(obj, tg.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                                     out_stride=SL, fixed_aad_len=5))
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tg.open_batch(obj, tg.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L,
                                     in_stride=SL, out_stride=L, fixed_aad_len=5,
                                     status=status))
    torch.cuda.synchronize()
    assert int(status.sum()) == n
    assert torch.equal(back, inp)
    del back
    import fullcheck
    recs, nbytes = fullcheck.check_all(
        torch, oracle_mod, alg, np.frombuffer(key, np.uint8), inp, np.arange(n) * L,
        np.full(n, L), sealed, np.arange(n) * SL, fullcheck.tls13_nonces(iv, 0, n),
        np.frombuffer(bytes(tls13_aad(L)), np.uint8), np.zeros(n), np.full(n, 5))
    assert recs == n and nbytes == n * (L + 16)
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 62)]))
    for i in idx:
        i = int(i)
        pt = inp[i * L:(i + 1) * L].cpu().numpy().tobytes()
        nonce = bytes(tls13_nonce(iv, i))
        want = (oracle_mod.gcm_seal if alg == "aesgcm" else oracle_mod.chacha_seal)(
            key, nonce, pt, bytes(tls13_aad(L)))
        got = sealed[i * SL:i * SL + L + 16].cpu().numpy().tobytes()
        assert got == bytes(want), i
    del inp, sealed
    torch.cuda.empty_cache()
