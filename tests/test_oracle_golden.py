"""Pin the oracle (C restatement + pure-Python restatement) to the reference.

Fixtures in tests/golden/ were produced by running the tlslite-ng reference
itself (tests/golden/make_golden.py); kat.json holds the reference's own
known-answer vectors (unit_tests/test_tlslite_utils_{aesgcm,chacha20_poly1305,
poly1305,chacha}.py).
"""
import hashlib

import pytest

from vectors import (FULL_HEX_MAX, config1_inputs, detbytes, load, tls13_aad,
                     tls13_nonce)
from oracle import pyaead

KAT = load("kat.json")
VECS = load("aead_vectors.json")
NEG = load("negative.json")
BATCH = load("record_batch.json")
H = bytes.fromhex


def _c_pair(oracle, alg):
    if alg.startswith("chacha"):
        return oracle.chacha_seal, oracle.chacha_open
    return oracle.gcm_seal, oracle.gcm_open


def _py(alg, key):
    return pyaead.CHACHA20_POLY1305(key) if alg.startswith("chacha") else pyaead.AESGCM(key)


def _inputs(v):
    tag = "%s-%d-%d" % (v["alg"], v["len"], v["aadlen"])
    return (detbytes("key-" + tag, v["keylen"]), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, v["aadlen"]), detbytes("pt-" + tag, v["len"]))


@pytest.mark.parametrize("i", range(len(KAT["aead"])))
def test_kat_aead(oracle_mod, i):
    v = KAT["aead"][i]
    seal, open_ = _c_pair(oracle_mod, v["alg"])
    key, nonce, pt, aad = H(v["key"]), H(v["nonce"]), H(v["pt"]), H(v["aad"])
    assert seal(key, nonce, pt, aad).hex() == v["ct_tag"]
    assert open_(key, nonce, H(v["ct_tag"]), aad) == pt
    py = _py(v["alg"], bytearray(key))
    assert py.seal(bytearray(nonce), bytearray(pt), bytearray(aad)).hex() == v["ct_tag"]


@pytest.mark.parametrize("i", range(12))
def test_kat_poly1305(oracle_mod, i):
    v = KAT["poly1305"][i]
    assert oracle_mod.poly1305(H(v["key"]), H(v["msg"])).hex() == v["tag"]
    assert pyaead.poly1305(H(v["key"]), H(v["msg"])).hex() == v["tag"]


def test_kat_chacha20(oracle_mod):
    for v in KAT["chacha20"]:
        got = oracle_mod.chacha20_xor(H(v["key"]), H(v["nonce"]), v["counter"], H(v["data"]))
        assert got.hex() == v["out"]
        assert pyaead.chacha20_xor(H(v["key"]), H(v["nonce"]), v["counter"],
                                   H(v["data"])).hex() == v["out"]


def test_aes_fips197(oracle_mod):
    # FIPS-197 C.1 / C.3 example vectors (AES-128, AES-256)
    pt = H("00112233445566778899aabbccddeeff")
    assert oracle_mod.aes_block(H("000102030405060708090a0b0c0d0e0f"), pt).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert oracle_mod.aes_block(H("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f"),
                                pt).hex() == "8ea2b7ca516745bfeafc49904b496089"


@pytest.mark.parametrize("i", range(len(VECS)))
def test_golden_grid_c_oracle(oracle_mod, i):
    v = VECS[i]
    key, nonce, aad, pt = _inputs(v)
    seal, open_ = _c_pair(oracle_mod, v["alg"])
    sealed = seal(key, nonce, pt, aad)
    assert sealed[-16:].hex() == v["tag"]
    assert hashlib.sha256(bytes(sealed[:-16])).hexdigest() == v["ct_sha256"]
    if "ct_tag" in v:
        assert sealed.hex() == v["ct_tag"]
    assert open_(key, nonce, sealed, aad) == pt


@pytest.mark.parametrize("i", [i for i, v in enumerate(VECS) if v["len"] <= 1025])
def test_golden_grid_pyaead(i):
    v = VECS[i]
    key, nonce, aad, pt = _inputs(v)
    sealed = _py(v["alg"], key).seal(nonce, pt, aad)
    assert sealed[-16:].hex() == v["tag"]
    if "ct_tag" in v:
        assert sealed.hex() == v["ct_tag"]


@pytest.mark.parametrize("i", range(len(NEG)))
def test_negative(oracle_mod, i):
    v = NEG[i]
    _, open_ = _c_pair(oracle_mod, v["alg"])
    assert open_(H(v["key"]), H(v["nonce"]), H(v["ct_tag"]), H(v["aad"])) is None
    assert _py(v["alg"], bytearray(H(v["key"]))).open(
        bytearray(H(v["nonce"])), bytearray(H(v["ct_tag"])), bytearray(H(v["aad"]))) is None


def test_error_conventions(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.gcm_seal(bytes(16), bytes(11), b"x")
    with pytest.raises(ValueError):
        oracle_mod.chacha_open(bytes(32), bytes(16), bytes(64))
    with pytest.raises(AssertionError):
        oracle_mod.gcm_seal(bytes(8), bytes(12), b"x")
    assert oracle_mod.gcm_open(bytes(16), bytes(12), bytes(15)) is None
    assert oracle_mod.chacha_open(bytes(32), bytes(12), bytes(15)) is None


def test_record_batches(oracle_mod):
    import numpy as np
    for b in BATCH["batches"]:
        key, iv = H(b["key"]), H(b["iv"])
        alg = "chacha" if b["alg"].startswith("chacha") else "aesgcm"
        recs = b["records"]
        n = len(recs)
        pts = [detbytes("batch-pt-%s-%d" % (b["alg"], r["seq"]), r["len"]) for r in recs]
        lens = np.array([r["len"] for r in recs], dtype=np.uint32)
        in_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        out_off = np.concatenate([[0], np.cumsum(lens + 16)[:-1]]).astype(np.uint64)
        nonces = np.frombuffer(b"".join(bytes(tls13_nonce(iv, r["seq"])) for r in recs), np.uint8)
        aad = np.frombuffer(b"".join(bytes(tls13_aad(r["len"])) for r in recs), np.uint8)
        out, _ = oracle_mod.batch(alg, "seal", np.frombuffer(key, np.uint8), nonces, aad,
                                  np.arange(n) * 5, np.full(n, 5), np.frombuffer(b"".join(
                                      bytes(p) for p in pts), np.uint8), in_off, lens,
                                  int(lens.sum()) + 16 * n, out_off, nthreads=3)
        for i, r in enumerate(recs):
            o = int(out_off[i])
            L = r["len"]
            assert out[o + L:o + L + 16].tobytes().hex() == r["tag"]
            assert hashlib.sha256(out[o:o + L].tobytes()).hexdigest() == r["ct_sha256"]
        back, status = oracle_mod.batch(alg, "open", np.frombuffer(key, np.uint8), nonces, aad,
                                        np.arange(n) * 5, np.full(n, 5), out, out_off,
                                        lens + 16, int(lens.sum()), in_off, nthreads=2)
        assert status.all()


def test_config1_digest(oracle_mod):
    key, iv, pts = config1_inputs()
    h = hashlib.sha256()
    for seq, pt in enumerate(pts):
        h.update(oracle_mod.chacha_seal(key, tls13_nonce(iv, seq), pt, tls13_aad(len(pt))))
    assert h.hexdigest() == BATCH["config1"]["sealed_sha256"]


# ---- GHASH / Poly1305 edge vectors (tests/golden/make_golden_ghash.py) ----

def test_ghash_golden_pyaead():
    """pyaead's GHASH (the 4-bit-table restatement) against the reference's
    AESGCM._auth values for edge-case H and lengths."""
    gold = load("ghash.json")["ghash"]
    for v in gold:
        h = int.from_bytes(bytes.fromhex(v["h"]), "big")
        tbl = pyaead._ghash_table(h)
        aad = detbytes("ghash-aad-%d" % v["aad_len"], v["aad_len"])
        ct = detbytes("ghash-ct-%d" % v["ct_len"], v["ct_len"])
        y = pyaead._ghash(tbl, 0, aad)
        y = pyaead._ghash(tbl, y, ct)
        y = pyaead._gmul(tbl, y ^ ((len(aad) * 8) << 64 | len(ct) * 8))
        assert y.to_bytes(16, "big").hex() == v["ghash"], (v["h_label"], v["aad_len"], v["ct_len"])


def test_ghash_golden_c_oracle(oracle_mod):
    """The C oracle's byte-wise GHASH multiply (the one its batch checks use)
    against the reference's AESGCM._auth values for edge-case H and lengths."""
    for v in load("ghash.json")["ghash"]:
        aad = detbytes("ghash-aad-%d" % v["aad_len"], v["aad_len"])
        ct = detbytes("ghash-ct-%d" % v["ct_len"], v["ct_len"])
        got = oracle_mod.ghash(bytes.fromhex(v["h"]), aad, ct)
        assert bytes(got).hex() == v["ghash"], (v["h_label"], v["aad_len"], v["ct_len"])


def test_oracle_fast_forms_selfcheck(oracle_mod):
    """T-table AES against byte-wise SubBytes/ShiftRows/MixColumns, and the
    byte-wise GHASH multiply against the reference's nibble-wise _mul, on
    20 000 random keys and blocks (AES-128 and AES-256 alternating)."""
    assert oracle_mod.selfcheck(20000) == 0


def test_poly1305_golden_extra(oracle_mod):
    """C and Python oracles against the reference's Poly1305 tags with r and s
    at their clamped maxima over long all-0xff messages."""
    for v in load("ghash.json")["poly1305_extra"]:
        key = bytes.fromhex(v["key"])
        msg = b"\xff" * v["len"] if v["msg_label"] == "ff" else bytes(detbytes(v["msg_label"], v["len"]))
        assert bytes(pyaead.poly1305(key, msg)).hex() == v["tag"]
        assert bytes(oracle_mod.poly1305(key, msg)).hex() == v["tag"]
