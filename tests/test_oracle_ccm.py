"""Pin the AES-CCM oracle (oracle/aead_oracle.c ccm_*) to the reference.

tests/golden/ccm.json was produced by running the reference's AESCCM
(tlslite/utils/aesccm.py) through tests/golden/make_golden_ccm.py; its ``kat``
entries are the known answers of unit_tests/test_tlslite_utils_aesccm.py.
"""
import numpy as np
import pytest

from vectors import FULL_HEX_MAX, detbytes, load, sha256hex, tls13_nonce

CCM = load("ccm.json")
H = bytes.fromhex


def ccm_inputs(v):
    tag = "%s-%d-%d" % (v["alg"], v["len"], v["aadlen"])
    return (detbytes("key-" + tag, v["keylen"]), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, v["aadlen"]), detbytes("pt-" + tag, v["len"]))


@pytest.mark.parametrize("i", range(len(CCM["kat"])))
def test_kat(oracle_mod, i):
    v = CCM["kat"][i]
    key, nonce, pt, aad, tl = H(v["key"]), H(v["nonce"]), H(v["pt"]), H(v["aad"]), v["taglen"]
    assert oracle_mod.ccm_seal(key, nonce, pt, aad, tl).hex() == v["ct_tag"]
    assert oracle_mod.ccm_open(key, nonce, H(v["ct_tag"]), aad, tl) == pt


def test_vectors(oracle_mod):
    for v in CCM["vectors"]:
        key, nonce, aad, pt = ccm_inputs(v)
        tl = v["taglen"]
        sealed = oracle_mod.ccm_seal(key, nonce, pt, aad, tl)
        assert sealed[-tl:].hex() == v["tag"], (v["alg"], v["len"], v["aadlen"])
        assert sha256hex(sealed[:-tl]) == v["ct_sha256"]
        if v["len"] <= FULL_HEX_MAX:
            assert sealed.hex() == v["ct_tag"]
        assert oracle_mod.ccm_open(key, nonce, sealed, aad, tl) == pt


def test_negative(oracle_mod):
    for v in CCM["negative"]:
        got = oracle_mod.ccm_open(H(v["key"]), H(v["nonce"]), H(v["ct_tag"]), H(v["aad"]),
                                  v["taglen"])
        assert got is None, (v["alg"], v["case"])


def test_errors(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.ccm_seal(bytes(16), bytes(11), b"")
    with pytest.raises(AssertionError):
        oracle_mod.ccm_seal(bytes(24), bytes(12), b"")


@pytest.mark.parametrize("bi", range(4))
def test_batch_form(oracle_mod, bi):
    """oracle.batch (the sampled checker of the GPU tests) against the fixtures."""
    b = CCM["batch"][bi]
    tl = b["taglen"]
    key, iv = H(b["key"]), H(b["iv"])
    recs = b["records"]
    n = len(recs)
    pts = [detbytes("ccm-batch-pt-%s-%d" % (b["alg"], r["seq"]), r["len"]) for r in recs]
    lens = np.array([r["len"] for r in recs], np.uint32)
    in_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    out_off = np.concatenate([[0], np.cumsum(lens + tl)[:-1]]).astype(np.uint64)
    nonces = np.frombuffer(b"".join(bytes(tls13_nonce(iv, r["seq"])) for r in recs), np.uint8)
    aad = np.frombuffer(b"".join(bytes([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff])
                                 for L in lens), np.uint8)
    alg = "aesccm" if tl == 16 else "aesccm8"
    out, _ = oracle_mod.batch(alg, "seal", np.frombuffer(key, np.uint8), nonces, aad,
                              np.arange(n, dtype=np.uint64) * 5, np.full(n, 5, np.uint32),
                              np.frombuffer(b"".join(bytes(p) for p in pts), np.uint8),
                              in_off, lens, int(out_off[-1] + lens[-1] + tl), out_off,
                              nthreads=2)
    for r, o, L in zip(recs, out_off, lens):
        rec = out[int(o):int(o) + int(L) + tl].tobytes()
        assert rec[-tl:].hex() == r["tag"]
        assert sha256hex(rec[:-tl]) == r["ct_sha256"]
