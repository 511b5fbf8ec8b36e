"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where the read-only tlslite-ng reference is
importable through ``refloader``.  The reference never
travels to the GPU box; the JSON files written here do.

    python tests/golden/make_golden.py            # write fixtures
    python tests/golden/make_golden.py --timing   # also time reference vs pyaead

Fixtures:
  kat.json           known-answer vectors from the reference's own unit tests
                     (inputs + expected outputs), re-verified against the
                     reference before writing;
  aead_vectors.json  seal/open over the LENGTHS x AAD_LENGTHS x ALGS grid with
                     inputs from vectors.detbytes, outputs from the reference;
  negative.json      tampered tag / ciphertext / aad / nonce -> None;
  record_batch.json  TLS 1.3 framed batches (nonce = iv xor seq, 5-byte AAD)
                     and the config-1 workload digest.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refloader  # noqa: E402
from vectors import (AAD_LENGTHS, ALGS, FULL_HEX_MAX, LENGTHS, config1_inputs,  # noqa: E402
                     detbytes, sha256hex, tls13_aad, tls13_nonce)

refloader.load()
from tlslite.utils import python_aesgcm, python_chacha20_poly1305  # noqa: E402
from tlslite.utils.chacha import ChaCha  # noqa: E402
from tlslite.utils.poly1305 import Poly1305  # noqa: E402


def ref_new(alg, key):
    if alg == "chacha20-poly1305":
        return python_chacha20_poly1305.new(key)
    return python_aesgcm.new(key)


H = bytes.fromhex

# Known answers held by the reference's unit tests (cited per entry).
KAT_AEAD = [
    # unit_tests/test_tlslite_utils_aesgcm.py:30-43
    ("aes128gcm", "01" * 16, "02" * 12, b"text to encrypt.".hex(), "",
     "27816817e65a295cf28e6d46cb910e757a313af67da75c40ba11d872df234bd4"),
    # :123-138 (GCM spec test case 1)
    ("aes128gcm", "00" * 16, "00" * 12, "", "", "58e2fccefa7e3061367f1d57a4e7455a"),
    # :140-156 (case 2)
    ("aes128gcm", "00" * 16, "00" * 12, "00" * 16, "",
     "0388dace60b6a392f328c2b971b2fe78ab6e47d42cec13bdf53a67b21257bddf"),
    # :158-189 (case 3)
    ("aes128gcm", "feffe9928665731c6d6a8f9467308308", "cafebabefacedbaddecaf888",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
     "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255", "",
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e"
     "21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091473f5985"
     "4d5c2af327cd64a62cf35abd2ba6fab4"),
    # :191-226 (case 4)
    ("aes128gcm", "feffe9928665731c6d6a8f9467308308", "cafebabefacedbaddecaf888",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
     "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39",
     "feedfacedeadbeeffeedfacedeadbeefabaddad2",
     "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e"
     "21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091"
     "5bc94fbc3221a5db94fae95ae7121a47"),
    # :228-242 (case 13)
    ("aes256gcm", "00" * 32, "00" * 12, "", "", "530f8afbc74536b9a963b4f1c4cb738b"),
    # :244-258 (case 14)
    ("aes256gcm", "00" * 32, "00" * 12, "00" * 16, "",
     "cea7403d4d606b6e074ec5d3baf39d18d0d1c8a799996bf0265b98b5d48ab919"),
    # unit_tests/test_tlslite_utils_chacha20_poly1305.py:29-55 (RFC 7539 2.8.2)
    ("chacha20-poly1305",
     "808182838485868788898a8b8c8d8e8f909192939495969798999a9b9c9d9e9f",
     "070000004041424344454647",
     b"Ladies and Gentlemen of the class of '99: If I could offer you only one "
     b"tip for the future, sunscreen would be it.".hex(),
     "50515253c0c1c2c3c4c5c6c7",
     "d31a8d34648e60db7b86afbc53ef7ec2a4aded51296e08fea9e2b5a736ee62d6"
     "3dbea45e8ca9671282fafb69da92728b1a71de0a9e060b2905d6a5b67ecd3b36"
     "92ddbd7f2d778b8c9803aee328091b58fab324e4fad675945585808b4831d7bc"
     "3ff4def08e4b7a9de576d26586cec64b6116"
     "1ae10b594f09e26a7e902ecbd0600691"),
    # :63-109 (RFC 7539 A.5, open direction)
    ("chacha20-poly1305",
     "1c9240a5eb55d38af333888604f6b5f0473917c1402b80099dca5cbc207075c0",
     "000000000102030405060708",
     (b"Internet-Drafts are draft documents valid for a maximum of six months "
      b"and may be updated, replaced, or obsoleted by other documents at any "
      b"time. It is inappropriate to use Internet-Drafts as reference material "
      b"or to cite them other than as /\xe2\x80\x9cwork in progress./\xe2\x80\x9d").hex(),
     "f33388860000000000004e91",
     "64a0861575861af460f062c79be643bd5e805cfd345cf389f108670ac76c8cb2"
     "4c6cfc18755d43eea09ee94e382d26b0bdb7b73c321b0100d4f03b7f355894cf"
     "332f830e710b97ce98c8a84abd0b948114ad176e008d33bd60f982b1ff37c855"
     "9797a06ef4f0ef61c186324e2b3506383606907b6a7c02b0f9f6157b53c867e4"
     "b9166c767b804d46a59b5216cde7a4e99040c5a40433225ee282a1b0a06c523e"
     "af4534d7f83fa1155b0047718cbc546a0d072b04b3564eea1b422273f548271a"
     "0bb2316053fa76991955ebd63159434ecebb4e466dae5a1073a6727627097a10"
     "49e617d91d361094fa68f0ff77987130305beaba2eda04df997b714d6c6f2c29"
     "a6ad5cb4022b02709b"
     "eead9d67890cbb22392336fea1851f38"),
]

IETF_TEXT = (b"Any submission to the IETF intended by the Contributor for publi"
             b"cation as all or part of an IETF Internet-Draft or RFC and any s"
             b"tatement made within the context of an IETF activity is consider"
             b"ed an \"IETF Contribution\". Such statements include oral statemen"
             b"ts in IETF sessions, as well as written and electronic communica"
             b"tions made at any time or place, which are addressed to")

# unit_tests/test_tlslite_utils_poly1305.py:52-210 (RFC 7539 2.5.2, A.3 #1-11)
KAT_POLY = [
    ("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b",
     b"Cryptographic Forum Research Group".hex(), "a8061dc1305136c6c22b8baf0c0127a9"),
    ("00" * 32, "00" * 64, "00" * 16),
    ("00" * 16 + "36e5f6b5c5e06070f0efca96227a863e", IETF_TEXT.hex(),
     "36e5f6b5c5e06070f0efca96227a863e"),
    ("36e5f6b5c5e06070f0efca96227a863e" + "00" * 16, IETF_TEXT.hex(),
     "f3477e7cd95417af89a6b8794c310cf0"),
    ("1c9240a5eb55d38af333888604f6b5f0473917c1402b80099dca5cbc207075c0",
     (b"'Twas brillig, and the slithy toves\nDid gyre and gimble in the wabe:\n"
      b"All mimsy were the borogoves,\nAnd the mome raths outgrabe.").hex(),
     "4541669a7eaaee61e708dc7cbcc5eb62"),
    ("02" + "00" * 31, "ff" * 16, "03" + "00" * 15),
    ("02" + "00" * 15 + "ff" * 16, "02" + "00" * 15, "03" + "00" * 15),
    ("01" + "00" * 31, "ff" * 16 + "f0" + "ff" * 15 + "11" + "00" * 15, "05" + "00" * 15),
    ("01" + "00" * 31, "ff" * 16 + "fb" + "fe" * 15 + "01" * 16, "00" * 16),
    ("02" + "00" * 31, "fd" + "ff" * 15, "fa" + "ff" * 15),
    ("01" + "00" * 7 + "04" + "00" * 23,
     "e33594d7505e43b90000000000000000" "3394d7505e4379cd0100000000000000"
     "00000000000000000000000000000000" "01000000000000000000000000000000",
     "14" + "00" * 7 + "55" + "00" * 7),
    ("01" + "00" * 7 + "04" + "00" * 23,
     "e33594d7505e43b90000000000000000" "3394d7505e4379cd0100000000000000"
     "00000000000000000000000000000000", "13" + "00" * 15),
]


def make_kat():
    out = {"aead": [], "poly1305": [], "chacha20": []}
    for alg, key, nonce, pt, aad, expect in KAT_AEAD:
        c = ref_new(alg, bytearray(H(key)))
        got = c.seal(bytearray(H(nonce)), bytearray(H(pt)), bytearray(H(aad)))
        assert got.hex() == expect, (alg, key)
        assert c.open(bytearray(H(nonce)), got, bytearray(H(aad))) == bytearray(H(pt))
        out["aead"].append({"alg": alg, "key": key, "nonce": nonce, "pt": pt,
                            "aad": aad, "ct_tag": expect})
    for key, msg, expect in KAT_POLY:
        m = bytearray(H(msg))
        tag = Poly1305(bytearray(H(key))).create_tag(m).hex()
        assert tag == expect, key
        out["poly1305"].append({"key": key, "msg": m.hex(), "tag": tag})
    # ChaCha20 block function, RFC 7539 2.3.2 / 2.4.2
    # (unit_tests/test_tlslite_utils_chacha.py:122-349 exercise these)
    for key, nonce, ctr, n in (
            ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
             "000000090000004a00000000", 1, 64),
            ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
             "000000000000004a00000000", 1, 114),
            ("00" * 32, "00" * 12, 0, 64),
            ("00" * 31 + "01", "00" * 11 + "02", 1, 375)):
        data = detbytes("chacha-kat-%d" % n, n)
        ct = ChaCha(bytearray(H(key)), bytearray(H(nonce)), counter=ctr).encrypt(data)
        out["chacha20"].append({"key": key, "nonce": nonce, "counter": ctr,
                                "data": data.hex(), "out": ct.hex()})
    return out


def vec_inputs(alg, klen, L, A):
    tag = "%s-%d-%d" % (alg, L, A)
    return (detbytes("key-" + tag, klen), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, A), detbytes("pt-" + tag, L))


def make_vectors():
    vecs = []
    for alg, klen in ALGS:
        for L in LENGTHS:
            for A in AAD_LENGTHS:
                key, nonce, aad, pt = vec_inputs(alg, klen, L, A)
                c = ref_new(alg, key)
                sealed = c.seal(nonce, pt, aad)
                assert c.open(nonce, sealed, aad) == pt
                v = {"alg": alg, "keylen": klen, "len": L, "aadlen": A,
                     "tag": sealed[-16:].hex(), "ct_sha256": sha256hex(sealed[:-16])}
                if L <= FULL_HEX_MAX:
                    v["ct_tag"] = sealed.hex()
                vecs.append(v)
    return vecs


def make_negative():
    neg = []
    for alg, klen in ALGS:
        for L in (0, 1, 16, 17, 1024):
            key, nonce, aad, pt = vec_inputs(alg, klen, L, 13)
            c = ref_new(alg, key)
            sealed = c.seal(nonce, pt, aad)
            cases = [("tag_bit", nonce, sealed[:-1] + bytearray([sealed[-1] ^ 1]), aad),
                     ("aad_bit", nonce, sealed, bytearray([aad[0] ^ 0x80]) + aad[1:]),
                     ("nonce_bit", bytearray([nonce[0] ^ 1]) + nonce[1:], sealed, aad),
                     ("short", nonce, sealed[:15], aad)]
            if L:
                cases.append(("ct_bit", nonce, bytearray([sealed[0] ^ 4]) + sealed[1:], aad))
            for name, n2, ct2, aad2 in cases:
                assert c.open(n2, ct2, aad2) is None, (alg, L, name)
                neg.append({"alg": alg, "key": key.hex(), "case": name, "nonce": n2.hex(),
                            "ct_tag": ct2.hex(), "aad": aad2.hex(), "expect": None})
    return neg


BATCH_LENGTHS = [16384, 0, 1, 16385, 1024, 5, 16, 4096, 100, 16384, 63, 64, 65,
                 2000, 16383, 31]


def make_batches():
    out = {"batches": []}
    for alg, klen in ALGS:
        key = detbytes("batch-key-" + alg, klen)
        iv = detbytes("batch-iv-" + alg, 12)
        recs = []
        for seq, L in enumerate(BATCH_LENGTHS):
            pt = detbytes("batch-pt-%s-%d" % (alg, seq), L)
            sealed = ref_new(alg, key).seal(tls13_nonce(iv, seq), pt, tls13_aad(L))
            recs.append({"seq": seq, "len": L, "tag": sealed[-16:].hex(),
                         "ct_sha256": sha256hex(sealed[:-16])})
        out["batches"].append({"alg": alg, "key": key.hex(), "iv": iv.hex(), "records": recs})
    # BASELINE configs[0]: 4096 x 1 KiB ChaCha20-Poly1305 (digest only).
    key, iv, pts = config1_inputs()
    c = python_chacha20_poly1305.new(key)
    h = hashlib.sha256()
    t0 = time.time()
    for seq, pt in enumerate(pts):
        sealed = c.seal(tls13_nonce(iv, seq), pt, tls13_aad(len(pt)))
        h.update(sealed)
    out["config1"] = {"n": len(pts), "len": 1024, "sealed_sha256": h.hexdigest(),
                      "ref_seal_seconds_1core": round(time.time() - t0, 2)}
    return out


def timing():
    """Per-core speed of the reference vs oracle/pyaead on one 16 KiB record."""
    sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
    import pyaead
    res = {}
    for alg, klen in (("aes128gcm", 16), ("chacha20-poly1305", 32)):
        key, nonce, aad, pt = vec_inputs(alg, klen, 16384, 5)
        ref = ref_new(alg, key)
        mine = pyaead.CHACHA20_POLY1305(key) if alg.startswith("chacha") else pyaead.AESGCM(key)
        for name, obj in (("reference", ref), ("pyaead", mine)):
            t0 = time.perf_counter()
            for _ in range(3):
                s = obj.seal(nonce, pt, aad)
            res["%s/%s" % (alg, name)] = (time.perf_counter() - t0) / 3
            assert s == ref.seal(nonce, pt, aad)
    print(json.dumps(res, indent=1))
    return res


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    if "--timing" in sys.argv:
        timing()
        sys.exit(0)
    dump("kat.json", make_kat())
    dump("aead_vectors.json", make_vectors())
    dump("negative.json", make_negative())
    dump("record_batch.json", make_batches())
    print("fixtures written to", HERE)
