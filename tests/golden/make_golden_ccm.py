"""Generate tests/golden/ccm.json from the REFERENCE's AESCCM (build container only).

SURVEY.md section 8(f) row 2: AES-CCM / CCM_8 (tlslite/utils/aesccm.py:11-155,
python_aesccm.py, cipherfactory.createAESCCM/createAESCCM_8 :102-142).

    python tests/golden/make_golden_ccm.py

Contents:
  kat        known answers held by unit_tests/test_tlslite_utils_aesccm.py
             (inputs + expected outputs, re-checked against the reference);
  vectors    seal over LENGTHS x AAD_LENGTHS x {aes128ccm, aes256ccm,
             aes128ccm_8, aes256ccm_8}, inputs from vectors.detbytes,
             outputs from the reference;
  negative   tampered records the reference's open rejects (None);
  batch      TLS 1.3 framed batches (nonce = iv xor seq, 5-byte header AAD).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refloader  # noqa: E402
from vectors import AAD_LENGTHS, FULL_HEX_MAX, LENGTHS, detbytes, sha256hex, tls13_nonce  # noqa: E402

refloader.load()
from tlslite.utils import cipherfactory, python_aesccm  # noqa: E402

CCM_ALGS = [("aes128ccm", 16, 16), ("aes256ccm", 32, 16), ("aes128ccm_8", 16, 8),
            ("aes256ccm_8", 32, 8)]

# unit_tests/test_tlslite_utils_aesccm.py: (line, key, taglen, nonce, pt, aad, expected)
KAT = [
    (70, b"\x01" * 16, 16, b"\x02" * 12, b"text to encrypt.", b"",
     b"%}Q.\x99\xa3\r\xae\xcbMc\xf2\x16,^\xff\xa0I\x8e\xf9\xc9F>\xbf\xa4\x00Y\x02p"
     b"\xe3\xb8\xa2"),
    (85, b"\x01" * 32, 16, b"\x02" * 12, b"text to encrypt.", b"",
     b"IN\x1c\x06\xb8\x0b9SD<\xf8RL\xb4,=\xd6&d\xae^1\xf8\xbf\xfa8D\x98\xdd\x14\xb51"),
    (100, b"\x01" * 16, 8, b"\x02" * 12, b"text to encrypt.", b"",
     b"%}Q.\x99\xa3\r\xae\xcbMc\xf2\x16,^\xff\x14\xb8-?\x7f\xac\x8bI"),
    (114, b"\x01" * 32, 8, b"\x02" * 12, b"text to encrypt.", b"",
     b"IN\x1c\x06\xb8\x0b9SD<\xf8RL\xb4,=\xa2\x91\x84j1*\x0f\xeb"),
    (246, b"\x00" * 16, 16, b"\x00" * 12, b"", b"",
     b"\xb9\xf6P\xfb<9\xbb\x1b\xee\x0e)\x1d3\xf6\xae("),
    (259, b"\x00" * 16, 16, b"\x00" * 12, b"\x00" * 16, b"",
     b"n\xc7_\xb2\xe2\xb4\x87F\x1e\xdd\xcb\xb8\x97\x11\x92\xbaMO\xa3\xaf\x0b\xf6\xd3E"
     b"Aq0o\xfa\xdd\x9a\xfd"),
    (274, bytes.fromhex("feffe9928665731c6d6a8f9467308308"), 16,
     bytes.fromhex("cafebabefacedbaddecaf888"),
     bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
                   "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255"), b"",
     b"\x08\x93\xe9K\x91H\x80\x1a\xf0\xf74&\xab\xb0\x0e<\xa4\x9b\xf0\x9dy\xa2\x01'\xa7"
     b"\xeb\x19&\xfa\x89\x057\x87\xff\x02\xd0}q\x81;\x88[\x85\xe7\xf9lN\xed\xf4 \xdb"
     b"\x12j\x04Q\xce\x13\xbdA\xba\x01\x8d\x1b\xa7\xfc\xece\x99Dg\xa7{\x8b&B\xde\x91,"
     b"\x01."),
    (302, bytes.fromhex("feffe9928665731c6d6a8f9467308308"), 16,
     bytes.fromhex("cafebabefacedbaddecaf888"),
     bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
                   "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39"),
     bytes.fromhex("feedfacedeadbeeffeedfacedeadbeefabaddad2"),
     b"\x08\x93\xe9K\x91H\x80\x1a\xf0\xf74&\xab\xb0\x0e<\xa4\x9b\xf0\x9dy\xa2\x01'\xa7"
     b"\xeb\x19&\xfa\x89\x057\x87\xff\x02\xd0}q\x81;\x88[\x85\xe7\xf9lN\xed\xf4 \xdb"
     b"\x12j\x04Q\xce\x13\xbdA\xba\x028\xc3&\xb4{4\xf7\x8fe\x9eu\x10\x96\xcd\""),
    (333, b"\x00" * 32, 16, b"\x00" * 12, b"", b"",
     b"\xa8\x90&^C\xa2hU\xf2i\xb9?\xf4\xdd\xde\xf6"),
    (347, b"\x00" * 32, 16, b"\x00" * 12, b"\x00" * 16, b"",
     b"\xc1\x94@D\xc8\xe7\xaa\x95\xd2\xde\x95\x13\xc7\xf3\xdd\x8cK\n>^Q\xf1Q\xeb\x0f"
     b"\xfa\xe7\xc4=\x01\x0f\xdb"),
]


def ref(key, taglen):
    return python_aesccm.new(bytearray(key), taglen)


def make_kat():
    out = []
    for line, key, taglen, nonce, pt, aad, expect in KAT:
        c = ref(key, taglen)
        got = c.seal(bytearray(nonce), bytearray(pt), bytearray(aad))
        assert bytes(got) == expect, line
        assert c.open(bytearray(nonce), got, bytearray(aad)) == bytearray(pt)
        out.append({"line": line, "name": c.name, "key": key.hex(), "taglen": taglen,
                    "nonce": nonce.hex(), "pt": pt.hex(), "aad": aad.hex(),
                    "ct_tag": expect.hex()})
    # the factory surface (cipherfactory.py:102-142) names the objects
    for key, fn, name in ((b"\x01" * 16, cipherfactory.createAESCCM, "aes128ccm"),
                          (b"\x01" * 32, cipherfactory.createAESCCM_8, "aes256ccm_8")):
        assert fn(bytearray(key), ["python"]).name == name
    return out


def vec_inputs(alg, klen, L, A):
    tag = "%s-%d-%d" % (alg, L, A)
    return (detbytes("key-" + tag, klen), detbytes("nonce-" + tag, 12),
            detbytes("aad-" + tag, A), detbytes("pt-" + tag, L))


def make_vectors():
    vecs = []
    for alg, klen, taglen in CCM_ALGS:
        for L in LENGTHS:
            for A in AAD_LENGTHS:
                key, nonce, aad, pt = vec_inputs(alg, klen, L, A)
                c = ref(key, taglen)
                assert c.name == alg
                sealed = c.seal(nonce, pt, aad)
                assert c.open(nonce, sealed, aad) == pt
                v = {"alg": alg, "keylen": klen, "taglen": taglen, "len": L, "aadlen": A,
                     "tag": sealed[-taglen:].hex(), "ct_sha256": sha256hex(sealed[:-taglen])}
                if L <= FULL_HEX_MAX:
                    v["ct_tag"] = sealed.hex()
                vecs.append(v)
    # long AAD: the 0xfffe || be32 length form (aesccm.py:52-55)
    for alg, klen, taglen in CCM_ALGS[:1]:
        key, nonce, aad, pt = vec_inputs(alg, klen, 100, 0xff00)
        c = ref(key, taglen)
        sealed = c.seal(nonce, pt, aad)
        vecs.append({"alg": alg, "keylen": klen, "taglen": taglen, "len": 100,
                     "aadlen": 0xff00, "tag": sealed[-taglen:].hex(),
                     "ct_sha256": sha256hex(sealed[:-taglen]), "ct_tag": sealed.hex()})
    return vecs


def make_negative():
    neg = []
    for alg, klen, taglen in CCM_ALGS:
        for L in (0, 1, 16, 17, 1024):
            key, nonce, aad, pt = vec_inputs(alg, klen, L, 13)
            c = ref(key, taglen)
            sealed = c.seal(nonce, pt, aad)
            cases = [("tag_bit", nonce, sealed[:-1] + bytearray([sealed[-1] ^ 1]), aad),
                     ("aad_bit", nonce, sealed, bytearray([aad[0] ^ 0x80]) + aad[1:]),
                     ("nonce_bit", bytearray([nonce[0] ^ 1]) + nonce[1:], sealed, aad),
                     ("short", nonce, sealed[:taglen - 1], aad)]
            if L:
                cases.append(("ct_bit", nonce, bytearray([sealed[0] ^ 4]) + sealed[1:], aad))
            for name, n2, ct2, aad2 in cases:
                assert c.open(n2, ct2, aad2) is None, (alg, L, name)
                neg.append({"alg": alg, "taglen": taglen, "key": key.hex(), "case": name,
                            "nonce": n2.hex(), "ct_tag": ct2.hex(), "aad": aad2.hex()})
    return neg


BATCH_LENGTHS = [16384, 0, 1, 16385, 1024, 5, 16, 4096, 100, 63, 64, 65, 2000, 16383, 31]


def make_batches():
    out = []
    for alg, klen, taglen in CCM_ALGS:
        key = detbytes("ccm-batch-key-" + alg, klen)
        iv = detbytes("ccm-batch-iv-" + alg, 12)
        recs = []
        for seq, L in enumerate(BATCH_LENGTHS):
            pt = detbytes("ccm-batch-pt-%s-%d" % (alg, seq), L)
            n = L + taglen
            aad = bytearray([0x17, 3, 3, n >> 8, n & 0xff])
            sealed = ref(key, taglen).seal(tls13_nonce(iv, seq), pt, aad)
            recs.append({"seq": seq, "len": L, "tag": sealed[-taglen:].hex(),
                         "ct_sha256": sha256hex(sealed[:-taglen])})
        out.append({"alg": alg, "taglen": taglen, "key": key.hex(), "iv": iv.hex(),
                    "records": recs})
    return out


if __name__ == "__main__":
    obj = {"kat": make_kat(), "vectors": make_vectors(), "negative": make_negative(),
           "batch": make_batches()}
    with open(os.path.join(HERE, "ccm.json"), "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")
    print("wrote", os.path.join(HERE, "ccm.json"))
