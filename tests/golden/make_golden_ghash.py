"""Generate tests/golden/ghash.json from the REFERENCE itself (build container
only; see make_golden.py and SURVEY.md section 8c).

  ghash           GHASH_H(aad, ct) computed by the reference's own
                  AESGCM._auth (tlslite/utils/aesgcm.py:60-99) with a zero tag
                  mask, for edge-case H values (0, the GCM unit element, x^127,
                  all ones, E_K(0) of the reference unit tests' keys, random)
                  and AAD / ciphertext lengths around every block and table
                  boundary.  H is installed by handing AESGCM a raw "cipher"
                  that returns H for the all-zero block (aesgcm.py:45).
  poly1305_extra  Poly1305 tags from the reference (poly1305.py:32-48) for
                  keys with r and s at their clamped maxima and long all-0xff
                  messages (the accumulator stays near 2^130 - 5 for many
                  blocks), plus random keys at AEAD-sized lengths.
Inputs are vectors.detbytes(label, n): the fixture stores labels and lengths.

    python tests/golden/make_golden_ghash.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refloader  # noqa: E402
from vectors import detbytes  # noqa: E402

refloader.load()
from tlslite.utils.aesgcm import AESGCM  # noqa: E402
from tlslite.utils.poly1305 import Poly1305  # noqa: E402
from tlslite.utils.rijndael import Rijndael  # noqa: E402

H_VALUES = [
    ("zero", bytes(16)),
    ("one", bytes([0x80]) + bytes(15)),          # x^0 in GCM bit order
    ("x127", bytes(15) + bytes([0x01])),
    ("ones", bytes([0xff]) * 16),
    ("aes128-zero-key", None),                     # test_tlslite_utils_aesgcm.py cases 1-4
    ("aes256-zero-key", None),                     # cases 13-14
    ("aes128-kat-key", None),                      # feffe9928665731c6d6a8f9467308308
] + [("rand%d" % i, None) for i in range(5)]

SHAPES = [(0, 0), (0, 16), (16, 0), (0, 1), (13, 1), (5, 15), (20, 60), (17, 33), (5, 64),
          (0, 127), (13, 256), (5, 1024), (0, 1039), (5, 4096), (13, 16383), (5, 16384),
          (5, 16385), (20, 16400), (300, 500), (0, 65535)]


def h_for(label, h):
    if h is not None:
        return bytearray(h)
    if label == "aes128-zero-key":
        return bytearray(Rijndael(bytearray(16), 16).encrypt(bytearray(16)))
    if label == "aes256-zero-key":
        return bytearray(Rijndael(bytearray(32), 16).encrypt(bytearray(16)))
    if label == "aes128-kat-key":
        key = bytearray.fromhex("feffe9928665731c6d6a8f9467308308")
        return bytearray(Rijndael(key, 16).encrypt(bytearray(16)))
    return detbytes("ghash-h-" + label, 16)


def main():
    out = {"ghash": [], "poly1305_extra": []}
    for label, h in H_VALUES:
        hb = h_for(label, h)
        obj = AESGCM(bytearray(16), "python", lambda block, hb=hb: bytearray(hb))
        for alen, clen in SHAPES:
            if label.startswith("rand") and clen > 16400:
                continue
            aad = detbytes("ghash-aad-%d" % alen, alen)
            ct = detbytes("ghash-ct-%d" % clen, clen)
            g = obj._auth(ct, aad, bytearray(16))
            out["ghash"].append({"h_label": label, "h": hb.hex(), "aad_len": alen, "ct_len": clen,
                                 "ghash": bytes(g).hex()})
    # Poly1305: r = 0x0ffffffc0ffffffc0ffffffc0fffffff (clamped max), s = 2^128 - 1
    maxkey = bytearray([0xff] * 32)
    for n in (16, 17, 32, 64, 255, 256, 1024, 4096, 16400, 16417):
        msg = bytearray([0xff] * n)
        tag = Poly1305(maxkey).create_tag(msg)
        out["poly1305_extra"].append({"key": maxkey.hex(), "msg_label": "ff", "len": n,
                                      "tag": bytes(tag).hex()})
    for i, n in enumerate((0, 1, 15, 16, 31, 63, 64, 65, 1000, 1040, 4097, 16400, 16417)):
        key = detbytes("poly-key-%d" % i, 32)
        msg = detbytes("poly-msg-%d" % n, n)
        tag = Poly1305(key).create_tag(msg)
        out["poly1305_extra"].append({"key": key.hex(), "msg_label": "poly-msg-%d" % n, "len": n,
                                      "tag": bytes(tag).hex()})
    with open(os.path.join(HERE, "ghash.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote ghash.json: %d GHASH, %d Poly1305 vectors" % (len(out["ghash"]),
                                                               len(out["poly1305_extra"])))


if __name__ == "__main__":
    main()
