"""TLS 1.3 key-setup fixtures from the REFERENCE (build container only).

SURVEY.md section 8(f) row 4.  Writes tests/golden/keys.json:
  rfc8448  the HKDF-Expand-Label values unit_tests/test_tls1_3_vectors.py
           asserts (RFC 8448 simple 1-RTT handshake), re-checked against the
           reference's cryptomath.HKDF_expand_label;
  suites   calcTLS1_3PendingState (recordlayer.py:1268-1323) of every TLS 1.3
           suite on deterministic secrets: the client/server key and fixed IV
           the reference RecordLayer installs, and _calcTLS1_3KeyUpdate's
           next secret / key / IV;
  grid     HKDF_expand_label outputs over labels x contexts x lengths x
           {sha256, sha384} on deterministic secrets.

    python tests/golden/make_golden_keys.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import refloader  # noqa: E402
from vectors import detbytes  # noqa: E402

refloader.load()
from tlslite.constants import CipherSuite  # noqa: E402
from tlslite.recordlayer import RecordLayer  # noqa: E402
from tlslite.utils.cryptomath import HKDF_expand_label  # noqa: E402
from mocksock import MockSocket  # noqa: E402  (reference unit_tests/mocksock.py)

H = bytes.fromhex

# unit_tests/test_tls1_3_vectors.py (line, secret name, secret, label, length, expected)
RFC8448 = [
    (300, "s_hs_traffic", "b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38",
     b"key", 16, "3fce516009c21727d0f2e4e86ee403bc"),
    (309, "s_hs_traffic", "b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38",
     b"iv", 12, "5d313eb2671276ee13000b30"),
    (318, "s_hs_traffic", "b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38",
     b"finished", 32, "008d3b66f816ea559f96b537e885c31fc068bf492c652f01f288a1d8cdc19fc8"),
    (374, "s_ap_traffic", "a11af9f05531f856ad47116b45a950328204b4f44bfb6b3a4b4f1f3fcb631643",
     b"key", 16, "9f02283b6c9c07efc26bb9f2ac92e356"),
    (383, "s_ap_traffic", "a11af9f05531f856ad47116b45a950328204b4f44bfb6b3a4b4f1f3fcb631643",
     b"iv", 12, "cf782b88dd83549aadf1e984"),
    (392, "c_hs_traffic", "b3eddb126e067f35a780b3abf45e2d8f3b1a950738f52e9600746a0e27a55a21",
     b"key", 16, "dbfaa693d1762c5b666af5d950258d01"),
    (401, "c_hs_traffic", "b3eddb126e067f35a780b3abf45e2d8f3b1a950738f52e9600746a0e27a55a21",
     b"iv", 12, "5bd3c71b836e0b76bb73265f"),
]

SUITES = [("TLS_AES_128_GCM_SHA256", 32), ("TLS_AES_256_GCM_SHA384", 48),
          ("TLS_CHACHA20_POLY1305_SHA256", 32), ("TLS_AES_128_CCM_SHA256", 32),
          ("TLS_AES_128_CCM_8_SHA256", 32)]


def make_rfc8448():
    out = []
    for line, name, secret, label, length, expect in RFC8448:
        got = HKDF_expand_label(bytearray(H(secret)), label, b"", length, "sha256")
        assert got.hex() == expect, line
        out.append({"line": line, "name": name, "secret": secret, "label": label.decode(),
                    "length": length, "out": expect, "hash": "sha256"})
    return out


def make_suites():
    out = []
    for name, slen in SUITES:
        suite = getattr(CipherSuite, name)
        for k in range(4):
            cts, sts = detbytes("c-secret-%s-%d" % (name, k), slen), \
                detbytes("s-secret-%s-%d" % (name, k), slen)
            rl = RecordLayer(MockSocket(bytearray(0)))
            rl.version = (3, 4)
            rl.client = True
            rl.calcTLS1_3PendingState(suite, cts, sts, None)
            w, r = rl._pendingWriteState, rl._pendingReadState
            new_secret, upd = rl._calcTLS1_3KeyUpdate(suite, cts)
            out.append({"suite": suite, "name": name, "k": k, "client_secret": cts.hex(),
                        "server_secret": sts.hex(), "alg": w.encContext.name,
                        "client_key": bytes(w.encContext.key).hex(),
                        "client_iv": bytes(w.fixedNonce).hex(),
                        "server_key": bytes(r.encContext.key).hex(),
                        "server_iv": bytes(r.fixedNonce).hex(),
                        "update_secret": bytes(new_secret).hex(),
                        "update_key": bytes(upd.encContext.key).hex(),
                        "update_iv": bytes(upd.fixedNonce).hex()})
    return out


def make_grid():
    out = []
    for prf, hl in (("sha256", 32), ("sha384", 48)):
        for label in (b"key", b"iv", b"traffic upd", b"finished", b"c ap traffic",
                      b"a-much-longer-label-for-hkdf-expand-label-tests"):
            for ctxlen in (0, hl):
                for length in sorted({1, 12, 16, 32, hl}):
                    ctx = bytes(detbytes("ctx-%s-%d" % (prf, ctxlen), ctxlen))
                    secrets = [detbytes("grid-%s-%s-%d-%d-%d" % (prf, label.decode(), ctxlen,
                                                                 length, i), hl)
                               for i in range(3)]
                    outs = [HKDF_expand_label(s, label, ctx, length, prf).hex() for s in secrets]
                    out.append({"hash": prf, "label": label.decode(), "ctx": ctx.hex(),
                                "length": length, "secrets": [s.hex() for s in secrets],
                                "outs": outs})
    return out


if __name__ == "__main__":
    obj = {"rfc8448": make_rfc8448(), "suites": make_suites(), "grid": make_grid()}
    with open(os.path.join(HERE, "keys.json"), "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")
    print("wrote keys.json")
