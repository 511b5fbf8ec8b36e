"""Pin the key-setup oracle (oracle/keysetup.py) to the reference
(tests/golden/keys.json: RFC 8448 values of unit_tests/test_tls1_3_vectors.py
and reference RecordLayer / cryptomath outputs)."""
from vectors import load
from oracle import keysetup as K

KEYS = load("keys.json")
H = bytes.fromhex


def test_rfc8448():
    for v in KEYS["rfc8448"]:
        got = K.hkdf_expand_label(H(v["secret"]), v["label"].encode(), b"", v["length"], v["hash"])
        assert got.hex() == v["out"], v["line"]


def test_suites_match_reference_recordlayer():
    for v in KEYS["suites"]:
        alg = K.SUITES[v["suite"]][0]
        assert v["alg"] == ("chacha20-poly1305" if alg.startswith("chacha") else
                            alg.replace("aes", "aes%d" % (8 * K.SUITES[v["suite"]][1])))
        ck, civ = K.traffic_keys(v["suite"], H(v["client_secret"]))
        sk, siv = K.traffic_keys(v["suite"], H(v["server_secret"]))
        assert (ck.hex(), civ.hex(), sk.hex(), siv.hex()) == \
            (v["client_key"], v["client_iv"], v["server_key"], v["server_iv"]), v["name"]
        new = K.key_update(v["suite"], H(v["client_secret"]))
        assert new.hex() == v["update_secret"]
        uk, uiv = K.traffic_keys(v["suite"], new)
        assert (uk.hex(), uiv.hex()) == (v["update_key"], v["update_iv"])


def test_grid():
    for v in KEYS["grid"]:
        for s, o in zip(v["secrets"], v["outs"]):
            assert K.hkdf_expand_label(H(s), v["label"].encode(), H(v["ctx"]), v["length"],
                                       v["hash"]).hex() == o
