"""The device Poly1305 and GHASH arithmetic against the reference's own known
answers: RFC 7539 2.5.2 and A.3 #1-11
(unit_tests/test_tlslite_utils_poly1305.py:52-210, tests/golden/kat.json) and
reference-computed edge cases (tests/golden/ghash.json, make_golden_ghash.py:
r and s at their clamped maxima over long all-0xff messages; GHASH for H = 0,
1, x^127, all ones, the unit tests' E_K(0) and random H over lengths around
every block and table boundary), through every device code path the AEAD
kernels use (tlsgpu.selftest.POLY_MODES / GHASH_MODES)."""
import pytest

from vectors import detbytes, load

pytestmark = pytest.mark.gpu

KAT = load("kat.json")["poly1305"]
GOLD = load("ghash.json")


@pytest.fixture(scope="module")
def st():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tlsgpu import selftest
    return selftest


def _extra_msgs():
    keys, msgs, tags = [], [], []
    for v in GOLD["poly1305_extra"]:
        keys.append(bytes.fromhex(v["key"]))
        msgs.append(b"\xff" * v["len"] if v["msg_label"] == "ff" else bytes(detbytes(v["msg_label"], v["len"])))
        tags.append(bytes.fromhex(v["tag"]))
    return keys, msgs, tags


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_poly1305_rfc7539_kats(st, mode):
    keys = [bytes.fromhex(v["key"]) for v in KAT]
    msgs = [bytes.fromhex(v["msg"]) for v in KAT]
    got = st.poly1305(mode, keys, msgs)
    for i, v in enumerate(KAT):
        assert got[i].hex() == v["tag"], (st.POLY_MODES[mode], i)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_poly1305_reduction_edges(st, mode):
    keys, msgs, tags = _extra_msgs()
    got = st.poly1305(mode, keys, msgs)
    for i in range(len(msgs)):
        assert got[i] == tags[i], (st.POLY_MODES[mode], i, len(msgs[i]))


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5, 6])
def test_ghash_reference_values(st, mode):
    vecs = GOLD["ghash"]
    hs = [bytes.fromhex(v["h"]) for v in vecs]
    aads = [bytes(detbytes("ghash-aad-%d" % v["aad_len"], v["aad_len"])) for v in vecs]
    cts = [bytes(detbytes("ghash-ct-%d" % v["ct_len"], v["ct_len"])) for v in vecs]
    got = st.ghash(mode, hs, aads, cts)
    for i, v in enumerate(vecs):
        assert got[i].hex() == v["ghash"], (st.GHASH_MODES[mode], v["h_label"], v["aad_len"], v["ct_len"])


def test_poly1305_octet_striping_every_shape(st):
    """The octet striping (mode 4: r within a 64-byte chunk, r^29 across the
    other lanes' chunks, the lift r^(4 (d - 1) + mlast), the octet sum) on
    every message length 0 .. 1200 and a spread of longer ones (all chunk
    counts mod 8, every last-chunk fill), against the lane Horner (mode 0),
    which the RFC 7539 vectors above pin."""
    import random
    rng = random.Random(4)
    lens = list(range(0, 1201)) + [rng.randint(1201, 70000) for _ in range(200)]
    keys = [bytes(detbytes("oct-key-%d" % i, 32)) for i in range(len(lens))]
    keys[:4] = [b"\xff" * 32] * 4     # clamped-maximum r, s
    msgs = [bytes(detbytes("oct-msg-%d" % i, n)) for i, n in enumerate(lens)]
    msgs[:4] = [b"\xff" * n for n in lens[:4]]
    a = st.poly1305(4, keys, msgs)
    b = st.poly1305(0, keys, msgs)
    bad = [i for i in range(len(lens)) if a[i] != b[i]]
    assert not bad, [(i, lens[i]) for i in bad[:8]]
