"""GPU: bulk TLS 1.3 key setup -- tg_hkdf_expand_label
and tg_key_create_device against the reference's values (tests/golden/
keys.json) and the oracle, bit-exact; key tables built on the device must
seal exactly like tables built on the host."""
import numpy as np
import pytest

from vectors import load, tls13_aad

pytestmark = pytest.mark.gpu

KEYS = load("keys.json")
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


def _dev(torch, rows):
    a = np.frombuffer(b"".join(bytes(r) for r in rows), np.uint8).reshape(len(rows), -1)
    return torch.from_numpy(a.copy()).cuda()


def test_rfc8448(torch, tg):
    for v in KEYS["rfc8448"]:
        out = tg.keysetup.hkdf_expand_label(_dev(torch, [H(v["secret"])]), v["label"].encode(),
                                            b"", v["length"], 32)
        assert out.cpu().numpy().tobytes().hex() == v["out"], v["line"]


def test_grid(torch, tg):
    for v in KEYS["grid"]:
        hl = 32 if v["hash"] == "sha256" else 48
        out = tg.keysetup.hkdf_expand_label(_dev(torch, [H(s) for s in v["secrets"]]),
                                            v["label"].encode(), H(v["ctx"]), v["length"], hl)
        got = out.cpu().numpy()
        for row, o in zip(got, v["outs"]):
            assert row.tobytes().hex() == o, (v["hash"], v["label"], v["length"])


def test_suites_match_reference_recordlayer(torch, tg):
    for v in KEYS["suites"]:
        secrets = _dev(torch, [H(v["client_secret"]), H(v["server_secret"])])
        table, keys, ivs = tg.keysetup.traffic_keys(v["suite"], secrets)
        k, iv = keys.cpu().numpy(), ivs.cpu().numpy()
        assert (k[0].tobytes().hex(), iv[0].tobytes().hex()) == (v["client_key"], v["client_iv"])
        assert (k[1].tobytes().hex(), iv[1].tobytes().hex()) == (v["server_key"], v["server_iv"])
        new = tg.keysetup.key_update(v["suite"], secrets[:1].contiguous())
        assert new.cpu().numpy().tobytes().hex() == v["update_secret"], v["name"]
        _, uk, uiv = tg.keysetup.traffic_keys(v["suite"], new)
        assert uk.cpu().numpy().tobytes().hex() == v["update_key"]
        assert uiv.cpu().numpy().tobytes().hex() == v["update_iv"]
        assert table.nkeys == 2


@pytest.mark.parametrize("alg,klen", [("aesgcm", 16), ("aesgcm", 32), ("aesccm", 16),
                                      ("aesccm_8", 32), ("chacha20-poly1305", 32)])
@pytest.mark.parametrize("nkeys", [1, 300])
def test_device_table_seals_like_host_table(torch, tg, alg, klen, nkeys):
    """tg_key_create_device (schedule, H, GHASH tables on the GPU) vs
    tg_key_create (host) on one ragged batch: identical ciphertext and tags."""
    from batchpack import HostBatch
    rng = np.random.default_rng(nkeys + klen)
    keys = [rng.bytes(klen) for _ in range(nkeys)]
    tl = 8 if alg == "aesccm_8" else 16
    lens = [0, 1, 15, 16, 17, 1000, 16384] + list(rng.integers(0, 5000, 200))
    hb = HostBatch(lens, payload_seed=3, align=16, aad_mode="tls12", key_count=nkeys, tag=tl)
    host_t = tg.KeyTable(alg, keys)
    dev_t = tg.KeyTable.from_device(alg, _dev(torch, keys), nkeys, klen)
    outs = []
    for t in (host_t, dev_t):
        d = hb.to_device(torch)
        tg.seal_batch(t, hb.batch_kwargs(d))
        torch.cuda.synchronize()
        outs.append(d["out"].cpu().numpy())
    assert np.array_equal(outs[0], outs[1])


def test_many_sessions_end_to_end(torch, tg, oracle_mod):
    """65 536 TLS 1.3 AES-128-GCM sessions: secrets -> keys/IVs -> device key
    table -> one record per session sealed.  Every session's key and IV
    against the host key schedule (oracle/keysetup.py, pinned to keys.json),
    and every record against the C oracle (tests/fullcheck.py)."""
    import fullcheck
    from oracle import keysetup as K
    n, L = 1 << 16, 1024
    g = torch.Generator(device="cuda").manual_seed(0x7716)
    secrets = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    table, keys, ivs = tg.keysetup.traffic_keys(0x1301, secrets)
    pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    # record seq 0 of every session: nonce = iv (xor 0)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    out = torch.zeros(n * (L + 16), dtype=torch.uint8, device="cuda")
    kidx = torch.arange(n, dtype=torch.int32, device="cuda")
    tg.seal_batch(table, tg.make_batch(n, pt, out, ivs, aad=aad, fixed_len=L, in_stride=L,
                                       out_stride=L + 16, fixed_aad_len=5, key_idx=kidx))
    torch.cuda.synchronize()
    s_h, k_h, iv_h = secrets.cpu().numpy(), keys.cpu().numpy(), ivs.cpu().numpy()
    host = [K.traffic_keys(0x1301, s_h[i].tobytes()) for i in range(n)]
    hk = np.frombuffer(b"".join(k for k, _ in host), np.uint8).reshape(n, 16)
    hiv = np.frombuffer(b"".join(v for _, v in host), np.uint8).reshape(n, 12)
    assert np.array_equal(k_h, hk) and np.array_equal(iv_h, hiv)
    recs, nbytes = fullcheck.check_all(torch, oracle_mod, "aesgcm", hk, pt, np.arange(n) * L, np.full(n, L),
                                       out, np.arange(n) * (L + 16), hiv,
                                       np.frombuffer(bytes(tls13_aad(L)), np.uint8), np.zeros(n),
                                       np.full(n, 5), key_idx=np.arange(n, dtype=np.uint32))
    assert recs == n and nbytes == n * (L + 16)


def test_argument_errors(torch, tg):
    s = _dev(torch, [bytes(32)])
    with pytest.raises(tg.TlsGpuError):
        tg.keysetup.hkdf_expand_label(s, b"key", b"", 33, 32)      # > hash length
    with pytest.raises(tg.TlsGpuError):
        tg.keysetup.hkdf_expand_label(s, b"key", b"", 16, 40)      # no such hash
    with pytest.raises(tg.TlsGpuError):                             # AES key of 24 bytes
        tg.KeyTable.from_device("aesgcm", _dev(torch, [bytes(24)]), 1, 24)
