"""The whole-batch checker (tests/fullcheck.py) on the CPU: a batch sealed by
the oracle itself passes, nonces match the per-record restatement, and a
single flipped ciphertext or tag byte anywhere is reported with its record."""
import numpy as np
import pytest

import fullcheck
from vectors import detbytes, tls13_aad, tls13_nonce


def test_tls13_nonces_vectorised():
    iv = bytes(detbytes("fc-iv", 12))
    got = fullcheck.tls13_nonces(iv, 2 ** 40 - 3, 7)
    want = [bytes(tls13_nonce(iv, 2 ** 40 - 3 + i)) for i in range(7)]
    assert [r.tobytes() for r in got] == want


@pytest.mark.parametrize("alg,klen,stride", [("aesgcm", 16, 1000), ("chacha", 32, 1040),
                                             ("aesgcm", 32, None)])
def test_check_all_detects_flips(oracle_mod, alg, klen, stride):
    import torch
    rng = np.random.default_rng(klen)
    n = 300
    if stride is None:   # ragged, packed back to back
        lens = rng.integers(0, 3000, n)
        in_off = np.concatenate([[0], np.cumsum(lens)[:-1]])
        out_off = np.concatenate([[0], np.cumsum(lens + 16)[:-1]])
    else:
        lens = np.full(n, 984 if stride == 1000 else 1024)
        in_off = np.arange(n) * int(lens[0])
        out_off = np.arange(n) * stride
    key = rng.integers(0, 256, klen, dtype=np.uint8)
    iv = rng.bytes(12)
    inp = rng.integers(0, 256, int(in_off[-1] + lens[-1]) + 16, dtype=np.uint8)
    nonces = fullcheck.tls13_nonces(iv, 5, n)
    aad = np.frombuffer(b"".join(bytes(tls13_aad(int(L))) for L in lens), np.uint8).copy()
    aad_off, aad_len = np.arange(n) * 5, np.full(n, 5)
    out, _ = oracle_mod.batch(alg, "seal", key, nonces, aad, aad_off, aad_len, inp, in_off, lens,
                              int(out_off[-1] + lens[-1]) + 16, out_off, nthreads=4)
    d_in, d_out = torch.from_numpy(inp), torch.from_numpy(out.copy())
    args = (torch, oracle_mod, alg, key, d_in, in_off, lens, d_out, out_off, nonces, aad,
            aad_off, aad_len)
    assert fullcheck.check_all(*args, chunk=64, nthreads=4)[0] == n
    for i, where in ((0, 0), (n - 1, -1), (137, 3)):
        o = int(out_off[i]) + (where if where >= 0 else int(lens[i]) + 16 + where)
        d_out[o] ^= 1
        with pytest.raises(fullcheck.Mismatch, match=r"first \[%d\]" % i):
            fullcheck.check_all(*args, chunk=64, nthreads=4)
        d_out[o] ^= 1


def test_check_all_inner_type(oracle_mod):
    """Config 5's form: the device sealed fragment || 0x17 behind a header."""
    import torch
    rng = np.random.default_rng(3)
    n, L, DS, WS = 200, 100, 128, 256
    key, iv = rng.integers(0, 256, 16, dtype=np.uint8), rng.bytes(12)
    data = rng.integers(0, 256, n * DS, dtype=np.uint8)
    nonces = fullcheck.tls13_nonces(iv, 2 ** 40, n)
    hdr = np.frombuffer(bytes([0x17, 3, 3, 0, L + 17]), np.uint8)
    wire = np.zeros(n * WS, dtype=np.uint8)
    for i in range(n):
        inner = data[i * DS:i * DS + L].tobytes() + b"\x17"
        w = oracle_mod.gcm_seal(key.tobytes(), nonces[i].tobytes(), inner, hdr.tobytes())
        wire[i * WS + 5:i * WS + 5 + len(w)] = np.frombuffer(bytes(w), np.uint8)
    args = (torch, oracle_mod, "aesgcm", key, torch.from_numpy(data), np.arange(n) * DS,
            np.full(n, L), torch.from_numpy(wire), np.arange(n) * WS + 5, nonces, hdr,
            np.zeros(n), np.full(n, 5))
    assert fullcheck.check_all(*args, chunk=64, nthreads=2, inner_type=0x17)[0] == n
    with pytest.raises(fullcheck.Mismatch):
        fullcheck.check_all(*args, chunk=64, nthreads=2, inner_type=0x16)
