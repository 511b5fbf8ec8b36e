"""The per-record drop-in objects under threads: copies of one AEAD object
(copy.copy shares the device key, as recordlayer.py:262 / :913 copy the
cipher state) used from several threads at once.  ctypes releases the GIL
around every tg_seal / tg_open, so the calls really overlap; each takes its
own staging slot (api.hip take_stage), so every output must still equal the
oracle's."""
import copy
import threading

import numpy as np
import pytest

from vectors import tls13_aad

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("alg", ["aesgcm", "chacha", "aesccm"])
def test_copies_in_threads_vs_oracle(oracle_mod, alg):
    import torch
    import tlsgpu
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    rng = np.random.default_rng(17)
    key = rng.bytes(32 if alg == "chacha" else 16)
    base = {"aesgcm": tlsgpu.HipAESGCM, "chacha": tlsgpu.HipCHACHA20_POLY1305,
            "aesccm": tlsgpu.HipAESCCM}[alg](bytearray(key))
    seal = {"aesgcm": oracle_mod.gcm_seal, "chacha": oracle_mod.chacha_seal,
            "aesccm": oracle_mod.ccm_seal}[alg]
    nthreads, per = 4, 60
    jobs = [[(rng.bytes(12), rng.bytes(int(rng.integers(0, 20000)))) for _ in range(per)]
            for _ in range(nthreads)]
    results, errors = [None] * nthreads, []

    def work(t):
        try:
            obj = copy.copy(base)
            out = []
            for nonce, pt in jobs[t]:
                aad = bytes(tls13_aad(len(pt)))
                ct = obj.seal(nonce, pt, aad)
                back = obj.open(nonce, ct, aad)
                out.append((bytes(ct), back is not None and bytes(back) == pt))
            results[t] = out
        except Exception as e:   # surfaced below
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(nthreads):
        for (nonce, pt), (ct, opened) in zip(jobs[t], results[t]):
            assert ct == bytes(seal(key, nonce, pt, bytes(tls13_aad(len(pt))))), (t, len(pt))
            assert opened
