"""GPU parity of the bitsliced AES-GCM kernel (gcm_bs_kernel, aes_bs.h),
selected per launch with TLSGPU_GCM_VARIANT=4: ragged batches (lengths that
cut chunks of 32 blocks anywhere, 16-byte and byte alignment: the hooked and
the plain GHASH paths), tampered records, AES-128 and AES-256, and a
2^18 x 16 KiB round trip with sampled records checked against the oracle.
"""
import os

import numpy as np
import pytest

from vectors import detbytes, tls13_aad, tls13_nonce

pytestmark = pytest.mark.gpu

LEN_MIX = [0, 1, 15, 16, 17, 31, 496, 511, 512, 513, 527, 528, 1023, 1024, 1040, 4096, 8191,
           16383, 16384, 16385, 16400]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    return t


@pytest.fixture(scope="module")
def tg(torch):
    import tlsgpu
    return tlsgpu


@pytest.fixture
def bitsliced():
    old = os.environ.get("TLSGPU_GCM_VARIANT")
    os.environ["TLSGPU_GCM_VARIANT"] = "4"
    yield
    if old is None:
        del os.environ["TLSGPU_GCM_VARIANT"]
    else:
        os.environ["TLSGPU_GCM_VARIANT"] = old


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("align", [16, 1])
def test_bitsliced_ragged_vs_oracle(torch, tg, oracle_mod, bitsliced, klen, align):
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(31 * klen + align)
    lens = LEN_MIX * 4 + list(rng.integers(0, 16401, 150))
    hb = HostBatch(lens, payload_seed=align + 3, align=align, aad_mode="random")
    key = rng.bytes(klen)
    run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", np.frombuffer(key, np.uint8),
                  tg.HipAESGCM(bytearray(key)), tamper=(2, 40, 77))


def test_bitsliced_uniform_wave(torch, tg, oracle_mod, bitsliced):
    """Every lane of every wave the same long length (the fast path that
    loads a whole chunk at once), plus a final partial workgroup."""
    from batchpack import HostBatch, run_seal_open
    lens = [16384] * 1000 + [16385] * 40
    hb = HostBatch(lens, payload_seed=11, align=16, aad_mode="tls13")
    key = bytes(range(16))
    run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", np.frombuffer(key, np.uint8),
                  tg.HipAESGCM(bytearray(key)), tamper=(0, 999, 1039))


def test_bitsliced_full_size_samples(torch, tg, oracle_mod, bitsliced):
    n, L = 1 << 18, 16384
    g = torch.Generator(device="cuda").manual_seed(0x7715)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    key = bytes(detbytes("bitsliced-full", 16))
    iv = detbytes("bitsliced-iv", 12)
    obj = tg.HipAESGCM(bytearray(key))
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tg.make_nonces(iv, 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    S = 16512   # sealed stride: 128-byte aligned records, as the bench packs them
    sealed = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    tg.seal_batch(obj, tg.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                                     out_stride=S, fixed_aad_len=5))
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tg.open_batch(obj, tg.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L,
                                     in_stride=S, out_stride=L, fixed_aad_len=5, status=status))
    torch.cuda.synchronize()
    assert int(status.sum()) == n
    assert torch.equal(back, inp)
    rng = np.random.default_rng(2)
    for i in np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 30)])):
        i = int(i)
        want = oracle_mod.gcm_seal(key, bytes(tls13_nonce(iv, i)),
                                   inp[i * L:(i + 1) * L].cpu().numpy().tobytes(),
                                   bytes(tls13_aad(L)))
        assert sealed[i * S:i * S + L + 16].cpu().numpy().tobytes() == bytes(want), i
    del inp, back, sealed
    torch.cuda.empty_cache()
