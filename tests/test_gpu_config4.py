"""BASELINE configs[3] at full shape: AES-256-GCM,
65 536 session keys (PCG64 0x7716), 2^20 records with Zipf(1.2) lengths
64 B-16 KiB (PCG64 0x7717), TLS 1.2 AAD seq||0x17||0x0303||len and nonce
iv4||seq, records in arrival order (the engine's planner sorts the launch).
Every record's ciphertext and tag bit-exact against the threaded C oracle
(aesgcm.py:101-124 restated; tests/fullcheck.py), the seal -> open round trip
over the whole batch, and 128 sampled records through the oracle's
per-record entry point."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


# auto (length split: octet or wave-per-record kernel for the long records,
# lane kernel for the rest) / lane kernel for all / octet kernel for all
# (kt_hybrid -1: the bitsliced key-grouped kernel instead of the default
# T-table + bitsliced one for the long records)
@pytest.mark.parametrize("variant,lpr,hyb", [(0, 0, 0), (0, 0, -1), (0, 64, 0), (1, 0, 0), (14, 0, 0)])
def test_config4_full_shape_sampled(oracle_mod, variant, lpr, hyb):
    import torch
    import tlsgpu
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    with tlsgpu.options(gcm_table_variant=variant, kt_lpr=lpr, kt_hybrid=hyb):
        _run_config4(torch, tlsgpu, oracle_mod)


def _run_config4(torch, tlsgpu, oracle_mod):
    n, nkeys = 1 << 20, 65536
    rk = np.random.default_rng(0x7716)
    keys = rk.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    key_idx = rk.integers(0, nkeys, n).astype(np.uint32)
    lens = np.clip(64 * np.random.default_rng(0x7717).zipf(1.2, n), 64, 16384).astype(np.int64)
    seq = np.arange(n, dtype=np.uint64)
    in_sz = (lens + 15) // 16 * 16
    out_sz = (lens + 16 + 15) // 16 * 16
    in_off = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.int64)
    out_off = np.concatenate([[0], np.cumsum(out_sz)[:-1]]).astype(np.int64)
    aad = np.zeros((n, 13), dtype=np.uint8)
    aad[:, :8] = seq[:, None].view(np.uint8).reshape(n, 8)[:, ::-1]
    aad[:, 8], aad[:, 9], aad[:, 10] = 0x17, 3, 3
    aad[:, 11], aad[:, 12] = lens >> 8, lens & 0xff
    nonce = np.zeros((n, 12), dtype=np.uint8)
    nonce[:, :4] = rk.integers(0, 256, 4, dtype=np.uint8)
    nonce[:, 4:] = aad[:, :8]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    g = torch.Generator(device="cuda").manual_seed(0x7717)
    inp = torch.randint(0, 256, (int(in_sz.sum()),), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.zeros(int(out_sz.sum()), dtype=torch.uint8, device="cuda")
    back = torch.zeros_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d_lens, d_in, d_out = d(lens.astype(np.int32)), d(in_off), d(out_off)
    d_aad, d_nonce, d_kidx = d(aad.reshape(-1)), d(nonce.reshape(-1)), d(key_idx.view(np.int32))
    table = tlsgpu.KeyTable("aesgcm", [bytes(k) for k in keys])
    tlsgpu.seal_batch(table, tlsgpu.make_batch(n, inp, sealed, d_nonce, aad=d_aad, lens=d_lens,
                                               in_off=d_in, out_off=d_out, aad_stride=13,
                                               fixed_aad_len=13, key_idx=d_kidx))
    tlsgpu.open_batch(table, tlsgpu.make_batch(n, sealed, back, d_nonce, aad=d_aad, lens=d_lens,
                                               in_off=d_out, out_off=d_in, aad_stride=13,
                                               fixed_aad_len=13, key_idx=d_kidx, status=status))
    torch.cuda.synchronize()
    assert int(status.sum()) == n
    for lo in range(0, n, 1 << 18):   # round trip, in slices (the payload gaps are padding)
        hi = min(n, lo + (1 << 18))
        a, b = int(in_off[lo]), int(in_off[hi - 1] + in_sz[hi - 1])
        m = np.zeros(b - a, dtype=bool)
        for i in range(lo, hi):
            o = int(in_off[i]) - a
            m[o:o + int(lens[i])] = True
        mt = torch.from_numpy(m).cuda()
        assert torch.equal(back[a:b][mt], inp[a:b][mt])
    import fullcheck
    recs, nbytes = fullcheck.check_all(torch, oracle_mod, "aesgcm", keys, inp, in_off, lens, sealed,
                                       out_off, nonce, aad.reshape(-1), np.arange(n) * 13,
                                       np.full(n, 13), key_idx=key_idx)
    assert recs == n and nbytes == int(lens.sum()) + 16 * n
    pick = np.unique(np.concatenate([[0, n - 1, int(np.argmax(lens))],
                                     np.random.default_rng(4).integers(0, n, 125)]))
    for i in pick:
        i = int(i)
        L = int(lens[i])
        pt = inp[int(in_off[i]):int(in_off[i]) + L].cpu().numpy().tobytes()
        want = oracle_mod.gcm_seal(bytes(keys[key_idx[i]]), nonce[i].tobytes(), pt, aad[i].tobytes())
        got = sealed[int(out_off[i]):int(out_off[i]) + L + 16].cpu().numpy().tobytes()
        assert got == bytes(want), (i, L)
