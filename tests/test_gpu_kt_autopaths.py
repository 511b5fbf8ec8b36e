"""GPU: the key-table AES-GCM paths ``auto`` picks for one-length batches
(api.hip launch_gcm_table), every record against the C oracle
(tests/fullcheck.py), then opened back with tampered records
(aesgcm.py:101-154 per record, keys by key_idx as RecordLayer holds one
cipher per connection state):

* n > 2 048 records of one length with n L <= 16 MiB: one record per
  wavefront, no plan (4 096 x 2 KiB, 8 192 x 1 KiB);
* one length below the 2 048-byte split beyond 16 MiB: the lane kernel with
  no plan (32 768 x 1 KiB, 65 536 x 1 KiB);

and the planner's 64-bit sort keys (nkeys >= 2^17, planner.hip), with
out-of-range key indices, on the planned (hybrid + lane) path.
"""
import numpy as np
import pytest

from vectors import tls13_aad

pytestmark = pytest.mark.gpu


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


def _tamper_open(torch, tg, table, sealed, n, L, SL, nonces, aad, kidx, inp, bad):
    """Open every record back with the records in ``bad`` tampered (a
    ciphertext byte for even i, a tag byte for odd i): status 0 and zeroed
    plaintext for them, status 1 and the original plaintext for the rest."""
    s = sealed.clone()
    for i in bad:
        s[i * SL + (i * 37) % L if i % 2 == 0 else i * SL + L + i % 16] ^= 0x10
    back = torch.full_like(inp, 0xaa)
    status = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    tg.open_batch(table, tg.make_batch(n, s, back, nonces, aad=aad, fixed_len=L, in_stride=SL,
                                       out_stride=L, aad_stride=0, fixed_aad_len=5, key_idx=kidx,
                                       status=status))
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    want = np.ones(n, np.uint8)
    want[list(bad)] = 0
    assert np.array_equal(st, want), np.nonzero(st != want)[0][:8]
    ok = torch.ones(n, dtype=torch.bool, device="cuda")
    ok[list(bad)] = False
    bv, iv_ = back.view(n, L), inp.view(n, L)
    assert torch.equal(bv[ok], iv_[ok])
    assert not bv[~ok].any(), "rejected records must be zeroed"


@pytest.mark.parametrize("n,L", [(4096, 2048), (8192, 1024), (32768, 1024), (65536, 1024)])
@pytest.mark.parametrize("klen", [16, 32])
def test_one_length_key_table_whole_batch(torch, tg, oracle_mod, n, L, klen):
    import fullcheck
    nkeys = 977
    rng = np.random.default_rng(n + L + klen)
    keys = rng.integers(0, 256, (nkeys, klen), dtype=np.uint8)
    key_idx = rng.integers(0, nkeys, n).astype(np.uint32)
    iv = rng.bytes(12)
    SL = (L + 16 + 127) // 128 * 128
    g = torch.Generator(device="cuda").manual_seed(n + klen)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.zeros(n * SL, dtype=torch.uint8, device="cuda")
    nonces_h = fullcheck.tls13_nonces(iv, 1000, n)
    nonces = torch.from_numpy(nonces_h.reshape(-1).copy()).cuda()
    aad_h = np.frombuffer(bytes(tls13_aad(L)), np.uint8)
    aad = torch.from_numpy(aad_h.copy()).cuda()
    kidx = torch.from_numpy(key_idx.view(np.int32).copy()).cuda()
    table = tg.KeyTable("aesgcm", [bytes(k) for k in keys])
    tg.seal_batch(table, tg.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                                       out_stride=SL, aad_stride=0, fixed_aad_len=5, key_idx=kidx))
    torch.cuda.synchronize()
    recs, nbytes = fullcheck.check_all(torch, oracle_mod, "aesgcm", keys, inp, np.arange(n) * L,
                                       np.full(n, L), sealed, np.arange(n) * SL, nonces_h, aad_h,
                                       np.zeros(n), np.full(n, 5), key_idx=key_idx)
    assert recs == n and nbytes == n * (L + 16)
    bad = sorted(set([0, 1, n - 1] + list(rng.integers(0, n, 12))))
    _tamper_open(torch, tg, table, sealed, n, L, SL, nonces, aad, kidx, inp, bad)


def _planned_roundtrip(torch, tg, oracle_mod, opts, nkeys, lens, ki, out_of_range):
    """Seal a mixed-length key-table batch on the planned path, in-range
    records against the oracle, then open it back (out-of-range key indices:
    skipped, status 0, plaintext zeroed)."""
    from batchpack import HostBatch
    rng = np.random.default_rng(nkeys)
    keys = rng.integers(0, 256, (nkeys, 16), dtype=np.uint8)
    hb = HostBatch(lens, payload_seed=9, align=16, aad_mode="tls12", key_count=2)
    n = hb.n
    hb.key_idx = ki
    table = tg.KeyTable("aesgcm", [bytes(k) for k in keys])
    d = hb.to_device(torch)
    with tg.options(**opts):
        tg.seal_batch(table, hb.batch_kwargs(d))
        torch.cuda.synchronize()
        got = d["out"].cpu().numpy()
        inr = np.ones(n, bool)
        inr[out_of_range] = False
        ki_ok = np.where(inr, ki, 0).astype(np.uint32)
        hb.key_idx = ki_ok
        want, _ = hb.oracle(oracle_mod, "aesgcm", keys, "seal")
        hb.key_idx = ki
        for i in np.nonzero(inr)[0]:
            o, L = int(hb.out_off[i]), int(hb.lens[i])
            assert np.array_equal(got[o:o + L + 16], want[o:o + L + 16]), ("seal", int(i), L)
        pt = torch.full((hb.in_bytes,), 0xaa, dtype=torch.uint8, device="cuda")
        status = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        tg.open_batch(table, tg.make_batch(n, d["out"], pt, d["nonces"], aad=d["aad"], lens=d["lens"],
                                           in_off=d["out_off"], out_off=d["in_off"], aad_off=d["aad_off"],
                                           aad_len=d["aad_len"], key_idx=d["key_idx"], status=status))
        torch.cuda.synchronize()
    st, back = status.cpu().numpy(), pt.cpu().numpy()
    assert np.array_equal(st, inr.astype(np.uint8)), np.nonzero(st != inr)[0][:8]
    for i in range(n):
        o, L = int(hb.in_off[i]), int(hb.lens[i])
        if inr[i]:
            assert np.array_equal(back[o:o + L], hb.inp[o:o + L]), ("open", i)
        else:
            assert not back[o:o + L].any(), ("skipped record not zeroed", i)


@pytest.mark.parametrize("opts", [{}, {"kt_lpr": 32}, {"gcm_table_variant": 14}])
def test_planner_64bit_keys(torch, tg, oracle_mod, opts):
    """nkeys = 2^17 + 1 makes the plan sort on 64-bit keys (key | length
    packed beyond 32 bits; above the counting plan's key limit).  Per-record
    lengths around the 2 048-byte split, key indices over the whole table and
    some out of range (planned into the lane kernel's tail and skipped: open
    status 0).  In-range records against the oracle, then opened back."""
    nkeys = (1 << 17) + 1
    rng = np.random.default_rng(0x64b)
    lens = list(rng.integers(0, 5000, 5000)) + [2047, 2048, 2049, 16384, 16385, 0, 1]
    n = len(lens)
    ki = rng.integers(0, nkeys, n).astype(np.uint32)
    ki[:3] = [0, nkeys - 1, nkeys - 2]
    out_of_range = [5, 17, n - 2]
    ki[out_of_range] = [nkeys, nkeys + 12345, 0xfffffff0]
    _planned_roundtrip(torch, tg, oracle_mod, opts, nkeys, lens, ki, out_of_range)


@pytest.mark.parametrize("opts", [{}, {"kt_lpr": 32}, {"kt_lpr": 8}, {"gcm_table_variant": 14},
                                  {"kt_overlap": -1}])
def test_counting_plan_skewed_keys(torch, tg, oracle_mod, opts):
    """The counting plan (planner.hip key_job_plan_counting, up to 2^17 keys):
    records 0-299 on one key (about 265 of them long: above kBucketSortMax,
    left in scatter order), 64 and 65 records on two more keys, 40 records of
    one length on a fourth, the rest spread over 997 keys; lengths 0 .. 18 000
    around the split, and out-of-range key indices, one on a 40 000-byte
    record (the tail's length buckets clamp at 32 767).  Every in-range record
    against the oracle, then opened back."""
    nkeys = 997
    rng = np.random.default_rng(0xc0de)
    lens = list(rng.integers(0, 18000, 2600)) + [2047, 2048, 2049, 16384, 16385, 0, 1, 32766, 32767, 40000]
    lens += [4096] * 40
    n = len(lens)
    ki = rng.integers(0, nkeys, n).astype(np.uint32)
    ki[:300] = 3
    ki[300:364] = 5
    ki[364:429] = 7
    ki[n - 40:] = 11
    out_of_range = [400, 1000, 2609, n - 41]   # 2609: the 40 000-byte record
    ki[out_of_range] = [nkeys, nkeys + 5, nkeys + 1, 0xffffffff]
    _planned_roundtrip(torch, tg, oracle_mod, opts, nkeys, lens, ki, out_of_range)
