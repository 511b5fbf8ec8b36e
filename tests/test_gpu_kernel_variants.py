"""GPU parity of every kernel behind the same batch entry points: batches of
up to 2048 records run one record per wavefront, larger ones a record per
lane; each is forced here on ragged batches (lengths, alignment, AAD, tampered
records) and checked bit-exact against the oracle."""
import numpy as np
import pytest

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


LENS = [0, 1, 15, 16, 17, 63, 64, 65, 1000, 1024, 1040, 4095, 16383, 16384, 16385, 16400]


@pytest.mark.parametrize("alg,klen,opts", [
    ("aesgcm", 16, {"gcm_variant": 16}),          # T-table lane per record
    ("aesgcm", 32, {"gcm_variant": 16}),
    ("aesgcm", 16, {"gcm_variant": 6}),           # wave per record
    ("aesgcm", 32, {"gcm_variant": 6}),
    ("aesgcm", 16, {"gcm_variant": 14}),          # 8-block bitsliced, octet per record
    ("aesgcm", 32, {"gcm_variant": 14}),
    ("aesgcm", 16, {"gcm_variant": 15}),          # hybrid T-table + bitsliced (persistent)
    ("aesgcm", 32, {"gcm_variant": 15}),
    ("aesgcm", 16, {"gcm_variant": 15, "hy_threads": 768}),   # 3 waves / SIMD, payload prefetch
    ("aesgcm", 32, {"gcm_variant": 15, "hy_threads": 768}),
    ("aesgcm", 16, {"gcm_variant": 15, "hy_t": 8, "hy_prio": 1}),   # round 2's split
    ("aesgcm", 16, {"gcm_variant": 15, "hy_t": 16}),   # T-table waves only
    ("aesgcm", 32, {"gcm_variant": 15, "hy_t": -1}),   # bitsliced waves only
    ("chacha", 32, {"chacha_variant": 4}),        # lane per record, register-staged tile fill
    ("chacha", 32, {"chacha_variant": 5}),        # lane per record, LDS-DMA tile fill (auto)
    ("chacha", 32, {"chacha_variant": 3}),        # wave per record
    ("chacha", 32, {"chacha_variant": 6}),        # eight lanes per record (octets), no tile
])
@pytest.mark.parametrize("align", [16, 1])
def test_forced_kernel_vs_oracle(torch, tg, oracle_mod, alg, klen, opts, align):
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(hash((alg, klen, tuple(sorted(opts.items())), align)) & 0xffff)
    # + long records: many 256-counter windows (window-cache refreshes)
    lens = LENS * 5 + list(rng.integers(0, 16401, 120)) + [65520, 65536, 70001]
    hb = HostBatch(lens, payload_seed=align + 21, align=align, aad_mode="random")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    with tg.options(**opts):
        run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                      tamper=(1, 30, 111))


def test_unknown_variant_is_an_error(torch, tg):
    """A variant no launcher knows fails the launch instead of running auto."""
    from batchpack import HostBatch
    hb = HostBatch([100, 200], payload_seed=1)
    d = hb.to_device(torch)
    obj = tg.HipAESGCM(bytearray(16))
    with tg.options(gcm_variant=4):   # round 2's removed 32-block bitsliced kernel
        with pytest.raises(tg.TlsGpuError):
            tg.seal_batch(obj, hb.batch_kwargs(d))
    with pytest.raises(tg.TlsGpuError):
        tg.set_option("no_such_option", 1)


@pytest.mark.parametrize("alg,klen", [("aesgcm", 16), ("chacha", 32)])
def test_auto_wave_per_record_batch(torch, tg, oracle_mod, alg, klen):
    """A 2048-record batch (four waves per record for AES-GCM, one for ChaCha)."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(77 + klen)
    lens = list(rng.integers(0, 2049, 2048))
    hb = HostBatch(lens, payload_seed=5, align=16, aad_mode="tls13")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                  tamper=(0, 2047))


@pytest.mark.parametrize("alg,klen,keys,opts", [
    ("aesgcm", 16, 1, {"gcm_variant": 16}), ("aesgcm", 16, 1, {"gcm_variant": 14}),
    ("aesgcm", 16, 1, {"gcm_variant": 15}), ("aesgcm", 32, 1, {"gcm_variant": 15}),
    ("chacha", 32, 1, {"chacha_variant": 4}), ("chacha", 32, 1, {"chacha_variant": 5}),
    ("chacha", 32, 1, {"chacha_variant": 6}),
    ("chacha", 32, 29, {"chacha_variant": 4}),
    ("aesgcm", 32, 29, {"gcm_table_variant": 1}), ("aesgcm", 32, 29, {"gcm_table_variant": 0}),
    ("aesgcm", 16, 29, {"gcm_table_variant": 14}), ("chacha", 32, 29, {})])
@pytest.mark.parametrize("align", [16, 1])
def test_planned_mixed_batch(torch, tg, oracle_mod, alg, klen, keys, opts, align):
    """> 2048 records with per-record lengths on a lane-per-record or octet
    kernel run in a planned order (planner.hip): every record must still land
    in its own output slot.  Single-key batches of this size run a wave per
    record by default, so the other kernels are forced for them."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(1000 + klen + keys + align + sum(opts.values()))
    lens = list(rng.integers(0, 3000, 5000)) + [16384, 16400, 0, 1] * 5
    hb = HostBatch(lens, payload_seed=align, align=align, aad_mode="tls12", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    if keys == 1:
        obj = tg.HipAESGCM(bytearray(kb[0])) if alg == "aesgcm" else \
            tg.HipCHACHA20_POLY1305(bytearray(kb[0]))
        karr = np.frombuffer(kb[0], np.uint8)
    else:
        obj = tg.KeyTable("chacha20-poly1305" if alg == "chacha" else "aesgcm", kb)
        karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    with tg.options(**opts):
        run_seal_open(torch, tg, oracle_mod, hb, alg, karr, obj, tamper=(7, 2500, 5019))


def test_auto_mixed_batch_hybrid(torch, tg, oracle_mod):
    """A mixed-length single-key AES-GCM batch above kWaveMaxRecords runs the
    planner and the hybrid octet kernel by default (aes_gcm.hip)."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(77)
    lens = list(rng.integers(0, 3000, 26000)) + [16384, 16400, 0, 1] * 5
    hb = HostBatch(lens, payload_seed=11, align=16, aad_mode="tls13")
    key = rng.bytes(16)
    run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", np.frombuffer(key, np.uint8),
                  tg.HipAESGCM(bytearray(key)), tamper=(3, 13000, 26019))


@pytest.mark.parametrize("alg,klen", [("aesgcm", 16), ("chacha", 32)])
def test_auto_mixed_batch_wave_path(torch, tg, oracle_mod, alg, klen):
    """A mixed-length single-key batch above the old 2048-record limit runs a
    wave per record without planning."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(5 + klen)
    lens = list(rng.integers(0, 3000, 6000)) + [16384, 16400, 0, 1] * 5
    hb = HostBatch(lens, payload_seed=9, align=16, aad_mode="tls12")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                  tamper=(3, 4000, 6019))


@pytest.mark.parametrize("alg,klen", [("aesgcm", 16), ("aesgcm", 32), ("chacha", 32)])
@pytest.mark.parametrize("waves", [1, 4, 16])
@pytest.mark.parametrize("align", [16, 1])
def test_waves_per_record_forced(torch, tg, oracle_mod, alg, klen, waves, align):
    """The wave-per-record kernels with one, four or sixteen waves per record
    (option waves_per_record; auto picks 16 / 4 / 1 by batch size): the
    segment count changes every record's split point and H / r power."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(waves * 100 + klen + align)
    lens = LENS * 3 + list(rng.integers(0, 16401, 60)) + [20000, 65000]
    hb = HostBatch(lens, payload_seed=align + 40, align=align, aad_mode="random")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    kind = {"gcm_variant": 6} if alg == "aesgcm" else {"chacha_variant": 3}
    with tg.options(waves_per_record=waves, **kind):
        run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                      tamper=(2, 50, len(lens) - 1))


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("align", [16, 1])
def test_key_table_wave_kernel(torch, tg, oracle_mod, klen, align):
    """Many keys, mixed lengths, one wave per record (gcm_table_wave_kernel,
    gcm_table_variant 5): round keys from the record's key, GHASH powers from
    the key's precomputed table."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(300 + klen + align)
    lens = LENS * 4 + list(rng.integers(0, 16401, 300)) + [20000, 65000]
    keys = 37
    hb = HostBatch(lens, payload_seed=align + 77, align=align, aad_mode="random", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    obj = tg.KeyTable("aesgcm", kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    with tg.options(gcm_table_variant=5):
        run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", karr, obj, tamper=(4, 100, len(lens) - 1))


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("keys", [2, 37, 300])
@pytest.mark.parametrize("align", [16, 1])
@pytest.mark.parametrize("variant,split,lpr", [(14, 0, 0), (0, 0, 8), (0, 1000, 8), (0, 4097, 8),
                                              (0, 0, 16), (0, 1000, 32), (0, 4097, 64), (0, 0, 64),
                                              (6, 0, 0), (0, 1000, -1), (0, 4097, -1)])
def test_key_table_octet_kernel(torch, tg, oracle_mod, klen, keys, align, variant, split, lpr):
    """Many keys, ragged lengths, through the key-grouped octet kernel
    (aes_gcm_bs8.hip gcm_kt_kernel): jobs of at most eight records of one
    key, bitsliced keystream with the key's planes, GHASH through the wave's
    4-bit tables of the key's H^8.  Variant 14 sends every record there; the
    auto path (0) splits the batch by length at kt_split (0 = the default
    2048), runs the long ones through the key-grouped bitsliced kernel with
    kt_lpr = 8 / 16 / 32 / 64 lanes per record (jobs of 8 / 4 / 2 / 1 records
    of one key, GHASH stride H^lpr) or the wave-per-record T-table kernel with
    per-wave 4-bit GHASH tables (kt_lpr -1), and the shorter records through
    the lane kernel from the tail of the same plan; variant 6 sends every
    record to the wave-per-record kernel."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(700 + klen + keys + align + split + lpr)
    lens = LENS * 4 + list(rng.integers(0, 16401, 400)) + [999, 1000, 1001, 2047, 2048, 2049,
                                                            4096, 4097, 20000, 65000, 70001]
    hb = HostBatch(lens, payload_seed=align + 91, align=align, aad_mode="random", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    obj = tg.KeyTable("aesgcm", kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    with tg.options(gcm_table_variant=variant, kt_split=split, kt_lpr=lpr):
        run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", karr, obj, tamper=(4, 100, len(lens) - 1))


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("keys", [3, 300])
@pytest.mark.parametrize("split,hyb,kt_t,ovl", [(0, 0, 0, 0), (1000, 0, 0, 0), (0, 0, 1, 0), (1000, 0, 11, 0),
                                                (1000, -1, 0, 0), (1000, 0, 0, -1)])
def test_key_table_hybrid_kernel(torch, tg, oracle_mod, klen, keys, split, hyb, kt_t, ovl):
    """The key-table long records at 32 lanes per record on the persistent
    T-table + bitsliced kernel (aes_gcm_bs8.hip gcm_kth_kernel; kt_hybrid 0,
    the default): T-table waves at 32 lanes per record with per-half counter
    windows, bitsliced waves as in the key-grouped kernel, per-wave 4-bit
    GHASH tables rebuilt when a wave's key changes; kt_t 1 / 11 puts one / all
    waves on the T-table cipher; kt_hybrid -1 the bitsliced key-grouped
    kernel; kt_overlap -1 keeps the short records' lane kernel on the
    caller's stream instead of the engine's second stream.  Ragged lengths
    around the batch and window boundaries, AES-128 and AES-256, oracle-exact
    with tampered tags."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(900 + klen + keys + split + kt_t + hyb)
    lens = LENS * 3 + list(rng.integers(0, 16401, 500)) + [2047, 2048, 2049, 4095, 4096, 4097, 4111,
                                                           8191, 8192, 8209, 16384, 16400, 20000, 70001]
    hb = HostBatch(lens, payload_seed=keys + 5, align=16, aad_mode="random", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    obj = tg.KeyTable("aesgcm", kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    with tg.options(gcm_table_variant=0, kt_split=split, kt_lpr=32, kt_hybrid=hyb, kt_t=kt_t, kt_overlap=ovl):
        run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", karr, obj, tamper=(4, 100, len(lens) - 1))


@pytest.mark.parametrize("alg,opts", [("aesgcm", {"gcm_table_variant": 0}),
                                      ("aesgcm", {"gcm_table_variant": 0, "kt_lpr": -1}),
                                      ("aesgcm", {"gcm_table_variant": 0, "kt_lpr": 32}),
                                      ("aesgcm", {"gcm_table_variant": 0, "kt_hybrid": -1}),
                                      ("aesgcm", {"gcm_table_variant": 6}),
                                      ("aesgcm", {"gcm_table_variant": 1}),
                                      ("aesgcm", {"gcm_table_variant": 5}),
                                      ("aesgcm", {"gcm_table_variant": 14}),
                                      ("chacha", {}), ("chacha", {"chacha_variant": 4}),
                                      ("aesccm", {"ccm_variant": 2}),
                                      ("aesccm", {"ccm_variant": 3})])
def test_key_index_out_of_range_is_skipped(torch, tg, oracle_mod, alg, opts):
    """A key-table record whose key_idx is not below the table's size is
    never read past the table: seal leaves its output alone, open reports
    status 0 and zeroes its plaintext output (as a rejected record's; the
    output buffer starts filled with 0xaa); every other record is sealed and
    opened as usual."""
    from batchpack import HostBatch
    nk = 7
    rng = np.random.default_rng(55)
    lens = list(rng.integers(0, 5000, 3000)) + [16384] * 40
    hb = HostBatch(lens, payload_seed=3, align=16, aad_mode="tls12", key_count=nk)
    bad = np.array([0, 5, 17, 1500, 2999, 3020], dtype=np.int64)
    hb.key_idx[bad] = np.array([nk, nk + 1, 0xffffffff, nk, 1000, nk], dtype=np.uint32)
    klen = 32 if alg == "chacha" else 16
    kb = [rng.bytes(klen) for _ in range(nk)]
    name = {"aesgcm": "aesgcm", "chacha": "chacha20-poly1305", "aesccm": "aesccm"}[alg]
    table = tg.KeyTable(name, kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(nk, klen)
    good = np.setdiff1d(np.arange(hb.n), bad)
    with tg.options(**opts):
        d = hb.to_device(torch)
        tg.seal_batch(table, hb.batch_kwargs(d))
        torch.cuda.synchronize()
        got = d["out"].cpu().numpy()
        kidx = hb.key_idx.copy()
        hb.key_idx = np.where(kidx < nk, kidx, 0).astype(np.uint32)   # the oracle needs valid keys
        want, _ = hb.oracle(oracle_mod, alg, karr, "seal")
        hb.key_idx = kidx
        for i in good:
            o, L = int(hb.out_off[i]), int(hb.lens[i])
            assert np.array_equal(got[o:o + L + 16], want[o:o + L + 16]), ("seal", i)
        for i in bad:
            o, L = int(hb.out_off[i]), int(hb.lens[i])
            assert not got[o:o + L + 16].any(), ("skipped record written", i)
        # open: the good records' sealed bytes back, bad ones rejected
        src = d["out"].clone()
        pt = torch.full((hb.in_bytes,), 0xaa, dtype=torch.uint8, device="cuda")
        status = torch.full((hb.n,), 7, dtype=torch.uint8, device="cuda")
        tg.open_batch(table, tg.make_batch(hb.n, src, pt, d["nonces"], aad=d["aad"], lens=d["lens"],
                                           in_off=d["out_off"], out_off=d["in_off"], aad_off=d["aad_off"],
                                           aad_len=d["aad_len"], key_idx=d["key_idx"], status=status))
        torch.cuda.synchronize()
        st = status.cpu().numpy()
        assert (st[bad] == 0).all()
        assert (st[good] == 1).all()
        back = pt.cpu().numpy()
        for i in bad:
            o, L = int(hb.in_off[i]), int(hb.lens[i])
            assert not back[o:o + L].any(), ("skipped record's plaintext not zeroed", i)
        for i in good[::37]:
            o, L = int(hb.in_off[i]), int(hb.lens[i])
            assert np.array_equal(back[o:o + L], hb.inp[o:o + L]), ("open", i)


def test_hy_t_out_of_range_fails_launch(torch, tg):
    """hy_t above the hybrid workgroup's waves is TG_EINVAL at launch (no
    silent fallback to the default split); hy_t within range works."""
    n, L = 32768, 16    # above the wave kernel's limit: the hybrid kernel
    inp = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    out = torch.zeros(n * (L + 16), dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    key = tg.HipAESGCM(bytearray(16))
    b = tg.make_batch(n, inp, out, nonces, fixed_len=L, in_stride=L, out_stride=L + 16)
    with tg.options(gcm_variant=15, hy_t=17):
        with pytest.raises(tg.TlsGpuError):
            tg.seal_batch(key, b)
    with tg.options(gcm_variant=15, hy_t=16):
        tg.seal_batch(key, b)
    torch.cuda.synchronize()
