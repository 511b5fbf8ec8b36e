"""GPU parity of every kernel behind the same batch entry points: batches of
up to 2048 records run one record per wavefront, larger ones a record per
lane; each is forced here on ragged batches (lengths, alignment, AAD, tampered
records) and checked bit-exact against the oracle."""
import os

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


def _with_env(var, value):
    class Ctx(object):
        def __enter__(self):
            self.old = os.environ.get(var)
            os.environ[var] = value

        def __exit__(self, *a):
            if self.old is None:
                del os.environ[var]
            else:
                os.environ[var] = self.old
    return Ctx()


LENS = [0, 1, 15, 16, 17, 63, 64, 65, 1000, 1024, 1040, 4095, 16383, 16384, 16385, 16400]


@pytest.mark.parametrize("alg,klen,var,value", [
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "5"),          # lane per record, full rounds
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "5"),
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "7"),          # lane per record, counter windows
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "7"),
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "8"),          # windows, two blocks per group
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "9"),          # windows, rotated GHASH tables
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "13"),         # windows, three blocks per group
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "6"),          # wave per record
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "6"),
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "14"),         # 8-block bitsliced, octet per record
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "14"),
    ("aesgcm", 16, "TLSGPU_GCM_VARIANT", "15"),         # hybrid T-table + bitsliced (persistent)
    ("aesgcm", 32, "TLSGPU_GCM_VARIANT", "15"),
    ("chacha", 32, "TLSGPU_CHACHA_VARIANT", "4"),       # lane per record
    ("chacha", 32, "TLSGPU_CHACHA_VARIANT", "3"),       # wave per record
])
@pytest.mark.parametrize("align", [16, 1])
def test_forced_kernel_vs_oracle(torch, tg, oracle_mod, alg, klen, var, value, align):
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(hash((alg, klen, value, align)) & 0xffff)
    # + long records: many 256-counter windows (window-cache refreshes)
    lens = LENS * 5 + list(rng.integers(0, 16401, 120)) + [65520, 65536, 70001]
    hb = HostBatch(lens, payload_seed=align + 21, align=align, aad_mode="random")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    with _with_env(var, value):
        run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                      tamper=(1, 30, 111))


@pytest.mark.parametrize("keys", ["0", "1", "2"])   # LDS / scalar loads / row layout (default 4: folded)
@pytest.mark.parametrize("klen", [16, 32])
def test_hybrid_key_plane_sources(torch, tg, oracle_mod, keys, klen, monkeypatch):
    """The hybrid kernel's alternative key-plane providers (TLSGPU_HY_KEYS)."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(300 + klen + int(keys))
    lens = LENS * 3 + list(rng.integers(0, 16401, 60)) + [65536, 70001]
    hb = HostBatch(lens, payload_seed=31, align=16, aad_mode="random")
    key = rng.bytes(klen)
    monkeypatch.setenv("TLSGPU_GCM_VARIANT", "15")
    monkeypatch.setenv("TLSGPU_HY_KEYS", keys)
    run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", np.frombuffer(key, np.uint8),
                  tg.HipAESGCM(bytearray(key)), tamper=(2, 40))


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


@pytest.mark.parametrize("alg,klen,keys,gcmv", [("aesgcm", 16, 1, "7"), ("aesgcm", 16, 1, "14"),
                                               ("aesgcm", 16, 1, "15"), ("aesgcm", 32, 1, "15"),
                                               ("chacha", 32, 1, None), ("aesgcm", 32, 29, None),
                                               ("chacha", 32, 29, None)])
@pytest.mark.parametrize("align", [16, 1])
def test_planned_mixed_batch(torch, tg, oracle_mod, alg, klen, keys, gcmv, align):
    """> 2048 records with per-record lengths on a lane-per-record kernel run
    longest first (planner.hip): every record must still land in its own
    output slot.  Single-key batches of this size run a wave per record by
    default, so the lane kernel is forced for them."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(1000 + klen + keys + align + int(gcmv or 0))
    lens = list(rng.integers(0, 3000, 5000)) + [16384, 16400, 0, 1] * 5
    hb = HostBatch(lens, payload_seed=align, align=align, aad_mode="tls12", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    if keys == 1:
        obj = tg.HipAESGCM(bytearray(kb[0])) if alg == "aesgcm" else \
            tg.HipCHACHA20_POLY1305(bytearray(kb[0]))
        karr = np.frombuffer(kb[0], np.uint8)
        env = ("TLSGPU_GCM_VARIANT", gcmv) if alg == "aesgcm" else ("TLSGPU_CHACHA_VARIANT", "4")
    else:
        obj = tg.KeyTable("chacha20-poly1305" if alg == "chacha" else "aesgcm", kb)
        karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
        env = ("TLSGPU_GCM_TABLE_VARIANT", "0")   # AES: the lane kernel
    with _with_env(*env):
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
@pytest.mark.parametrize("waves", ["1", "4", "16"])
@pytest.mark.parametrize("align", [16, 1])
def test_waves_per_record_forced(torch, tg, oracle_mod, alg, klen, waves, align):
    """The wave-per-record kernels with one or four waves per record
    (TLSGPU_WAVES_PER_RECORD; auto picks 16 / 4 / 1 by batch size):
    the segment count changes every record's split point and H / r power."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(int(waves) * 100 + klen + align)
    lens = LENS * 3 + list(rng.integers(0, 16401, 60)) + [20000, 65000]
    hb = HostBatch(lens, payload_seed=align + 40, align=align, aad_mode="random")
    key = rng.bytes(klen)
    obj = tg.HipAESGCM(bytearray(key)) if alg == "aesgcm" else tg.HipCHACHA20_POLY1305(bytearray(key))
    var = "TLSGPU_GCM_VARIANT" if alg == "aesgcm" else "TLSGPU_CHACHA_VARIANT"
    with _with_env(var, "6" if alg == "aesgcm" else "3"), \
            _with_env("TLSGPU_WAVES_PER_RECORD", waves):
        run_seal_open(torch, tg, oracle_mod, hb, alg, np.frombuffer(key, np.uint8), obj,
                      tamper=(2, 50, len(lens) - 1))


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("threads", ["512", "768", "1024"])
@pytest.mark.parametrize("align", [16, 1])
def test_key_table_wave_kernel(torch, tg, oracle_mod, klen, threads, align):
    """Many keys, mixed lengths, one wave per record (gcm_table_wave_kernel,
    key-table variant 5): round keys from the record's key, GHASH powers from
    the key's precomputed table."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(300 + klen + int(threads) + align)
    lens = LENS * 4 + list(rng.integers(0, 16401, 300)) + [20000, 65000]
    keys = 37
    hb = HostBatch(lens, payload_seed=align + 77, align=align, aad_mode="random", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    obj = tg.KeyTable("aesgcm", kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    with _with_env("TLSGPU_GCM_TABLE_WAVE_THREADS", threads), \
            _with_env("TLSGPU_GCM_TABLE_VARIANT", "5"):
        run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", karr, obj, tamper=(4, 100, len(lens) - 1))


@pytest.mark.parametrize("klen", [16, 32])
@pytest.mark.parametrize("keys", [2, 37, 300])
@pytest.mark.parametrize("align", [16, 1])
def test_key_table_octet_kernel(torch, tg, oracle_mod, klen, keys, align, monkeypatch):
    """Many keys, ragged lengths, through the key-grouped octet kernel
    (aes_gcm_bs8.hip gcm_kt_kernel, TLSGPU_GCM_TABLE_VARIANT=14): jobs of at
    most eight records of one key, bitsliced keystream with the key's planes,
    GHASH through the wave's 4-bit tables of the key's H^8."""
    from batchpack import HostBatch, run_seal_open
    rng = np.random.default_rng(700 + klen + keys + align)
    lens = LENS * 4 + list(rng.integers(0, 16401, 400)) + [20000, 65000, 70001]
    hb = HostBatch(lens, payload_seed=align + 91, align=align, aad_mode="random", key_count=keys)
    kb = [rng.bytes(klen) for _ in range(keys)]
    obj = tg.KeyTable("aesgcm", kb)
    karr = np.frombuffer(b"".join(kb), np.uint8).reshape(keys, klen)
    monkeypatch.setenv("TLSGPU_GCM_TABLE_VARIANT", "14")
    run_seal_open(torch, tg, oracle_mod, hb, "aesgcm", karr, obj, tamper=(4, 100, len(lens) - 1))
