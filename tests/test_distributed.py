"""World-size-2 checks of the record sharding on CPU (gloo), driving the same
tlsgpu.distributed functions bench.py runs for N > 1: process setup, the weak
shard plan (rank g seals seq [g n, (g+1) n)), the rank-offset nonces (host
mirror of tg_make_nonces), the barrier-bracketed timed region, the counter
reduction and the per-rank gather.  Each rank seals its shard with the oracle
(the GPU kernels are the -m gpu tests' job); concatenated per-rank nonces and
records must equal a single-rank run.
"""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tlsgpu import distributed as tgd
from vectors import tls13_aad, tls13_nonce


def test_shard_range_partitions():
    for n in (0, 1, 7, 1 << 20, 1000003):
        for w in (1, 2, 3, 8):
            spans = [tgd.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            for (a, na), (b, _) in zip(spans, spans[1:]):
                assert a + na == b
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_weak_shard_is_bench_plan():
    for w in (1, 2, 4, 8):
        spans = [tgd.weak_shard(1 << 20, w, r) for r in range(w)]
        assert spans == [(r << 20, 1 << 20) for r in range(w)]
    with pytest.raises(ValueError):
        tgd.weak_shard(10, 2, 2)


def test_host_nonces_match_record_layer():
    iv = bytes(range(12))
    got = tgd.tls13_nonces(iv, 2 ** 33 - 2, 5)
    assert got == b"".join(bytes(tls13_nonce(iv, 2 ** 33 - 2 + i)) for i in range(5))


def test_nccl_needs_a_device_per_rank(monkeypatch):
    """init_process refuses LOCAL_RANK >= device count under nccl instead of
    wrapping several ranks onto one GPU."""
    class FakeCuda(object):
        @staticmethod
        def device_count():
            return 1

        @staticmethod
        def set_device(d):
            raise AssertionError("must not be reached")

    class FakeTorch(object):
        cuda = FakeCuda()

    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    with pytest.raises(tgd.DistError):
        tgd.init_process(FakeTorch(), None, backend="nccl")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


N_PER_RANK, LEN, STEPS = 19, 300, 2
KEY, IV = bytes(range(32)), bytes(range(100, 112))


def _pt(s):
    return (hashlib.sha256(b"pt%d" % s).digest() * (LEN // 32 + 1))[:LEN]


def _worker(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                       "RANK": str(rank), "LOCAL_RANK": str(rank)})
    w, r, local, dev = tgd.init_process(torch, dist, backend="gloo", use_gpu=False)
    assert (w, r, local, dev) == (world, rank, rank, None)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle
    first, count = tgd.weak_shard(N_PER_RANK, world, rank)
    nonces = tgd.tls13_nonces(IV, first, count)
    out = {}

    def step(k):
        for i in range(count):
            s = first + i
            out[s] = bytes(oracle.chacha_seal(KEY, nonces[12 * i:12 * i + 12], _pt(s), tls13_aad(LEN)))

    elapsed = tgd.timed(torch, dist, world, step, STEPS)
    sums, tmax = tgd.reduce_counters(torch, dist, [count * STEPS, count * LEN * STEPS, 0], elapsed)
    rows = tgd.gather_rows(torch, dist, [rank, count, first])
    assert tgd.selftest_collectives(torch, dist)["ok"]
    with open(os.path.join(outdir, "rank%d" % rank), "w") as f:
        f.write("%d %d %d %.6f %.6f\n" % (sums[0], sums[1], sums[2], tmax, elapsed))
        f.write(repr(rows) + "\n")
    with open(os.path.join(outdir, "nonces%d" % rank), "wb") as f:
        f.write(nonces)
    for s, rec in out.items():
        with open(os.path.join(outdir, "rec%05d" % s), "wb") as f:
            f.write(rec)
    tgd.barrier(torch, dist, world)
    dist.destroy_process_group()


def test_world2_sharded_seal_equals_single(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    total = world * N_PER_RANK
    tmaxes = []
    for r in range(world):
        lines = open(tmp_path / ("rank%d" % r)).read().splitlines()
        recs, payload, fails, tmax, mine = lines[0].split()
        assert int(float(recs)) == total * STEPS and int(float(payload)) == total * LEN * STEPS
        assert int(float(fails)) == 0
        assert float(tmax) >= float(mine)
        tmaxes.append(float(tmax))
        rows = eval(lines[1])   # noqa: S307 -- our own repr of a list of float lists
        assert [int(x[0]) for x in rows] == list(range(world))
        assert [int(x[2]) for x in rows] == [g * N_PER_RANK for g in range(world)]
    assert tmaxes[0] == tmaxes[1]                       # every rank reports the max
    # concatenated per-rank nonces == one rank covering all seqs
    cat = b"".join(open(tmp_path / ("nonces%d" % r), "rb").read() for r in range(world))
    assert cat == tgd.tls13_nonces(IV, 0, total)
    from oracle import oracle
    for s in range(total):
        want = oracle.chacha_seal(KEY, tls13_nonce(IV, s), _pt(s), tls13_aad(LEN))
        assert open(tmp_path / ("rec%05d" % s), "rb").read() == bytes(want)


def _world1_worker(_, outdir):
    for k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    os.environ["TLSGPU_DIST_SELFTEST"] = "1"
    w, r, _, dev = tgd.init_process(torch, dist, backend="gloo", use_gpu=False)
    assert (w, r, dev) == (1, 0, None) and tgd.group_active(dist)
    info = tgd.selftest_collectives(torch, dist)
    sums, tmax = tgd.reduce_counters(torch, dist, [3, 4, 0], 1.5)
    rows = tgd.gather_rows(torch, dist, [7.0, 8.0])
    dist.destroy_process_group()
    with open(os.path.join(outdir, "world1"), "w") as f:
        f.write(repr((info["ok"], info["backend"], info["world"], sums, tmax, rows)))


def test_world1_group_selftest(tmp_path):
    """bench.py --dist-selftest at world size 1: the group is created anyway
    (tcp rendezvous on 127.0.0.1 outside torch.distributed.run) and the
    counter reduction, rate gather and collective self-test go through the
    backend (gloo here; RCCL in the -m gpu test)."""
    mp.spawn(_world1_worker, args=(str(tmp_path),), nprocs=1, join=True)
    got = eval(open(tmp_path / "world1").read())   # noqa: S307 -- our own repr
    assert got == (True, "gloo", 1, [3.0, 4.0, 0.0], 1.5, [[7.0, 8.0]])


def test_world2_without_master_addr_refused(monkeypatch):
    """At world > 1 the free-port fallback would give every rank its own
    port and hang the rendezvous: without MASTER_ADDR it is a
    DistError before any process group is created."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.delenv("MASTER_ADDR", raising=False)
    with pytest.raises(tgd.DistError, match="MASTER_ADDR"):
        tgd.init_process(torch, dist, backend="gloo", use_gpu=False)
    assert not dist.is_initialized()
