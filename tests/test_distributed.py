"""World-size-2 checks of the record sharding on CPU (gloo).

Each rank seals its contiguous seq shard of one connection with the oracle
(the GPU path is exercised by bench.py on real devices); concatenated per-rank
output must equal a single-rank run, and the counter reduction must add up.
"""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tlsgpu.distributed import reduce_counters, shard_range, tls13_nonces
from vectors import tls13_aad, tls13_nonce


def test_shard_range_partitions():
    for n in (0, 1, 7, 1 << 20, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0
            for (a, na), (b, _) in zip(spans, spans[1:]):
                assert a + na == b
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_host_nonces_match_record_layer():
    iv = bytes(range(12))
    got = tls13_nonces(iv, 2 ** 33 - 2, 5)
    assert got == b"".join(bytes(tls13_nonce(iv, 2 ** 33 - 2 + i)) for i in range(5))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


N_TOTAL, LEN = 37, 300


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle
    key, iv = bytes(range(32)), bytes(range(100, 112))
    first, count = shard_range(N_TOTAL, world, rank)
    h = hashlib.sha256()
    for s in range(first, first + count):
        pt = hashlib.sha256(b"pt%d" % s).digest() * (LEN // 32 + 1)
        out = oracle.chacha_seal(key, tls13_nonce(iv, s), pt[:LEN], tls13_aad(LEN))
        h.update(bytes(out))
        with open(os.path.join(outdir, "rec%05d" % s), "wb") as f:
            f.write(bytes(out))
    sums, tmax = reduce_counters(torch, dist, [count, count * LEN, 0], 0.1 * (rank + 1))
    with open(os.path.join(outdir, "rank%d" % rank), "w") as f:
        f.write("%d %d %d %.3f" % (sums[0], sums[1], sums[2], tmax))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_sharded_seal_equals_single(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        recs, payload, fails, tmax = open(tmp_path / ("rank%d" % r)).read().split()
        assert int(recs) == N_TOTAL and int(payload) == N_TOTAL * LEN and int(fails) == 0
        assert float(tmax) == pytest.approx(0.2)
    from oracle import oracle
    key, iv = bytes(range(32)), bytes(range(100, 112))
    for s in range(N_TOTAL):
        pt = hashlib.sha256(b"pt%d" % s).digest() * (LEN // 32 + 1)
        want = oracle.chacha_seal(key, tls13_nonce(iv, s), pt[:LEN], tls13_aad(LEN))
        assert open(tmp_path / ("rec%05d" % s), "rb").read() == bytes(want)
