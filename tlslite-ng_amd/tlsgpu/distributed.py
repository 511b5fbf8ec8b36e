"""Multi-GPU sharding of record batches (one process per GPU).

A connection's records are independent AEAD calls keyed by (key, fixed IV,
seq) -- tlslite/recordlayer.py:251-256 (seq), :522-534 (nonce) -- so a batch
shards by contiguous sequence-number range with no data exchange: rank r of W
seals seq [seq0_r, seq0_r + n_r).  The only collectives are reductions of the
per-rank counters (records, payload bytes, auth failures), of the timing max,
and a gather of the per-rank kernel rates for the report -- bench.py runs them
over RCCL (backend "nccl") on GPUs, tests/test_distributed.py over gloo on CPU.

Everything bench.py does for N > 1 lives here (process setup, the shard plan,
the per-rank nonces, the barrier-bracketed timed region, the reductions), so
the world-size-2 CPU test drives the same functions.
"""
import os
import time


class DistError(RuntimeError):
    pass


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def init_process(torch, dist, backend=None, use_gpu=True, group_at_world1=None):
    """One process per GPU.  backend None = TLSGPU_DIST_BACKEND or "nccl"
    (= RCCL over xGMI on ROCm).  Under nccl every rank needs its own device:
    LOCAL_RANK >= device count is an error (no silent oversubscription).  gloo
    is the CPU rehearsal backend; with use_gpu it may map several ranks to one
    device (rank % device count), which is only for rehearsals.

    A process group is created for world > 1, and also at world 1 when
    ``group_at_world1`` (default: TLSGPU_DIST_SELFTEST=1) asks for it, so the
    collectives below run through the backend on a one-GPU box too (the RCCL
    self-test, bench.py --dist-selftest).  Without MASTER_ADDR the world-1
    group rendezvouses on tcp://127.0.0.1 at a free port; at world > 1 every
    rank would pick a different port and hang, so that is a DistError.
    Returns (world, rank, local_rank, device or None)."""
    world, rank, local = env_rank()
    backend = backend or os.environ.get("TLSGPU_DIST_BACKEND", "nccl")
    if group_at_world1 is None:
        group_at_world1 = os.environ.get("TLSGPU_DIST_SELFTEST") == "1"
    device = None
    if use_gpu:
        ndev = torch.cuda.device_count()
        if ndev < 1:
            raise DistError("no GPU visible")
        if backend == "nccl" and local >= ndev:
            raise DistError("LOCAL_RANK %d >= %d visible GPUs: one process per GPU needs a device "
                            "per local rank" % (local, ndev))
        device = local if backend == "nccl" else local % ndev
        torch.cuda.set_device(device)
    elif backend == "nccl":
        raise DistError("the nccl backend needs a GPU per rank")
    if world > 1 or group_at_world1:
        kw = {}
        if "MASTER_ADDR" not in os.environ:
            if world > 1:
                raise DistError("WORLD_SIZE=%d without MASTER_ADDR: launch the ranks with "
                                "torch.distributed.run (--master-addr 127.0.0.1)" % world)
            kw = {"init_method": "tcp://127.0.0.1:%d" % _free_port(), "world_size": world,
                  "rank": rank}
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device), **kw)
        else:
            dist.init_process_group(backend, **kw)
    return world, rank, local, device


def group_active(dist):
    """True when a process group exists (world > 1, or the world-1 self-test):
    the collectives below then go through the backend."""
    return dist.is_available() and dist.is_initialized()


def selftest_collectives(torch, dist, device=None):
    """The collectives bench.py uses, checked on known values: an all_reduce
    SUM and MAX of rank-dependent tensors and an all_gather of a per-rank row.
    Returns a dict for the bench line; ``ok`` is False on any mismatch."""
    if not group_active(dist):
        raise DistError("no process group")
    world, rank = dist.get_world_size(), dist.get_rank()
    c = torch.tensor([1.0, float(rank), 2.0 ** 40 + rank], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    t = torch.tensor([float(rank) * 3.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    row = torch.tensor([float(rank), float(rank) + 0.5], dtype=torch.float64, device=device)
    rows = [torch.zeros_like(row) for _ in range(world)]
    dist.all_gather(rows, row)
    if device is not None:
        torch.cuda.synchronize()
    want_sum = [float(world), float(world * (world - 1) // 2),
                world * 2.0 ** 40 + world * (world - 1) // 2]
    ok = (c.tolist() == want_sum and t.item() == 3.0 * (world - 1) and
          [r.tolist() for r in rows] == [[float(g), g + 0.5] for g in range(world)])
    return {"backend": dist.get_backend(), "world": world, "all_reduce_sum": c.tolist(),
            "all_reduce_max": t.item(), "all_gather_rows": world, "ok": bool(ok)}


def shard_range(n_total, world, rank):
    """Contiguous partition of ``n_total`` records: returns (first, count)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def weak_shard(n_per_rank, world, rank, seq_base=0):
    """Weak scaling (bench.py, BASELINE configs[4]): every rank seals
    ``n_per_rank`` records, rank g the seqs [g n, (g + 1) n).  (first, count)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return seq_base + rank * int(n_per_rank), int(n_per_rank)


def tls13_nonces(iv, seq0, n):
    """Host mirror of tg_make_nonces mode 0 (iv xor (0^4 || be64(seq)))."""
    iv = bytes(iv)
    out = bytearray()
    for s in range(seq0, seq0 + n):
        pad = bytes(4) + s.to_bytes(8, "big")
        out += bytes(a ^ b for a, b in zip(iv, pad))
    return bytes(out)


def shard_nonces(tlsgpu, iv, first, count, out):
    """This rank's nonces on the device (tg_make_nonces with the rank's seq
    offset); tls13_nonces(iv, first, count) is the host mirror."""
    tlsgpu.make_nonces(iv, first, count, out)
    return out


def _sync(torch):
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def barrier(torch, dist, world):
    """Device sync, then (N > 1) a process barrier, then device sync."""
    _sync(torch)
    if group_active(dist):
        dist.barrier()
    _sync(torch)


def timed(torch, dist, world, fn, steps):
    """The bench contract's timed region: barrier + device sync on both sides
    of exactly ``steps`` calls of ``fn(step)``; returns this rank's seconds."""
    barrier(torch, dist, world)
    t0 = time.perf_counter()
    for s in range(steps):
        fn(s)
    barrier(torch, dist, world)
    return time.perf_counter() - t0


def reduce_counters(torch, dist, counters, elapsed, device=None):
    """Sum ``counters`` (list of numbers) and take the max of ``elapsed`` over
    all ranks.  Returns (summed list, max elapsed)."""
    c = torch.tensor([float(x) for x in counters], dtype=torch.float64, device=device)
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if group_active(dist):
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in c.tolist()], float(t.item())


def reduce_verification(torch, dist, ok, mismatches, checked, device=None):
    """The N > 1 line's verification over all ranks: ``ok`` is the MIN of the
    ranks' flags (one failing shard fails the line), ``mismatches`` and
    ``checked`` (oracle-compared records) the SUMs.  Returns
    (ok, mismatches, checked)."""
    if group_active(dist) and dist.get_backend() == "gloo":
        device = None   # gloo's MIN over CPU tensors (the rehearsal backend)
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=device)
    c = torch.tensor([float(mismatches), float(checked)], dtype=torch.float64, device=device)
    if group_active(dist):
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    m, n = c.tolist()
    return bool(t.item() == 1.0), int(m), int(n)


def gather_rows(torch, dist, row, device=None):
    """All ranks' ``row`` (list of numbers, same length everywhere) as a list
    of lists indexed by rank (the per-rank kernel rates of the report)."""
    t = torch.tensor([float(x) for x in row], dtype=torch.float64, device=device)
    if group_active(dist):
        out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        return [[float(x) for x in o.tolist()] for o in out]
    return [[float(x) for x in t.tolist()]]
