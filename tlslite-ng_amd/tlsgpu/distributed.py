"""Multi-GPU sharding of record batches (one process per GPU).

A connection's records are independent AEAD calls keyed by (key, fixed IV,
seq) -- tlslite/recordlayer.py:251-256 (seq), :522-534 (nonce) -- so a batch
shards by contiguous sequence-number range with no data exchange: rank r of W
seals seq [seq0_r, seq0_r + n_r).  The only collective is a reduction of the
per-rank counters (records, payload bytes, auth failures) and of the timing
max, which bench.py runs over RCCL (backend "nccl") on GPUs and the tests run
over gloo on CPU.
"""


def shard_range(n_total, world, rank):
    """Contiguous partition of ``n_total`` records: returns (first, count)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def tls13_nonces(iv, seq0, n):
    """Host mirror of tg_make_nonces mode 0 (iv xor (0^4 || be64(seq)))."""
    iv = bytes(iv)
    out = bytearray()
    for s in range(seq0, seq0 + n):
        pad = bytes(4) + s.to_bytes(8, "big")
        out += bytes(a ^ b for a, b in zip(iv, pad))
    return bytes(out)


def reduce_counters(torch, dist, counters, elapsed, device=None):
    """Sum ``counters`` (list of numbers) and take the max of ``elapsed`` over
    all ranks.  Returns (summed list, max elapsed)."""
    c = torch.tensor([float(x) for x in counters], dtype=torch.float64, device=device)
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in c.tolist()], float(t.item())
