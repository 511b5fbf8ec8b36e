"""The multi-GPU shard plan on one device: every rank's nonces, built on the
device by tg_make_nonces with the rank's seq offset (tlsgpu.distributed.
shard_nonces, what bench.py runs per rank), concatenate to the single-rank
nonces of the whole connection (host mirror of recordlayer.py:522-534)."""
import pytest
import torch

from tlsgpu import distributed as tgd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rank_offset_nonces_concatenate(world):
    import tlsgpu
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    iv = bytes(range(40, 52))
    n = 1000
    parts = []
    for rank in range(world):
        first, count = tgd.weak_shard(n, world, rank, seq_base=2 ** 40 - 1500)
        out = torch.zeros(12 * count, dtype=torch.uint8, device="cuda")
        tgd.shard_nonces(tlsgpu, iv, first, count, out)
        parts.append(out.cpu().numpy().tobytes())
    torch.cuda.synchronize()
    assert b"".join(parts) == tgd.tls13_nonces(iv, 2 ** 40 - 1500, world * n)
