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


def test_rccl_world1_collectives():
    """The RCCL code path on hardware: a world-size-1
    process group under the nccl backend (what bench.py --dist-selftest and
    every N > 1 rank create), then the collectives bench.py runs -- the counter
    all_reduce (SUM, MAX) and the rate all_gather -- on device tensors, in a
    child process so this test process keeps no group."""
    import subprocess
    import sys
    import os
    code = (
        "import os, sys, torch, torch.distributed as dist\n"
        "sys.path.insert(0, %r)\n"
        "from tlsgpu import distributed as tgd\n"
        "w, r, l, dev = tgd.init_process(torch, dist, backend='nccl', group_at_world1=True)\n"
        "assert tgd.group_active(dist) and dist.get_backend() == 'nccl'\n"
        "info = tgd.selftest_collectives(torch, dist, device='cuda')\n"
        "sums, t = tgd.reduce_counters(torch, dist, [5, 6, 0], 2.5, device='cuda')\n"
        "rows = tgd.gather_rows(torch, dist, [1.0, 2.0], device='cuda')\n"
        "tgd.barrier(torch, dist, w)\n"
        "dist.destroy_process_group()\n"
        "print('RESULT', info['ok'], info['backend'], sums, t, rows)\n"
    ) % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tlslite-ng_amd")
    env = dict(os.environ)
    for k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")][0]
    assert line == "RESULT True nccl [5.0, 6.0, 0.0] 2.5 [[1.0, 2.0]]", line
