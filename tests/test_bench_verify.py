"""bench.py's N > 1 verdict covers every rank: each rank
checks its own sampled records against the oracle at its own seq offset, and
``verified`` / ``oracle_mismatches`` are the MIN / SUM over ranks.  World
size 2 over gloo on the CPU, through the same bench functions
(tests/bench_verify_rank.py): a mismatch on rank 1 alone -- a flipped byte,
or records sealed without the rank's seq offset -- makes rank 0's line say
verified false and every rank exit 3."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _run(mode, corrupt_rank=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TLSGPU_BENCH_CORRUPT_RANK"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    if corrupt_rank is not None:
        env["TLSGPU_BENCH_CORRUPT_RANK"] = str(corrupt_rank)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "bench_verify_rank.py"), mode]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-3000:]
    return r.returncode, json.loads(lines[0]), r.stdout + r.stderr


def _both_ranks_fail(out):
    """torch.distributed.run's failure report: the first rank to exit has
    status 3; the other one either exits 3 too or, when the launcher's
    SIGTERM beats its own exit, -15.  No rank may exit 0 or crash otherwise."""
    codes = re.findall(r"exitcode  : (-?\d+)", out)
    assert "3" in codes and set(codes) <= {"3", "-15"} and len(codes) == 2, out[-3000:]


@pytest.mark.parametrize("mode", ["headline", "c5"])
def test_all_ranks_clean(mode):
    rc, line, out = _run(mode)
    assert rc == 0, out[-3000:]
    assert line["verified"] is True and line["oracle_mismatches"] == 0
    assert line["oracle_checked_records"] == 12 and line["n_gpus"] == 2


@pytest.mark.parametrize("mode", ["headline", "c5"])
def test_rank1_mismatch_fails_the_line(mode):
    rc, line, out = _run(mode, corrupt_rank=1)
    assert line["verified"] is False and line["oracle_mismatches"] == 1, line
    assert rc != 0
    _both_ranks_fail(out)


def test_missing_seq_offset_on_rank1_is_caught():
    """Rank 1 sealed its shard at seq 0.. instead of 6..: every one of its
    records differs from the oracle at its true seq."""
    rc, line, out = _run("c5-noshift")
    assert line["verified"] is False and line["oracle_mismatches"] == 6, line
    assert rc != 0
    _both_ranks_fail(out)
