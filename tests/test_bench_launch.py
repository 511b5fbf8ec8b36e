"""bench.py --gpus N starts N ranks itself (one process per GPU through
torch.distributed.run on 127.0.0.1) when no launcher set WORLD_SIZE, and a
rank refuses to run when the launcher's world size differs from --gpus.
CPU only: without a GPU the ranks stop in tlsgpu.distributed.init_process,
which proves they were started."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rank_launch_cmd():
    import bench
    cmd = bench.rank_launch_cmd(["--gpus", "4", "--steps", "3"], 4, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert "--nnodes=1" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3"]


def test_check_world():
    import bench
    assert bench.check_world(1, {}) is None
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) is None
    assert "WORLD_SIZE=1" in bench.check_world(8, {"WORLD_SIZE": "1"})
    assert "WORLD_SIZE=2" in bench.check_world(1, {"WORLD_SIZE": "2"})


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_starts_two_ranks():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--records", "64",
              "--no-cpu-baseline"], {"TLSGPU_DIST_BACKEND": "gloo"})
    assert r.returncode != 0
    out = r.stdout + r.stderr
    # both ranks reached init_process (no GPU here) under the launcher
    assert out.count("no GPU visible") >= 2, out[-3000:]
    assert "torch.distributed" in out or "ChildFailedError" in out or "rank" in out.lower()


def test_world_mismatch_refused():
    r = _run(["--gpus", "2", "--records", "64", "--no-cpu-baseline"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_nccl_needs_a_gpu_per_rank():
    """Under nccl (the default backend) --gpus N with fewer visible devices
    is refused before any rank starts."""
    r = _run(["--gpus", "2", "--records", "64", "--no-cpu-baseline"], {"TLSGPU_DIST_BACKEND": "nccl"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "needs one GPU per rank, 0 visible" in r.stderr


@pytest.mark.parametrize("config", ["c4", "ingest", "ccm", "c1"])
def test_single_gpu_configs_refuse_n(config):
    r = _run(["--gpus", "2", "--config", config])
    assert r.returncode == 2 and "runs on one GPU" in r.stderr


def test_cpu_config1_in_full_matches_reference_digest():
    """bench.py's config-1 CPU leg (BASELINE configs[0] in full, 4 096 x 1 KiB
    ChaCha20-Poly1305 with the pure-Python restatement, split over processes):
    the sealed stream equals the reference's own digest and opens back."""
    import bench
    r = bench.cpu_config1(4)
    assert r["digest_match"] and r["opened_ok"] and r["cores"] == 4 and r["records"] == 4096
    assert r["value"] > 0
