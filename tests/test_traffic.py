"""HBM traffic bookkeeping on the CPU: tools/traffic_summary.py turns the
rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/traffic.sh into calibrated
bytes per launch, and bench.py reads them back into roofline.traffic
(measured_traffic, c4_traffic, c5_traffic).  Synthetic counter files with known
values pin the arithmetic; the committed profiles/r03/traffic.json must give
every bench line a figure."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAL_BYTES = 16384 * (1 << 18)


def _pass(d, sub, rows):
    """One rocprofv3 --pmc pass directory: rows of (kernel name, counter, KB)."""
    os.makedirs(os.path.join(d, sub), exist_ok=True)
    with open(os.path.join(d, sub, "pass_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
        for r in rows:
            w.writerow(r)


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_summary_calibrates_per_shape(tmp_path):
    d = str(tmp_path)
    kb = CAL_BYTES / 1024
    # calibration: octet reads count half (factor 2), writes count whole;
    # lane reads count 1/1.9, writes 1/0.65 (MI355X_MICROARCH.md: FETCH_SIZE is shape-dependent)
    for c, oct_kb, lane_kb in (("FETCH_SIZE", kb / 2, kb / 1.9), ("WRITE_SIZE", kb, kb / 0.65)):
        _pass(d, "cal_" + c, [("k_octet(unsigned char const*, unsigned char*)", c, oct_kb),
                              ("k_lane(unsigned char const*, unsigned char*)", c, lane_kb)])
    # headline seal: 2 launches; config 5: its own directories with the same kernel name
    _pass(d, "bench_FETCH_SIZE", [("void tg::gcm_hy_kernel<10, false, 1024>(...)", "FETCH_SIZE", 8e6)] * 2)
    _pass(d, "bench_WRITE_SIZE", [("void tg::gcm_hy_kernel<10, false, 1024>(...)", "WRITE_SIZE", 16e6)] * 2)
    _pass(d, "c5_FETCH_SIZE", [("void tg::gcm_hy_kernel<10, false, 1024>(...)", "FETCH_SIZE", 9e6),
                               ("tg::seal_prep(tg_records, bool, unsigned int, tg::RecScratch)", "FETCH_SIZE", 100.0)])
    _pass(d, "c5_WRITE_SIZE", [("void tg::gcm_hy_kernel<10, false, 1024>(...)", "WRITE_SIZE", 17e6),
                               ("tg::seal_prep(tg_records, bool, unsigned int, tg::RecScratch)", "WRITE_SIZE", 200.0)])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_summary.py"), d],
                         capture_output=True, text=True, check=True).stdout
    t = json.loads(out)
    assert t["calibration"]["octet"]["fetch_factor"] == pytest.approx(2.0, rel=1e-4)
    assert t["calibration"]["lane"]["write_factor"] == pytest.approx(0.65, rel=1e-4)
    k = t["kernels"]
    assert k["aes128gcm_seal"]["launches"] == 2
    assert k["aes128gcm_seal"]["hbm_bytes"] == pytest.approx(8e6 * 1024 * 2 + 16e6 * 1024, rel=1e-4)
    # config 5's kernels come only from the c5_* passes, not from the headline's
    assert k["c5_seal"]["hbm_bytes"] == pytest.approx(9e6 * 1024 * 2 + 17e6 * 1024, rel=1e-4)
    assert k["c5_prep"]["hbm_bytes"] == pytest.approx(100 * 1024 * 1.9 + 200 * 1024 * 0.65, rel=1e-4)


def test_committed_traffic_feeds_every_bench_line(bench):
    path = os.path.join(ROOT, "profiles", "r03", "traffic.json")
    n, L = 1 << 20, 16384
    for kern in ("aes128gcm_seal", "aes128gcm_open", "chacha20-poly1305_seal", "chacha20-poly1305_open"):
        t = bench.measured_traffic(path, kern, n, L)
        assert t and 0.98 < t["traffic_over_algorithmic"] < 1.1, (kern, t)
    for op in ("seal", "open"):
        t = bench.c4_traffic(path, op)
        assert t and t["hbm_bytes"] > 1e10
    t = bench.c5_traffic(path, n, bench.C5_APP)
    assert t and 0.98 < t["traffic_over_algorithmic"] < 1.1
    # only the default shapes have a measured figure
    assert bench.measured_traffic(path, "aes128gcm_seal", n // 2, L) is None
    assert bench.c5_traffic(path, n // 2, bench.C5_APP) is None
