"""libtlsgpu's host half (csrc/host.cpp: AES key schedules, GHASH tables, the
GcmKeyDev image, the record scanner) built with g++ -fsanitize=address,undefined
and driven by tests/native/host_check.cpp (no GPU).  The scanner runs in
exactly-sized heap buffers against the RecordSocket.recv restatement of
test_ingest_host.py (recordlayer.py:169-237) on random, truncated and
oversize-header streams; the C++ fuzz mode adds 10^5 cases per seed with
invariant checks."""
import os
import random
import shutil
import struct
import subprocess

import pytest

from test_ingest_host import _stream, _walk
from tlsgpu import ingest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "tlslite-ng_amd", "csrc")


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("asan") / "host_check")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-Werror",
           "-I" + CSRC, "-I" + os.path.join(ROOT, "include"), "-o", exe,
           os.path.join(HERE, "native", "host_check.cpp"), os.path.join(CSRC, "host.cpp"),
           os.path.join(CSRC, "hostcopy.cpp")]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


def _env():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    return env


def _run(exe, *args, stdin=None):
    return subprocess.run([exe, *args], input=stdin, capture_output=True, timeout=300, env=_env())


def test_sanitizer_is_live(host_check):
    r = _run(host_check, "canary")
    assert r.returncode not in (0, 3, 4)
    # UBSan's object-size check or ASan's heap-buffer-overflow, whichever fires first
    assert b"heap-buffer-overflow" in r.stderr or b"insufficient space" in r.stderr


def test_parallel_copy_clean(host_check):
    """tg_host_copy(_rows)'s splits (hostcopy.cpp) against memcpy, two callers at once."""
    r = _run(host_check, "copy")
    assert r.returncode == 0, (r.stdout.decode()[-2000:], r.stderr.decode()[-3000:])
    assert b"copy ok" in r.stdout


def test_key_setup_clean(host_check):
    r = _run(host_check, "keys")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert r.stdout.strip() == b"keys ok"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_scanner_fuzz_clean(host_check, seed):
    r = _run(host_check, "fuzz", "100000", str(seed))
    assert r.returncode == 0, r.stderr.decode()[-3000:]


def _cases(rng):
    """(bytes, max_body, max_n): well-formed streams cut anywhere, corrupted
    content types, oversize and at-limit lengths, empty input, max_n 0..3."""
    out = []
    limits = (2 ** 14, 2 ** 14 + 256, 2 ** 14 + 2048)
    for i in range(60):
        max_body = limits[i % 3]
        buf = bytearray(_stream(rng, rng.randint(0, 8), max_body))
        kind = i % 6
        if kind == 1 and buf:
            buf = buf[:rng.randrange(len(buf))]                       # truncated anywhere
        elif kind == 2 and buf:
            buf[0] = rng.choice([0, 19, 25, 0x80, 0xff])               # bad content type
        elif kind == 3:
            L = max_body + rng.randint(1, 300)                         # oversize header
            buf += bytes([23, 3, 3, L >> 8, L & 0xff]) + bytes(min(L, 100))
        elif kind == 4:
            buf += bytes([23, 3, 3, max_body >> 8, max_body & 0xff])  # at the limit, body missing
        elif kind == 5:
            buf += bytes([22, 3, 1])                                   # partial header
        for max_n in (64, rng.randint(0, 3)):
            out.append((bytes(buf), max_body, max_n))
    out.append((b"", 2 ** 14, 64))
    out.append((bytes([23, 3, 3, 0, 0]), 0, 64))
    out.append((bytes([23, 3, 3, 0xff, 0xff]) + bytes(0xffff), 0xffff, 64))
    return out


def _expect(buf, max_body, max_n):
    try:
        recs, _ = _walk(buf, max_body)
    except ingest.TLSIllegalParameterException:
        recs, err = None, 1
    except ingest.TLSRecordOverflow:
        recs, err = None, 2
    if recs is None:
        # the scanner stops after max_n records, before reaching a later bad header
        good, pos = [], 0
        while len(good) < max_n and len(buf) - pos >= 5 and buf[pos] in (20, 21, 22, 23, 24) \
                and (buf[pos + 3] << 8 | buf[pos + 4]) <= max_body:
            L = 5 + (buf[pos + 3] << 8 | buf[pos + 4])
            if len(buf) - pos < L:
                break
            good.append((pos, L))
            pos += L
        if len(good) == max_n or len(buf) - pos < 5 or (len(buf) - pos >= 5 and buf[pos] in (
                20, 21, 22, 23, 24) and (buf[pos + 3] << 8 | buf[pos + 4]) <= max_body):
            return "ok %d %d%s" % (len(good), pos, "".join(" %d:%d" % r for r in good))
        return "err %d %d" % (err, len(good))
    recs = recs[:max_n]
    used = sum(r[1] for r in recs)
    return "ok %d %d%s" % (len(recs), used, "".join(" %d:%d" % r for r in recs))


def test_scanner_matches_restatement(host_check):
    cases = _cases(random.Random(2024))
    data = b"".join(struct.pack("<III", mb, mn, len(b)) + b for b, mb, mn in cases)
    r = _run(host_check, "scan", stdin=data)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = r.stdout.decode().splitlines()
    assert len(lines) == len(cases)
    for (buf, mb, mn), line in zip(cases, lines):
        want = _expect(buf, mb, mn)
        got = line if line.startswith("ok") else " ".join(line.split()[:3])
        assert got == want, (mb, mn, len(buf))
