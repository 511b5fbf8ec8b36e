"""A library built with a measurement-only flag (tools/build_variant.sh
-DTG_CHACHA_NO_IO / TG_CHACHA_ILV / TG_KT_NO_GHASH / TG_KT_NO_BUILD /
TG_NT_IO) may return wrong bytes; it carries a marker in tg_version() and
tlsgpu.load() refuses it unless TLSGPU_ALLOW_MEASUREMENT_BUILD=1.  The
default build carries no marker.  CPU only: loading needs no GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = ("import sys; sys.path.insert(0, %r); import tlsgpu\n"
         "try:\n    l = tlsgpu._lib.load()\nexcept OSError as e:\n    print('REFUSED', e); sys.exit(0)\n"
         "print('LOADED', l.tg_version().decode())\n") % os.path.join(ROOT, "tlslite-ng_amd")


def _probe(lib=None, allow=False):
    env = dict(os.environ)
    env.pop("TLSGPU_LIB", None)
    env.pop("TLSGPU_ALLOW_MEASUREMENT_BUILD", None)
    if lib:
        env["TLSGPU_LIB"] = lib
    if allow:
        env["TLSGPU_ALLOW_MEASUREMENT_BUILD"] = "1"
    return subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True,
                          check=True).stdout


def test_default_build_has_no_marker():
    out = _probe()
    assert out.startswith("LOADED") and "MEASUREMENT" not in out


@pytest.mark.parametrize("flag", ["TG_NT_IO", "TG_KT_NO_GHASH"])
def test_measurement_build_refused(tmp_path, flag):
    if not os.path.isdir(os.path.join(ROOT, "tlslite-ng_amd", "csrc", "obj")):
        pytest.skip("library objects not built")
    # selftest.hip is the smallest translation unit; the marker comes from
    # common.h, which every .hip includes
    so = str(tmp_path / "libtlsgpu_meas.so")
    subprocess.run(["bash", os.path.join(ROOT, "tools", "build_variant.sh"), "selftest", so,
                    "-D" + flag], check=True, capture_output=True)
    out = _probe(so)
    assert out.startswith("REFUSED") and flag in out
    out = _probe(so, allow=True)
    assert out.startswith("LOADED") and "MEASUREMENT BUILD" in out and flag in out
