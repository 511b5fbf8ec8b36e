"""CPU checks of the C-ABI boundary: the library loads, exports every symbol
include/tlsgpu.h declares, the ctypes struct matches the C layout, and the
host-side argument conventions (reference error classes) hold without a GPU.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tlsgpu.h")


def _declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(tg_\w+)\s*\(", text, re.M)))


def test_header_matches_binding_list():
    from tlsgpu import _lib
    assert _declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    from tlsgpu import _lib
    lib = _lib.load()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert lib.tg_version().startswith(b"tlsgpu")


def test_no_device_is_reported_not_crashed():
    from tlsgpu import _lib
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    assert _lib.device_count() == 0


def test_struct_layout_matches_c(tmp_path):
    from tlsgpu import _lib
    fields = [f[0] for f in _lib.TgBatch._fields_]
    cnames = ["in" if f == "inp" else f for f in fields]
    src = tmp_path / "layout.c"
    body = "".join('printf("%%zu\\n", offsetof(tg_batch, %s));\n' % c for c in cnames)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tlsgpu.h"\n'
                   'int main(void){printf("%%zu\\n", sizeof(tg_batch));\n%sreturn 0;}\n' % body)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert out[0] == ctypes.sizeof(_lib.TgBatch)
    for (name, _), off in zip(_lib.TgBatch._fields_, out[1:]):
        assert getattr(_lib.TgBatch, name).offset == off, name


def test_records_struct_layout_matches_c(tmp_path):
    from tlsgpu import _lib
    names = [f[0] for f in _lib.TgRecords._fields_]
    body = "".join('printf("%%zu\\n", offsetof(tg_records, %s));\n' % c for c in names)
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tlsgpu.h"\n'
                   'int main(void){printf("%%zu\\n", sizeof(tg_records));\n%sreturn 0;}\n' % body)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert out[0] == ctypes.sizeof(_lib.TgRecords)
    for name, off in zip(names, out[1:]):
        assert getattr(_lib.TgRecords, name).offset == off, name


def test_key_length_errors_match_reference():
    from tlsgpu import HipAESGCM, HipCHACHA20_POLY1305
    with pytest.raises(AssertionError):        # aesgcm.py:37-38
        HipAESGCM(bytearray(8))
    with pytest.raises(AssertionError):
        HipAESGCM(bytearray(24))
    with pytest.raises(ValueError):            # chacha20_poly1305.py:21-22
        HipCHACHA20_POLY1305(bytearray(16))


def test_factory_without_backend_raises_not_implemented():
    from tlsgpu import cipherfactory, device_count
    if device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(NotImplementedError):
        cipherfactory.createAESGCM(bytearray(16))
    with pytest.raises(NotImplementedError):
        cipherfactory.createCHACHA20(bytearray(32), ["python"])


def test_header_compiles_as_c_and_cpp():
    with tempfile.TemporaryDirectory() as d:
        for comp, ext in (("gcc", "c"), ("g++", "cpp")):
            src = os.path.join(d, "h." + ext)
            with open(src, "w") as f:
                f.write('#include "tlsgpu.h"\nint main(void){tg_batch b; (void)b; return 0;}\n')
            subprocess.check_call([comp, "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                                   src, "-o", os.path.join(d, "h_" + ext)])
