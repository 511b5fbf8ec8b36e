"""CPU check of the 8-block bitsliced AES core (csrc/aes_bs8.h) that the
bitsliced AES-GCM kernel runs: compiled with g++ against the C oracle's AES
(rijndael.py:922-1038 restated) for AES-128/256, every lane start the kernel
uses and batch indices around every counter carry (tests/native/bs8_check.cpp),
with the round keys added plainly and folded into MixColumns (keymath.h
bs8_fold_word, the hybrid kernel's default).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bs8_core_matches_oracle(tmp_path):
    exe = str(tmp_path / "bs8_check")
    subprocess.check_call(
        ["g++", "-O2", "-Wall", "-Wno-unknown-pragmas", "-I",
         os.path.join(ROOT, "tlslite-ng_amd", "csrc"), "-I", os.path.join(ROOT, "oracle"),
         "-o", exe, os.path.join(ROOT, "tests", "native", "bs8_check.cpp"),
         "-x", "c", os.path.join(ROOT, "oracle", "aead_oracle.c"), "-lpthread"])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK")
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("NR=")]
    assert lines and all(ln.endswith("bad=0") for ln in lines), out.stdout
    assert any("fold=1" in ln for ln in lines) and any("fold=0" in ln for ln in lines)
