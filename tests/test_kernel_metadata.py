"""CPU check of the built library's code-object metadata:
the default headline kernels -- the hybrid AES-GCM kernel at 1 024 threads and
the ChaCha20-Poly1305 lane kernel with the LDS-DMA tile, single key, seal and
open -- spill no VGPRs and have no private segment.  A kernel with a private
segment makes the HIP runtime allocate scratch for every queue it runs on
(3.0 MiB per stream, profiles/r06/x10/stream_mem.jsonl); without one, device
memory stays flat however many streams a caller uses (test_gpu_scratch.py).

The metadata comes out of the library's offload bundle with the ROCm LLVM
tools (llvm-objcopy, clang-offload-bundler, llvm-readelf); no GPU is needed.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "tlslite-ng_amd", "tlsgpu", "libtlsgpu.so")


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    tools = [_tool(n) for n in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(tools) or not os.path.exists(LIB):
        pytest.skip("ROCm LLVM tools or the built library not present")
    objcopy, bundler, readelf = tools
    d = tmp_path_factory.mktemp("meta")
    fb = str(d / "fb.bin")
    subprocess.run([objcopy, "--dump-section=.hip_fatbin=" + fb, LIB, str(d / "j.so")], check=True)
    # the section holds one offload bundle per object file, back to back
    blob = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    assert starts, "no offload bundle in " + LIB
    notes = ""
    for n, a in enumerate(starts):
        part, co = str(d / ("b%d.bin" % n)), str(d / ("k%d.co" % n))
        open(part, "wb").write(blob[a:starts[n + 1] if n + 1 < len(starts) else len(blob)])
        subprocess.run([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + part,
                        "--output=" + co, "--unbundle"], check=True)
        notes += subprocess.run([readelf, "--notes", co], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|vgpr_spill_count|private_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name":
            cur = out.setdefault(v, {})
        elif cur is not None:
            cur[k] = int(v)
    return out


# mangled-name fragments: gcm_hy_kernel<NR, OPEN, 1024>, chacha_kernel<OPEN, false, 4, true>
HEADLINE = {
    "gcm_hy_kernel<10, seal, 1024>": "13gcm_hy_kernelILi10ELb0ELi1024EE",
    "gcm_hy_kernel<10, open, 1024>": "13gcm_hy_kernelILi10ELb1ELi1024EE",
    "gcm_hy_kernel<14, seal, 1024>": "13gcm_hy_kernelILi14ELb0ELi1024EE",
    "gcm_hy_kernel<14, open, 1024>": "13gcm_hy_kernelILi14ELb1ELi1024EE",
    "chacha_kernel<seal, single key, DMA>": "13chacha_kernelILb0ELb0ELi4ELb1EE",
    "chacha_kernel<open, single key, DMA>": "13chacha_kernelILb1ELb0ELi4ELb1EE",
}


@pytest.mark.parametrize("label", sorted(HEADLINE))
def test_headline_kernel_has_no_private_segment(kernels, label):
    frag = HEADLINE[label]
    found = [v for k, v in kernels.items() if frag in k]
    assert len(found) == 1, (label, len(found))
    meta = found[0]
    assert meta["vgpr_spill_count"] == 0, (label, meta)
    assert meta["private_segment_fixed_size"] == 0, (label, meta)
