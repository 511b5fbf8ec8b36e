"""Time the ChaCha20-Poly1305 lane kernel (seal and open) at the headline shape
(2^20 x 16 KiB, TLS 1.3 AAD, 128-byte aligned sealed records), HIP events on
the launch stream, without checking results -- for A/B runs of measurement
builds (TLSGPU_LIB), e.g. the I/O ablations.  usage: python tools/chacha_time_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import tlsgpu  # noqa: E402
from vectors import tls13_aad  # noqa: E402

n, L = 1 << 20, 16384
so = (L + 16 + 127) // 128 * 128
inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
back = torch.empty_like(inp)
status = torch.zeros(n, dtype=torch.uint8, device="cuda")
nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
tlsgpu.make_nonces(bytes(range(12)), 0, n, nonces)
aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
key = tlsgpu.HipCHACHA20_POLY1305(bytearray(range(32)))
sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=so, fixed_aad_len=5)
ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=so, out_stride=L,
                       fixed_aad_len=5, status=status)
res = []
for name, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
    fn(key, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        fn(key, b)
    e1.record()
    torch.cuda.synchronize()
    res.append("%s %.3f ms" % (name, e0.elapsed_time(e1) / 3))
print("%-40s %s" % (os.environ.get("TLSGPU_LIB", "tree"), "  ".join(res)), flush=True)
