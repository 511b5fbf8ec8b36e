"""AES-128-CCM latency of small batches and the per-record call: the wave-per-
record kernel (ccm_variant 2) against the lane kernel (3), HIP-event
times on the launch stream, and createAESCCM(...).seal / open wall time for one
16 KiB record (host buffers, the drop-in path).  usage: python tools/ccm_wave_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tlslite-ng_amd"))
import torch  # noqa: E402

import tlsgpu  # noqa: E402

L, tl = 16384, 16
o = tlsgpu.HipAESCCM(bytearray(range(16)))
for n in (1, 8, 64, 512, 2048, 4096, 8192):
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(12), 0, n, nonces)
    aad = torch.tensor([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff], dtype=torch.uint8, device="cuda")
    sealed = torch.empty(n * (L + tl), dtype=torch.uint8, device="cuda")
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                           out_stride=L + tl, fixed_aad_len=5)
    ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=L + tl,
                           out_stride=L, fixed_aad_len=5, status=status)
    line = []
    ref = None
    for variant in ("2", "3"):
        tlsgpu.set_option("ccm_variant", int(variant))
        for name, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
            fn(o, b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn(o, b)
            e1.record()
            torch.cuda.synchronize()
            line.append("v%s %s %.3f ms" % (variant, name, e0.elapsed_time(e1) / 3))
        assert torch.equal(back, inp) and int(status.sum()) == n
        if ref is None:
            ref = sealed.clone()
        else:
            assert torch.equal(ref, sealed)
    print("n=%5d x 16 KiB: %s" % (n, "  ".join(line)), flush=True)
tlsgpu.set_option("ccm_variant", 0)
c = tlsgpu.createAESCCM(bytearray(range(16)))
pt = bytearray(os.urandom(L))
nonce = bytearray(12)
hdr = bytearray([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff])
for _ in range(3):
    ct = c.seal(nonce, pt, hdr)
t0 = time.perf_counter()
for _ in range(20):
    ct = c.seal(nonce, pt, hdr)
t1 = time.perf_counter()
for _ in range(20):
    back = c.open(nonce, ct, hdr)
t2 = time.perf_counter()
assert back == pt
print("per-record 16 KiB AES-128-CCM: seal %.3f ms  open %.3f ms (host buffers)" %
      ((t1 - t0) / 20 * 1e3, (t2 - t1) / 20 * 1e3), flush=True)
