"""Kernel time of the AES-CCM wave kernel for 1 .. 64 records of 16 KiB
(HIP events on the launch stream), for A/B runs of alternative library builds
(TLSGPU_LIB).  usage: python tools/ccm_latency_ab.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tlslite-ng_amd"))
import torch  # noqa: E402

import tlsgpu  # noqa: E402

L, tl = 16384, 16
os.environ["TLSGPU_CCM_VARIANT"] = "2"
o = tlsgpu.HipAESCCM(bytearray(range(16)))
for n in (1, 8, 64):
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
    for name, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
        fn(o, b)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(o, b)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        line.append("%s %.3f ms" % (name, best))
    ok = torch.equal(back, inp) and int(status.sum()) == n
    print("%s n=%3d x 16 KiB: %s roundtrip %s" % (os.environ.get("TLSGPU_LIB", "tree"), n, "  ".join(line), ok),
          flush=True)
