"""AES-128-CCM batch throughput, 2^18 x 16 KiB records, counter-window cache
(default) against full rounds (TLSGPU_CCM_VARIANT=1); HIP-event times on the
launch stream.  usage: python tools/ccm_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tlslite-ng_amd"))
import torch  # noqa: E402

import tlsgpu  # noqa: E402

n, L, tl = 1 << 18, 16384, 16
inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
o = tlsgpu.HipAESCCM(bytearray(range(16)))
nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
tlsgpu.make_nonces(bytes(12), 0, n, nonces)
aad = torch.tensor([0x17, 3, 3, (L + tl) >> 8, (L + tl) & 0xff], dtype=torch.uint8, device="cuda")
sealed = torch.empty(n * (L + tl), dtype=torch.uint8, device="cuda")
back = torch.empty_like(inp)
sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                       out_stride=L + tl, fixed_aad_len=5)
status = torch.zeros(n, dtype=torch.uint8, device="cuda")
ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=L + tl,
                       out_stride=L, fixed_aad_len=5, status=status)
for variant in ("0", "1", "0", "1"):
    os.environ["TLSGPU_CCM_VARIANT"] = variant
    res = []
    for name, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
        fn(o, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn(o, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        res.append("%s %.2f ms %.1f GiB/s" % (name, ms, n * L / ms / 1e-3 / 2 ** 30))
    assert torch.equal(back, inp) and int(status.sum()) == n
    print("variant %s (%s): %s" % (variant, "windows" if variant == "0" else "full rounds",
                                   "  ".join(res)), flush=True)
