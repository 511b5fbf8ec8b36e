"""Device-resident AES-128-GCM seal of n x 16 KiB records: the wave-per-record
kernel (TLSGPU_GCM_VARIANT=6) against the hybrid octet kernel (15), to place
kWaveMaxRecords (aes_gcm.hip).  usage: python tools/hy_crossover_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tlslite-ng_amd"))
import torch  # noqa: E402
import tlsgpu  # noqa: E402

L, S = 16384, 16512
obj = tlsgpu.HipAESGCM(bytearray(16))
for n in (256, 1024, 4096, 8192, 16384, 32768, 65536, 131072, 196608):
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytearray(12), 0, n, nonces)
    aad = torch.tensor([23, 3, 3, 0x40, 0x11], dtype=torch.uint8, device="cuda")
    b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L,
                          out_stride=S, fixed_aad_len=5)
    res, ref = [], None
    for v in ("6", "15"):
        os.environ["TLSGPU_GCM_VARIANT"] = v
        for _ in range(2):
            tlsgpu.seal_batch(obj, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            tlsgpu.seal_batch(obj, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        res.append("v%s %.3f ms %.0f GiB/s" % (v, ms, n * L / ms / 1e-3 / 2 ** 30))
        if ref is None:
            ref = out.clone()
        else:
            assert torch.equal(ref, out)
    print("n=%6d  %s" % (n, "   ".join(res)), flush=True)
    del inp, out
