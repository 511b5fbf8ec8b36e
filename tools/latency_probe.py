"""Per-record latency of the drop-in objects (tg_seal / tg_open through the
factory objects, the path recordlayer.py calls once per record)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tlslite-ng_amd"))
import tlsgpu  # noqa: E402

for name, obj in (("aes128gcm", tlsgpu.HipAESGCM(bytearray(16))),
                  ("chacha20-poly1305", tlsgpu.HipCHACHA20_POLY1305(bytearray(32)))):
    for L in (64, 1024, 16384):
        pt = bytearray(os.urandom(L))
        nonce, aad = bytearray(12), bytearray(b"\x17\x03\x03\x40\x10")
        ct = obj.seal(nonce, pt, aad)
        t0 = time.perf_counter()
        for _ in range(50):
            ct = obj.seal(nonce, pt, aad)
        t1 = time.perf_counter()
        for _ in range(50):
            assert obj.open(nonce, ct, aad) == pt
        t2 = time.perf_counter()
        print("%-18s %6d B  seal %7.1f us  open %7.1f us" % (name, L, (t1 - t0) / 50 * 1e6,
                                                          (t2 - t1) / 50 * 1e6))
