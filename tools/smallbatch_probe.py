"""Device-resident throughput of small batches of 16 KiB records by kernel
choice: record per lane (GCM variant 7 / ChaCha 4), one wave per record, four
waves per record.  Sets the auto thresholds in aes_gcm.hip / chacha_poly.hip."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tlslite-ng_amd"))
import torch  # noqa: E402
import tlsgpu  # noqa: E402

L, S = 16384, 16512
REPS = 5


def run(obj, n, opts):
    with tlsgpu.options(**opts):
        inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
        out = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
        tlsgpu.make_nonces(bytearray(12), 0, n, nonces)
        aad = torch.tensor([23, 3, 3, 0x40, 0x11], dtype=torch.uint8, device="cuda")
        b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L,
                              out_stride=S, fixed_aad_len=5)
        for _ in range(3):
            tlsgpu.seal_batch(obj, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            tlsgpu.seal_batch(obj, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / REPS * 1e3
        return us, n * L / (us * 1e-6) / 2 ** 30


for name, obj, var, lane_v, wave_v in (
        ("aes128gcm", tlsgpu.HipAESGCM(bytearray(16)), "gcm_variant", 16, 6),
        ("chacha20-poly1305", tlsgpu.HipCHACHA20_POLY1305(bytearray(32)),
         "chacha_variant", 4, 3)):
    for n in (1, 4, 16, 64, 128, 256, 512, 1024, 2048, 4096, 16384, 65536):
        cols = []
        for label, env in (("lane", {var: lane_v}),
                           ("wave1", {var: wave_v, "waves_per_record": 1}),
                           ("wave4", {var: wave_v, "waves_per_record": 4}),
                           ("wave16", {var: wave_v, "waves_per_record": 16})):
            us, g = run(obj, n, env)
            cols.append("%s %8.1f us %7.1f GiB/s" % (label, us, g))
        print("%-18s n=%5d  %s" % (name, n, "  ".join(cols)), flush=True)

# where a record per lane overtakes a wave per record
for name, obj, var, lane_v, wave_v in (
        ("aes128gcm", tlsgpu.HipAESGCM(bytearray(16)), "gcm_variant", 16, 6),
        ("chacha20-poly1305", tlsgpu.HipCHACHA20_POLY1305(bytearray(32)),
         "chacha_variant", 4, 3)):
    for n in (32768, 65536, 98304, 131072, 163840, 196608, 262144, 524288, 1048576):
        cols = []
        for label, env in (("lane", {var: lane_v}),
                           ("wave1", {var: wave_v, "waves_per_record": 1})):
            us, g = run(obj, n, env)
            cols.append("%s %8.1f us %7.1f GiB/s" % (label, us, g))
        print("%-18s n=%7d  %s" % (name, n, "  ".join(cols)), flush=True)
        torch.cuda.empty_cache()
