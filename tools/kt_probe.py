"""Key-table AES-256-GCM seal time by record length: the lane-per-record
kernel (gcm_table_variant 1) against the key-grouped octet kernel (14)
on 65 536 keys with uniformly random key_idx, fixed-length batches of
64 B .. 16 KiB.  HIP-event times on the launch stream (torch's current).
usage: python tools/kt_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tlslite-ng_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tlsgpu  # noqa: E402

nkeys = 65536
rng = np.random.default_rng(1)
table = tlsgpu.KeyTable("aesgcm", [bytes(k) for k in rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)])
for L, n in ((16384, 1 << 18), (4096, 1 << 20), (1024, 1 << 20), (256, 1 << 20), (64, 1 << 20)):
    kidx = torch.from_numpy(rng.integers(0, nkeys, n).astype(np.int32)).cuda()
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(12), 0, n, nonces)
    aad = torch.zeros(13, dtype=torch.uint8, device="cuda")
    out = torch.empty(n * (L + 16), dtype=torch.uint8, device="cuda")
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, lens=lens, in_stride=L, out_stride=L + 16,
                          fixed_aad_len=13, key_idx=kidx)
    row = []
    for v in ("1", "14"):
        tlsgpu.set_option("gcm_table_variant", int(v))
        tlsgpu.seal_batch(table, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            tlsgpu.seal_batch(table, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        row.append("v%s %.3f ms %.1f GiB/s" % (v, ms, n * L / ms / 1e-3 / 2 ** 30))
    print("L=%5d n=%7d  %s" % (L, n, "   ".join(row)), flush=True)
    del inp, out
