"""Key-table cost at the long-record end of config 4: AES-256-GCM seal of
2^20 x 16 KiB records (80 % of config 4's bytes are 16 KiB records) through
the key-grouped kernel at each lanes-per-record choice over 65 536 keys,
against the same records under one key (bs8 octet kernel alone, and the
hybrid).  HIP-event times on torch's current stream, mean of 3.
usage: python tools/kt_ceiling_probe.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tlslite-ng_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tlsgpu  # noqa: E402

nkeys, L, n = 65536, 16384, 1 << 20
rng = np.random.default_rng(1)
keys = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
table = tlsgpu.KeyTable("aesgcm", [bytes(k) for k in keys])
single = tlsgpu.HipAESGCM(bytearray(bytes(keys[0])))
kidx = torch.from_numpy(rng.integers(0, nkeys, n).astype(np.int32)).cuda()
inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
tlsgpu.make_nonces(bytes(12), 0, n, nonces)
aad = torch.zeros(13, dtype=torch.uint8, device="cuda")
out = torch.empty(n * (L + 16), dtype=torch.uint8, device="cuda")
lens = torch.full((n,), L, dtype=torch.int32, device="cuda")


def timed(key, b):
    tlsgpu.seal_batch(key, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        tlsgpu.seal_batch(key, b)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 3


bk = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, lens=lens, in_stride=L, out_stride=L + 16,
                       fixed_aad_len=13, key_idx=kidx)
bs = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=L + 16,
                       fixed_aad_len=13)
rows = []
for name, key, b, opts in (("single hybrid", single, bs, {}),
                           ("single bs8", single, bs, {"gcm_variant": 14}),
                           ("kt lpr 8", table, bk, {"kt_lpr": 8}),
                           ("kt lpr 16", table, bk, {"kt_lpr": 16}),
                           ("kt lpr 32", table, bk, {"kt_lpr": 32}),
                           ("kt lpr 64", table, bk, {"kt_lpr": 64})):
    for o, v in opts.items():
        tlsgpu.set_option(o, v)
    ms = timed(key, b)
    for o in opts:
        tlsgpu.set_option(o, 0)
    print("%-14s %7.3f ms %7.1f GiB/s" % (name, ms, n * L / ms / 1e-3 / 2 ** 30), flush=True)
