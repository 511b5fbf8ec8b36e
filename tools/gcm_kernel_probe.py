"""Time the single-key AES-GCM kernels against each other at the headline
shape (2^20 x 16 KiB, TLS 1.3 AAD, 128-byte aligned sealed records), device
resident, and check that every kernel's sealed bytes equal the first one's
(the T-table kernel, itself pinned to the oracle by the -m gpu tests).

    python tools/gcm_kernel_probe.py "0" "14" "15:hy_t=8" ...

Each argument is VARIANT[:OPTION=VALUE,...] (the gcm_variant option and extra
tlsgpu options, include/tlsgpu.h tg_set_option).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import tlsgpu  # noqa: E402
from vectors import tls13_aad  # noqa: E402


def main():
    n = int(os.environ.get("PROBE_RECORDS", 1 << 20))
    L = 16384
    steps = int(os.environ.get("PROBE_STEPS", 3))
    klen = int(os.environ.get("PROBE_KEYLEN", 16))
    so = (L + 16 + 127) // 128 * 128
    g = torch.Generator(device="cuda").manual_seed(0x7715)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(range(12)), 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    key = tlsgpu.HipAESGCM(bytearray(range(klen)))
    sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                           out_stride=so, fixed_aad_len=5)
    ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=so,
                           out_stride=L, fixed_aad_len=5, status=status)
    ref = None
    for arg in sys.argv[1:]:
        var, _, extra = arg.partition(":")
        opts = {"gcm_variant": int(var)}
        for kv in filter(None, extra.split(",")):
            k, v = kv.split("=")
            opts[k] = int(v)
        ctx = tlsgpu.options(**opts)
        ctx.__enter__()
        times = {}
        for name, batch, fn in (("seal", sb, tlsgpu.seal_batch), ("open", ob, tlsgpu.open_batch)):
            fn(key, batch)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(steps):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fn(key, batch)
                b.record()
                b.synchronize()
                best = min(best, a.elapsed_time(b))
            times[name] = best
        ok_rt = bool(torch.equal(back, inp)) and int(status.sum()) == n
        digest = torch.stack([sealed[i * so:i * so + L + 16].to(torch.int64).sum()
                              for i in range(0, n, max(1, n // 64))]).cpu()
        tags = sealed.view(n, so)[:, L:L + 16].clone()
        if ref is None:
            ref = (digest, tags)
        same = bool(torch.equal(digest, ref[0])) and bool(torch.equal(tags, ref[1]))
        gib = n * L / 2**30
        print("%-24s seal %7.3f ms (%6.1f GiB/s)  open %7.3f ms (%6.1f GiB/s)  roundtrip %s  same-as-first %s"
              % (arg, times["seal"], gib / times["seal"] * 1e3, times["open"],
                 gib / times["open"] * 1e3, ok_rt, same), flush=True)
        ctx.__exit__(None, None, None)


if __name__ == "__main__":
    main()
