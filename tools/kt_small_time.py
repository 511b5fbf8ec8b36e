"""Latency of small key-table AES-GCM batches (the key-job plan's
cost on them): the same records -- ``n`` TLS 1.3 records of L bytes, 64
AES-128 session keys, random key_idx -- through the automatic choice (with one
fixed length and with a per-record length array), the lane kernel after the
plan (gcm_table_variant 1), and the wave-per-record kernels (variants 5, 6).  HIP events around each call on
the launch stream; mean and best of --reps calls after one warm-up; every run
opens its records back.

    python tools/kt_small_time.py [--reps 20] [--len 1024]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--len", type=int, default=1024)
    ap.add_argument("--max-records", type=int, default=65536)
    ap.add_argument("--alg", default="aesgcm", choices=["aesgcm", "chacha20-poly1305"])
    args = ap.parse_args()
    import torch
    import tlsgpu
    from vectors import tls13_aad
    L, so = args.len, (args.len + 16 + 15) // 16 * 16
    keys = [bytes([k]) * (16 if args.alg == "aesgcm" else 32) for k in range(64)]
    kt = tlsgpu.KeyTable(args.alg, keys)
    stream = torch.cuda.current_stream()
    out = []
    for n in [m for m in (1, 16, 256, 2048, 8192, 16384, 65536) if m <= args.max_records]:
        g = torch.Generator(device="cuda").manual_seed(n)
        inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
        sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
        back = torch.empty_like(inp)
        status = torch.zeros(n, dtype=torch.uint8, device="cuda")
        nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
        tlsgpu.make_nonces(bytes(range(12)), 0, n, nonces)
        aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
        kidx = torch.randint(0, 64, (n,), dtype=torch.int32, device="cuda", generator=g)
        lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
        row = {"records": n, "len": L}
        modes = ((("auto, one length", True, {}), ("auto, length array", False, {}),
                  ("lane kernel after the plan (variant 1, length array)", False, {"gcm_table_variant": 1}),
                  ("wave kernel, table-free GHASH (variant 5)", True, {"gcm_table_variant": 5}),
                  ("wave kernel, 4-bit tables (variant 6)", True, {"gcm_table_variant": 6}))
                 if args.alg == "aesgcm" else
                 (("auto, one length", True, {}), ("auto, length array", False, {}),
                  ("lane kernel (chacha_variant 5)", False, {"chacha_variant": 5}),
                  ("wave kernel (chacha_variant 3)", True, {"chacha_variant": 3})))
        for mode, fixed, opts in modes:
            kw = {"fixed_len": L} if fixed else {"lens": lens}
            sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, in_stride=L, out_stride=so,
                                   fixed_aad_len=5, key_idx=kidx, **kw)
            ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, in_stride=so, out_stride=L,
                                   fixed_aad_len=5, key_idx=kidx, status=status, **kw)
            with tlsgpu.options(**opts):
                tlsgpu.seal_batch(kt, sb, stream)
                ev = []
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    tlsgpu.seal_batch(kt, sb, stream)
                    b.record(stream)
                    ev.append((a, b))
                status.zero_()
                back.zero_()
                tlsgpu.open_batch(kt, ob, stream)
                torch.cuda.synchronize()
            ms = [a.elapsed_time(b) for a, b in ev]
            row[mode] = {"mean_ms": round(sum(ms) / len(ms), 4), "best_ms": round(min(ms), 4),
                         "roundtrip_ok": int(status.sum()) == n and bool(torch.equal(back, inp))}
        out.append(row)
        print(json.dumps(row))


if __name__ == "__main__":
    main()
