"""Time the headline AES-128-GCM seal and open (2^20 x 16 KiB records, TLS 1.3
AAD, sealed records at a 128-byte stride, device resident) with HIP events on
the launch stream: best and mean of --reps launches each.  For same-box A/B
runs of alternative builds (TLSGPU_LIB); correctness is the -m gpu tests' job,
but every run checks its own round trip (status and plaintext).

    python tools/aes_time.py [--reps 5] [--records N] [--keylen 16]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--keylen", type=int, default=16)
    ap.add_argument("--chacha", action="store_true")
    args = ap.parse_args()
    import torch
    import tlsgpu
    from vectors import tls13_aad
    n, L = args.records, 16384
    so = (L + 16 + 127) // 128 * 128
    g = torch.Generator(device="cuda").manual_seed(0x7715)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(range(12)), 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    key = (tlsgpu.HipCHACHA20_POLY1305(bytearray(range(32))) if args.chacha
           else tlsgpu.HipAESGCM(bytearray(range(args.keylen))))
    sb = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                           out_stride=so, fixed_aad_len=5)
    ob = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=so,
                           out_stride=L, fixed_aad_len=5, status=status)
    stream = torch.cuda.current_stream()
    res = {}
    for name, batch, fn in (("seal", sb, tlsgpu.seal_batch), ("open", ob, tlsgpu.open_batch)):
        fn(key, batch, stream)
        ev = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn(key, batch, stream)
            b.record(stream)
            ev.append((a, b))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        res[name] = {"best": round(min(ms), 3), "mean": round(sum(ms) / len(ms), 3)}
    ok = int(status.sum()) == n and bool(torch.equal(back, inp))
    res["roundtrip_ok"] = ok
    res["lib"] = os.environ.get("TLSGPU_LIB", "tree")
    opts = {k: v for k, v in os.environ.items() if k.startswith("TLSGPU_") and k != "TLSGPU_LIB"}
    if opts:
        res["options"] = opts
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
