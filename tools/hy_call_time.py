"""Per-call time of the single-key hybrid AES-GCM kernel on mid-size batches
(the per-launch scratch): 24 577 .. 65 536 records of
16 KiB, seal and open, back-to-back calls on one stream timed with HIP events
(launch overheads included) and the host wall time per call.

    python tools/hy_call_time.py [n ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import tlsgpu  # noqa: E402

L, S, REPS = 16384, 16512, 20


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [24577, 32768, 65536]
    key = tlsgpu.HipAESGCM(bytearray(range(16)))
    res = {"lib": os.environ.get("TLSGPU_LIB", "tree")}
    for n in sizes:
        inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
        out = torch.empty(n * S, dtype=torch.uint8, device="cuda")
        back = torch.empty_like(inp)
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
        tlsgpu.make_nonces(bytearray(12), 0, n, nonces)
        aad = torch.tensor([23, 3, 3, 0x40, 0x10], dtype=torch.uint8, device="cuda")
        sb = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=S,
                               fixed_aad_len=5)
        ob = tlsgpu.make_batch(n, out, back, nonces, aad=aad, fixed_len=L, in_stride=S, out_stride=L,
                               fixed_aad_len=5, status=st)
        stream = torch.cuda.current_stream()
        row = {}
        for name, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
            for _ in range(3):
                fn(key, b, stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            for _ in range(REPS):
                fn(key, b, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / REPS * 1e3
            row[name] = {"ms": round(e0.elapsed_time(e1) / REPS, 4), "wall_ms": round(wall, 4)}
        row["roundtrip_ok"] = int(st.sum()) == n and bool(torch.equal(back, inp))
        res[str(n)] = row
        del inp, out, back
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
