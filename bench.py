"""bench.py -- device-resident TLS record seal/open throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident record seal/open, AES-128-GCM +
ChaCha20-Poly1305, 16 KiB records.  Workload: BASELINE configs[1] and [2]
(single session key, 2^20 x 16 KiB TLS 1.3 records per GPU, nonce = iv xor
seq, 5-byte AAD) -- one "step" seals the whole batch and opens it back, for
AES-128-GCM and for ChaCha20-Poly1305 (4 kernel launches, 4 x 16 GiB of
payload).  ``value`` = payload bytes (plaintext for seal, same L for open)
of all ranks / max-over-ranks time, in GiB/s.

Multi-GPU (``torch.distributed.run``): every rank seals its own contiguous
seq range (weak scaling); the only collective is an RCCL all-reduce of the
per-rank counters {records, payload bytes, auth failures} and the timing max.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--records R] [--len L]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
AAD_LEN = 5
NONCE_LEN = 12
TAG_LEN = 16


def algorithmic_bytes(n, L, op):
    """seal reads L + A + 12, writes L + 16; open reads
    L + 16 + A + 12, writes L (+1 status byte)."""
    per = 2 * L + AAD_LEN + NONCE_LEN + TAG_LEN + (1 if op == "open" else 0)
    return n * per


# ------------------------------------------------------------- CPU baseline

def _cpu_worker(args):
    nrec, L, seed = args
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import pyaead
    from vectors import tls13_aad, tls13_nonce
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    done = 0
    for alg in ("aes128gcm", "chacha20-poly1305"):
        key = rng.bytes(16 if alg == "aes128gcm" else 32)
        iv = rng.bytes(12)
        c = pyaead.AESGCM(key) if alg == "aes128gcm" else pyaead.CHACHA20_POLY1305(key)
        for i in range(nrec):
            pt = rng.bytes(L)
            nonce = tls13_nonce(iv, i)
            aad = tls13_aad(L)
            sealed = c.seal(nonce, pt, aad)
            assert c.open(nonce, sealed, aad) == pt
            done += 2 * L
    return done, time.perf_counter() - t0


def cpu_baseline(L, cores, nrec):
    """The reference's pure-Python path (oracle/pyaead.py restates it; it runs
    at 0.6-1.0x the reference's own per-core speed) on ``cores``
    host processes, seal+open of ``nrec`` records per algorithm per process."""
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(nrec, L, 1000 + c) for c in range(cores)])
    wall = time.perf_counter() - t0
    total = sum(r[0] for r in res)
    return {"value": total / wall / 2 ** 30, "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": "%d procs x %d x %d B records, AES-128-GCM + ChaCha20-Poly1305 seal+open, "
                      "oracle/pyaead.py (pure-Python restatement of the reference path); "
                      "%.1f s wall" % (cores, nrec, L, wall)}


# -------------------------------------------------------------- GPU bench

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--len", type=int, default=16384)
    ap.add_argument("--cpu-cores", type=int, default=16)
    ap.add_argument("--cpu-records", type=int, default=6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time the host<->device path")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "r01", "traffic.json"),
                    help="per-launch HBM bytes from tools/traffic.sh (rocprofv3 FETCH_SIZE / "
                         "WRITE_SIZE passes at this config) for roofline.traffic")
    ap.add_argument("--record-align", type=int, default=128,
                    help="byte alignment of each sealed record (ct||tag) in the packed batch")
    ap.add_argument("--config", default="headline", choices=["headline", "c4", "c5", "ingest"],
                    help="headline = BASELINE configs[1]+[2] (the metric); c4 = configs[3] "
                         "(AES-256-GCM, 65536 keys, Zipf lengths); c5 = configs[4] (TLS 1.3 "
                         "AES-128-GCM seal, 16385-byte inner plaintext, seq-sharded); ingest = "
                         "the host ingest pipeline (tlsgpu.ingest, SURVEY 8(f) row 3), host "
                         "memory to host memory")
    ap.add_argument("--c4-presorted", action="store_true",
                    help="config 4: pack records longest first on the host")
    ap.add_argument("--ingest-mib", type=int, default=2048,
                    help="application data per direction for --config ingest")
    args = ap.parse_args()
    if args.config == "ingest":
        return run_ingest(args)
    if args.config == "c4":
        return run_config4(args)
    if args.config == "c5":
        return run_config5(args)

    import torch
    import torch.distributed as dist
    import tlsgpu
    from vectors import tls13_aad

    world, rank, local = init_dist(torch, dist)

    n, L = args.records, args.len
    # sealed records are ct||tag (the wire form), packed at a stride rounded up
    # to --record-align bytes so every record starts on an HBM line boundary
    SL = (L + TAG_LEN + args.record_align - 1) // args.record_align * args.record_align
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0x7715 + rank)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    sealed = torch.empty(n * SL, dtype=torch.uint8, device=dev)
    back = torch.empty(n * L, dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    nonces = torch.empty(NONCE_LEN * n, dtype=torch.uint8, device=dev)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device=dev)
    hrng = torch.Generator().manual_seed(0x7716)
    iv = bytes(torch.randint(0, 256, (12,), dtype=torch.uint8, generator=hrng).tolist())
    keys = {"aes128gcm": bytes(torch.randint(0, 256, (16,), dtype=torch.uint8, generator=hrng).tolist()),
            "chacha20-poly1305": bytes(torch.randint(0, 256, (32,), dtype=torch.uint8,
                                                     generator=hrng).tolist())}
    ciphers = {"aes128gcm": tlsgpu.HipAESGCM(bytearray(keys["aes128gcm"])),
               "chacha20-poly1305": tlsgpu.HipCHACHA20_POLY1305(bytearray(keys["chacha20-poly1305"]))}
    # this rank's records are seq [rank*n, (rank+1)*n) of one connection
    tlsgpu.make_nonces(iv, rank * n, n, nonces)
    seal_b = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                               out_stride=SL, fixed_aad_len=AAD_LEN)
    open_b = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L,
                               in_stride=SL, out_stride=L, fixed_aad_len=AAD_LEN,
                               status=status)
    stream = torch.cuda.current_stream()
    kinds = [(a, op) for a in ciphers for op in ("seal", "open")]
    ev = {k: [] for k in kinds}

    def step(record):
        for a, c in ciphers.items():
            for op, fn, b in (("seal", tlsgpu.seal_batch, seal_b), ("open", tlsgpu.open_batch, open_b)):
                if record:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                fn(c, b, stream)
                if record:
                    e1.record(stream)
                    ev[(a, op)].append((e0, e1))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # correctness of the timed work (not timed): every record authentic, round trip exact
    ok = int(status.sum().item()) == n and torch.equal(back, inp)
    # the only collective: counters summed and the timed span max-reduced (RCCL)
    from tlsgpu.distributed import reduce_counters
    nfail = n - int(status.sum().item())
    sums, elapsed = reduce_counters(torch, dist, [n * args.steps * len(kinds),
                                                  n * L * args.steps * len(kinds), nfail],
                                    elapsed, device=dev)
    payload_bytes = sums[1]
    per_kernel = {}
    for (a, op), lst in ev.items():
        ms = sum(e0.elapsed_time(e1) for e0, e1 in lst) / len(lst)
        alg_bytes = algorithmic_bytes(n, L, op)
        per_kernel["%s_%s" % (a, op)] = {
            "ms": round(ms, 3), "payload_GiBps": round(n * L / (ms / 1e3) / 2 ** 30, 1),
            "algorithmic_GBps": round(alg_bytes / (ms / 1e3) / 1e9, 1)}
    dom = max(per_kernel, key=lambda k: per_kernel[k]["ms"])
    dom_op = "open" if dom.endswith("open") else "seal"
    dom_achieved = algorithmic_bytes(n, L, dom_op) / (per_kernel[dom]["ms"] / 1e3) / 1e9

    e2e = None
    if args.e2e and rank == 0:
        e2e = end_to_end(torch, tlsgpu, ciphers, aad, nonces, L, min(n, 1 << 16))

    if rank == 0:
        line = {
            "metric": "GiB/s device-resident record seal/open, AES-128-GCM + ChaCha20-Poly1305 16KiB",
            "value": round(payload_bytes / elapsed / 2 ** 30, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint payloads, seeded per rank)",
            "config": {"workload": "BASELINE configs[1]+[2]: 2^20 x 16 KiB TLS 1.3 records per GPU, "
                                   "single key, AES-128-GCM and ChaCha20-Poly1305, seal+open",
                       "records_per_gpu": n, "record_len": L, "aad_len": AAD_LEN,
                       "sealed_stride": SL,
                       "parallelism": "records sharded by seq range, %d rank(s)" % world},
            "per_kernel": per_kernel,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(dom_achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dom_achieved / HBM_PEAK_GBS, 4),
                         "traffic": measured_traffic(args.traffic_file, dom, n, L),
                         "bytes_per_record": algorithmic_bytes(1, L, dom_op),
                         "algorithmic_bytes_per_launch": algorithmic_bytes(n, L, dom_op)},
            "verified": bool(ok),
            "auth_failures": int(sums[2]),
        }
        if e2e:
            line["end_to_end"] = e2e
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(L, args.cpu_cores, args.cpu_records)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def measured_traffic(path, kernel, n, L):
    """HBM bytes per launch of ``kernel`` from a committed tools/traffic.sh
    summary (PMC passes cannot run inside the timed process), or None when
    there is none for this exact config (2^20 x 16 KiB headline records)."""
    if n != 1 << 20 or L != 16384 or not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    return round(t[kernel]["hbm_bytes"]) if kernel in t else None


def init_dist(torch, dist):
    """One process per GPU (torch.distributed.run sets RANK/LOCAL_RANK/
    WORLD_SIZE); backend "nccl" = RCCL over xGMI.  TLSGPU_DIST_BACKEND=gloo
    and a device count below the world size are for rehearsal only."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    if world > 1:
        backend = os.environ.get("TLSGPU_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def run_config5(args):
    """BASELINE configs[4]: TLS 1.3 AES-128-GCM record seal, inner plaintext
    L = 16385 (16384 application bytes + content type 0x17, recordlayer.py:
    606-617), AAD 17 03 03 40 11, 2^20 records per GPU; rank g seals seq
    [g*2^20, (g+1)*2^20) of one connection.  RCCL carries only the counters."""
    import torch
    import torch.distributed as dist
    import tlsgpu
    from tlsgpu.distributed import reduce_counters
    from vectors import tls13_aad
    world, rank, _ = init_dist(torch, dist)
    n, L = args.records, 16385
    SL = (L + TAG_LEN + args.record_align - 1) // args.record_align * args.record_align
    IL = (L + 127) // 128 * 128
    g = torch.Generator(device="cuda").manual_seed(0x7715 + rank)
    inp = torch.randint(0, 256, (n * IL,), dtype=torch.uint8, device="cuda", generator=g)
    inp.view(n, IL)[:, L - 1] = 0x17                       # TLS 1.3 inner content type
    sealed = torch.empty(n * SL, dtype=torch.uint8, device="cuda")
    nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    hrng = torch.Generator().manual_seed(0x7716)
    iv = bytes(torch.randint(0, 256, (12,), dtype=torch.uint8, generator=hrng).tolist())
    key = bytes(torch.randint(0, 256, (16,), dtype=torch.uint8, generator=hrng).tolist())
    tlsgpu.make_nonces(iv, rank * n, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    c = tlsgpu.HipAESGCM(bytearray(key))
    b = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=IL,
                          out_stride=SL, fixed_aad_len=AAD_LEN)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        tlsgpu.seal_batch(c, b, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tlsgpu.seal_batch(c, b, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sums, elapsed = reduce_counters(torch, dist, [n * args.steps, n * L * args.steps, 0],
                                    time.perf_counter() - t0, device="cuda")
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s device-resident TLS 1.3 AES-128-GCM record seal (BASELINE configs[4])",
            "value": round(sums[1] / elapsed / 2 ** 30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "dtype": "u8", "data": "synthetic",
            "config": {"workload": "configs[4]", "records_per_gpu": n, "inner_plaintext": L,
                       "records_total": int(sums[0] / args.steps)}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_config4(args):
    """BASELINE configs[3]: AES-256-GCM, 65 536 independent session keys
    (PCG64 0x7716), 2^20 records with Zipf(1.2) lengths 64 B-16 KiB (PCG64
    0x7717), TLS 1.2 AAD seq||0x17||0x0303||len and nonce iv4||seq.  Records
    are packed in arrival (seq) order; the engine's planner (planner.hip)
    launches them longest first.  --c4-presorted packs them in descending
    length order on the host instead (what the planner does, for comparison).
    Reports payload GiB/s of seal and of open, and the byte-weighted mean length."""
    import numpy as np
    import torch
    import tlsgpu
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    n, nkeys = args.records, 65536
    rk = np.random.default_rng(0x7716)
    keys = rk.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    key_idx = rk.integers(0, nkeys, n).astype(np.uint32)
    rl = np.random.default_rng(0x7717)
    lens = np.clip(64 * rl.zipf(1.2, n), 64, 16384).astype(np.int64)
    order = np.argsort(-lens, kind="stable") if args.c4_presorted else np.arange(n)
    lens, key_idx = lens[order], key_idx[order]
    seq = order.astype(np.uint64)           # record identity = its original seq number
    in_sz = (lens + 15) // 16 * 16
    out_sz = (lens + 16 + 15) // 16 * 16
    in_off = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.int64)
    out_off = np.concatenate([[0], np.cumsum(out_sz)[:-1]]).astype(np.int64)
    aad = np.zeros((n, 13), dtype=np.uint8)
    aad[:, :8] = seq[:, None].view(np.uint8).reshape(n, 8)[:, ::-1]
    aad[:, 8], aad[:, 9], aad[:, 10] = 0x17, 3, 3
    aad[:, 11], aad[:, 12] = lens >> 8, lens & 0xff
    nonce = np.zeros((n, 12), dtype=np.uint8)
    nonce[:, :4] = rk.integers(0, 256, 4, dtype=np.uint8)
    nonce[:, 4:] = aad[:, :8]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    total_in, total_out = int(in_sz.sum()), int(out_sz.sum())
    g = torch.Generator(device="cuda").manual_seed(0x7717)
    inp = torch.randint(0, 256, (total_in,), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.empty(total_out, dtype=torch.uint8, device="cuda")
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d_lens, d_in_off, d_out_off = d(lens.astype(np.int32)), d(in_off), d(out_off)
    d_aad, d_nonce, d_kidx = d(aad.reshape(-1)), d(nonce.reshape(-1)), d(key_idx.view(np.int32))
    table = tlsgpu.KeyTable("aesgcm", [bytes(k) for k in keys])
    sb = tlsgpu.make_batch(n, inp, sealed, d_nonce, aad=d_aad, lens=d_lens, in_off=d_in_off,
                           out_off=d_out_off, aad_stride=13, fixed_aad_len=13, key_idx=d_kidx)
    ob = tlsgpu.make_batch(n, sealed, back, d_nonce, aad=d_aad, lens=d_lens, in_off=d_out_off,
                           out_off=d_in_off, aad_stride=13, fixed_aad_len=13, key_idx=d_kidx,
                           status=status)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        tlsgpu.seal_batch(table, sb, stream)
        tlsgpu.open_batch(table, ob, stream)
    ms = {"seal": [], "open": []}
    for _ in range(args.steps):
        for op, fn, b in (("seal", tlsgpu.seal_batch, sb), ("open", tlsgpu.open_batch, ob)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn(table, b, stream)
            e1.record(stream)
            ms[op].append((e0, e1))
    torch.cuda.synchronize()
    ok = int(status.sum().item()) == n and torch.equal(back, inp)
    payload = float(lens.sum())
    res = {}
    for op, lst in ms.items():
        t = sum(a.elapsed_time(b) for a, b in lst) / len(lst)
        res[op] = {"ms": round(t, 3), "payload_GiBps": round(payload / (t / 1e3) / 2 ** 30, 1)}
    line = {"metric": "GiB/s device-resident record seal/open, AES-256-GCM, 65536 keys, "
                      "Zipf 64B-16KiB (BASELINE configs[3])",
            "value": round(2 * payload / ((res["seal"]["ms"] + res["open"]["ms"]) / 1e3) / 2 ** 30, 2),
            "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "dtype": "u8", "data": "synthetic", "records": n, "keys": nkeys,
            "record_order": "host-presorted" if args.c4_presorted else "arrival (engine planner)",
            "mean_len": round(float(lens.mean()), 1),
            "byte_weighted_mean_len": round(float((lens * lens).sum() / lens.sum()), 1),
            "per_op": res, "verified": bool(ok)}
    print(json.dumps(line), flush=True)
    if not ok:
        sys.exit(3)


class _NullSink(object):
    """A socket stand-in that takes the wire bytes without copying them."""

    def __init__(self):
        self.bytes = 0

    def sendall(self, mv):
        self.bytes += len(mv)


class _MemSink(object):
    def __init__(self):
        self.parts = []

    def sendall(self, mv):
        self.parts.append(bytes(mv))


def run_ingest(args):
    """Host ingest pipeline (tlsgpu.ingest): application data in host memory
    -> RecordWriter (pinned slots, H2D, device framing + AEAD, device pack,
    D2H) -> wire bytes; and wire bytes -> RecordReader (header scan, H2D,
    device spread + open, D2H) -> application data.  TLS 1.3, 16 KiB records.
    Reported in DESIGN.md (end-to-end row), never as the headline value."""
    import hashlib
    import numpy as np
    import torch
    import tlsgpu
    torch.cuda.set_device(0)
    total = args.ingest_mib << 20
    blk = np.random.default_rng(0x7718).integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    data = blk * (total // len(blk))
    want = hashlib.sha256(data).hexdigest()
    iv = bytes(range(12))
    res = {}
    for alg, obj in (("aes128gcm", lambda: tlsgpu.HipAESGCM(bytearray(16))),
                     ("chacha20-poly1305", lambda: tlsgpu.HipCHACHA20_POLY1305(bytearray(32)))):
        mv = memoryview(data)
        # warm-up: build the wire stream once (also the reader's input)
        ms = _MemSink()
        w = tlsgpu.RecordWriter(ms, obj(), tlsgpu.TLS13, iv, batch_records=8192)
        for p in range(0, len(data), 64 << 20):
            w.write(mv[p:p + (64 << 20)])
        w.flush()
        wire = b"".join(ms.parts)
        del ms
        ns = _NullSink()
        w = tlsgpu.RecordWriter(ns, obj(), tlsgpu.TLS13, iv, batch_records=8192)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for p in range(0, len(data), 64 << 20):
            w.write(mv[p:p + (64 << 20)])
        w.flush()
        t_w = time.perf_counter() - t0
        r = tlsgpu.RecordReader(obj(), tlsgpu.TLS13, iv, batch_records=8192,
                                buffer_bytes=160 << 20)
        wv = memoryview(wire)
        outbuf = np.empty(total, np.uint8)
        ov, pos = memoryview(outbuf), 0
        t0 = time.perf_counter()
        for p in range(0, len(wire), 128 << 20):   # socket reads of 128 MiB
            r.feed(wv[p:p + (128 << 20)])
            pos += len(r.read_application_data(out=ov[pos:]))
        t_r = time.perf_counter() - t0
        ok = (pos == total and hashlib.sha256(outbuf).hexdigest() == want
              and ns.bytes == len(wire))
        res[alg] = {"write_GiBps": round(total / t_w / 2 ** 30, 2),
                    "read_GiBps": round(total / t_r / 2 ** 30, 2),
                    "records": w.records_sent, "wire_bytes": len(wire), "verified": ok}
        del wire, outbuf, ov
    line = {"metric": "GiB/s host ingest pipeline (RecordWriter / RecordReader), TLS 1.3, "
                      "16 KiB records, host memory to host memory",
            "unit": "GiB/s", "n_gpus": 1, "app_data_bytes": total, "dtype": "u8",
            "data": "synthetic", "per_alg": res}
    print(json.dumps(line), flush=True)


def end_to_end(torch, tlsgpu, ciphers, aad, nonces, L, n):
    """Records start and end in pinned host memory (socket buffers): H2D copy,
    seal, D2H copy, pipelined over chunks on two streams.  Reported in
    DESIGN.md, never as ``value``."""
    chunk = 8192
    host_in = torch.randint(0, 256, (n * L,), dtype=torch.uint8).pin_memory()
    host_out = torch.empty(n * (L + TAG_LEN), dtype=torch.uint8).pin_memory()
    res = {}
    for a, c in ciphers.items():
        streams = [torch.cuda.Stream() for _ in range(2)]
        bufs = [(torch.empty(chunk * L, dtype=torch.uint8, device="cuda"),
                 torch.empty(chunk * (L + TAG_LEN), dtype=torch.uint8, device="cuda"))
                for _ in streams]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ci, s0 in enumerate(range(0, n, chunk)):
            k = min(chunk, n - s0)
            s = streams[ci % 2]
            din, dout = bufs[ci % 2]
            with torch.cuda.stream(s):
                din[:k * L].copy_(host_in[s0 * L:(s0 + k) * L], non_blocking=True)
                b = tlsgpu.make_batch(k, din, dout, nonces[12 * s0:], aad=aad, fixed_len=L,
                                      in_stride=L, out_stride=L + TAG_LEN, fixed_aad_len=AAD_LEN)
                tlsgpu.seal_batch(c, b, s)
                host_out[s0 * (L + TAG_LEN):(s0 + k) * (L + TAG_LEN)].copy_(
                    dout[:k * (L + TAG_LEN)], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[a + "_seal"] = {"GiBps_payload": round(n * L / dt / 2 ** 30, 2), "records": n}
    return res


if __name__ == "__main__":
    main()
