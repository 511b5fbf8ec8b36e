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


# The JSON line goes to the process's original stdout, and only it: once the
# arguments are parsed, fd 1 is pointed at stderr, so library banners (RCCL
# prints its version block to fd 1 when a communicator is created) cannot
# land in the driver's one-line output.
_JSON_FD = None


def emit(line):
    """Print the bench's one JSON line on the original stdout."""
    os.write(_JSON_FD if _JSON_FD is not None else 1, (json.dumps(line) + "\n").encode())


def quiet_stdout():
    """Keep fd 1 for the JSON line (emit) and send everything else to stderr."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def algorithmic_bytes(n, L, op):
    """seal reads L + A + 12, writes L + 16; open reads
    L + 16 + A + 12, writes L (+1 status byte)."""
    per = 2 * L + AAD_LEN + NONCE_LEN + TAG_LEN + (1 if op == "open" else 0)
    return n * per


# ------------------------------------------------------------- CPU baseline

def host_cores():
    """CPUs this process may actually use: the affinity mask, capped by a
    cgroup-v2 CPU quota when one is set (the GPU box gives a job a share of
    a larger machine).  Returns (cores, os.cpu_count())."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            cores = max(1, min(cores, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return cores, os.cpu_count()


def _cpu_worker(L, seed, seconds, start, q):
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import pyaead
    from vectors import tls13_aad, tls13_nonce
    rng = np.random.default_rng(seed)
    ciphers = {"aes128gcm": pyaead.AESGCM(rng.bytes(16)),
               "chacha20-poly1305": pyaead.CHACHA20_POLY1305(rng.bytes(32))}
    iv = rng.bytes(12)
    pt = rng.bytes(L)
    aad = tls13_aad(L)
    start.wait()
    t0 = time.perf_counter()
    done, i = 0, 0
    while time.perf_counter() - t0 < seconds:
        for c in ciphers.values():
            nonce = tls13_nonce(iv, i)
            sealed = c.seal(nonce, pt, aad)
            assert c.open(nonce, sealed, aad) == pt
            done += 2 * L
        i += 1
    q.put((done, time.perf_counter() - t0))


def cpu_baseline(L, cores, seconds, gpu_samples):
    """The reference's pure-Python path, restated in oracle/pyaead.py, on
    ``cores`` host processes started together, each sealing and opening
    L-byte records with both AEADs for ``seconds``.  pyaead is not slower
    than the reference: a 16 KiB seal takes 44.4 ms against the reference's
    63.5 ms for AES-128-GCM (1.43x faster) and 39.9 against 37.3 ms for
    ChaCha20-Poly1305 (0.93x; tests/golden/make_golden.py --timing), so this
    baseline overstates the reference's own CPU rate, if anything.  The same leg re-seals ``gpu_samples``
    (records the GPU sealed in this run: key, nonce, plaintext, GPU output)
    and reports whether the GPU bytes match."""
    ctx = mp.get_context("spawn")
    start, q = ctx.Barrier(cores + 1), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(L, 1000 + c, seconds, start, q))
             for c in range(cores)]
    for p in procs:
        p.start()
    start.wait()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    from oracle import pyaead
    match = True
    for alg, key, nonce, pt, aad, got in gpu_samples:
        c = pyaead.AESGCM(key) if alg == "aes128gcm" else pyaead.CHACHA20_POLY1305(key)
        match = match and bytes(c.seal(nonce, pt, aad)) == bytes(got)
    cap, ncpu = host_cores()
    return {"value": total / wall / 2 ** 30, "unit": "GiB/s", "cores": cores, "kind": "port",
            "host_cpus": ncpu, "usable_cpus": cap,
            "sample": "%d processes x %.0f s each (%d records of %d B per process on average), "
                      "AES-128-GCM + ChaCha20-Poly1305 seal+open, oracle/pyaead.py (pure-Python "
                      "restatement of the reference path)" % (cores, seconds,
                                                               total // (2 * L) // max(cores, 1), L),
            "gpu_records_rechecked": len(gpu_samples), "gpu_records_match": bool(match)}


# ------------------------------------------- per-rank checks (every N)

def headline_check(samples):
    """Every rank's own sampled records (alg, key, nonce, plaintext, aad, GPU
    output) re-sealed with the C oracle (oracle/aead_oracle.c, pinned to the
    reference's vectors): the number of records whose bytes differ."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    bad = 0
    for alg, key, nonce, pt, aad, got in samples:
        seal = O.gcm_seal if alg.startswith("aes") else O.chacha_seal
        bad += int(bytes(seal(key, nonce, pt, aad)) != bytes(got))
    return bad


def corrupt_for_test(samples, rank, field):
    """Test hook (tests/test_bench_verify.py): TLSGPU_BENCH_CORRUPT_RANK=r
    flips one byte of the first sample's GPU bytes on rank r before the
    oracle check, so a one-shard failure must surface in the reduced
    ``verified``.  ``field`` indexes the GPU bytes in a sample tuple."""
    if not samples or os.environ.get("TLSGPU_BENCH_CORRUPT_RANK") != str(rank):
        return samples
    s0 = list(samples[0])
    b = bytearray(s0[field])
    b[len(b) // 2] ^= 0x01
    s0[field] = bytes(b)
    return [tuple(s0)] + list(samples[1:])


def verify_shards(torch, dist, local_ok, bad, checked, device=None):
    """The line's verification over ALL ranks (tlsgpu.distributed.
    reduce_verification): MIN of each rank's own round-trip flag and oracle
    agreement, SUM of the oracle mismatches and of the records checked.
    Every rank returns the same (ok, mismatches, checked)."""
    from tlsgpu import distributed as tgd
    return tgd.reduce_verification(torch, dist, bool(local_ok) and bad == 0, bad, checked, device=device)


def finish(dist, ok):
    """Tear down the process group; exit 3 on every rank when any shard
    failed its checks."""
    from tlsgpu import distributed as tgd
    if tgd.group_active(dist):
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# ---------------------------------------------- BASELINE configs[0], in full

C1_RECORDS, C1_LEN = 4096, 1024


def _cpu_worker_c1(lo, hi, start, q):
    """Records [lo, hi) of config 1: CHACHA20_POLY1305.seal then .open
    (chacha20_poly1305.py:48,68) with the pure-Python restatement, TLS 1.3
    nonce iv xor seq and AAD 17 03 03 04 10."""
    sys.path.insert(0, ROOT)
    from oracle import pyaead
    from vectors import config1_inputs, tls13_aad, tls13_nonce
    key, iv, pts = config1_inputs(C1_RECORDS, C1_LEN)
    c = pyaead.CHACHA20_POLY1305(key)
    start.wait()
    t0 = time.perf_counter()
    sealed = [bytes(c.seal(tls13_nonce(iv, s), pts[s], tls13_aad(len(pts[s])))) for s in range(lo, hi)]
    t_seal = time.perf_counter() - t0
    ok = all(c.open(tls13_nonce(iv, s), bytearray(w), tls13_aad(len(pts[s]))) == pts[s]
             for s, w in zip(range(lo, hi), sealed))
    q.put((lo, sealed, ok, t_seal, time.perf_counter() - t0))


def cpu_config1(cores):
    """BASELINE configs[0] run in full on the host: 4 096 x 1 KiB
    ChaCha20-Poly1305 records sealed and opened back with oracle/pyaead.py (the
    reference's pure-Python path restated), split over ``cores`` processes
    started together.  The sealed stream's SHA-256 is compared with the digest
    the reference itself produced (tests/golden/record_batch.json
    config1.sealed_sha256)."""
    import hashlib
    from vectors import load
    ctx = mp.get_context("spawn")
    cores = max(1, min(cores, C1_RECORDS))
    start, q = ctx.Barrier(cores + 1), ctx.Queue()
    bounds = [(C1_RECORDS * k // cores, C1_RECORDS * (k + 1) // cores) for k in range(cores)]
    procs = [ctx.Process(target=_cpu_worker_c1, args=(lo, hi, start, q)) for lo, hi in bounds]
    for p in procs:
        p.start()
    start.wait()
    res = sorted(q.get() for _ in procs)
    for p in procs:
        p.join()
    h = hashlib.sha256()
    for r in res:
        for w in r[1]:
            h.update(w)
    want = load("record_batch.json")["config1"]["sealed_sha256"]
    wall = max(r[4] for r in res)
    payload = 2 * C1_RECORDS * C1_LEN
    return {"value": round(payload / wall / 2 ** 20, 3), "unit": "MiB/s", "cores": cores,
            "kind": "port", "records": C1_RECORDS, "record_len": C1_LEN,
            "seconds": round(wall, 3), "seal_seconds": round(max(r[3] for r in res), 3),
            "records_per_s": round(2 * C1_RECORDS / wall, 1),
            "sample": "BASELINE configs[0] in full: %d x %d B ChaCha20-Poly1305 seal + open, "
                      "oracle/pyaead.py on %d processes" % (C1_RECORDS, C1_LEN, cores),
            "sealed_sha256": h.hexdigest(), "digest_match": h.hexdigest() == want,
            "opened_ok": all(r[2] for r in res)}


# -------------------------------------------------------------- GPU bench

def read_bytes(n, L, op):
    """The read half of algorithmic_bytes: seal reads L + A + 12, open
    L + 16 + A + 12 (north_star's "HBM-read roofline")."""
    return n * (L + AAD_LEN + NONCE_LEN + (TAG_LEN if op == "open" else 0))


def free_port():
    """A TCP port free on 127.0.0.1 right now (the rendezvous of the ranks)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_launch_cmd(argv, gpus, port):
    """The command that runs this bench as ``gpus`` ranks, one process per
    GPU: torch.distributed.run on one node, rendezvous on 127.0.0.1, the
    same bench arguments.  (The driver's own N > 1 runs start the ranks
    themselves; then WORLD_SIZE is set and no launch happens.)"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
            str(gpus), "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env=None):
    """Inside a rank: the launcher's world size must be what --gpus asked
    for.  Returns an error message or None."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        return "--gpus %d but WORLD_SIZE=%d: launch one rank per GPU (bench.py --gpus N starts them)" % (
            gpus, world)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--len", type=int, default=16384)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU baseline processes (0 = every usable host core, host_cores())")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU baseline: seconds each process seals/opens")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time the host<->device path")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "r06", "traffic.json"),
                    help="per-launch HBM bytes from tools/traffic.sh (rocprofv3 FETCH_SIZE / "
                         "WRITE_SIZE passes at this config, calibrated per access shape) for "
                         "roofline.traffic")
    ap.add_argument("--record-align", type=int, default=128,
                    help="byte alignment of each sealed record (ct||tag) in the packed batch")
    ap.add_argument("--config", default="headline", choices=["headline", "c1", "c4", "c5", "ingest", "ccm"],
                    help="headline = BASELINE configs[1]+[2] (the metric); c1 = configs[0] "
                         "(4096 x 1 KiB ChaCha20-Poly1305, the device path beside the host CPU "
                         "run in full); c4 = configs[3] "
                         "(AES-256-GCM, 65536 keys, Zipf lengths); c5 = configs[4] (TLS 1.3 "
                         "AES-128-GCM record seal through the framing path, seq-sharded); "
                         "ingest = the host ingest pipeline (tlsgpu.ingest, SURVEY 8(f) row 3), "
                         "host memory to host memory; ccm = AES-128-CCM and CCM_8 seal/open "
                         "(SURVEY 8(f) row 2) at the headline's record shape")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="create the process group even at world size 1 (TLSGPU_DIST_SELFTEST=1) "
                         "so the counter reduction and the rate gather run through the backend "
                         "(RCCL under nccl) on a one-GPU box; the line then carries dist_backend "
                         "and dist_selftest")
    ap.add_argument("--c4-presorted", action="store_true",
                    help="config 4: pack records longest first on the host")
    ap.add_argument("--ingest-mib", type=int, default=2048,
                    help="application data per direction for --config ingest")
    ap.add_argument("--ingest-batch", type=int, default=2048,
                    help="--config ingest: records per pipeline batch (writer and reader)")
    ap.add_argument("--ingest-slots", type=int, default=4,
                    help="--config ingest: pipeline slots per direction")
    ap.add_argument("--ingest-read-mib", type=int, default=512,
                    help="--config ingest: bytes per socket read handed to the reader")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # N ranks, one process per GPU, started here before anything in this
        # process touches the GPU; this process only waits and passes on the
        # ranks' exit status (rank 0 prints the JSON line)
        if args.config in ("c1", "c4", "ingest", "ccm"):
            ap.error("--config %s runs on one GPU (BASELINE configs[3] / the host pipeline)" % args.config)
        backend = os.environ.get("TLSGPU_DIST_BACKEND", "nccl")
        if backend == "nccl":
            import torch   # device_count() does not initialise the GPU
            ndev = torch.cuda.device_count()
            if ndev < args.gpus:
                print("--gpus %d under nccl needs one GPU per rank, %d visible "
                      "(TLSGPU_DIST_BACKEND=gloo rehearses the ranks on fewer)" % (args.gpus, ndev),
                      file=sys.stderr)
                sys.exit(2)
        import subprocess
        sys.stdout.flush()
        sys.exit(subprocess.call(rank_launch_cmd(sys.argv[1:], args.gpus, free_port())))
    err = check_world(args.gpus)
    if err:
        print(err, file=sys.stderr)
        sys.exit(2)
    quiet_stdout()
    if args.dist_selftest:
        os.environ["TLSGPU_DIST_SELFTEST"] = "1"
    if args.config == "ingest":
        return run_ingest(args)
    if args.config == "c1":
        return run_config1(args)
    if args.config == "c4":
        return run_config4(args)
    if args.config == "c5":
        return run_config5(args)
    if args.config == "ccm":
        return run_ccm(args)

    import torch
    import torch.distributed as dist
    import tlsgpu
    from tlsgpu import distributed as tgd
    from vectors import tls13_aad

    try:
        world, rank, local, device = tgd.init_process(torch, dist)
    except tgd.DistError as e:
        print("rank setup: %s" % e, file=sys.stderr)
        sys.exit(2)
    n, L = args.records, args.len
    first, _ = tgd.weak_shard(n, world, rank)   # this rank: seq [rank n, (rank + 1) n)
    # sealed records are ct||tag (the wire form), packed at a stride rounded up
    # to --record-align bytes so every record starts on an HBM line boundary
    SL = (L + TAG_LEN + args.record_align - 1) // args.record_align * args.record_align
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0x7715 + rank)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    sealed = torch.empty(n * SL, dtype=torch.uint8, device=dev)
    back = torch.empty(n * L, dtype=torch.uint8, device=dev)
    nonces = torch.empty(NONCE_LEN * n, dtype=torch.uint8, device=dev)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device=dev)
    hrng = torch.Generator().manual_seed(0x7716)
    iv = bytes(torch.randint(0, 256, (12,), dtype=torch.uint8, generator=hrng).tolist())
    keys = {"aes128gcm": bytes(torch.randint(0, 256, (16,), dtype=torch.uint8, generator=hrng).tolist()),
            "chacha20-poly1305": bytes(torch.randint(0, 256, (32,), dtype=torch.uint8,
                                                     generator=hrng).tolist())}
    ciphers = {"aes128gcm": tlsgpu.HipAESGCM(bytearray(keys["aes128gcm"])),
               "chacha20-poly1305": tlsgpu.HipCHACHA20_POLY1305(bytearray(keys["chacha20-poly1305"]))}
    tgd.shard_nonces(tlsgpu, iv, first, n, nonces)
    # each cipher opens into its own status array: the verdicts of both AEADs
    # survive the step (the payload buffers are shared)
    status = {a: torch.zeros(n, dtype=torch.uint8, device=dev) for a in ciphers}
    seal_b = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                               out_stride=SL, fixed_aad_len=AAD_LEN)
    open_b = {a: tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=SL,
                                   out_stride=L, fixed_aad_len=AAD_LEN, status=status[a])
              for a in ciphers}
    stream = torch.cuda.current_stream()
    kinds = [(a, op) for a in ciphers for op in ("seal", "open")]
    ev = {k: [] for k in kinds}

    def step(record):
        for a, c in ciphers.items():
            for op, fn, b in (("seal", tlsgpu.seal_batch, seal_b), ("open", tlsgpu.open_batch, open_b[a])):
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
    elapsed = tgd.timed(torch, dist, world, lambda s: step(True), args.steps)

    # correctness of the timed work (untimed): every record of both AEADs
    # authentic in the last step, then per cipher a fresh seal -> open round
    # trip (the shared payload buffers hold only the last cipher's output)
    fails = {a: n - int(status[a].sum().item()) for a in ciphers}
    samples, verified = [], {}
    pick = sorted(set([0, n - 1, n // 2, (n * 7) // 11]))
    for a, c in ciphers.items():
        status[a].zero_()
        back.zero_()
        tlsgpu.seal_batch(c, seal_b, stream)
        tlsgpu.open_batch(c, open_b[a], stream)
        torch.cuda.synchronize()
        verified[a] = int(status[a].sum().item()) == n and bool(torch.equal(back, inp))
        for i in pick:   # for the CPU leg's re-check
            samples.append((a, keys[a], tgd.tls13_nonces(iv, first + i, 1),
                            inp[i * L:(i + 1) * L].cpu().numpy().tobytes(), bytes(tls13_aad(L)),
                            sealed[i * SL:i * SL + L + TAG_LEN].cpu().numpy().tobytes()))
    # every rank checks its own sampled records against the C oracle, and the
    # line's verdict is reduced over all ranks (a wrong seq offset on rank g
    # is symmetric in seal and open, so only the oracle sees it)
    samples = corrupt_for_test(samples, rank, 5)
    bad = headline_check(samples)
    ok, bad_all, checked_all = verify_shards(torch, dist, all(verified.values()), bad, len(samples), device=dev)
    # the only collectives: counters summed, the timed span max-reduced and
    # the per-rank kernel times gathered (RCCL)
    sums, elapsed = tgd.reduce_counters(torch, dist, [n * args.steps * len(kinds),
                                                      n * L * args.steps * len(kinds),
                                                      sum(fails.values())], elapsed, device=dev)
    payload_bytes = sums[1]
    per_kernel, my_ms = {}, []
    for (a, op), lst in ev.items():
        ms = sum(e0.elapsed_time(e1) for e0, e1 in lst) / len(lst)
        my_ms.append(ms)
        alg_bytes = algorithmic_bytes(n, L, op)
        per_kernel["%s_%s" % (a, op)] = {
            "ms": round(ms, 3), "payload_GiBps": round(n * L / (ms / 1e3) / 2 ** 30, 1),
            "algorithmic_GBps": round(alg_bytes / (ms / 1e3) / 1e9, 1),
            "frac": round(alg_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_read": round(read_bytes(n, L, op) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    rows = tgd.gather_rows(torch, dist, my_ms, device=dev)
    dist_info = tgd.selftest_collectives(torch, dist, device=dev) if tgd.group_active(dist) else None
    dom = max(per_kernel, key=lambda k: per_kernel[k]["ms"])
    dom_op = "open" if dom.endswith("open") else "seal"
    dom_s = per_kernel[dom]["ms"] / 1e3
    dom_achieved = algorithmic_bytes(n, L, dom_op) / dom_s / 1e9
    traffic = measured_traffic(args.traffic_file, dom, n, L)

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
                         "frac_read": round(read_bytes(n, L, dom_op) / dom_s / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": traffic["hbm_bytes"] if traffic else None,
                         "traffic_detail": traffic,
                         "bytes_per_record": algorithmic_bytes(1, L, dom_op),
                         "read_bytes_per_record": read_bytes(1, L, dom_op),
                         "algorithmic_bytes_per_launch": algorithmic_bytes(n, L, dom_op)},
            "verified": bool(ok),
            "verified_scope": "all %d rank(s): MIN of each rank's round trip and oracle agreement" % world,
            "verified_per_cipher_rank0": verified,
            "oracle_checked_records": checked_all, "oracle_mismatches": bad_all,
            "auth_failures": int(sums[2]),
            "auth_failures_per_cipher": fails,
            "dist_backend": dist.get_backend() if tgd.group_active(dist) else None,
        }
        if dist_info:
            line["dist_selftest"] = dist_info
        if world > 1:
            names = ["%s_%s" % k for k in kinds]
            line["per_rank"] = [{nm: {"ms": round(ms, 3),
                                      "frac": round(algorithmic_bytes(n, L, nm.rsplit("_", 1)[1]) /
                                                    (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
                                 for nm, ms in zip(names, r)} for r in rows]
        if e2e:
            line["end_to_end"] = e2e
        if not args.no_cpu_baseline:
            # rank 0 only, after the collectives, at any N (the other ranks
            # go on to tear down their process group)
            cores = args.cpu_cores or host_cores()[0]
            line["cpu_baseline"] = cpu_baseline(L, cores, args.cpu_seconds, samples)
            line["cpu_baseline"]["config1"] = cpu_config1(cores)
        emit(line)
    finish(dist, ok)


def measured_traffic(path, kernel, n, L):
    """HBM bytes per launch of ``kernel`` from a committed tools/traffic.sh
    summary (PMC passes cannot run inside the timed process): the calibrated
    figure with the raw counters and the factors behind it, or None when
    there is none for this exact config (2^20 x 16 KiB headline records)."""
    if n != 1 << 20 or L != 16384 or not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    k = t.get("kernels", {}).get(kernel)
    if not k:
        return None
    return {"hbm_bytes": round(k["hbm_bytes"]), "fetch_size_bytes": round(k["fetch_size_bytes"]),
            "write_size_bytes": round(k["write_size_bytes"]), "access_shape": k["shape"],
            "fetch_factor": k["fetch_factor"], "write_factor": k["write_factor"],
            "traffic_over_algorithmic": round(k["hbm_bytes"] / algorithmic_bytes(n, L, kernel.rsplit("_", 1)[1]), 3),
            # the launch's other kernel (AES-GCM: hy_mask_kernel, round 4), not in hbm_bytes
            "mask_kernel_bytes": (round(t["kernels"]["aes128gcm_masks"]["hbm_bytes"])
                                  if kernel.startswith("aes128gcm") and "aes128gcm_masks" in t.get("kernels", {})
                                  else None),
            "source": os.path.relpath(path, ROOT)}


def c4_traffic(path, op):
    """Config 4's HBM bytes per ``op`` (one seal or open of the whole batch:
    the long-record and the short-record kernel together) from the
    tools/traffic.sh summary, or None."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        ks = json.load(f).get("kernels", {})
    kt, lane = ks.get("c4_kt_" + op), ks.get("c4_lane_" + op)
    if not kt:
        return None
    if lane:   # a separate lane kernel for the short records (before round 6's fusion)
        kernels = {"long_records (gcm_kth_kernel)": round(kt["hbm_bytes"]),
                   "gcm_table_vkernel": round(lane["hbm_bytes"])}
    else:      # the key-table hybrid takes the short records too
        kernels = {"all_records (gcm_kth_kernel)": round(kt["hbm_bytes"])}
    # the per-record keystream precompute and per-job keys (round 4), one
    # launch each per seal or open, when the summary has them
    for lab, name in (("c4_masks", "kt_mask_kernel"), ("c4_jobkey", "kth_jobkey_kernel")):
        if ks.get(lab):
            kernels[name] = round(ks[lab]["hbm_bytes"])
    return {"hbm_bytes": sum(kernels.values()), "kernels": kernels,
            "source": os.path.relpath(path, ROOT)}


def c5_traffic(path, n, L_app):
    """Config 5's HBM bytes per record seal of the whole batch (the framing
    kernel and the AEAD kernel together) from the tools/traffic.sh summary,
    or None (only for the default 2^20 x 16 KiB shape)."""
    if n != 1 << 20 or L_app != C5_APP or not os.path.exists(path):
        return None
    with open(path) as f:
        ks = json.load(f).get("kernels", {})
    parts = [ks.get("c5_prep"), ks.get("c5_seal")]
    if not all(parts):
        return None
    hbm = sum(k["hbm_bytes"] for k in parts)
    return {"hbm_bytes": round(hbm),
            "kernels": {"seal_prep": round(parts[0]["hbm_bytes"]), "gcm_hy_kernel": round(parts[1]["hbm_bytes"])},
            "traffic_over_algorithmic": round(hbm / c5_algorithmic_bytes(n, L_app, "seal"), 3),
            "source": os.path.relpath(path, ROOT)}


def c5_algorithmic_bytes(n, L_app, op):
    """Config 5's record seal through the framing path (recordlayer.py:
    606-617 then 536-565): reads the L application bytes, writes the 5-byte
    header, the inner plaintext's ciphertext (L + 1, content type appended)
    and the tag.  The nonce and AAD rows the framing kernel builds for the
    AEAD are scratch, not counted.  Open: reads the wire record, writes the
    L + 1 inner plaintext (+ status, type, length)."""
    wire = 5 + L_app + 1 + TAG_LEN
    return n * (L_app + wire) if op == "seal" else n * (wire + L_app + 1 + 6)


C5_APP = 16384


def c5_layout(L=C5_APP):
    """Config 5's buffers: fragment i at i * DS (DS = L + 1 rounded up to a
    128-byte line: the inner content type is appended in place), wire record
    i at i * WS + 123, so its ciphertext after the 5-byte header starts on a
    128-byte line.  Returns (DS, WS, header offset)."""
    DS = (L + 1 + 127) // 128 * 128
    WS = (5 + L + 1 + TAG_LEN + 123 + 127) // 128 * 128
    return DS, WS, 123


def c5_pick(n, count=128, seed=0xc5):
    """Records checked against the framing oracle: the first, the last and
    random others (count in all, fewer when n is smaller)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    idx = set([0, n - 1])
    while len(idx) < min(count, n):
        idx.add(int(rng.integers(0, n)))
    return sorted(idx)


def c5_samples(data, wire, wire_len, idx, L=C5_APP):
    """Host copies of the picked records: (i, fragment, wire record)."""
    DS, WS, H = c5_layout(L)
    wl = wire_len.cpu().numpy()
    out = []
    for i in idx:
        frag = data[i * DS:i * DS + L].cpu().numpy().tobytes()
        w = wire[i * WS + H:i * WS + H + int(wl[i])].cpu().numpy().tobytes()
        out.append((i, frag, w))
    return out


def c5_check(samples, key, iv, seq0):
    """CPU leg, checker part: every sampled wire record equals
    oracle/records.seal_record (recordlayer.py:606-617, :536-565 restated,
    pinned to the reference RecordLayer's wire bytes) for its seq, and opens
    back there to (ok, 0x17, fragment).  Returns the number of mismatches."""
    sys.path.insert(0, ROOT)
    from oracle import records as R
    bad = 0
    for i, frag, w in samples:
        want = R.seal_record("tls13", "aes128gcm", key, iv, seq0 + i, 0x17, frag)
        got_open = R.open_record("tls13", "aes128gcm", key, iv, seq0 + i, w)
        bad += int(w != want or got_open != (R.OK, 0x17, frag))
    return bad


def _cpu_worker_c5(L, seed, seconds, start, q):
    """sendRecord + _encryptThenSeal for TLS 1.3 AES-128-GCM (recordlayer.py:
    606-617, :536-565) with the pure-Python AEAD restatement."""
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import pyaead
    from vectors import tls13_nonce
    rng = np.random.default_rng(seed)
    c = pyaead.AESGCM(rng.bytes(16))
    iv = rng.bytes(12)
    data = rng.bytes(L)
    start.wait()
    t0 = time.perf_counter()
    done, i = 0, 0
    while time.perf_counter() - t0 < seconds:
        inner = data + b"\x17"
        n = len(inner) + TAG_LEN
        hdr = bytes([0x17, 3, 3, n >> 8, n & 0xff])
        wire = hdr + bytes(c.seal(tls13_nonce(iv, i), inner, hdr))
        assert len(wire) == 5 + n
        done += L
        i += 1
    q.put((done, time.perf_counter() - t0))


def cpu_baseline_c5(L, cores, seconds):
    ctx = mp.get_context("spawn")
    start, q = ctx.Barrier(cores + 1), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker_c5, args=(L, 2000 + c, seconds, start, q))
             for c in range(cores)]
    for p in procs:
        p.start()
    start.wait()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    cap, ncpu = host_cores()
    return {"value": total / wall / 2 ** 30, "unit": "GiB/s", "cores": cores, "kind": "port",
            "host_cpus": ncpu, "usable_cpus": cap,
            "sample": "%d processes x %.0f s each, TLS 1.3 AES-128-GCM record seal (inner type, "
                      "header, AEAD) of %d-byte fragments, oracle/pyaead.py (pure-Python restatement "
                      "of the reference path)" % (cores, seconds, L)}


def _cpu_worker_c4(seed, seconds, start, q):
    """Config 4's mix on one host process: AES-256-GCM sessions (a cipher
    object per session, as RecordLayer keeps one per connection state,
    recordlayer.py:1268-1323), Zipf(1.2) record lengths 64 B-16 KiB, TLS 1.2
    nonce iv4 || seq and AAD seq || 0x17 0303 || len, seal then open with the
    pure-Python restatement."""
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import pyaead
    rng = np.random.default_rng(seed)
    sessions = [(pyaead.AESGCM(rng.bytes(32)), rng.bytes(4)) for _ in range(16)]
    lens = np.clip(64 * rng.zipf(1.2, 4096), 64, 16384)
    data = rng.bytes(16384)
    start.wait()
    t0 = time.perf_counter()
    done, i = 0, 0
    while time.perf_counter() - t0 < seconds:
        c, iv4 = sessions[i % len(sessions)]
        L = int(lens[i % len(lens)])
        seq = i.to_bytes(8, "big")
        aad = seq + bytes([0x17, 3, 3, L >> 8, L & 0xff])
        sealed = c.seal(iv4 + seq, data[:L], aad)
        assert c.open(iv4 + seq, sealed, aad) == data[:L]
        done += 2 * L
        i += 1
    q.put((done, time.perf_counter() - t0, i))


def cpu_baseline_c4(cores, seconds):
    """BASELINE configs[3] on the host cores: ``cores`` processes started
    together, each sealing and opening config-4-shaped records (_cpu_worker_c4)
    for ``seconds``; payload GiB/s counted like the GPU line (seal + open)."""
    ctx = mp.get_context("spawn")
    start, q = ctx.Barrier(cores + 1), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker_c4, args=(3000 + c, seconds, start, q)) for c in range(cores)]
    for p in procs:
        p.start()
    start.wait()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    total, wall, recs = sum(r[0] for r in res), max(r[1] for r in res), sum(r[2] for r in res)
    cap, ncpu = host_cores()
    return {"value": total / wall / 2 ** 30, "unit": "GiB/s", "cores": cores, "kind": "port",
            "host_cpus": ncpu, "usable_cpus": cap,
            "sample": "%d processes x %.0f s each (%d records in all), AES-256-GCM seal+open, 16 "
                      "sessions per process, Zipf(1.2) lengths 64 B-16 KiB, TLS 1.2 nonce and AAD, "
                      "oracle/pyaead.py (pure-Python restatement of the reference path)"
                      % (cores, seconds, recs)}


def run_config1(args):
    """BASELINE configs[0] (ChaCha20-Poly1305 seal + open of 4 096 x 1 KiB
    records, chacha20_poly1305.py:48,68): the device batch path, timed per
    step with HIP events on the launch stream, its sealed stream checked
    against the reference's digest (record_batch.json config1.sealed_sha256)
    and every record opened back; beside it the same workload run in full on
    the host cores with the pure-Python restatement (cpu_config1)."""
    import hashlib
    import numpy as np
    import torch
    import tlsgpu
    from vectors import config1_inputs, load, tls13_aad
    key, iv, pts = config1_inputs(C1_RECORDS, C1_LEN)
    n, L = C1_RECORDS, C1_LEN
    inp = torch.from_numpy(np.frombuffer(b"".join(bytes(p) for p in pts), np.uint8).copy()).cuda()
    out = torch.zeros(n * (L + TAG_LEN), dtype=torch.uint8, device="cuda")
    back = torch.zeros_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(NONCE_LEN * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(iv, 0, n, nonces)
    aad = torch.from_numpy(np.frombuffer(bytes(tls13_aad(L)), np.uint8).copy()).cuda()
    c = tlsgpu.HipCHACHA20_POLY1305(key)
    sb = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L,
                           out_stride=L + TAG_LEN, fixed_aad_len=AAD_LEN)
    ob = tlsgpu.make_batch(n, out, back, nonces, aad=aad, fixed_len=L, in_stride=L + TAG_LEN,
                           out_stride=L, fixed_aad_len=AAD_LEN, status=status)
    stream = torch.cuda.current_stream()
    evs = []
    for k in range(args.warmup + args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        tlsgpu.seal_batch(c, sb, stream)
        tlsgpu.open_batch(c, ob, stream)
        e1.record(stream)
        if k >= args.warmup:
            evs.append((e0, e1))
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    want = load("record_batch.json")["config1"]["sealed_sha256"]
    ok = digest == want and int(status.sum()) == n and bool(torch.equal(back, inp))
    line = {"metric": "MiB/s ChaCha20-Poly1305 seal+open, 4096 x 1 KiB (BASELINE configs[0])",
            "value": round(2 * n * L / (ms / 1e3) / 2 ** 20, 1), "unit": "MiB/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "none", "dtype": "u8",
            "data": "config1_inputs(): random.Random(0) key, iv and plaintexts",
            "config": {"workload": "configs[0]: 4096 x 1 KiB ChaCha20-Poly1305 seal + open, "
                                   "TLS 1.3 nonce and AAD", "records": n, "record_len": L},
            "sealed_sha256": digest, "digest_match": digest == want, "verified": bool(ok)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_config1(args.cpu_cores or host_cores()[0])
    emit(line)
    if not ok:
        sys.exit(3)


def run_config5(args):
    """BASELINE configs[4]: TLS 1.3 AES-128-GCM record seal, 2^20 records per
    GPU of L = 16384 application bytes through the device framing path
    (tg_seal_records: inner plaintext = data || 0x17, header 17 03 03 40 11,
    ct || tag behind it; recordlayer.py:606-617, :536-565); rank g seals seq
    [g 2^20, (g + 1) 2^20) of one connection (tlsgpu.distributed).  RCCL
    carries only the counters.  Checked (untimed) by opening every wire record
    back with tg_open_records (status, content type, plaintext), and on rank 0
    by the CPU leg: 128 sampled wire records (the first and the last among
    them) compared byte for byte with the framing oracle."""
    import torch
    import torch.distributed as dist
    import tlsgpu
    from tlsgpu import distributed as tgd
    try:
        world, rank, _, _ = tgd.init_process(torch, dist)
    except tgd.DistError as e:
        print("rank setup: %s" % e, file=sys.stderr)
        sys.exit(2)
    n, L = args.records, C5_APP
    first, _ = tgd.weak_shard(n, world, rank)
    DS, WS, H = c5_layout(L)
    g = torch.Generator(device="cuda").manual_seed(0x7715 + rank)
    data = torch.randint(0, 256, (n * DS,), dtype=torch.uint8, device="cuda", generator=g)
    orig = data.view(n, DS)[:, :L].clone()
    data_off = torch.arange(n, dtype=torch.int64, device="cuda") * DS
    data_len = torch.full((n,), L, dtype=torch.int32, device="cuda")
    ctype = torch.full((n,), 0x17, dtype=torch.uint8, device="cuda")
    wire_off = torch.arange(n, dtype=torch.int64, device="cuda") * WS + H
    wire = torch.empty(n * WS, dtype=torch.uint8, device="cuda")
    wire_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    hrng = torch.Generator().manual_seed(0x7716)
    iv = bytes(torch.randint(0, 256, (12,), dtype=torch.uint8, generator=hrng).tolist())
    key = bytes(torch.randint(0, 256, (16,), dtype=torch.uint8, generator=hrng).tolist())
    c = tlsgpu.HipAESGCM(bytearray(key))
    stream = torch.cuda.current_stream()
    evs = []

    def step(record):
        if record:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        tlsgpu.seal_records(c, tlsgpu.TLS13, iv, first, n, data, data_off, data_len, ctype, wire,
                            wire_off, wire_len, stream=stream)
        if record:
            e1.record(stream)
            evs.append((e0, e1))

    for _ in range(args.warmup):
        step(False)
    elapsed = tgd.timed(torch, dist, world, lambda s: step(True), args.steps)
    # untimed check: every wire record opens back to its fragment and type
    wl = int(wire_len[0].item())
    samples = c5_samples(data, wire, wire_len, c5_pick(n), L)   # every rank: its own shard
    back = torch.zeros(n * DS, dtype=torch.uint8, device="cuda")
    o_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    o_ct = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 255, dtype=torch.uint8, device="cuda")
    tlsgpu.open_records(c, tlsgpu.TLS13, iv, first, n, wire, wire_off, wire_len, back, data_off,
                        o_len, o_ct, st, stream=stream)
    torch.cuda.synchronize()
    ok = (bool((wire_len == 5 + L + 1 + TAG_LEN).all()) and int((st == 0).sum()) == n and
          bool((o_ct == 0x17).all()) and bool((o_len == L).all()) and
          bool(torch.equal(back.view(n, DS)[:, :L], orig)))
    hdr = wire[H:H + 5].cpu().numpy().tobytes()
    ok = ok and hdr == bytes([0x17, 0x03, 0x03, (L + 17) >> 8, (L + 17) & 0xff])
    # each rank's 128 sampled wire records against the framing oracle at its
    # own seq offset (first = g n), reduced over all ranks
    bad = c5_check(corrupt_for_test(samples, rank, 2), key, iv, first)
    ok, bad_all, checked_all = verify_shards(torch, dist, ok, bad, len(samples), device="cuda")
    sums, elapsed = tgd.reduce_counters(torch, dist, [n * args.steps, n * L * args.steps, 0],
                                        elapsed, device="cuda")
    dist_info = tgd.selftest_collectives(torch, dist, device="cuda") if tgd.group_active(dist) else None
    ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    ach = c5_algorithmic_bytes(n, L, "seal") / (ms / 1e3) / 1e9
    rows = tgd.gather_rows(torch, dist, [ms, float(first)], device="cuda")
    if rank == 0:
        line = {
            "metric": "GiB/s device-resident TLS 1.3 AES-128-GCM record seal (BASELINE configs[4])",
            "value": round(sums[1] / elapsed / 2 ** 30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "dtype": "u8", "data": "synthetic",
            "config": {"workload": "configs[4]: tg_seal_records (header + inner type + AEAD)",
                       "records_per_gpu": n, "app_bytes": L, "wire_record": wl,
                       "records_total": int(sums[0] / args.steps),
                       "layout": "fragment stride %d, wire stride %d, header at +%d" % (DS, WS, H)},
            "roofline": {"bound": "hbm", "kernel": "seal_records (framing + AEAD launches)",
                         "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4),
                         "frac_read": round(n * L / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes_per_record": c5_algorithmic_bytes(1, L, "seal"), "traffic": None,
                         "ms": round(ms, 3)},
            "oracle_checked_records": checked_all, "oracle_mismatches": bad_all,
            "verified": bool(ok),
            "verified_scope": "all %d rank(s): MIN of each rank's open-back check and its %d sampled "
                              "wire records against the framing oracle" % (world, len(samples)),
            "dist_backend": dist.get_backend() if tgd.group_active(dist) else None}
        if world > 1:
            line["per_rank"] = [{"rank": g, "seq0": int(r[1]), "ms": round(r[0], 3),
                                 "frac": round(c5_algorithmic_bytes(n, L, "seal") / (r[0] / 1e3) / 1e9 /
                                               HBM_PEAK_GBS, 4)} for g, r in enumerate(rows)]
        if dist_info:
            line["dist_selftest"] = dist_info
        tr = c5_traffic(args.traffic_file, n, L) if world == 1 else None
        if tr:
            line["roofline"]["traffic"] = tr["hbm_bytes"]
            line["roofline"]["traffic_detail"] = tr
        if not args.no_cpu_baseline:   # rank 0, after the collectives, at any N
            cores = args.cpu_cores or host_cores()[0]
            line["cpu_baseline"] = cpu_baseline_c5(L, cores, args.cpu_seconds)
        emit(line)
    finish(dist, ok)


def run_ccm(args):
    """SURVEY 8(f) row 2 (aesccm.py:11-155): AES-128-CCM and AES-128-CCM_8
    seal + open of ``--records`` TLS 1.3 records of ``--len`` bytes (default
    the headline's 2^20 x 16 KiB), single key, records resident in HBM, one
    GPU.  Not a BASELINE config (the reference publishes no CCM figure); the
    row measures the CCM kernels at the headline's shape.  Checked untimed:
    every record opens back (status and plaintext), and 64 sampled sealed
    records equal the C oracle's AESCCM restatement byte for byte.  CPU
    baseline: the C oracle's batch entry (the restatement, threaded) on the
    usable cores over a bounded sample."""
    import numpy as np
    import torch
    import tlsgpu
    from vectors import tls13_aad
    from tlsgpu import distributed as tgd
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    n, L = args.records, args.len
    SLc = (L + TAG_LEN + args.record_align - 1) // args.record_align * args.record_align
    g = torch.Generator(device="cuda").manual_seed(0x7715)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    sealed = torch.empty(n * SLc, dtype=torch.uint8, device="cuda")
    back = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    nonces = torch.empty(NONCE_LEN * n, dtype=torch.uint8, device="cuda")
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    hrng = torch.Generator().manual_seed(0x7716)
    iv = bytes(torch.randint(0, 256, (12,), dtype=torch.uint8, generator=hrng).tolist())
    key = bytes(torch.randint(0, 256, (16,), dtype=torch.uint8, generator=hrng).tolist())
    tgd.shard_nonces(tlsgpu, iv, 0, n, nonces)
    stream = torch.cuda.current_stream()
    per_op, ok, total_ms, mism = {}, True, 0.0, 0
    for tl, name in ((16, "aes128ccm"), (8, "aes128ccm_8")):
        c = tlsgpu.HipAESCCM(bytearray(key), tag_length=tl)
        status = torch.zeros(n, dtype=torch.uint8, device="cuda")
        seal_b = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L,
                                   out_stride=SLc, fixed_aad_len=AAD_LEN)
        open_b = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=SLc,
                                   out_stride=L, fixed_aad_len=AAD_LEN, status=status)
        ev = {"seal": [], "open": []}
        for it in range(args.warmup + args.steps):
            for op, fn, bt in (("seal", tlsgpu.seal_batch, seal_b), ("open", tlsgpu.open_batch, open_b)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn(c, bt, stream)
                e1.record(stream)
                if it >= args.warmup:
                    ev[op].append((e0, e1))
        torch.cuda.synchronize()
        good = int(status.sum().item()) == n and bool(torch.equal(back, inp))
        pick = sorted(set(list(range(0, n, max(1, n // 63)))[:63] + [n - 1]))
        for i in pick:
            nonce = tgd.tls13_nonces(iv, i, 1)
            want = O.ccm_seal(key, nonce, inp[i * L:(i + 1) * L].cpu().numpy().tobytes(),
                              bytes(tls13_aad(L)), taglen=tl)
            got = sealed[i * SLc:i * SLc + L + tl].cpu().numpy().tobytes()
            mism += int(bytes(want) != got)
        ok = ok and good
        for op in ("seal", "open"):
            ms = sum(a.elapsed_time(b) for a, b in ev[op]) / len(ev[op])
            total_ms += ms
            alg = 2 * L + AAD_LEN + NONCE_LEN + tl
            per_op["%s_%s" % (name, op)] = {
                "ms": round(ms, 3), "payload_GiBps": round(n * L / (ms / 1e3) / 2 ** 30, 1),
                "algorithmic_GBps": round(n * alg / (ms / 1e3) / 1e9, 1),
                "frac": round(n * alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    dom = max(per_op, key=lambda k: per_op[k]["ms"])
    line = {
        "metric": "GiB/s device-resident record seal/open, AES-128-CCM + AES-128-CCM_8 %d B" % L,
        "value": round(4 * n * L / (total_ms / 1e3) / 2 ** 30, 2), "unit": "GiB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "none",
        "dtype": "u8", "data": "synthetic (torch.randint payloads)",
        "config": {"workload": "SURVEY 8(f) row 2: %d x %d B TLS 1.3 records, single key, "
                               "AES-128-CCM and CCM_8, seal+open (not a BASELINE config)" % (n, L),
                   "records": n, "record_len": L, "sealed_stride": SLc},
        "per_op": per_op,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": per_op[dom]["algorithmic_GBps"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": per_op[dom]["frac"], "traffic": None},
        "oracle_checked_records": 2 * len(pick), "oracle_mismatches": mism,
        "verified": bool(ok and mism == 0)}
    if not args.no_cpu_baseline:
        cores = args.cpu_cores or host_cores()[0]
        m = 4096 if n >= 4096 else n
        x = inp[:m * L].view(m, L).cpu().numpy()
        keys = np.frombuffer(key, np.uint8).reshape(1, 16)
        nn = np.frombuffer(b"".join(tgd.tls13_nonces(iv, i, 1) for i in range(m)), np.uint8)
        ad = np.frombuffer(bytes(tls13_aad(L)) * m, np.uint8)
        obuf = np.zeros(m * (L + TAG_LEN), np.uint8)   # reused: no page faults in the timed loop
        t0, reps = time.perf_counter(), 0
        while True:
            O.batch("aesccm", "seal", keys, nn, ad, np.arange(m, dtype=np.uint64) * AAD_LEN,
                    np.full(m, AAD_LEN, np.uint32), x.reshape(-1), np.arange(m, dtype=np.uint64) * L,
                    np.full(m, L, np.uint32), m * (L + TAG_LEN),
                    np.arange(m, dtype=np.uint64) * (L + TAG_LEN), nthreads=cores, out=obuf)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": reps * m * L / dt / 2 ** 30, "unit": "GiB/s", "cores": cores,
                                "kind": "port",
                                "sample": "AES-128-CCM seal of %d x %d B records, repeated for %.1f s, "
                                          "oracle/aead_oracle.c (the C restatement of aesccm.py) "
                                          "threaded over %d cores" % (m, L, dt, cores)}
    emit(line)
    if not line["verified"]:
        sys.exit(3)


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
    # 64 sampled records (the first, the last, spread over the batch) re-sealed
    # with the C oracle under their own session key
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    mism, pick = 0, sorted(set(list(range(0, n, max(1, n // 62)))[:62] + [n - 1]))
    for i in pick:
        L_i = int(lens[i])
        pt = inp[int(in_off[i]):int(in_off[i]) + L_i].cpu().numpy().tobytes()
        got = sealed[int(out_off[i]):int(out_off[i]) + L_i + TAG_LEN].cpu().numpy().tobytes()
        want = O.gcm_seal(bytes(keys[key_idx[i]]), bytes(nonce[i]), pt, bytes(aad[i]))
        mism += int(bytes(want) != got)
    ok = ok and mism == 0
    payload = float(lens.sum())
    res = {}
    for op, lst in ms.items():
        t = sum(a.elapsed_time(b) for a, b in lst) / len(lst)
        # SURVEY 8(d) + the 4-byte key index: seal reads L + 13 + 12 + 4,
        # writes L + 16; open reads L + 16 + 13 + 12 + 4, writes L + 1
        alg = 2 * payload + n * (13 + NONCE_LEN + TAG_LEN + 4 + (1 if op == "open" else 0))
        rd = payload + n * (13 + NONCE_LEN + 4 + (TAG_LEN if op == "open" else 0))
        res[op] = {"ms": round(t, 3), "payload_GiBps": round(payload / (t / 1e3) / 2 ** 30, 1),
                   "algorithmic_GBps": round(alg / (t / 1e3) / 1e9, 1),
                   "frac": round(alg / (t / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                   "frac_read": round(rd / (t / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    dom = max(res, key=lambda k: res[k]["ms"])
    line = {"metric": "GiB/s device-resident record seal/open, AES-256-GCM, 65536 keys, "
                      "Zipf 64B-16KiB (BASELINE configs[3])",
            "value": round(2 * payload / ((res["seal"]["ms"] + res["open"]["ms"]) / 1e3) / 2 ** 30, 2),
            "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "dtype": "u8", "data": "synthetic", "records": n, "keys": nkeys,
            "record_order": "host-presorted" if args.c4_presorted else "arrival (engine planner)",
            "mean_len": round(float(lens.mean()), 1),
            "byte_weighted_mean_len": round(float((lens * lens).sum() / lens.sum()), 1),
            "per_op": res,
            "roofline": {"bound": "hbm", "kernel": "aes256gcm_%s (key table)" % dom,
                         "achieved": res[dom]["algorithmic_GBps"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": res[dom]["frac"], "frac_read": res[dom]["frac_read"],
                         "traffic": None},
            "oracle_checked_records": len(pick), "oracle_mismatches": mism,
            "verified": bool(ok)}
    tr = c4_traffic(args.traffic_file, dom) if n == 1 << 20 and not args.c4_presorted else None
    if tr:
        alg = 2 * payload + n * (13 + NONCE_LEN + TAG_LEN + 4 + (1 if dom == "open" else 0))
        tr["traffic_over_algorithmic"] = round(tr["hbm_bytes"] / alg, 3)
        line["roofline"]["traffic"] = tr["hbm_bytes"]
        line["roofline"]["traffic_detail"] = tr
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_c4(args.cpu_cores or host_cores()[0], args.cpu_seconds)
    emit(line)
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
        w = tlsgpu.RecordWriter(ms, obj(), tlsgpu.TLS13, iv, batch_records=2048)
        for p in range(0, len(data), 64 << 20):
            w.write(mv[p:p + (64 << 20)])
        w.flush()
        wire = b"".join(ms.parts)
        del ms
        ns = _NullSink()
        w = tlsgpu.RecordWriter(ns, obj(), tlsgpu.TLS13, iv, batch_records=args.ingest_batch,
                                nslots=args.ingest_slots)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for p in range(0, len(data), 64 << 20):
            w.write(mv[p:p + (64 << 20)])
        w.flush()
        t_w = time.perf_counter() - t0
        wv = memoryview(wire)
        rates, ok = {}, ns.bytes == len(wire)
        # the caller's buffer pinned (packed plaintext lands in it by DMA) or
        # pageable; socket reads of 128 MiB handed to read_application_data
        # (data=: copied into the pinned buffer a batch at a time while the
        # batches before run), or fed first (feed(): one threaded copy, then
        # the pipeline)
        for kind in ("pinned", "pageable", "pinned_feed"):
            outbuf = (np.empty(total, np.uint8) if kind == "pageable"
                      else torch.empty(total, dtype=torch.uint8).pin_memory().numpy())
            rd = args.ingest_read_mib << 20
            r = tlsgpu.RecordReader(obj(), tlsgpu.TLS13, iv, batch_records=args.ingest_batch,
                                    buffer_bytes=rd + (32 << 20), nslots=args.ingest_slots)
            ov, pos = memoryview(outbuf), 0
            t0 = time.perf_counter()
            for p in range(0, len(wire), rd):   # socket reads of --ingest-read-mib
                if kind == "pinned_feed":
                    r.feed(wv[p:p + rd])
                    pos += len(r.read_application_data(out=ov[pos:]))
                else:
                    pos += len(r.read_application_data(out=ov[pos:], data=wv[p:p + rd]))
            rates[kind] = round(total / (time.perf_counter() - t0) / 2 ** 30, 2)
            ok = ok and pos == total and hashlib.sha256(outbuf).hexdigest() == want
            del r, ov, outbuf
        res[alg] = {"write_GiBps": round(total / t_w / 2 ** 30, 2),
                    "read_GiBps": rates["pinned"], "read_pageable_out_GiBps": rates["pageable"],
                    "read_feed_first_GiBps": rates["pinned_feed"],
                    "records": w.records_sent, "wire_bytes": len(wire), "verified": ok}
        del wire
    # the bounds beside it: pinned host <-> device copies, and host copies
    # into pinned memory on 1 and on the pipeline's threads (tg_host_copy)
    from tlsgpu import ingest as _ing
    pin = torch.empty(1 << 30, dtype=torch.uint8).pin_memory().numpy()
    page = np.frombuffer(blk * 16, np.uint8)
    hc = {}
    for th in (1, _ing.COPY_THREADS):
        keep, _ing.COPY_THREADS = _ing.COPY_THREADS, th
        _ing.host_copy(pin, page)
        t0 = time.perf_counter()
        for _ in range(3):
            _ing.host_copy(pin, page)
        hc["threads_%d" % th] = round(3 * (1 << 30) / (time.perf_counter() - t0) / 2 ** 30, 2)
        _ing.COPY_THREADS = keep
    del pin, page
    line = {"metric": "GiB/s host ingest pipeline (RecordWriter / RecordReader), TLS 1.3, "
                      "16 KiB records, host memory to host memory",
            "unit": "GiB/s", "n_gpus": 1, "app_data_bytes": total, "dtype": "u8",
            "data": "synthetic", "per_alg": res, "pcie_GBps": pcie_ceiling(torch),
            "pipeline": {"batch_records": args.ingest_batch, "slots": args.ingest_slots,
                         "socket_read_bytes": args.ingest_read_mib << 20,
                         "copy_threads": _ing.COPY_THREADS},
            "host_copy_to_pinned_GiBps": hc}
    emit(line)


def pcie_ceiling(torch, nbytes=1 << 30):
    """Raw pinned-host <-> device copy rates on this box (hipMemcpyAsync via
    torch): H2D alone, D2H alone, and both at once on two streams."""
    h_in = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def t(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3

    h2d = t(lambda: d_a.copy_(h_in, non_blocking=True))
    d2h = t(lambda: h_out.copy_(d_b, non_blocking=True))

    def both():
        with torch.cuda.stream(s1):
            d_a.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_b, non_blocking=True)
    bi = t(both)
    return {"h2d_GBps": round(nbytes / h2d / 1e9, 1), "d2h_GBps": round(nbytes / d2h / 1e9, 1),
            "bidir_GBps_each_way": round(nbytes / bi / 1e9, 1), "bytes": nbytes}


def end_to_end(torch, tlsgpu, ciphers, aad, nonces, L, n):
    """Records start and end in pinned host memory (socket buffers): chunk k
    is copied in on an H2D stream, sealed on a compute stream and copied out
    on a D2H stream, each stage waiting on the previous one's event, with
    three buffer slots so H2D(k+1) || seal(k) || D2H(k-1).  Reported in
    DESIGN.md against the measured PCIe ceiling, never as ``value``."""
    chunk, slots = 8192, 3
    ceil = pcie_ceiling(torch)
    host_in = torch.randint(0, 256, (n * L,), dtype=torch.uint8).pin_memory()
    host_out = torch.empty(n * (L + TAG_LEN), dtype=torch.uint8).pin_memory()
    res = {"pcie": ceil}
    sh2d, scomp, sd2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    bufs = [(torch.empty(chunk * L, dtype=torch.uint8, device="cuda"),
             torch.empty(chunk * (L + TAG_LEN), dtype=torch.uint8, device="cuda")) for _ in range(slots)]
    for a, c in ciphers.items():
        # warm-up: the first launch of a kernel loads its code object
        b = tlsgpu.make_batch(chunk, bufs[0][0], bufs[0][1], nonces, aad=aad, fixed_len=L,
                              in_stride=L, out_stride=L + TAG_LEN, fixed_aad_len=AAD_LEN)
        tlsgpu.seal_batch(c, b, scomp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = [None] * slots          # D2H-finished event of the chunk that last used a slot
        for ci, s0 in enumerate(range(0, n, chunk)):
            k = min(chunk, n - s0)
            sl = ci % slots
            din, dout = bufs[sl]
            if done[sl] is not None:
                sh2d.wait_event(done[sl])
            with torch.cuda.stream(sh2d):
                din[:k * L].copy_(host_in[s0 * L:(s0 + k) * L], non_blocking=True)
                e_in = torch.cuda.Event()
                e_in.record(sh2d)
            scomp.wait_event(e_in)
            b = tlsgpu.make_batch(k, din, dout, nonces[12 * s0:], aad=aad, fixed_len=L,
                                  in_stride=L, out_stride=L + TAG_LEN, fixed_aad_len=AAD_LEN)
            tlsgpu.seal_batch(c, b, scomp)
            e_c = torch.cuda.Event()
            e_c.record(scomp)
            sd2h.wait_event(e_c)
            with torch.cuda.stream(sd2h):
                host_out[s0 * (L + TAG_LEN):(s0 + k) * (L + TAG_LEN)].copy_(dout[:k * (L + TAG_LEN)],
                                                                            non_blocking=True)
                done[sl] = torch.cuda.Event()
                done[sl].record(sd2h)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        bound = max(n * L / (ceil["bidir_GBps_each_way"] * 1e9),
                    n * (L + TAG_LEN) / (ceil["bidir_GBps_each_way"] * 1e9))
        res[a + "_seal"] = {"GiBps_payload": round(n * L / dt / 2 ** 30, 2), "records": n,
                            "frac_of_pcie_bidir": round(bound / dt, 3)}
    return res


if __name__ == "__main__":
    main()
