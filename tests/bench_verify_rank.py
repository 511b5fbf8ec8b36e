"""One rank of tests/test_bench_verify.py (started by torch.distributed.run,
gloo, CPU): the tail of bench.py's headline / config-5 legs -- every rank's
own sampled records checked against the C oracle at its own seq offset,
the verdict reduced over all ranks (bench.verify_shards), rank 0's JSON line
and the exit status (bench.finish) -- on records the oracle itself sealed for
this rank's shard (the GPU's part is the -m gpu tests' job).

    mode "headline" | "c5": correct records; TLSGPU_BENCH_CORRUPT_RANK=r
        flips a byte of one record on rank r (bench.corrupt_for_test);
    mode "c5-noshift": rank 1 seals its records at seq i instead of
        first + i, the wrong-offset bug a seal -> open round trip cannot see.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import records as R  # noqa: E402
from tlsgpu import distributed as tgd  # noqa: E402
from vectors import tls13_aad  # noqa: E402


def main():
    mode = sys.argv[1]
    world, rank, _, _ = tgd.init_process(torch, dist, backend="gloo", use_gpu=False)
    n = 6
    first, _ = tgd.weak_shard(n, world, rank)
    key, iv = bytes(range(16)), bytes(range(100, 112))
    frags = [bytes((rank * 31 + i * 7 + j) & 0xff for j in range(300 + 17 * i)) for i in range(n)]
    if mode == "headline":
        samples = []
        for i, pt in enumerate(frags):
            nonce = tgd.tls13_nonces(iv, first + i, 1)
            aad = bytes(tls13_aad(len(pt)))
            samples.append(("aes128gcm", key, nonce, pt, aad, bytes(O.gcm_seal(key, nonce, pt, aad))))
        bad = bench.headline_check(bench.corrupt_for_test(samples, rank, 5))
    else:
        shift = 0 if (mode == "c5-noshift" and rank == 1) else first
        samples = [(i, f, R.seal_record("tls13", "aes128gcm", key, iv, shift + i, 0x17, f))
                   for i, f in enumerate(frags)]
        bad = bench.c5_check(bench.corrupt_for_test(samples, rank, 2), key, iv, first)
    # each rank's own round trip passed (the device part is not run here)
    ok, mism, checked = bench.verify_shards(torch, dist, True, bad, len(samples))
    if rank == 0:
        bench.emit({"mode": mode, "n_gpus": world, "verified": ok, "oracle_mismatches": mism,
                    "oracle_checked_records": checked})
    bench.finish(dist, ok)


if __name__ == "__main__":
    main()
