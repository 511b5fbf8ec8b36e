"""Run each AEAD kernel once on a fixed batch, for rocprofv3 counter passes.

    rocprofv3 --pmc <counters> --output-format csv -d out -- python tools/prof_kernels.py

PROF_RECORDS / PROF_LEN: batch shape (2^18 x 16 KiB); sealed records at
bench.py's 128-byte aligned stride; PROF_REPS: seal + open rounds (1);
PROF_ALGS: which AEADs (aes128gcm, chacha20-poly1305, aes128ccm); PROF_OPTS: tlsgpu options as name=value,... (e.g.
hy_t=16 for a hybrid kernel of T-table waves only, hy_t=-1 for bitsliced
waves only).
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
    n = int(os.environ.get("PROF_RECORDS", 1 << 18))
    L = int(os.environ.get("PROF_LEN", 16384))
    algs = os.environ.get("PROF_ALGS", "aes128gcm,chacha20-poly1305").split(",")
    for kv in filter(None, os.environ.get("PROF_OPTS", "").split(",")):
        k, v = kv.split("=")
        tlsgpu.set_option(k, int(v))
    reps = int(os.environ.get("PROF_REPS", 1))
    so = (L + 16 + 127) // 128 * 128
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
    back = torch.empty_like(inp)
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(12), 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    for a in algs:
        c = (tlsgpu.HipAESGCM(bytearray(16)) if a == "aes128gcm" else
             tlsgpu.HipAESCCM(bytearray(16)) if a == "aes128ccm" else
             tlsgpu.HipCHACHA20_POLY1305(bytearray(32)))
        for _ in range(reps):
            tlsgpu.seal_batch(c, tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L,
                                                   in_stride=L, out_stride=so, fixed_aad_len=5))
            tlsgpu.open_batch(c, tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L,
                                                   in_stride=so, out_stride=L, fixed_aad_len=5,
                                                   status=status))
        torch.cuda.synchronize()
        # PROF_NOCHECK=1: measurement builds whose output is not the AEAD's
        assert os.environ.get("PROF_NOCHECK") == "1" or int(status.sum()) == n
    print("prof_kernels done", n, L, algs)


if __name__ == "__main__":
    main()
