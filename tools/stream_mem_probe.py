"""Device memory per new stream: what a first launch on a fresh stream costs
(VERDICT r05 item 6).

For each launch kind, 24 fresh torch streams each run one launch; the
device's used memory (hipMemGetInfo through torch.cuda.mem_get_info) is read
before and after, and the scratch the library itself holds
(tg_scratch_info) is subtracted.  Kinds:

  torch      a torch elementwise kernel (no library call, no private segment)
  nonces     tg_make_nonces (a library kernel with no private segment)
  chacha     ChaCha20-Poly1305 batch (lane kernel: private segment 40 B in
             round 5, none since round 6)
  aesgcm     AES-128-GCM batch (hybrid kernel: private segment 92 B in
             round 5, none since round 6)

usage: python tools/stream_mem_probe.py  -> one JSON line per kind
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)


def hip_streams(k):
    """k fresh HIP streams (raw handles: torch's own pool hands out 32
    streams round robin, so its streams would be warm after the first kind)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = []
    for _ in range(k):
        h = ctypes.c_void_p()
        if hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) != 0:
            raise RuntimeError("hipStreamCreateWithFlags failed")
        out.append(h.value)
    return out


def main():
    import torch
    import tlsgpu
    from vectors import tls13_aad
    n, L = 65536, 1024
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    out = torch.zeros(n * (L + 16), dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(bytes(12), 0, n, nonces)
    b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=L + 16,
                          fixed_aad_len=5)
    gcm = tlsgpu.HipAESGCM(bytearray(16))
    cc = tlsgpu.HipCHACHA20_POLY1305(bytearray(32))
    x = torch.zeros(1 << 20, device="cuda")
    kinds = {
        "torch": lambda st: x.add_(1.0),   # on torch.cuda.ExternalStream(st)
        "nonces": lambda st: tlsgpu.make_nonces(bytes(12), 0, n, nonces, stream=st),
        "chacha": lambda st: tlsgpu.seal_batch(cc, b, st),
        "aesgcm": lambda st: tlsgpu.seal_batch(gcm, b, st),
    }
    for f in kinds.values():
        f(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for name, f in kinds.items():
        torch.cuda.synchronize()
        free_pre = torch.cuda.mem_get_info()[0]
        streams = hip_streams(24)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        lib0 = tlsgpu.scratch_info()[0]
        for h in streams:
            st = torch.cuda.ExternalStream(h)
            with torch.cuda.stream(st):
                f(h)
            st.synchronize()
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info()[0]
        lib1 = tlsgpu.scratch_info()[0]
        used = (free0 - free1) - (lib1 - lib0)
        print(json.dumps({"kind": name, "streams": 24, "create_bytes": free_pre - free0, "device_bytes": free0 - free1,
                          "library_scratch_bytes": lib1 - lib0,
                          "other_per_stream_mib": round(used / 24 / 2**20, 3)}), flush=True)


def torch_pool(kinds):
    """The same on torch's own stream pool (32 streams per device, created
    together on first use, handed out round robin), as tests/test_gpu_scratch.py
    uses: a separate process per kind, so every kind meets fresh pool streams."""
    import subprocess
    for name in kinds:
        code = (
            "import sys, json; sys.path[:0] = %r\n"
            "import torch, tlsgpu\n"
            "from vectors import tls13_aad\n"
            "n, L = 65536, 1024\n"
            "inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device='cuda')\n"
            "out = torch.zeros(n * (L + 16), dtype=torch.uint8, device='cuda')\n"
            "nonces = torch.zeros(12 * n, dtype=torch.uint8, device='cuda')\n"
            "aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device='cuda')\n"
            "b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=L + 16, fixed_aad_len=5)\n"
            "gcm = tlsgpu.HipAESGCM(bytearray(16))\n"
            "f = {'nonces': lambda st: tlsgpu.make_nonces(bytes(12), 0, n, nonces, stream=st),"
            " 'aesgcm': lambda st: tlsgpu.seal_batch(gcm, b, st)}[%r]\n"
            "f(None); torch.cuda.synchronize()\n"
            "streams = [torch.cuda.Stream() for _ in range(40)]\n"
            "torch.cuda.synchronize(); free0 = torch.cuda.mem_get_info()[0]; lib0 = tlsgpu.scratch_info()[0]\n"
            "for st in streams:\n"
            "    f(st); st.synchronize()\n"
            "torch.cuda.synchronize(); free1 = torch.cuda.mem_get_info()[0]; lib1 = tlsgpu.scratch_info()[0]\n"
            "print(json.dumps({'kind': 'torch_pool_' + %r, 'streams': 40, 'device_bytes': free0 - free1,"
            " 'library_scratch_bytes': lib1 - lib0, 'per_pool_stream_mib': round((free0 - free1 - (lib1 - lib0)) / 32 / 2**20, 3)}))\n"
        ) % ([ROOT, os.path.join(ROOT, "tlslite-ng_amd"), os.path.join(ROOT, "tests", "golden")], name, name)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
        print(r.stdout.strip() or r.stderr[-500:], flush=True)


if __name__ == "__main__":
    if "--torch-pool" in sys.argv:
        torch_pool(["nonces", "aesgcm"])
        sys.exit(0)
    main()
