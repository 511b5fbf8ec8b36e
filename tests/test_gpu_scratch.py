"""GPU: the per-launch scratch of the hybrid AES-GCM kernel (job counter,
batch copy and the per-record keystream masks) comes from the library's
scratch cache and goes back behind each launch: batches
launched on many streams leave the library's memory and device memory as a
whole flat, and their records stay right."""
import numpy as np
import pytest

from vectors import tls13_aad

pytestmark = pytest.mark.gpu


def test_many_streams_memory_flat(oracle_mod):
    import torch
    import tlsgpu
    import fullcheck
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    n, L = 32768, 256          # above the wave-kernel range: the hybrid kernel (1 MiB of masks)
    key, iv = bytes(range(16)), bytes(range(40, 52))
    obj = tlsgpu.HipAESGCM(bytearray(key))
    g = torch.Generator(device="cuda").manual_seed(11)
    inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.zeros(n * (L + 16), dtype=torch.uint8, device="cuda")
    nonces = torch.zeros(12 * n, dtype=torch.uint8, device="cuda")
    tlsgpu.make_nonces(iv, 0, n, nonces)
    aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
    b = tlsgpu.make_batch(n, inp, out, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=L + 16,
                          fixed_aad_len=5)
    # torch hands out its pool of 32 streams round robin: 40 streams use all
    # of them.  The library's own scratch must not grow with the streams: at
    # most the buffers of the launches in flight (one here, plus the first).
    streams = [torch.cuda.Stream() for _ in range(40)]
    # each pool stream set up by a torch op first: the queue's own memory
    # (1.2 MiB per pool stream, profiles/r06/y1/stream_mem.jsonl) is torch's
    for st in streams:
        with torch.cuda.stream(st):
            torch.zeros(1, device="cuda").add_(1)
    tlsgpu.seal_batch(obj, b)
    torch.cuda.synchronize()
    bytes0, bufs0 = tlsgpu.scratch_info()
    free0 = torch.cuda.mem_get_info()[0]
    for st in streams:
        tlsgpu.seal_batch(obj, b, st)
        st.synchronize()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    bytes1, bufs1 = tlsgpu.scratch_info()
    # per-stream buffers kept for the process would hold 32 more here
    assert bufs1 <= bufs0 + 1 and bytes1 <= bytes0 + (2 << 20), (bytes0, bufs0, bytes1, bufs1)
    # Device memory as a whole stays flat.  A kernel with a private segment
    # (register spills) makes the HIP runtime allocate scratch for every queue
    # it first runs on: 3.0 MiB per stream for the hybrid AES-GCM kernel while
    # it spilled 22 VGPRs (profiles/r06/x10/stream_mem.jsonl).  The default
    # hybrid and ChaCha20-Poly1305 kernels have none since round 6
    # (tests/test_kernel_metadata.py), and tools/stream_mem_probe.py measures 0
    # per stream for them (profiles/r06/y1/stream_mem.jsonl).  So only the
    # library's own scratch, checked above, may grow, plus slack.
    grew = free0 - free1
    bound = (bytes1 - bytes0) + (8 << 20)
    assert grew <= bound, (grew / 2**20, bound / 2**20)
    # many launches in flight on one stream reuse one buffer (stream order)
    for _ in range(20):
        tlsgpu.seal_batch(obj, b, streams[0])
    torch.cuda.synchronize()
    assert tlsgpu.scratch_info()[1] == bufs1
    tlsgpu.seal_batch(obj, b)
    torch.cuda.synchronize()
    recs, _ = fullcheck.check_all(torch, oracle_mod, "aesgcm", np.frombuffer(key, np.uint8), inp,
                                  np.arange(n) * L, np.full(n, L), out, np.arange(n) * (L + 16),
                                  fullcheck.tls13_nonces(iv, 0, n),
                                  np.frombuffer(bytes(tls13_aad(L)), np.uint8), np.zeros(n), np.full(n, 5))
    assert recs == n
