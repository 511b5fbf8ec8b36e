"""GPU: the per-launch scratch of the hybrid AES-GCM kernel (job counter,
batch copy and the per-record keystream masks) comes from the library's
scratch cache and goes back behind each launch: batches
launched on many streams leave device memory flat, and their records stay
right."""
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
    # of them.  Each stream first runs a ChaCha20-Poly1305 batch (no
    # per-launch scratch), so whatever the runtime keeps per stream is there
    # before the count starts; then one AES-GCM batch per stream.
    chacha = tlsgpu.HipCHACHA20_POLY1305(bytearray(32))
    streams = [torch.cuda.Stream() for _ in range(40)]
    tlsgpu.seal_batch(obj, b)                 # the cache's first buffer
    for st in streams:
        tlsgpu.seal_batch(chacha, b, st)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for st in streams:
        tlsgpu.seal_batch(obj, b, st)
        st.synchronize()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    # per-stream buffers kept for the process would hold 32 x 1 MiB here
    assert free0 - free1 < 8 << 20, (free0, free1)
    tlsgpu.seal_batch(obj, b)
    torch.cuda.synchronize()
    recs, _ = fullcheck.check_all(torch, oracle_mod, "aesgcm", np.frombuffer(key, np.uint8), inp,
                                  np.arange(n) * L, np.full(n, L), out, np.arange(n) * (L + 16),
                                  fullcheck.tls13_nonces(iv, 0, n),
                                  np.frombuffer(bytes(tls13_aad(L)), np.uint8), np.zeros(n), np.full(n, 5))
    assert recs == n
