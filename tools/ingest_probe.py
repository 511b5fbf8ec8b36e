"""Phase timing of the ingest RecordReader on one 128 MiB feed (design probe)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tlslite-ng_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tlsgpu  # noqa: E402
from tlsgpu import ingest  # noqa: E402

iv = bytes(range(12))
data = np.random.default_rng(1).integers(0, 256, 256 << 20, dtype=np.uint8).tobytes()


class Mem(object):
    def __init__(self):
        self.p = []

    def sendall(self, mv):
        self.p.append(bytes(mv))


m = Mem()
w = tlsgpu.RecordWriter(m, tlsgpu.HipAESGCM(bytearray(16)), tlsgpu.TLS13, iv, batch_records=8192)
w.write(data)
w.flush()
wire = b"".join(m.p)
r = tlsgpu.RecordReader(tlsgpu.HipAESGCM(bytearray(16)), tlsgpu.TLS13, iv, batch_records=8192,
                        buffer_bytes=160 << 20)
T = {}


def tm(name, f, *a):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    v = f(*a)
    torch.cuda.synchronize()
    T[name] = T.get(name, 0) + time.perf_counter() - t0
    return v


orig_open, orig_scan = r._open, r._scan
r._open = lambda n, used: tm("open", orig_open, n, used)
r._scan = lambda: tm("scan", orig_scan)
wv = memoryview(wire)
out = np.empty(len(data), np.uint8)
pos = 0
for p in range(0, len(wire), 128 << 20):
    tm("feed", r.feed, wv[p:p + (128 << 20)])
    pos += len(tm("read_app", r.read_application_data, memoryview(out)[pos:]))
assert pos == len(data) and out.tobytes() == data
print({k: round(v * 1e3, 1) for k, v in T.items()}, "ms for", len(data) >> 20, "MiB")
