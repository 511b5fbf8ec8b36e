"""Pack record batches for the GPU tests and the bench (host numpy -> device).

A batch is described by host numpy arrays (offsets, lengths, nonces, aad) so
the same description drives libtlsgpu (device copies) and the C oracle
(host arrays) on identical inputs.
"""
import numpy as np

from vectors import tls12_aad, tls13_aad, tls13_nonce


class HostBatch(object):
    """Packed records: payloads back to back at ``in_off`` (optionally
    16-byte aligned), outputs at ``out_off``, 12-byte nonces, AAD rows."""

    def __init__(self, lens, payload_seed=0, align=16, aad_mode="tls13", key_count=1,
                 iv=None, seq0=0, open_input=None, tag=16):
        rng = np.random.default_rng(payload_seed)
        self.n = n = len(lens)
        self.tag = tag
        self.lens = np.asarray(lens, dtype=np.uint32)
        step = lambda L: ((L + align - 1) // align) * align if align > 1 else L  # noqa: E731
        in_sizes = np.array([step(int(L) + (tag if open_input is not None else 0))
                             for L in self.lens], dtype=np.uint64)
        out_sizes = np.array([step(int(L) + tag) for L in self.lens], dtype=np.uint64)
        self.in_off = np.concatenate([[0], np.cumsum(in_sizes)[:-1]]).astype(np.uint64)
        self.out_off = np.concatenate([[0], np.cumsum(out_sizes)[:-1]]).astype(np.uint64)
        self.in_bytes = int(in_sizes.sum()) + 16
        self.out_bytes = int(out_sizes.sum()) + 16
        self.inp = rng.integers(0, 256, self.in_bytes, dtype=np.uint8)
        self.iv = np.frombuffer(bytes(iv) if iv is not None else rng.bytes(12), np.uint8)
        self.seq = np.arange(seq0, seq0 + n, dtype=np.uint64)
        self.nonces = np.frombuffer(b"".join(bytes(tls13_nonce(bytes(self.iv), int(s)))
                                             for s in self.seq), np.uint8).copy()
        if aad_mode == "tls13":
            rows = [bytes(tls13_aad(int(L))) for L in self.lens]
        elif aad_mode == "tls12":
            rows = [bytes(tls12_aad(int(s), int(L))) for s, L in zip(self.seq, self.lens)]
        else:  # random lengths 0..40
            rows = [rng.bytes(int(rng.integers(0, 41))) for _ in range(n)]
        self.aad_len = np.array([len(r) for r in rows], dtype=np.uint32)
        self.aad_off = np.concatenate([[0], np.cumsum(self.aad_len)[:-1]]).astype(np.uint64)
        self.aad = np.frombuffer(b"".join(rows) + bytes(16), np.uint8).copy()
        self.key_idx = (rng.integers(0, key_count, n).astype(np.uint32)
                        if key_count > 1 else None)

    def to_device(self, torch, dev="cuda"):
        t = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        d = {
            "inp": t(self.inp), "in_off": t(self.in_off.view(np.int64)),
            "lens": t(self.lens.view(np.int32)), "out_off": t(self.out_off.view(np.int64)),
            "nonces": t(self.nonces), "aad": t(self.aad), "aad_off": t(self.aad_off.view(np.int64)),
            "aad_len": t(self.aad_len.view(np.int32)),
            "out": torch.zeros(self.out_bytes, dtype=torch.uint8, device=dev),
            "status": torch.zeros(self.n, dtype=torch.uint8, device=dev),
        }
        if self.key_idx is not None:
            d["key_idx"] = t(self.key_idx.view(np.int32))
        return d

    def batch_kwargs(self, d, open_=False):
        from tlsgpu import make_batch
        return make_batch(self.n, d["inp"], d["out"], d["nonces"], aad=d["aad"], lens=d["lens"],
                          in_off=d["in_off"], out_off=d["out_off"], aad_off=d["aad_off"],
                          aad_len=d["aad_len"], key_idx=d.get("key_idx"),
                          status=d["status"] if open_ else None)

    def oracle(self, oracle_mod, alg, keys, op="seal", inp=None, in_off=None, nthreads=8):
        src = self.inp if inp is None else inp
        off = self.in_off if in_off is None else in_off
        inlen = self.lens + (self.tag if op == "open" else 0)
        out_off = self.out_off
        return oracle_mod.batch(alg, op, keys, self.nonces, self.aad, self.aad_off, self.aad_len,
                                src, off, inlen, self.out_bytes, out_off, key_idx=self.key_idx,
                                nthreads=nthreads)


def run_seal_open(torch, tg, oracle_mod, hb, alg, keys, key_obj, tamper=()):
    """Seal ``hb`` on the GPU, compare with the oracle bit-exact, open the
    sealed records back (tag bits flipped in ``tamper``) and check status and
    plaintext (rejected records zeroed)."""
    T = hb.tag
    d = hb.to_device(torch)
    tg.seal_batch(key_obj, hb.batch_kwargs(d))
    torch.cuda.synchronize()
    got = d["out"].cpu().numpy()
    want, _ = hb.oracle(oracle_mod, alg, keys, "seal")
    for i in range(hb.n):
        o, L = int(hb.out_off[i]), int(hb.lens[i])
        assert np.array_equal(got[o:o + L + T], want[o:o + L + T]), ("seal mismatch", i, L)
    # open the sealed records back (input = ct||tag at out_off)
    sealed = got.copy()
    for i in tamper:
        o, L = int(hb.out_off[i]), int(hb.lens[i])
        sealed[o + L + (i % T)] ^= 0x20  # flip a tag bit
    src = torch.from_numpy(sealed).cuda()
    pt = torch.zeros(hb.in_bytes, dtype=torch.uint8, device="cuda")
    status = torch.zeros(hb.n, dtype=torch.uint8, device="cuda")
    b = tg.make_batch(hb.n, src, pt, d["nonces"], aad=d["aad"], lens=d["lens"],
                      in_off=d["out_off"], out_off=d["in_off"], aad_off=d["aad_off"],
                      aad_len=d["aad_len"], key_idx=d.get("key_idx"), status=status)
    tg.open_batch(key_obj, b)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    back = pt.cpu().numpy()
    for i in range(hb.n):
        o, L = int(hb.in_off[i]), int(hb.lens[i])
        if i in tamper:
            assert st[i] == 0, i
            assert not back[o:o + L].any(), "rejected record must be zeroed"
        else:
            assert st[i] == 1, i
            assert np.array_equal(back[o:o + L], hb.inp[o:o + L]), ("open mismatch", i)
