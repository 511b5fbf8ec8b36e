"""Whole-batch parity: every record of a device batch against the C oracle.

The full-size GPU tests (2^20 records) seal on the device and then hand the
whole batch to ``check_all``: it walks the records in chunks of ``chunk``
(2^16 by default, about 1 GiB of payload), copies the chunk's inputs and the
device's outputs to the host, seals the same inputs with the threaded C
oracle (``oracle.batch``, aead_oracle.c: aesgcm.py:101-124 and
chacha20_poly1305.py:48-66 restated) and compares every record byte for byte,
ciphertext and tag.  Host memory stays bounded by a few chunks.  The nonces
and AADs given here are computed on the host independently of the device
(``vectors.tls13_nonce`` semantics, vectorised), so a device nonce bug shows
as a mismatch too.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def host_threads():
    """The cores this process may use (cgroup quota aware, as bench.py's
    CPU leg): 16 on the GPU box, 8 here."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from bench import host_cores
    return host_cores()[0]


def tls13_nonces(iv, seq0, n):
    """nonce_i = iv xor (0^4 || be64(seq0 + i)) for i < n (recordlayer.py:525-530),
    as an (n, 12) uint8 array."""
    seq = (np.uint64(seq0) + np.arange(n, dtype=np.uint64)).astype(">u8")
    out = np.tile(np.frombuffer(bytes(iv), np.uint8), (n, 1))
    out[:, 4:] ^= seq.view(np.uint8).reshape(n, 8)
    return out


class Mismatch(AssertionError):
    pass


def _span(off, size, lo, hi):
    a = int(off[lo])
    b = int((off[lo:hi] + size[lo:hi]).max())
    return a, b


def check_all(torch, oracle_mod, alg, keys, d_in, in_off, lens, d_out, out_off, nonces,
              aad, aad_off, aad_len, key_idx=None, chunk=1 << 16, nthreads=None,
              inner_type=None, tag=16):
    """Seal records [0, n) of the device batch again with the C oracle and
    compare every output record (ciphertext and tag) with the device's.

    ``d_in`` / ``d_out``: device uint8 tensors; ``in_off`` / ``out_off`` /
    ``lens`` / ``aad_off`` / ``aad_len``: host arrays (record i's plaintext at
    ``d_in[in_off[i]:in_off[i] + lens[i]]``, its ct || tag at ``d_out[out_off[i]:]``);
    ``nonces``: host (n, 12); ``aad``: host uint8 buffer.  ``inner_type``: if
    set, the sealed plaintext is the TLS 1.3 inner plaintext fragment || type
    (recordlayer.py:606-617; config 5, equal fragment lengths), so the device
    record at ``out_off[i]`` is lens[i] + 1 + 16 bytes.  Returns the number of
    records and bytes checked; raises Mismatch naming the first records that
    differ.  ``tag``: the tag length (8 for AES-CCM_8)."""
    n = len(lens)
    nthreads = nthreads or host_threads()
    in_off = np.asarray(in_off, dtype=np.int64)
    out_off = np.asarray(out_off, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    aad_off = np.asarray(aad_off, dtype=np.int64)
    aad_len = np.asarray(aad_len, dtype=np.int64)
    if len(in_off) != n or len(out_off) != n or len(nonces) != n:
        raise ValueError("batch arrays disagree on n")
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    extra = 0 if inner_type is None else 1
    if extra and not (lens == lens[0]).all():
        raise ValueError("inner_type needs equal fragment lengths")
    obuf = None
    checked = 0
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        ia, ib = _span(in_off, lens, lo, hi)
        oa, ob = _span(out_off, lens + extra + tag, lo, hi)
        h_in = d_in[ia:ib].cpu().numpy()
        h_out = d_out[oa:ob].cpu().numpy()
        r_in_off = in_off[lo:hi] - ia
        r_lens = lens[lo:hi]
        if extra:
            m, L = hi - lo, int(lens[0])
            st = int(r_in_off[1] - r_in_off[0]) if m > 1 else L
            rows = np.lib.stride_tricks.as_strided(h_in[int(r_in_off[0]):], (m, L), (st, 1))
            inner = np.empty((m, L + 1), dtype=np.uint8)
            inner[:, :L] = rows
            inner[:, L] = inner_type
            h_in, r_in_off, r_lens = inner.reshape(-1), np.arange(m) * (L + 1), r_lens + 1
        r_out_off = out_off[lo:hi] - oa
        if obuf is None or obuf.size < ob - oa:
            obuf = np.zeros(ob - oa, dtype=np.uint8)
        want, _ = oracle_mod.batch(alg, "seal", keys, nonces[lo:hi], aad, aad_off[lo:hi],
                                   aad_len[lo:hi], h_in, r_in_off, r_lens, ob - oa, r_out_off,
                                   key_idx=None if key_idx is None else key_idx[lo:hi],
                                   nthreads=nthreads, out=obuf)
        rl = r_lens + tag
        m = hi - lo
        stride = int(r_out_off[1] - r_out_off[0]) if m > 1 else int(rl[0])
        uniform = bool((rl == rl[0]).all()) and stride >= int(rl[0]) and \
            (m == 1 or bool((np.diff(r_out_off) == stride).all()))
        if uniform:
            # equal records at a fixed stride: compare as one 2-D view
            o0, w = int(r_out_off[0]), int(rl[0])
            span = stride * (m - 1) + w
            g2 = np.lib.stride_tricks.as_strided(h_out[o0:o0 + span], (m, w), (stride, 1))
            w2 = np.lib.stride_tricks.as_strided(want[o0:o0 + span], (m, w), (stride, 1))
            bad = np.concatenate([r + np.nonzero((g2[r:r + 2048] != w2[r:r + 2048]).any(axis=1))[0]
                                  for r in range(0, m, 2048)])
        else:
            bad = [j for j in range(m)
                   if not np.array_equal(h_out[r_out_off[j]:r_out_off[j] + rl[j]],
                                         want[r_out_off[j]:r_out_off[j] + rl[j]])]
        if len(bad):
            first = [int(lo + j) for j in bad[:8]]
            raise Mismatch("%s: %d of records [%d, %d) differ from the oracle, first %s"
                           % (alg, len(bad), lo, hi, first))
        checked += int(rl.sum())
    return n, checked
