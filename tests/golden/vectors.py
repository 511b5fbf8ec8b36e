"""Deterministic inputs shared by the golden generator and the tests.

Inputs are expanded from short labels with SHA-256 in counter mode, so the
fixtures only need to store labels, lengths and the reference's outputs; the
GPU box regenerates the same bytes without the reference.
"""
import hashlib
import json
import os

GOLDEN_DIR = os.path.dirname(os.path.abspath(__file__))


def detbytes(label, n):
    """n deterministic bytes derived from ``label`` (str)."""
    out = bytearray()
    ctr = 0
    seed = label.encode()
    while len(out) < n:
        out += hashlib.sha256(seed + ctr.to_bytes(8, "big")).digest()
        ctr += 1
    return bytearray(out[:n])


def sha256hex(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def load(name):
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return json.load(f)


def tls13_nonce(iv, seq):
    """fixed IV xor (0^4 || seq_be64) -- tlslite/recordlayer.py:525-530."""
    pad = bytes(4) + int(seq).to_bytes(8, "big")
    return bytearray(a ^ b for a, b in zip(iv, pad))


def tls13_aad(ct_len):
    """TLS 1.3 record header 0x17 0x0303 len(ct||tag) -- recordlayer.py:546-552."""
    n = ct_len + 16
    return bytearray([0x17, 0x03, 0x03, (n >> 8) & 0xff, n & 0xff])


def tls12_aad(seq, ptlen, ctype=0x17, version=(3, 3)):
    """seq || type || version || len -- tlslite/recordlayer.py:540-545."""
    return bytearray(int(seq).to_bytes(8, "big") + bytes([ctype, version[0], version[1],
                                                         (ptlen >> 8) & 0xff, ptlen & 0xff]))


# Vector grid.
LENGTHS = [0, 1, 15, 16, 17, 63, 64, 65, 255, 256, 1023, 1024, 1025,
           16383, 16384, 16385, 16400]
AAD_LENGTHS = [0, 5, 13, 20]
ALGS = [("aes128gcm", 16), ("aes256gcm", 32), ("chacha20-poly1305", 32)]
FULL_HEX_MAX = 256   # store the whole ct||tag up to this plaintext length


def config1_inputs(n=4096, length=1024):
    """BASELINE.json configs[0]: ChaCha20-Poly1305, n x 1 KiB, random.Random(0).

    key 32 B, iv 12 B, then one fresh plaintext per record; nonce_i =
    iv xor seq_i, AAD_i = TLS 1.3 header.
    """
    import random
    rng = random.Random(0)
    key = bytearray(rng.randbytes(32))
    iv = bytearray(rng.randbytes(12))
    pts = [bytearray(rng.randbytes(length)) for _ in range(n)]
    return key, iv, pts
