"""Pure-Python restatement of tlslite-ng's pure-Python AEAD path.

TEST INFRASTRUCTURE ONLY (checker / reported CPU baseline; never shipped or
measured as the product).  This is what ``bench.py`` times on the GPU box's
host cores as the stand-in for the reference's own pure-Python path, which
cannot travel to the box.  It keeps the reference's algorithmic shape so its
speed is representative of the reference, checked in this container by
``tests/golden/make_golden.py --timing`` (ratio recorded in DESIGN.md):

* AES: 32-bit T-table rounds over big-endian column words, like
  ``Rijndael.encrypt`` (tlslite/utils/rijndael.py:995-1038);
* CTR: one block encryption per 16 bytes, counter incremented as a 128-bit
  big-endian integer (tlslite/utils/python_aes.py:101-116);
* GHASH: 4-bit product table of H over Python ints in the bit-reflected
  representation (tlslite/utils/aesgcm.py:46-99);
* ChaCha20: list-of-words double rounds (tlslite/utils/chacha.py:68-153);
* Poly1305: bigint Horner mod 2^130-5 (tlslite/utils/poly1305.py:32-48).
"""
import struct

# --------------------------------------------------------------------- AES

def _xt(a):
    a <<= 1
    return (a ^ 0x11b) if a & 0x100 else a


def _tables():
    exp, log = [0] * 512, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= _xt(x)          # multiply by the generator 3
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    sbox = []
    for v in range(256):
        inv = 0 if v == 0 else exp[255 - log[v]]
        s = inv
        for _ in range(4):
            inv = ((inv << 1) | (inv >> 7)) & 0xff
            s ^= inv
        sbox.append(s ^ 0x63)
    te = [[0] * 256 for _ in range(4)]
    for v in range(256):
        s = sbox[v]
        s2 = _xt(s)
        w = (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s)
        for k in range(4):
            te[k][v] = ((w >> (8 * k)) | (w << (32 - 8 * k))) & 0xffffffff
    return sbox, te


_SBOX, _TE = _tables()


def expand_key(key):
    """AES key schedule as 32-bit big-endian words (rijndael.py:922-993)."""
    nk = len(key) // 4
    if nk not in (4, 6, 8):
        raise ValueError("bad key length")
    nr = nk + 6
    w = list(struct.unpack(">%dI" % nk, bytes(key)))
    rcon = 1
    for i in range(nk, 4 * (nr + 1)):
        t = w[i - 1]
        if i % nk == 0:
            t = ((t << 8) | (t >> 24)) & 0xffffffff
            t = ((_SBOX[t >> 24] << 24) | (_SBOX[(t >> 16) & 0xff] << 16) |
                 (_SBOX[(t >> 8) & 0xff] << 8) | _SBOX[t & 0xff])
            t ^= rcon << 24
            rcon = _xt(rcon)
        elif nk > 6 and i % nk == 4:
            t = ((_SBOX[t >> 24] << 24) | (_SBOX[(t >> 16) & 0xff] << 16) |
                 (_SBOX[(t >> 8) & 0xff] << 8) | _SBOX[t & 0xff])
        w.append(w[i - nk] ^ t)
    return nr, w


def aes_encrypt(ks, block):
    nr, w = ks
    t0, t1, t2, t3 = _TE
    s0, s1, s2, s3 = struct.unpack(">4I", bytes(block))
    s0 ^= w[0]; s1 ^= w[1]; s2 ^= w[2]; s3 ^= w[3]
    k = 4
    for _ in range(nr - 1):
        a0 = t0[s0 >> 24] ^ t1[(s1 >> 16) & 255] ^ t2[(s2 >> 8) & 255] ^ t3[s3 & 255] ^ w[k]
        a1 = t0[s1 >> 24] ^ t1[(s2 >> 16) & 255] ^ t2[(s3 >> 8) & 255] ^ t3[s0 & 255] ^ w[k + 1]
        a2 = t0[s2 >> 24] ^ t1[(s3 >> 16) & 255] ^ t2[(s0 >> 8) & 255] ^ t3[s1 & 255] ^ w[k + 2]
        a3 = t0[s3 >> 24] ^ t1[(s0 >> 16) & 255] ^ t2[(s1 >> 8) & 255] ^ t3[s2 & 255] ^ w[k + 3]
        s0, s1, s2, s3 = a0, a1, a2, a3
        k += 4
    sb = _SBOX
    out = []
    for c, (x0, x1, x2, x3) in enumerate(((s0, s1, s2, s3), (s1, s2, s3, s0),
                                          (s2, s3, s0, s1), (s3, s0, s1, s2))):
        v = ((sb[x0 >> 24] << 24) | (sb[(x1 >> 16) & 255] << 16) |
             (sb[(x2 >> 8) & 255] << 8) | sb[x3 & 255]) ^ w[k + c]
        out.append(v)
    return bytearray(struct.pack(">4I", *out))


# ------------------------------------------------------------------- GHASH

_RED = [0x0000, 0x1c20, 0x3840, 0x2460, 0x7080, 0x6ca0, 0x48c0, 0x54e0,
        0xe100, 0xfd20, 0xd940, 0xc560, 0x9180, 0x8da0, 0xa9c0, 0xb5e0]


def _rev4(i):
    return ((i & 1) << 3) | ((i & 2) << 1) | ((i & 4) >> 1) | ((i & 8) >> 3)


def _ghash_table(h):
    tbl = [0] * 16
    tbl[_rev4(1)] = h
    for i in range(2, 16, 2):
        v = tbl[_rev4(i // 2)]
        v = (v >> 1) ^ (0xe1 << 120) if v & 1 else v >> 1
        tbl[_rev4(i)] = v
        tbl[_rev4(i + 1)] = v ^ h
    return tbl


def _gmul(tbl, y):
    r = 0
    for _ in range(32):
        r = (r >> 4) ^ (_RED[r & 15] << 112) ^ tbl[y & 15]
        y >>= 4
    return r


def _ghash(tbl, y, data):
    n = len(data)
    for i in range(0, n - n % 16, 16):
        y = _gmul(tbl, y ^ int.from_bytes(data[i:i + 16], "big"))
    if n % 16:
        y = _gmul(tbl, y ^ int.from_bytes(bytes(data[n - n % 16:]).ljust(16, b"\0"), "big"))
    return y


class AESGCM(object):
    """Same object contract as tlslite/utils/aesgcm.py:27-57."""

    def __init__(self, key):
        if len(key) not in (16, 32):
            raise AssertionError()
        self.key = bytearray(key)
        self._ks = expand_key(key)
        self._tbl = _ghash_table(int.from_bytes(aes_encrypt(self._ks, bytes(16)), "big"))

    def _ctr(self, nonce, data):
        base = int.from_bytes(bytes(nonce) + b"\0\0\0\2", "big")
        out = bytearray(len(data))
        for j in range(0, len(data), 16):
            ks = aes_encrypt(self._ks, ((base + j // 16) % (1 << 128)).to_bytes(16, "big"))
            chunk = data[j:j + 16]
            out[j:j + len(chunk)] = bytes(a ^ b for a, b in zip(chunk, ks))
        return out

    def _tag(self, nonce, ct, aad):
        mask = aes_encrypt(self._ks, bytes(nonce) + b"\0\0\0\1")
        y = _ghash(self._tbl, 0, aad)
        y = _ghash(self._tbl, y, ct)
        y = _gmul(self._tbl, y ^ ((len(aad) << 67) | (len(ct) << 3)))
        return bytearray((y ^ int.from_bytes(mask, "big")).to_bytes(16, "big"))

    def seal(self, nonce, plaintext, data):
        if len(nonce) != 12:
            raise ValueError("Bad nonce length")
        ct = self._ctr(nonce, plaintext)
        return ct + self._tag(nonce, ct, data)

    def open(self, nonce, ciphertext, data):
        if len(nonce) != 12:
            raise ValueError("Bad nonce length")
        if len(ciphertext) < 16:
            return None
        ct, tag = ciphertext[:-16], ciphertext[-16:]
        if self._tag(nonce, ct, data) != tag:
            return None
        return self._ctr(nonce, ct)


# ---------------------------------------------------------------- ChaCha20

def _chacha_block(kw, ctr, nw):
    st = [0x61707865, 0x3320646e, 0x79622d32, 0x6b206574] + kw + [ctr] + nw
    x = st[:]
    m = 0xffffffff
    for _ in range(10):
        for a, b, c, d in ((0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
                           (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)):
            xa, xb, xc, xd = x[a], x[b], x[c], x[d]
            xa = (xa + xb) & m; xd ^= xa; xd = ((xd << 16) & m) | (xd >> 16)
            xc = (xc + xd) & m; xb ^= xc; xb = ((xb << 12) & m) | (xb >> 20)
            xa = (xa + xb) & m; xd ^= xa; xd = ((xd << 8) & m) | (xd >> 24)
            xc = (xc + xd) & m; xb ^= xc; xb = ((xb << 7) & m) | (xb >> 25)
            x[a], x[b], x[c], x[d] = xa, xb, xc, xd
    return struct.pack("<16I", *[(p + q) & m for p, q in zip(st, x)])


def chacha20_xor(key, nonce, counter, data):
    kw = list(struct.unpack("<8I", bytes(key)))
    nw = list(struct.unpack("<3I", bytes(nonce)))
    out = bytearray(len(data))
    for j in range(0, len(data), 64):
        ks = _chacha_block(kw, counter + j // 64, nw)
        chunk = data[j:j + 64]
        out[j:j + len(chunk)] = bytes(a ^ b for a, b in zip(chunk, ks))
    return out


_P1305 = (1 << 130) - 5


def poly1305(key, data):
    r = int.from_bytes(bytes(key[:16]), "little") & 0x0ffffffc0ffffffc0ffffffc0fffffff
    s = int.from_bytes(bytes(key[16:32]), "little")
    acc = 0
    for j in range(0, len(data), 16):
        chunk = bytes(data[j:j + 16]) + b"\x01"
        acc = ((acc + int.from_bytes(chunk, "little")) * r) % _P1305
    return bytearray(((acc + s) & ((1 << 128) - 1)).to_bytes(16, "little"))


def _pad16(n):
    return bytes((16 - n % 16) % 16)


class CHACHA20_POLY1305(object):
    """Same object contract as tlslite/utils/chacha20_poly1305.py:19-32."""

    def __init__(self, key):
        if len(key) != 32:
            raise ValueError("Key must be 256 bit long")
        self.key = bytearray(key)

    def _tag(self, nonce, ct, aad):
        otk = chacha20_xor(self.key, nonce, 0, bytes(32))
        mac = (bytes(aad) + _pad16(len(aad)) + bytes(ct) + _pad16(len(ct)) +
               struct.pack("<QQ", len(aad), len(ct)))
        return poly1305(otk, mac)

    def seal(self, nonce, plaintext, data):
        if len(nonce) != 12:
            raise ValueError("Nonce must be 96 bit large")
        ct = chacha20_xor(self.key, nonce, 1, plaintext)
        return ct + self._tag(nonce, ct, data)

    def open(self, nonce, ciphertext, data):
        if len(nonce) != 12:
            raise ValueError("Nonce must be 96 bit long")
        if len(ciphertext) < 16:
            return None
        ct, tag = ciphertext[:-16], ciphertext[-16:]
        if self._tag(nonce, ct, data) != tag:
            return None
        return chacha20_xor(self.key, nonce, 1, ct)
