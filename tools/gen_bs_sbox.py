"""Generate csrc/aes_bs_sbox.h: Boyar and Peralta's 113-gate AES S-box circuit
(32 AND, 77 XOR, 4 XNOR; top linear layer Y*, nonlinear core T2..T45 / Z*,
bottom linear layer) with single-use XOR/AND chains fused into 3-input
v_bitop3_b32 gates (any 3-input boolean function is one full-rate
instruction on gfx950).  The circuit is checked against the AES S-box for all
256 inputs before anything is written.  (Round 1 used their depth-16,
128-gate circuit: 84 fused gates; this one fuses to 76.)  A gate is recomputed inside its
consumers (and dropped) whenever every consumer still has at most three
distinct inputs afterwards; repeated to a fixed point.

    python3 tools/gen_bs_sbox.py > tlslite-ng_amd/csrc/aes_bs_sbox.h
"""
import itertools

CIRCUIT = """
Y14=U3^U5 Y13=U0^U6 Y9=U0^U3 Y8=U0^U5 T0=U1^U2 Y1=T0^U7 Y4=Y1^U3 Y12=Y13^Y14 Y2=Y1^U0 Y5=Y1^U6
Y3=Y5^Y8 T1=U4^Y12 Y15=T1^U5 Y20=T1^U1 Y6=Y15^U7 Y10=Y15^T0 Y11=Y20^Y9 Y7=U7^Y11 Y17=Y10^Y11
Y19=Y10^Y8 Y16=T0^Y11 Y21=Y13^Y16 Y18=U0^Y16
T2=Y12&Y15 T3=Y3&Y6 T4=T3^T2 T5=Y4&U7 T6=T5^T2 T7=Y13&Y16 T8=Y5&Y1 T9=T8^T7 T10=Y2&Y7 T11=T10^T7
T12=Y9&Y11 T13=Y14&Y17 T14=T13^T12 T15=Y8&Y10 T16=T15^T12 T17=T4^T14 T18=T6^T16 T19=T9^T14
T20=T11^T16 T21=T17^Y20 T22=T18^Y19 T23=T19^Y21 T24=T20^Y18 T25=T21^T22 T26=T21&T23 T27=T24^T26
T28=T25&T27 T29=T28^T22 T30=T23^T24 T31=T22^T26 T32=T31&T30 T33=T32^T24 T34=T23^T33 T35=T27^T33
T36=T24&T35 T37=T36^T34 T38=T27^T36 T39=T29&T38 T40=T25^T39 T41=T40^T37 T42=T29^T33 T43=T29^T40
T44=T33^T37 T45=T42^T41
Z0=T44&Y15 Z1=T37&Y6 Z2=T33&U7 Z3=T43&Y16 Z4=T40&Y1 Z5=T29&Y7 Z6=T42&Y11 Z7=T45&Y17 Z8=T41&Y10
Z9=T44&Y12 Z10=T37&Y3 Z11=T33&Y4 Z12=T43&Y13 Z13=T40&Y5 Z14=T29&Y2 Z15=T42&Y9 Z16=T45&Y14 Z17=T41&Y8
T46=Z15^Z16 T47=Z10^Z11 T48=Z5^Z13 T49=Z9^Z10 T50=Z2^Z12 T51=Z2^Z5 T52=Z7^Z8 T53=Z0^Z3 T54=Z6^Z7
T55=Z16^Z17 T56=Z12^T48 T57=T50^T53 T58=Z4^T46 T59=Z3^T54 T60=T46^T57 T61=Z14^T57 T62=T52^T58
T63=T49^T58 T64=Z4^T59 T65=T61^T62 T66=Z1^T63 S0=T59^T63 S6=T56^T62 S7=T48^T60 T67=T64^T65
S3=T53^T66 S4=T51^T66 S5=T47^T65 S1=T64^S3 S2=T55^T67
"""
# U0 = input bit 7 .. U7 = bit 0, S0 = output bit 7 .. S7 = bit 0; the four
# XNORs (S1, S2, S6, S7) are written as XORs, so the circuit computes
# S(x) ^ 0x63 (the constant is folded into the round keys, aes_bs.h)

gates, order = {}, []
for tok in CIRCUIT.split():
    out, expr = tok.split("=")
    op = "^" if "^" in expr else "&"
    x, y = expr.split(op)
    gates[out] = (op, x, y)
    order.append(out)
INPUTS = ["U%d" % i for i in range(8)]   # U0 = bit 7 ... U7 = bit 0


def _aes_sbox(v):
    def xt(a):
        return ((a << 1) ^ (0x1b if a & 0x80 else 0)) & 0xff
    exp, log, x = [0] * 256, [0] * 256, 1
    for i in range(255):
        exp[i], log[x] = x, i
        x ^= xt(x)
    inv = exp[(255 - log[v]) % 255] if v else 0
    s, r = inv, inv
    for _ in range(4):
        r = ((r << 1) | (r >> 7)) & 0xff
        s ^= r
    return s ^ 0x63


for _v in range(256):
    _env = {"U%d" % i: (_v >> (7 - i)) & 1 for i in range(8)}
    for _g in order:
        _op, _a, _b = gates[_g]
        _env[_g] = _env[_a] ^ _env[_b] if _op == "^" else _env[_a] & _env[_b]
    assert sum(_env["S%d" % i] << (7 - i) for i in range(8)) == _aes_sbox(_v) ^ 0x63, _v

# expression trees: node -> ("^"|"&", left, right) with leaves = names of
# live nodes / inputs.  A node is absorbed (recomputed inside each consumer)
# when every consumer still has at most three distinct leaves afterwards;
# repeat until nothing changes.
tree = {g: (gates[g][0], gates[g][1], gates[g][2]) for g in order}
live = set(order)


def leaves_of(t):
    if isinstance(t, str):
        return {t}
    return leaves_of(t[1]) | leaves_of(t[2])


def subst(t, name, rep):
    if isinstance(t, str):
        return rep if t == name else t
    return (t[0], subst(t[1], name, rep), subst(t[2], name, rep))


def cover(cand_order):
    tr = dict(tree)
    lv = set(order)
    changed = True
    while changed:
        changed = False
        for n in cand_order:
            if n not in lv or n.startswith("S"):
                continue
            cons = [c for c in order if c in lv and n in leaves_of(tr[c])]
            if cons and all(len((leaves_of(tr[c]) - {n}) | leaves_of(tr[n])) <= 3 for c in cons):
                for c in cons:
                    tr[c] = subst(tr[c], n, tr[n])
                lv.discard(n)
                changed = True
    return tr, lv


# the absorption order matters: keep the best of a few seeded shuffles
import random
best = cover(order)
for seed in range(4000):
    co = list(order)
    random.Random(seed).shuffle(co)
    cand = cover(co)
    if len(cand[1]) < len(best[1]):
        best = cand
tree, live = best


def evaluate(t, env):
    if isinstance(t, str):
        return env[t]
    x, y = evaluate(t[1], env), evaluate(t[2], env)
    return x ^ y if t[0] == "^" else x & y


def key(v):
    return (v[0], int(v[1:]))


def var(n):   # outputs are emitted as o0..o7 (an output may feed another)
    return "o" + n[1:] if n.startswith("S") else n


lines = []
for g in order:
    if g not in live:
        continue
    t = tree[g]
    name = g if not g.startswith("S") else "o" + g[1:]
    leaves = sorted(leaves_of(t), key=key)
    if isinstance(t[1], str) and isinstance(t[2], str):
        lines.append("    const uint32_t %s = %s %s %s;" % (name, var(t[1]), t[0], var(t[2])))
        continue
    while len(leaves) < 3:
        leaves.append(leaves[0])
    tt = 0
    for a, b, c in itertools.product((0, 1), repeat=3):
        if evaluate(t, {leaves[0]: a, leaves[1]: b, leaves[2]: c}):
            tt |= 1 << (a * 4 + b * 2 + c)
    lines.append("    const uint32_t %s = bop3(%s, %s, %s, 0x%02x);" % (name, var(leaves[0]), var(leaves[1]),
                                                                         var(leaves[2]), tt))

nodes = len(live)
print("// aes_bs_sbox.h -- GENERATED by tools/gen_bs_sbox.py; do not edit.")
print("// Boyar-Peralta 113-gate AES S-box fused into %d 2- and 3-input" % nodes)
print("// gates (bop3 = one v_bitop3_b32).  x[b] = plane of bit b; the output is")
print("// S(x) ^ 0x63 (the circuit's four XNORs dropped, see aes_bs.h).")
print("#pragma once")
print("TG_BS_HD void sbox(uint32_t* x) {")
print("    const uint32_t " + ", ".join("U%d = x[%d]" % (i, 7 - i) for i in range(8)) + ";")
print("\n".join(lines))
for b in range(8):
    print("    x[%d] = o%d;" % (b, 7 - b))   # S0 is bit 7
print("}")
