"""Generate csrc/aes_bs_sbox.h: Boyar and Peralta's 113-gate AES S-box circuit
(32 AND, 77 XOR, 4 XNOR; top linear layer Y*, nonlinear core T2..T45 / Z*,
bottom linear layer) covered by the fewest 2- and 3-input gates (any
3-input boolean function is one full-rate v_bitop3_b32 on gfx950).

* XOR chains of the circuit are re-associated (REASSOC, found by
  tools/sbox_reassoc_search.py: (a ^ b) ^ c -> (a ^ c) ^ b where a ^ b has
  one consumer); the gates keep Boyar-Peralta's names, not their meanings.
* The cover is an exact minimum-area 3-LUT mapping: every 3-feasible cut of
  every gate is enumerated and a 0/1 program (scipy.optimize.milp, HiGHS)
  picks the fewest materialised gates such that each one is computed from at
  most three inputs or materialised gates (a gate may be recomputed inside
  several covers).
* Both the rewritten circuit and the emitted cover are checked against the
  AES S-box for all 256 inputs before anything is written.

Round 1: the depth-16 128-gate circuit, greedy fusion, 84 gates; round 2:
this circuit with greedy fusion, 76; with the exact cover, 74; with the
re-association, 72.

    python3 tools/gen_bs_sbox.py > tlslite-ng_amd/csrc/aes_bs_sbox.h
"""
import itertools
import sys

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
REASSOC = """
Y21=Y13^T9 Y18=T16^T10 T4=T17^T2 T6=Y19^T2 T9=T14^T8 T11=Y18^U0 T17=T3^Y20 T18=T6^T5 T19=Y21^T7
T20=T11^T7 T21=T4^T14 T22=T18^T16 T23=T19^Y16 T24=T20^Y16 T37=T34^T36 T50=Z2^T53 T51=Z5^T66
T52=Z8^Z7 T54=Z3^Z7 T55=T67^Z16 T56=T62^T48 T57=T50^Z12 T59=T54^Z6 T61=T62^Z14 T65=T61^T57
S6=T56^Z12 S7=T60^T48 T67=Z17^T65 S4=T51^Z2 S2=T55^T64
"""
INPUTS = ["U%d" % i for i in range(8)]   # U0 = bit 7 ... U7 = bit 0


def parse(text):
    out = {}
    for tok in text.split():
        name, expr = tok.split("=")
        op = "^" if "^" in expr else "&"
        x, y = expr.split(op)
        out[name] = (op, x, y)
    return out


def topo(gates):
    done, out, pending = set(INPUTS), [], list(gates)
    while pending:
        rest = []
        for n in pending:
            if gates[n][1] in done and gates[n][2] in done:
                out.append(n)
                done.add(n)
            else:
                rest.append(n)
        if len(rest) == len(pending):
            raise ValueError("cyclic circuit")
        pending = rest
    return out


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


def check(gates, order):
    for v in range(256):
        env = {"U%d" % i: (v >> (7 - i)) & 1 for i in range(8)}
        for g in order:
            op, a, b = gates[g]
            env[g] = env[a] ^ env[b] if op == "^" else env[a] & env[b]
        assert sum(env["S%d" % i] << (7 - i) for i in range(8)) == _aes_sbox(v) ^ 0x63, v


def cuts_of(gates, order, k=3):
    """Non-trivial k-feasible cuts of every gate, dominated ones dropped."""
    cuts = {u: [frozenset([u])] for u in INPUTS}
    nontriv = {}
    for n in order:
        _, a, b = gates[n]
        cs = {c1 | c2 for c1 in cuts[a] for c2 in cuts[b] if len(c1 | c2) <= k}
        cs = sorted((c for c in cs if not any(o < c for o in cs)), key=sorted)
        nontriv[n] = cs
        cuts[n] = [frozenset([n])] + cs
    return nontriv


def min_cover(gates, order, time_limit=600):
    """Exact minimum number of materialised gates: x_n (gate n materialised),
    y_nc (n computed from cut c); sum_c y_nc = x_n, y_nc <= x_l for the gate
    leaves l of c, x = 1 at the outputs."""
    import numpy as np
    from scipy.optimize import Bounds, LinearConstraint, milp
    from scipy.sparse import coo_matrix
    nontriv = cuts_of(gates, order)
    idx = {("x", n): i for i, n in enumerate(order)}
    for n in order:
        for c in nontriv[n]:
            idx[("y", n, c)] = len(idx)
    ri, ci, vv, lo, hi = [], [], [], [], []

    def row(coefs, lb, ub):
        r = len(lo)
        for key, v in coefs:
            ri.append(r)
            ci.append(idx[key])
            vv.append(v)
        lo.append(lb)
        hi.append(ub)
    for n in order:
        row([(("y", n, c), 1) for c in nontriv[n]] + [(("x", n), -1)], 0, 0)
        for c in nontriv[n]:
            for leaf in c:
                if leaf in gates:
                    row([(("y", n, c), 1), (("x", leaf), -1)], -np.inf, 0)
        if n.startswith("S"):
            row([(("x", n), 1)], 1, 1)
    cost = np.zeros(len(idx))
    for n in order:
        cost[idx[("x", n)]] = 1
    res = milp(cost, constraints=LinearConstraint(coo_matrix((vv, (ri, ci)), shape=(len(lo), len(idx))).tocsr(),
                                                  lo, hi),
               integrality=np.ones(len(idx)), bounds=Bounds(0, 1), options={"time_limit": time_limit})
    if res.x is None:
        raise RuntimeError("milp: " + res.message)
    return {n: next(c for c in nontriv[n] if res.x[idx[("y", n, c)]] > 0.5)
            for n in order if res.x[idx[("x", n)]] > 0.5}, res


def cone(gates, n, leaves):
    """Expression tree of gate n down to the leaves of its cut."""
    op, a, b = gates[n]
    sub = [x if (x in leaves or x in INPUTS) else cone(gates, x, leaves) for x in (a, b)]
    return (op, sub[0], sub[1])


def leaves_of(t):
    if isinstance(t, str):
        return {t}
    return leaves_of(t[1]) | leaves_of(t[2])


def evaluate(t, env):
    if isinstance(t, str):
        return env[t]
    x, y = evaluate(t[1], env), evaluate(t[2], env)
    return x ^ y if t[0] == "^" else x & y


def key(v):
    return (v[0], int(v[1:]))


def var(n):   # outputs are emitted as o0..o7 (an output may feed another)
    return "o" + n[1:] if n.startswith("S") else n


def main():
    gates = parse(CIRCUIT)
    check(gates, topo(gates))
    gates.update(parse(REASSOC))
    order = topo(gates)
    check(gates, order)
    roots, res = min_cover(gates, order)
    if res.status != 0:
        print("warning: cover not proven optimal (%s)" % res.message, file=sys.stderr)
    trees = {n: cone(gates, n, roots[n]) for n in roots}
    lines = []
    for g in order:
        if g not in roots:
            continue
        t = trees[g]
        name = var(g)
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
    # the emitted cover itself, for all 256 inputs
    for v in range(256):
        env = {"U%d" % i: (v >> (7 - i)) & 1 for i in range(8)}
        for g in order:
            if g in roots:
                env[g] = evaluate(trees[g], env)
        assert sum(env["S%d" % i] << (7 - i) for i in range(8)) == _aes_sbox(v) ^ 0x63, v
    print("// aes_bs_sbox.h -- GENERATED by tools/gen_bs_sbox.py; do not edit.")
    print("// Boyar-Peralta 113-gate AES S-box, XOR-reassociated and covered by %d" % len(roots))
    print("// 2- and 3-input gates (bop3 = one v_bitop3_b32).  x[b] = plane of bit b;")
    print("// the output is S(x) ^ 0x63 (the circuit's four XNORs dropped, see aes_bs.h).")
    print("#pragma once")
    print("TG_BS_HD void sbox(uint32_t* x) {")
    print("    const uint32_t " + ", ".join("U%d = x[%d]" % (i, 7 - i) for i in range(8)) + ";")
    print("\n".join(lines))
    for b in range(8):
        print("    x[%d] = o%d;" % (b, 7 - b))   # S0 is bit 7
    print("}")


if __name__ == "__main__":
    main()
