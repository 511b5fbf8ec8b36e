"""Search other circuits for the bitsliced AES S-box's 3-input-gate cover
(VERDICT r04 item 2).  tools/gen_bs_sbox.py's 0/1 program is an exact cover
of ONE circuit; this tool re-synthesises the linear layers of Boyar and
Peralta's circuit and covers each candidate with the same program:

* bottom layer: the eight outputs S_i are XORs of the 18 products Z_k
  (rows of B below); a candidate is a randomised Paar network (repeatedly
  materialise a pair of signals that occurs together in the most targets,
  ties broken at random, optionally a random non-maximal pair with
  probability ``eps``), so the cover sees XOR trees BP's own SLP heuristic
  did not produce;
* top layer: the 22 linear signals the nonlinear core and the products read
  (Y1..Y21, T1-level combinations of U0..U7) re-synthesised the same way
  from the eight inputs;
* middle: BP's nonlinear core T2..T45 as published (the GF(2^4) inversion),
  optionally with its XOR chains re-associated at random.

Each candidate is checked against the AES S-box on all 256 inputs before it
is covered.  Output: one JSON line per candidate (seed, layer choice, cover
size) and the best circuit.

    python3 tools/sbox_circuit_search.py SEED COUNT [bottom|top|both|none] [CIRCUIT] > log.jsonl

CIRCUIT: bp113 (default; gen_bs_sbox.CIRCUIT), bp113r (with REASSOC, the
shipped 72-gate start) or bpd16 (Boyar and Peralta's depth-16, 128-gate
circuit, round 1's starting point); mode "none" covers the circuit as it is.
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bs_sbox as gb  # noqa: E402


# Boyar and Peralta, "A depth-16 circuit for the AES S-box" (2011): 128
# gates; S7..S0 here are output bits 7..0 (renamed below to this tool's
# S0 = bit 7 convention), the four XNORs written as XORs like CIRCUIT.
DEPTH16 = """
T1=U0^U3 T2=U0^U5 T3=U0^U6 T4=U3^U5 T5=U4^U6 T6=T1^T5 T7=U1^U2 T8=U7^T6 T9=U7^T7 T10=T6^T7
T11=U1^U5 T12=U2^U5 T13=T3^T4 T14=T6^T11 T15=T5^T11 T16=T5^T12 T17=T9^T16 T18=U3^U7 T19=T7^T18
T20=T1^T19 T21=U6^U7 T22=T7^T21 T23=T2^T22 T24=T2^T10 T25=T20^T17 T26=T3^T16 T27=T1^T12
M1=T13&T6 M2=T23&T8 M3=T14^M1 M4=T19&U7 M5=M4^M1 M6=T3&T16 M7=T22&T9 M8=T26^M6 M9=T20&T17
M10=M9^M6 M11=T1&T15 M12=T4&T27 M13=M12^M11 M14=T2&T10 M15=M14^M11 M16=M3^M2 M17=M5^T24
M18=M8^M7 M19=M10^M15 M20=M16^M13 M21=M17^M15 M22=M18^M13 M23=M19^T25 M24=M22^M23 M25=M22&M20
M26=M21^M25 M27=M20^M21 M28=M23^M25 M29=M28&M27 M30=M26&M24 M31=M20&M23 M32=M27&M31 M33=M27^M25
M34=M21&M22 M35=M24&M34 M36=M24^M25 M37=M21^M29 M38=M32^M33 M39=M23^M30 M40=M35^M36 M41=M38^M40
M42=M37^M39 M43=M37^M38 M44=M39^M40 M45=M42^M41 M46=M44&T6 M47=M40&T8 M48=M39&U7 M49=M43&T16
M50=M38&T9 M51=M37&T17 M52=M42&T15 M53=M45&T27 M54=M41&T10 M55=M44&T13 M56=M40&T23 M57=M39&T19
M58=M43&T3 M59=M38&T22 M60=M37&T20 M61=M42&T1 M62=M45&T4 M63=M41&T2
L0=M61^M62 L1=M50^M56 L2=M46^M48 L3=M47^M55 L4=M54^M58 L5=M49^M61 L6=M62^L5 L7=M46^L3 L8=M51^M59
L9=M52^M53 L10=M53^L4 L11=M60^L2 L12=M48^M51 L13=M50^L0 L14=M52^M61 L15=M55^L1 L16=M56^L0
L17=M57^L1 L18=M58^L8 L19=M63^L4 L20=L0^L1 L21=L1^L7 L22=L3^L12 L23=L18^L2 L24=L15^L9 L25=L6^L10
L26=L7^L9 L27=L8^L10 L28=L11^L14 L29=L11^L17
S7=L6^L24 S6=L16^L26 S5=L19^L28 S4=L6^L21 S3=L20^L22 S2=L25^L29 S1=L13^L27 S0=L6^L23
"""


def circuit(name):
    if name == "bpd16":
        g = gb.parse(DEPTH16)
        ren = {"S%d" % k: "S%d" % (7 - k) for k in range(8)}   # S_k = bit k -> S_(7-k)
        return {ren.get(n, n): (op, ren.get(a, a), ren.get(b, b)) for n, (op, a, b) in g.items()}
    g = gb.parse(gb.CIRCUIT)
    if name == "bp113r":
        g.update(gb.parse(gb.REASSOC))
    return g


def lin_forms(gates, order, basis):
    """Linear form (bitmask over ``basis``) of every XOR-only signal above the basis."""
    f = {b: 1 << i for i, b in enumerate(basis)}
    for n in order:
        op, a, c = gates[n]
        if op == "^" and a in f and c in f and n not in f:
            f[n] = f[a] ^ f[c]
    return f


def paar(targets, nbase, rng, eps):
    """Random-tie Paar XOR network: targets (name -> bitmask over nbase
    base signals) -> list of (new_name, left, right) with operands as base
    indices (int) or earlier new names; every target ends as one signal."""
    sig = [1 << i for i in range(nbase)]          # column masks of the current signals
    names = list(range(nbase))
    rows = {t: [j for j in range(nbase) if m >> j & 1] for t, m in targets.items()}
    out, k = [], 0
    # a target that already is a base signal needs no gate
    while True:
        cnt = {}
        for t, cols in rows.items():
            if len(cols) < 2:
                continue
            for x in range(len(cols)):
                for y in range(x + 1, len(cols)):
                    p = (cols[x], cols[y])
                    cnt[p] = cnt.get(p, 0) + 1
        if not cnt:
            break
        best = max(cnt.values())
        cands = [p for p, c in cnt.items() if c == best]
        if eps and rng.random() < eps:
            cands = list(cnt)
        a, b = rng.choice(cands)
        name = "N%d" % k
        k += 1
        out.append((name, names[a], names[b]))
        names.append(name)
        sig.append(sig[a] ^ sig[b])
        new = len(names) - 1
        for t, cols in rows.items():
            if a in cols and b in cols:
                cols.remove(a)
                cols.remove(b)
                cols.append(new)
    final = {t: names[cols[0]] for t, cols in rows.items()}
    return out, final


def rebuild(base_gates, layer, rng, eps):
    """A copy of the circuit with one linear layer re-synthesised."""
    g = dict(base_gates)
    order = gb.topo(g)
    if layer == "bottom":
        # the products that only XORs follow (BP113's Z0..Z17, depth-16's M46..M63)
        users = {}
        for n, (op, a, c) in g.items():
            users.setdefault(a, []).append(n)
            users.setdefault(c, []).append(n)

        def xor_only(n):
            return all(g[u][0] == "^" and xor_only(u) for u in users.get(n, []))
        basis = sorted((n for n, v in g.items() if v[0] == "&" and xor_only(n)), key=gb.key)
        f = lin_forms(g, order, basis)
        targets = {"S%d" % i: f["S%d" % i] for i in range(8)}
        drop = [n for n in g if n in f and n not in basis]
    else:   # top: every XOR-only function of U0..U7 that the rest of the circuit reads
        basis = gb.INPUTS
        f = lin_forms(g, order, basis)
        lin = [n for n in f if n not in basis]
        readers = set()
        for n, (op, a, c) in g.items():
            if n not in f:
                readers.update(x for x in (a, c) if x in f and x not in basis)
        targets = {n: f[n] for n in readers}
        drop = lin
    for n in drop:
        del g[n]
    net, final = paar(targets, len(basis), rng, eps)
    ren = {}
    for name, a, b in net:
        ren[name] = "L%s%s" % (layer[0], name[1:])
    for name, a, b in net:
        x = basis[a] if isinstance(a, int) else ren[a]
        y = basis[b] if isinstance(b, int) else ren[b]
        g[ren[name]] = ("^", x, y)
    # targets: alias each to its final signal (a target equal to a base
    # signal or another target's signal gets a copy through a rename)
    alias = {}
    for t, s in final.items():
        s = basis[s] if isinstance(s, int) else ren[s]
        alias[t] = s
    # rewrite readers of the dropped targets to their aliases; outputs keep names
    for n, (op, a, c) in list(g.items()):
        g[n] = (op, alias.get(a, a) if not a.startswith("S") else a,
                alias.get(c, c) if not c.startswith("S") else c)
    if layer == "bottom":
        for t, s in alias.items():   # S_i must exist as a gate
            if s in g and not s.startswith("S"):
                g[t] = g.pop(s)
                for n, (op, a, c) in list(g.items()):
                    g[n] = (op, t if a == s else a, t if c == s else c)
    return g


def main():
    seed, count = int(sys.argv[1]), int(sys.argv[2])
    mode = sys.argv[3] if len(sys.argv) > 3 else "bottom"
    cname = sys.argv[4] if len(sys.argv) > 4 else ("bp113r" if os.environ.get("SBOX_FROM_REASSOC") else "bp113")
    rng = random.Random(seed)
    base = circuit(cname)
    best, best_g = None, None
    for it in range(count):
        g = base
        eps = rng.choice([0.0, 0.05, 0.15])
        layers = ["bottom", "top"] if mode == "both" else [] if mode == "none" else [mode]
        for layer in layers:
            g = rebuild(g, layer, rng, eps)
        order = gb.topo(g)
        gb.check(g, order)
        roots, res = gb.min_cover(g, order, time_limit=120)
        n = len(roots)
        xor2 = sum(1 for v in g.values() if v[0] == "^")
        print(json.dumps({"seed": seed, "it": it, "circuit": cname, "mode": mode, "eps": eps, "xor2_gates": xor2,
                          "and_gates": sum(1 for v in g.values() if v[0] == "&"),
                          "cover": n, "optimal": res.status == 0}), flush=True)
        if best is None or n < best:
            best, best_g = n, g
    print(json.dumps({"best": best, "circuit": {k: list(v) for k, v in best_g.items()}}), flush=True)


if __name__ == "__main__":
    main()
