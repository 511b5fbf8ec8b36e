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

    python3 tools/sbox_circuit_search.py SEED COUNT [bottom|top|both] > log.jsonl
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bs_sbox as gb  # noqa: E402


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
        basis = ["Z%d" % i for i in range(18)]
        f = lin_forms(g, order, basis)
        targets = {"S%d" % i: f["S%d" % i] for i in range(8)}
        drop = [n for n in g if n in f and n not in basis and not n.startswith("Z")]
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
    rng = random.Random(seed)
    base = gb.parse(gb.CIRCUIT)
    if os.environ.get("SBOX_FROM_REASSOC"):
        base.update(gb.parse(gb.REASSOC))
    best, best_g = None, None
    for it in range(count):
        g = base
        eps = rng.choice([0.0, 0.05, 0.15])
        layers = ["bottom", "top"] if mode == "both" else [mode]
        for layer in layers:
            g = rebuild(g, layer, rng, eps)
        order = gb.topo(g)
        gb.check(g, order)
        roots, res = gb.min_cover(g, order, time_limit=120)
        n = len(roots)
        xor2 = sum(1 for v in g.values() if v[0] == "^")
        print(json.dumps({"seed": seed, "it": it, "mode": mode, "eps": eps, "xor2_gates": xor2,
                          "and_gates": sum(1 for v in g.values() if v[0] == "&"),
                          "cover": n, "optimal": res.status == 0}), flush=True)
        if best is None or n < best:
            best, best_g = n, g
    print(json.dumps({"best": best, "circuit": {k: list(v) for k, v in best_g.items()}}), flush=True)


if __name__ == "__main__":
    main()
