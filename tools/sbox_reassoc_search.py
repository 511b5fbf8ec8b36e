"""Search XOR re-associations of the Boyar-Peralta S-box circuit that lower
the exact 3-input gate cover of tools/gen_bs_sbox.py (random hill climb: 1-3
moves (a ^ b) ^ c -> (a ^ c) ^ b or (b ^ c) ^ a, where a ^ b feeds only this
gate, kept when the minimum cover does not grow).  Each cover is a 0/1
program of ~20 s; round 2 ran seeds 11-14 x 150 steps (about an hour on four
cores), all ending at 72 gates (from 74), and took one of them as REASSOC;
annealing from that circuit (SBOX_FROM_REASSOC=1, seeds 21-24, uphill 0.25,
~75 minutes each) found nothing below 72.

    python3 tools/sbox_reassoc_search.py SEED STEPS [UPHILL] > gates.json

SBOX_CIRCUIT=bpd16 starts from Boyar and Peralta's depth-16 circuit instead
(tools/sbox_circuit_search.py circuit(); round 5).
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bs_sbox as gb  # noqa: E402


def cover_size(gates):
    order = gb.topo(gates)
    roots, _ = gb.min_cover(gates, order, time_limit=90)
    return len(roots)


def moves(gates):
    fan = {}
    for _, a, b in gates.values():
        fan[a] = fan.get(a, 0) + 1
        fan[b] = fan.get(b, 0) + 1
    out = []
    for n, (op, a, b) in gates.items():
        if op != "^":
            continue
        for x, c in ((a, b), (b, a)):
            if x in gates and gates[x][0] == "^" and fan.get(x, 0) == 1 and not x.startswith("S"):
                out.append((n, x, c) + gates[x][1:])
    return out


def apply(gates, m, which):
    n, x, c, p, q = m
    g = dict(gates)
    g[x], g[n] = (("^", p, c), ("^", x, q)) if which == 0 else (("^", q, c), ("^", x, p))
    return g


def main():
    seed, steps = int(sys.argv[1]), int(sys.argv[2])
    rng = random.Random(seed)
    cur = gb.parse(gb.CIRCUIT)
    if os.environ.get("SBOX_FROM_REASSOC"):   # continue from the shipped re-association
        cur.update(gb.parse(gb.REASSOC))
    if os.environ.get("SBOX_CIRCUIT"):
        import sbox_circuit_search as scs
        cur = scs.circuit(os.environ["SBOX_CIRCUIT"])
    best = cover_size(cur)
    print("start %d" % best, file=sys.stderr, flush=True)
    # annealing: a cover one gate larger is accepted with probability ``uphill``
    uphill = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    cur_c, top = best, cur
    for it in range(steps):
        g = cur
        for _ in range(rng.randint(1, 3)):
            g = apply(g, rng.choice(moves(g)), rng.randint(0, 1))
        c = cover_size(g)
        if c <= cur_c or (c == cur_c + 1 and rng.random() < uphill):
            cur, cur_c = g, c
            if c < best:
                print("step %d -> %d" % (it, c), file=sys.stderr, flush=True)
                best, top = c, g
    gb.check(top, gb.topo(top))
    json.dump({"gates": best, "circuit": {k: list(v) for k, v in top.items()}}, sys.stdout)


if __name__ == "__main__":
    main()
