"""Issue-cost model of a kernel's hot loops from a hipcc -save-temps .s file.

usage: python tools/issue_model.py FILE.s SYMBOL_SUBSTRING [loops]

Finds the kernel whose symbol contains SYMBOL_SUBSTRING, takes its largest
innermost loops (basic-block cycles closed by a backward branch that hold no
other loop; ``loops`` of them, default 3) and prints, per loop, the VALU instructions by gfx950 issue class
and the LDS / global instructions, then the average SIMD cycles per VALU
instruction of their union.  Issue classes (wave64 on a 32-lane SIMD; rates
measured by tools/issue_probe3.hip):

  fast (2 cycles)   v_add_u32, v_xor_b32, v_or_b32, v_and_b32, v_lshrrev_b32,
                    v_bitop3_b32 with VGPR operands, v_mov, v_cndmask, ...
  half (4 cycles)   v_alignbit / v_alignbyte / v_perm, v_lshlrev_b32,
                    v_lshl_or / v_add3 / v_xad, multiplies, v_mad_*,
                    v_lshl_add_u64, v_pk_*, any VOP3 with an SGPR operand
                    (v_bitop3 / v_xor3 with an s register)

The model is the one DESIGN.md section 4 uses for the VALU ceiling: busy
cycles = sum over instructions of their class cost, per SIMD.
"""
import collections
import re
import sys

HALF_PREFIX = ("v_alignbit", "v_alignbyte", "v_perm", "v_lshlrev_b32", "v_lshl_or", "v_add3",
               "v_xad", "v_mul", "v_mad", "v_lshl_add", "v_pk_", "v_bfe", "v_bfi", "v_dot",
               "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64")
SGPR_HALF = ("v_bitop3", "v_xor3", "v_and_or", "v_or3")


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\w*:", l) and sub in l.split(":")[0]:
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found: " + sub)
    end = start
    while "s_endpgm" not in lines[end]:
        end += 1
    return lines[start:end + 1]


def loops(body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB[\w_]+):", l)
        if m:
            labels[m.group(1)] = i
    last = {}   # loop header -> its last backward branch (one loop per header)
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            last[labels[m.group(2)]] = i
    return sorted(last.items())


def classify(line):
    m = re.match(r"^\s+(v_\w+)\s+(.*)$", line)
    if not m:
        return None
    op, args = m.group(1), m.group(2)
    if op.startswith(HALF_PREFIX):
        return "half"
    if op.startswith(SGPR_HALF) and re.search(r"\bs\d+\b|\bs\[", args):
        return "half"
    return "fast"


def mix(body, a, b):
    c = collections.Counter()
    for l in body[a:b + 1]:
        k = classify(l)
        if k:
            c["valu_" + k] += 1
            continue
        m = re.match(r"^\s+((ds|global|buffer|scratch|s)_\w+)", l)
        if m:
            op = m.group(1)
            if op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_")):
                c["vmem"] += 1
            elif op.startswith("scratch_"):
                c["scratch"] += 1
            else:
                c["salu/smem"] += 1
    return c


def main():
    path, sub = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    body = kernel_lines(path, sub)
    allo = set(loops(body))
    inner = [(a, b) for a, b in allo if not any((c, d) != (a, b) and a <= c and d <= b for c, d in allo)]
    ls = sorted(inner, key=lambda ab: -sum(mix(body, *ab).values()))[:n]
    tot = collections.Counter()
    for a, b in ls:
        c = mix(body, a, b)
        tot += c
        v = c["valu_fast"] + c["valu_half"]
        print("loop lines %d-%d: %d VALU (%d fast, %d half), %d LDS, %d VMEM, %d scratch"
              % (a, b, v, c["valu_fast"], c["valu_half"], c["lds"], c["vmem"], c["scratch"]))
    v = tot["valu_fast"] + tot["valu_half"]
    if v:
        cyc = (2 * tot["valu_fast"] + 4 * tot["valu_half"]) / v
        print("all: %d VALU, %.1f %% half rate, %.2f SIMD cycles per VALU instruction"
              % (v, 100.0 * tot["valu_half"] / v, cyc))


if __name__ == "__main__":
    main()
