"""Per-basic-block opcode counts of one kernel in a hipcc -save-temps .s file:
the big blocks (loop bodies) with their VALU / LDS / SGPR-operand mix.

    python tools/asm_blocks.py FILE.s SYMBOL_SUBSTRING [min_valu]
"""
import re
import sys
from collections import Counter

HALF = ("v_perm_b32", "v_alignbit_b32", "v_alignbyte_b32", "v_lshlrev_b32", "v_lshl_or_b32",
        "v_add3_u32", "v_xad_u32", "v_mad_u32_u24", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
        "v_lshl_add_u32", "v_pk_add_u16", "v_lshl_add_u64", "v_bfe_u32", "v_and_or_b32", "v_or3_b32")


def blocks(path, sub):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if sub in l and l.split(":")[0].endswith(l.split(":")[0])
                 and not l.startswith("\t") and l.rstrip().endswith(sub.split()[-1]) is False
                 and ":" in l and not l.startswith(" ") and not l.startswith(";") and l.find(sub) == 0
                 or (l.startswith("_Z") and sub in l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    out, cur = [], None
    for i in range(start, end):
        l = lines[i]
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m or cur is None:
            cur = [i + 1, m.group(1) if m else "entry", []]
            out.append(cur)
            continue
        s = l.strip()
        if s and not s.startswith(";") and not s.startswith("."):
            cur[2].append(s)
    return out


def reads_sgpr(ins):
    """True if a VALU instruction reads an SGPR source (not vcc / exec, not the
    carry-out SGPR destination of the _co_ and 64-bit mad forms)."""
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return False
    ops = [o.strip() for o in parts[1].split(",")]
    srcs = ops[2:] if ("_co_" in parts[0] or "mad_u64" in parts[0] or "mad_i64" in parts[0]) else ops[1:]
    return any(re.match(r"s(\d+|\[)", o) for o in srcs)


def main():
    path, sub = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    for line, name, ins in blocks(path, sub):
        ops = [s.split()[0] for s in ins]
        valu = [s for s in ins if s.startswith("v_")]
        if len(valu) < mn:
            continue
        half = sum(1 for s in valu if s.split()[0].split("_e")[0] in HALF)
        # any VALU reading an SGPR issues at half rate on gfx950 (VOP2 included;
        # a literal does not: profiles/r04/probe4.txt)
        sgpr3 = sum(1 for s in valu if reads_sgpr(s))
        lit = sum(1 for s in valu if s.startswith("v_bitop3") and re.search(r",\s*(0x[0-9a-f]+|-?\d+)\s", s))
        ds = sum(1 for o in ops if o.startswith("ds_"))
        c = Counter(o for o in ops if o.startswith("v_") or o.startswith("ds_"))
        print("line %d %s: VALU %d (half-rate opcodes %d, with an SGPR operand %d, bitop3 with literal %d), DS %d"
              % (line, name, len(valu), half, sgpr3, lit, ds))
        print("   ", ", ".join("%s %d" % kv for kv in c.most_common(10)))


if __name__ == "__main__":
    main()
