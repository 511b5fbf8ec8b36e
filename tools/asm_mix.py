"""Instruction mix of the hottest loop of a kernel in a hipcc -save-temps .s file.

usage: python tools/asm_mix.py FILE.s SYMBOL_SUBSTRING [top]
Finds the kernel whose symbol contains SYMBOL_SUBSTRING, then the largest
basic-block cycle closed by a backward branch, and prints opcode counts.
"""
import collections
import re
import sys


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
    out = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            out.append((labels[m.group(2)], i))
    return out


def mix(body, a, b):
    c = collections.Counter()
    for l in body[a:b + 1]:
        m = re.match(r"^\s+([vsdgb][a-z_0-9]+)\b", l)
        if m:
            c[m.group(1)] += 1
    return c


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    body = kernel_lines(path, sub)
    ls = loops(body)
    if not ls:
        raise SystemExit("no loops")
    a, b = max(ls, key=lambda ab: sum(mix(body, *ab).values()))
    c = mix(body, a, b)
    print("loop lines %d-%d: %d instructions" % (a, b, sum(c.values())))
    for k, v in c.most_common(top):
        print("%6d  %s" % (v, k))
    cls = collections.Counter()
    for k, v in c.items():
        cls[k.split("_")[0] + ("_" + k.split("_")[1] if k.startswith(("ds", "global", "buffer")) else "")] += v
    print("by class:", dict(cls.most_common()))


if __name__ == "__main__":
    main()
