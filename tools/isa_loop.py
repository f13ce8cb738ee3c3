#!/usr/bin/env python3
"""Instruction mix of a kernel's largest loop in a hipcc --save-temps .s file:
tools/isa_loop.py <file.s> <kernel-name-regex>...
ISA_LOOP_RANK=k picks the k-th largest innermost loop instead (a kernel that
inlines two variants of its iteration loop, e.g. decode_small_kernel's
finite / non-finite sum-product forms, has one loop per variant)."""
import collections
import os
import re
import sys


def loop_mix(s, pat):
    m = re.search(r"^(\S*%s\S*):" % pat, s, re.M)
    start = m.end()
    body = s[start:s.index(".Lfunc_end", start)]
    lines = [l.strip() for l in body.split("\n")]
    labels = {}
    for i, l in enumerate(lines):
        lm = re.match(r"^(\.LBB\d+_\d+):", l)
        if lm:
            labels[lm.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        mm = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            loops.append((labels[mm.group(1)], i))
    # the iteration loop: the loop with the most f64 / VALU work that
    # contains no other loop
    def work(a, b):
        return sum(1 for l in lines[a:b] if l.startswith("v_"))
    inner = [(a, b) for a, b in loops
             if not any((a2 > a or b2 < b) and a <= a2 and b2 <= b for a2, b2 in loops)]
    inner.sort(key=lambda ab: -work(*ab))
    rank = int(os.environ.get("ISA_LOOP_RANK", "0"))  # 1: the second-largest loop, ...
    a, b = inner[min(rank, len(inner) - 1)]
    ins = [l.split()[0] for l in lines[a:b]
           if l and not l.startswith((".", ";", "s_nop")) and not re.match(r"^\S+:", l)]
    return m.group(1), collections.Counter(ins)


if __name__ == "__main__":
    s = open(sys.argv[1]).read()
    for pat in sys.argv[2:]:
        name, c = loop_mix(s, pat)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        f64 = sum(v for k, v in c.items() if k.startswith("v_") and "f64" in k)
        salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith("s_waitcnt"))
        ds = sum(v for k, v in c.items() if k.startswith("ds_"))
        print("%s\n  loop valu %d f64 %d salu %d ds %d waitcnt %d" %
              (name[:70], valu, f64, salu, ds, c["s_waitcnt"]))
        print("  ", c.most_common(16))
