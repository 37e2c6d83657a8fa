#!/usr/bin/env python3
"""Instruction mix of one kernel in two device-assembly files (hipcc --offload-device-only -S):
tools/isa_mix.py OLD.s NEW.s KERNEL_SUBSTRING [NEW_KERNEL_SUBSTRING] - total counts, loop-body
counts (the largest basic-block run between a label and its backward branch is not attempted: the
whole function is counted) and every opcode whose count differs."""
import re
import sys
from collections import Counter


def kern(path, name):
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(name) + r"\S*):", s, re.M)
    if not m:
        raise SystemExit(f"{name} not in {path}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    return [l.strip().split()[0] for l in s[i:j].splitlines()
            if l.startswith("\t") and not l.strip().startswith((".", ";"))], m.group(1)


o, on = kern(sys.argv[1], sys.argv[3])
n, nn = kern(sys.argv[2], sys.argv[4] if len(sys.argv) > 4 else sys.argv[3])
print(on, "->", nn)
print("instructions", len(o), len(n))
co, cn = Counter(o), Counter(n)
for k in sorted(set(co) | set(cn)):
    if co[k] != cn[k]:
        print(f"{k:32s} {co[k]:5d} {cn[k]:5d}")
