#!/usr/bin/env python3
"""Per-function VALU/SALU/memory instruction histogram of a gfx950 .s file
(hipcc --offload-device-only -S): static instruction counts, used to compare
field-arithmetic variants before spending GPU time on them.

  python tools/isa_hist.py build/kernels.s [function-substring ...]
"""
import re
import sys
from collections import Counter


def functions(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^([_A-Za-z][\w.$]*):", line)
        if m and not m.group(1).startswith(".L"):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            t = line.split()
            if t and re.match(r"^[sv]_|^(global|buffer|scratch|ds|flat)_", t[0]):
                body.append(t[0])
    if cur:
        yield cur, body


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    for name, body in functions(path):
        if pats and not any(p in name for p in pats):
            continue
        if not body:
            continue
        c = Counter(body)
        print(f"== {name}: {len(body)} instrs, {sum(v for k, v in c.items() if k.startswith('v_'))} VALU")
        for k, v in c.most_common(14):
            print(f"   {v:6d} {k}")


if __name__ == "__main__":
    main()
