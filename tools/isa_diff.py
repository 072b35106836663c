"""Compare the gfx950 ISA of every kernel between two `hipcc --cuda-device-only -S` dumps of a source
file (e.g. before and after a source cleanup that must not change any remaining kernel):

    python tools/isa_diff.py BEFORE.s AFTER.s

Prints, per kernel symbol of AFTER: identical / changed (+ first differing line) / new, and the symbols
of BEFORE that are gone.  Basic-block and temporary label numbers (function-order dependent) and
comments are normalised away."""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+|\w+_kernel\w*):\s*(;.*)?$", line)
        if m and cur is None:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                out[cur] = body
                cur = None
                continue
            s = line.split(";")[0].rstrip()
            if not s.strip():
                continue
            s = re.sub(r"\.LBB\d+_", ".LBB_", s)
            s = re.sub(r"\.Ltmp\d+", ".Ltmp", s)
            body.append(s)
    return out


def main(a, b):
    ka, kb = kernels(a), kernels(b)
    same = changed = 0
    for k, v in kb.items():
        if k not in ka:
            print(f"NEW      {k[:90]}")
        elif ka[k] == v:
            same += 1
        else:
            changed += 1
            d = next((i for i, (x, y) in enumerate(zip(ka[k], v)) if x != y), min(len(ka[k]), len(v)))
            print(f"CHANGED  {k[:90]}  ({len(ka[k])} -> {len(v)} lines; first diff at {d}: "
                  f"{ka[k][d].strip() if d < len(ka[k]) else '<end>'} | {v[d].strip() if d < len(v) else '<end>'})")
    for k in ka:
        if k not in kb:
            print(f"REMOVED  {k[:90]}")
    print(f"{same} identical, {changed} changed, {len(kb) - same - changed} new, {len(set(ka) - set(kb))} removed")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
