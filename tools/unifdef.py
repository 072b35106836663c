"""Resolve compile-time A/B switches of the HIP sources to their shipped defaults (a minimal unifdef):

    python tools/unifdef.py FILE...      (rewrites the files in place)

`#if` / `#ifdef` / `#ifndef` / `#elif` / `#else` / `#endif` whose conditions involve only the macros in
DEFAULTS (defined, with that value) or UNDEFINED are evaluated and the dead branches dropped, the
`#ifndef M / #define M v / #endif` default blocks of those macros included; any other conditional is kept
verbatim.  Remaining uses of a resolved macro in code are replaced by its value.  Used to cut the A/B
alternatives no test builds; tools/isa_diff.py then checks that every remaining
kernel compiles to the same ISA as before."""
import re
import sys

DEFAULTS = {
    "PDG_EFWD_X6F": 0, "PDG_EFWD_CX6": 1, "PDG_EBW_XCD": 0, "PDG_EBF_ONLY": 0, "PDG_EK_NT": 0,
    "PDG_EEB_2DEEP": 1, "PDG_EEB_MASK": 1, "PDG_EFC_DEFER": 1, "PDG_EFC_XCD": 1,
    "PDG_NN_LATE_STAGE": 1, "PDG_NODE_NET_X6": 1, "PDG_NODE_NET_PAIR": 1, "PDG_NODE_PQ_X6": 1,
    "PDG_EF_PREFETCH": 1, "PDG_EF_EARLY": 1, "PDG_EF_NEXT": 1, "PDG_EB_EARLY_A1E": 0, "PDG_EDGE_X6": 1,
    "PDG_WGJ_2DEEP": 1, "PDG_WGP_2DEEP": 1, "PDG_WGRAD_GROUPS": 3, "PDG_NT_ST": 1, "PDG_NT_ROWS": 0,
    "PDG_X6_SWZ": 2,
}
UNDEFINED = {"PDG_WGRAD_F32", "PDG_NO_XCD_REMAP", "PDG_NT_LD"}
KNOWN = set(DEFAULTS) | UNDEFINED
IDENT = re.compile(r"\b[A-Za-z_]\w*\b")


def evaluate(expr: str):
    """Value of a preprocessor expression over KNOWN macros, or None when it names anything else."""
    expr = expr.split("//")[0].strip()
    expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in DEFAULTS else
                  ("0" if m.group(1) in UNDEFINED else f"__unknown_{m.group(1)}"), expr)
    names = set(IDENT.findall(expr)) - {"and", "or", "not"}
    if any(n not in DEFAULTS for n in names):
        return None
    py = expr.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    for n in names:
        py = re.sub(rf"\b{n}\b", str(DEFAULTS[n]), py)
    return bool(eval(py))


def process(text: str) -> str:
    out = []
    # stack entries: [resolved (bool), emitting_parent, taken, active]
    stack = []

    def emitting():
        return all(e[3] for e in stack if e[0]) and (not stack or stack[-1][1])

    for line in text.splitlines(keepends=True):
        s = line.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b\s*(.*)", s)
        if not m:
            if emitting():
                out.append(line)
            continue
        kw, rest = m.group(1), m.group(2)
        parent = emitting()
        if kw in ("ifdef", "ifndef"):
            name = rest.split()[0] if rest else ""
            if name in KNOWN:
                val = (name in DEFAULTS) == (kw == "ifdef")
                stack.append([True, parent, val, val])
            else:
                stack.append([False, parent, True, True])
                if parent:
                    out.append(line)
        elif kw == "if":
            val = evaluate(rest)
            if val is None:
                stack.append([False, parent, True, True])
                if parent:
                    out.append(line)
            else:
                stack.append([True, parent, val, val])
        elif kw == "elif":
            top = stack[-1]
            if top[0]:
                val = evaluate(rest)
                if val is None:
                    raise SystemExit(f"unresolvable #elif after a resolved #if: {s}")
                top[3] = (not top[2]) and val
                top[2] = top[2] or val
            else:
                if top[1]:
                    out.append(line)
        elif kw == "else":
            top = stack[-1]
            if top[0]:
                top[3] = not top[2]
                top[2] = True
            elif top[1]:
                out.append(line)
        else:   # endif
            top = stack.pop()
            if not top[0] and top[1]:
                out.append(line)
    res = "".join(out)
    for n, v in DEFAULTS.items():
        res = re.sub(rf"\b{n}\b", str(v), res)
    return res


if __name__ == "__main__":
    for path in sys.argv[1:]:
        src = open(path).read()
        new = process(src)
        if new != src:
            open(path, "w").write(new)
            print(f"{path}: {len(src.splitlines())} -> {len(new.splitlines())} lines")
