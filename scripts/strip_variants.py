"""Resolve compile-time A/B switches to their shipped values in the engine sources (a small unifdef).

Each macro named in STRIP is treated as defined to its shipped value: `#if` / `#elif` conditions that
involve only such macros and integer literals are evaluated and their dead branches dropped, the
macro's own `#ifndef M / #define M v / #endif` default block is dropped, and remaining uses of M in code
are replaced by the value.  Conditions on any other macro are kept as they are.  The check that nothing
else changed: the preprocessed translation units (hipcc -E, host and device) are token-identical before
and after (scripts/strip_variants.py --check).

usage: python3 scripts/strip_variants.py [--check] file...
"""
import re
import subprocess
import sys

STRIP = {
    # measured, not kept (DESIGN.md and profiles/ name the A/B each one was)
    "H3C_AF_EARLY_OLD": 0, "H3C_AF_EXPERIMENT": 0, "H3C_AF_SKEW": 0, "H3C_AF_STATIC": 0, "H3C_FAST_FILL": 1,
    "H3C_FAST_GRAB": 1, "H3C_FX": 0, "H3C_LUT2": 1, "H3C_PERM_LAYOUT": 1, "H3C_SEG_ABS_ROWS": 1,
    "H3C_SEG_FOLD_TAB": 1, "H3C_SEG_FUSE_FIN": 1, "H3C_SMALL_EXP": 0, "H3C_UIO_FOLD_ILP": 0, "H3C_UIO_GRAB": 0,
    "H3C_UIO_IMG_NT": 0, "H3C_UIO_LATE_JOIN": 0, "H3C_UIO_SFIELDS": 1, "H3C_UIO_SOLO": 1, "H3C_UNI_DYNAMIC": 1,
    "H3C_UNI_PAIR": 0, "H3C_UPD_EXPERIMENT": 0, "H3C_UPD_SKEW": 0, "H3C_XOR3_ASM": 1, "H3C_AF_EARLY_FILL": 1,
    "H3C_UPD_EARLY_FILL": 1, "H3C_UIO_EARLY": 1, "H3C_UIO_SERIAL": 1, "H3C_AF_STORE_EARLY": 1, "H3C_SMALL_QUAD": 1,
    "H3C_UPD_WG_BAL": 1, "H3C_FAST_LPT": 1, "H3C_PINGPONG": 0,
    # printf traces no script uses (af_trace.py and fast_wg_trace.py use H3C_AF_TRACE / H3C_FAST_TRACE: kept)
    "H3C_BLOCK_TRACE": 0, "H3C_FRONT_TRACE": 0, "H3C_PB_TRACE": 0,
}
DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")
IDENT = re.compile(r"\b[A-Za-z_][A-Za-z0-9_]*\b")


def evaluate(expr):
    """True / False when the condition involves only STRIP macros and literals, else None."""
    e = re.sub(r"//.*$", "", expr)
    e = re.sub(r"/\*.*?\*/", "", e).strip()
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in STRIP else m.group(0), e)
    names = set(IDENT.findall(e))
    if not names <= set(STRIP):
        return None
    e = IDENT.sub(lambda m: str(STRIP[m.group(0)]), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    try:
        return bool(eval(e, {}))
    except Exception:
        return None


def strip(lines):
    out = []
    # stack entries: [kind, emit_now, taken, drop_directives]
    #   kind "known": every directive of the chain is dropped; emit_now = this branch is live
    #   kind "keep": directives kept; emit_now False for a branch found dead
    #   kind "default": the `#ifndef M` default block of a stripped macro (dropped whole)
    stack = []

    def live():
        return all(s[1] for s in stack)

    for line in lines:
        m = DIRECTIVE.match(line)
        if not m:
            w = line.split()
            if w[:1] == ["#define"] and len(w) > 1 and w[1] in STRIP:
                continue  # (a stripped macro's own definition)
            if live():
                out.append(subst(line))
            continue
        kw, rest = m.group(1), m.group(2)
        if kw in ("ifdef", "ifndef"):
            name = rest.split()[0] if rest.split() else ""
            if name in STRIP:
                stack.append(["known", kw == "ifdef", kw == "ifdef", True])
            else:
                stack.append(["keep", True, True, False])
                if live():
                    out.append(line)
            continue
        if kw == "if":
            v = evaluate(rest)
            if v is None:
                stack.append(["keep", True, True, False])
                if all(s[1] for s in stack[:-1]):
                    out.append(subst_directive(line))
            else:
                stack.append(["known", v, v, True])
            continue
        top = stack[-1]
        parent_live = all(s[1] for s in stack[:-1])
        if kw == "elif":
            v = evaluate(rest)
            if top[0] == "known":
                if top[2]:
                    top[1] = False
                elif v is None:
                    raise SystemExit(f"unresolvable #elif after resolved branches: {line.strip()}")
                else:
                    top[1], top[2] = v, v
            else:  # a kept chain
                if v is None:
                    top[1] = True
                    if parent_live:
                        out.append(subst_directive(line))
                elif v:
                    top[1] = True
                    if parent_live:
                        out.append(re.sub(r"#\s*elif.*$", "#else", line))
                    top[0] = "keep-else"
                else:
                    top[1] = False
            continue
        if kw == "else":
            if top[0] == "known":
                top[1] = not top[2]
            elif top[0] == "keep-else":
                top[1] = False
            else:
                top[1] = True
                if parent_live:
                    out.append(line)
            continue
        if kw == "endif":
            stack.pop()
            if top[0] != "known" and parent_live:
                out.append(line)
            continue
    if stack:
        raise SystemExit("unbalanced conditionals")
    return out


def subst(line):
    if "#define" in line or "#undef" in line:
        return IDENT.sub(lambda m: str(STRIP[m.group(0)]) if m.group(0) in STRIP else m.group(0), line)
    # code: replace macro uses (not inside // comments)
    code, sep, comment = line.partition("//")
    code = IDENT.sub(lambda m: str(STRIP[m.group(0)]) if m.group(0) in STRIP else m.group(0), code)
    return code + sep + comment


def subst_directive(line):
    return subst(line)


def preprocess(path, device):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-E", "-P", "-I", "include",
           "--cuda-device-only" if device else "--cuda-host-only", path]
    return re.findall(r"\S+", subprocess.run(cmd, check=True, capture_output=True, text=True).stdout)


def main():
    """Strips every file given; with --check, every .hip among them is preprocessed (host and device) before
    and after, and all files are restored unless every translation unit is token-identical."""
    args = sys.argv[1:]
    check = "--check" in args
    files = [a for a in args if a != "--check"]
    units = [f for f in files if f.endswith(".hip")]
    src = {f: open(f).read() for f in files}
    before = {(u, d): preprocess(u, d) for u in units for d in (False, True)} if check else {}
    for f in files:
        new = strip(src[f].split("\n"))
        open(f, "w").write("\n".join(new))
        print(f"{f}: {src[f].count(chr(10)) + 1} -> {len(new)} lines")
    for (u, d), toks in before.items():
        after = preprocess(u, d)
        if after != toks:
            for f in files:
                open(f, "w").write(src[f])
            bad = next(i for i, (a, b) in enumerate(zip(toks, after)) if a != b) if len(toks) == len(after) else -1
            raise SystemExit(f"{u}: preprocessed {'device' if d else 'host'} tokens differ (first at {bad}, "
                             f"{len(toks)} vs {len(after)} tokens); every file restored")
    if check:
        print("preprocessed translation units identical")


if __name__ == "__main__":
    main()
