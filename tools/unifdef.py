"""Resolve compile-time variant switches in csrc/ to their product values (a small unifdef).

    python tools/unifdef.py [--write] FILE...

Knob guards (`#ifndef X` / `#define X v` / `#endif`, comment lines allowed inside) become a plain
`#define X v` when X is still referenced elsewhere, and vanish otherwise.  Every `#if` /
`#ifdef` / `#ifndef` / `#elif` whose expression depends only on known macros (the knobs'
defaults, and the forced values below) is resolved: the losing branches are deleted, the
winner kept without its directives.  Conditions on unknown macros stay as they are.

The check that this changed nothing is the kernels' ISA: tools/isa_diff.sh disassembles the
code objects of two liborbx.so builds and compares them kernel by kernel.
"""
from __future__ import annotations

import pathlib
import re
import sys

# macros a product build never defines (diagnostics, tuning overrides)
FORCED_UNDEF = {"ORBX_TUNING", "FAST_COMPASS_PK", "ORBX_STAMPS", "ORBX_OCT_STAMPS", "ORBX_CHAIN_STAMPS"}
# macros whose value is fixed to the product one even though a guard would let a build change it
FORCED = {"OD_DIAG": 0, "ST_DIAG": 0, "FAST_DIAG": 0, "STRIP_DIAG": 0, "LEVEL_DIAG": 0,
          "CHAIN_DIAG": 0, "LEVEL_FORCE_GENERIC": 0}
# guards that stay (values a build passes on purpose)
KEEP = {"ORBX_SRC_HASH"}

DIR = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")
DEF = re.compile(r"^\s*#\s*define\s+([A-Za-z_]\w*)\s*(.*)$")


def strip_comment(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s)
    return s.split("//")[0].strip()


def knob_guards(lines):
    """Indices (i_ifndef, i_define, i_endif, name, value) of `#ifndef X / #define X v / #endif`."""
    out = []
    i = 0
    while i < len(lines):
        m = DIR.match(lines[i])
        if m and m.group(1) == "ifndef":
            name = strip_comment(m.group(2))
            j = i + 1
            d = None
            ok = True
            while j < len(lines):
                mj = DIR.match(lines[j])
                if mj:
                    ok = mj.group(1) == "endif"
                    break
                md = DEF.match(lines[j])
                if md:
                    if d is not None or md.group(1) != name:
                        ok = False
                        break
                    d = j
                elif lines[j].strip() and not lines[j].strip().startswith("//"):
                    ok = False
                    break
                j += 1
            if ok and d is not None and j < len(lines) and name not in KEEP:
                val = strip_comment(DEF.match(lines[d]).group(2))
                out.append((i, d, j, name, val))
                i = j + 1
                continue
        i += 1
    return out


def to_value(v: str):
    try:
        return int(v, 0)
    except ValueError:
        return None


def evaluate(expr: str, table: dict):
    """True / False, or None when the expression names a macro outside the table."""
    e = strip_comment(expr)
    unknown = False

    def dfn(m):
        nonlocal unknown
        n = m.group(1) or m.group(2)
        if n in table:
            return "1" if table[n] is not None else "0"
        unknown = True
        return "0"

    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)", dfn, e)

    def ident(m):
        nonlocal unknown
        n = m.group(0)
        if n in table:
            v = table[n]
            if v is None:
                return "0"
            iv = to_value(str(v))
            if iv is None:
                unknown = True
                return "0"
            return str(iv)
        unknown = True
        return "0"

    e = re.sub(r"\b[A-Za-z_]\w*\b", ident, e)
    if unknown:
        return None
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    try:
        return bool(eval(e, {}, {}))
    except Exception:
        return None


def process(text: str, table: dict, refs: set) -> str:
    lines = text.split("\n")
    guards = knob_guards(lines)
    drop = set()
    replace = {}
    for (i, d, j, name, val) in guards:
        drop.update(range(i, j + 1))
        if name in refs:
            replace[i] = lines[d]  # the define, without its guard (comments after it go too)
            # keep comment lines that sat inside the guard
            extra = [lines[k] for k in range(i + 1, j) if k != d]
            replace[i] = "\n".join([lines[d]] + extra)
    body = []
    for k, ln in enumerate(lines):
        md = DEF.match(ln)
        if k in replace:
            body.append(replace[k])
        elif k in drop:
            continue
        elif md and md.group(1) in table and md.group(1) not in refs:
            continue  # a knob define nothing reads any more
        else:
            body.append(ln)
    lines = "\n".join(body).split("\n")

    out = []
    # stack entries: dict(active_parent, taken, emitted, cur_keep)
    stack = []

    def keeping():
        return all(s["cur_keep"] for s in stack)

    for ln in lines:
        m = DIR.match(ln)
        if not m:
            if keeping():
                out.append(ln)
            continue
        kind, rest = m.group(1), m.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            name = strip_comment(rest)
            if kind == "ifdef":
                v = evaluate(f"defined({name})", table)
            elif kind == "ifndef":
                v = evaluate(f"defined({name})", table)
                v = None if v is None else (not v)
            else:
                v = evaluate(rest, table)
            parent = keeping()
            st = {"parent": parent, "taken": False, "emitted": False, "cur_keep": False}
            stack.append(st)
            if v is True:
                st["taken"] = True
                st["cur_keep"] = True
            elif v is False:
                st["cur_keep"] = False
            else:
                st["emitted"] = True
                st["cur_keep"] = True
                if parent:
                    out.append(ln)
        elif kind == "elif":
            st = stack[-1]
            if st["taken"]:
                st["cur_keep"] = False
                continue
            v = evaluate(rest, table)
            if v is False:
                st["cur_keep"] = False
            elif v is True:
                st["taken"] = True
                st["cur_keep"] = True
                if st["emitted"] and st["parent"]:
                    out.append(re.sub(r"#\s*elif\b.*", "#else", ln))
            else:
                st["cur_keep"] = True
                if st["parent"]:
                    if st["emitted"]:
                        out.append(ln)
                    else:
                        out.append(re.sub(r"#\s*elif\b", "#if", ln))
                st["emitted"] = True
        elif kind == "else":
            st = stack[-1]
            if st["taken"]:
                st["cur_keep"] = False
                continue
            st["taken"] = True
            st["cur_keep"] = True
            if st["emitted"] and st["parent"]:
                out.append(ln)
        else:  # endif
            st = stack.pop()
            if st["emitted"] and st["parent"]:
                out.append(ln)
    assert not stack, "unbalanced conditionals"
    return "\n".join(out)


def main(argv):
    write = "--write" in argv
    files = [pathlib.Path(a) for a in argv if not a.startswith("--")]
    texts = {f: f.read_text() for f in files}
    table = {n: None for n in FORCED_UNDEF}
    table.update({k: str(v) for k, v in FORCED.items()})
    for f, t in texts.items():
        for (_, _, _, name, val) in knob_guards(t.split("\n")):
            table.setdefault(name, val)
    # iterate: resolving conditions can drop the last reference of a knob
    for _ in range(4):
        allt = "\n".join(texts.values())
        refs = set()
        for name in table:
            n_ref = len(re.findall(r"\b%s\b" % re.escape(name), allt))
            n_def = len(re.findall(r"#\s*(?:define|ifndef)\s+%s\b" % re.escape(name), allt))
            if n_ref - n_def > 0:
                refs.add(name)
        new = {f: process(t, table, refs) for f, t in texts.items()}
        if new == texts:
            break
        texts = new
    for f, t in texts.items():
        if write:
            f.write_text(t)
        n = len(re.findall(r"^\s*#\s*if", t, re.M))
        print(f"{f}: {n} conditionals")


if __name__ == "__main__":
    main(sys.argv[1:])
